#!/bin/bash
# Round-4: per-kernel times (rocprofv3 --stats) of C3 Utf8 at 50 M records for env variants ($@).
set -u
ROOTDIR=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $ROOTDIR
i=0
for V in "$@"; do
  i=$((i+1)); D=gpurun_out/g$i; mkdir -p $D
  env $V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 -u bench.py --workload synstr200 --records 50000000 --strings offsets --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $D/b.json 2> $D/b.err || { tail -5 $D/b.err; exit 1; }
  echo "== $V $(python3 -c "import json; d=json.load(open('$D/b.json')); print(d['ms_per_step'])")"
  python3 - $D <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "cbx" in r["Name"]:
        print(f"  {r['Name'][:40]:40s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:.4f}")
PY
done
