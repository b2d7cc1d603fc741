#!/bin/bash
# rocprofv3 kernel trace of one bench workload.  Usage: tools/gpu_prof_workload.sh TAG WORKLOAD [bench args]
set -u
TAG=$1; W=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$W
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 -u bench.py --workload $W --no-cpu-baseline --no-end-to-end "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/run_kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:12]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs'])/1e6:9.3f} pct={float(r['Percentage']):6.2f}")
PY
