#!/bin/bash
# Round-4 A/B: C3 (50 M records) views + Utf8 with env variants ($@: "NAME=VALUE ..." specs, one per run).
set -u
mkdir -p gpurun_out
for V in "$@"; do
  for S in views offsets; do
    env $V timeout -k 10 300 python -u bench.py --workload synstr200 --records 50000000 --strings $S --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$V', '$S', d['ms_per_step'], d['roofline']['frac'])"
  done
done
