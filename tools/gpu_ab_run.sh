#!/bin/bash
# A/B of the product build against a variant (tools/build_variant.py) on bench workloads, alternating.
# Usage: tools/gpu_ab_run.sh VARIANT WORKLOAD...
set -u
V=$1; shift
mkdir -p gpurun_out
for W in "$@"; do
  for round in 1 2; do
    for lib in $V cur; do
      if [ "$lib" = cur ]; then unset CBX_LIB_VARIANT; else export CBX_LIB_VARIANT=$lib; fi
      timeout -k 10 200 python -u bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/ab_${W}_${lib}_$round.json 2>gpurun_out/ab_${W}_${lib}_$round.err || { echo "bench $W $lib failed"; tail -5 gpurun_out/ab_${W}_${lib}_$round.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab_${W}_${lib}_$round.json')); print('$W', '$lib', $round, d['ms_per_step'], d['kernel_ms'], d['roofline']['kernel'][:30])"
    done
  done
done
