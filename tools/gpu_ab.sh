#!/bin/bash
# A/B timing of two library builds in one GPU call: tools/gpu_ab.sh VARIANT WORKLOAD [bench args]
# (VARIANT: cobrix_amd/libcobrix_hip_<VARIANT>.so from tools/build_variant.py; "cur" = the product build)
set -u
V=$1; W=$2; shift 2
mkdir -p gpurun_out
for round in 1 2; do
  for lib in $V cur; do
    if [ "$lib" = cur ]; then unset CBX_LIB_VARIANT; else export CBX_LIB_VARIANT=$lib; fi
    timeout -k 10 200 python -u bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end "$@" > gpurun_out/ab_${lib}_$round.json 2>/dev/null || { echo "bench $lib failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${lib}_$round.json')); print('$lib', $round, d['ms_per_step'], d['kernel_ms'])"
  done
done
