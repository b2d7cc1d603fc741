#!/bin/bash
# Occupancy-hint sweep of the specialised kernel on one workload.  Usage: tools/gpu_wpe.sh WORKLOAD
set -u
W=${1:-syn200}
mkdir -p gpurun_out
for N in 0 3 4; do
  CBX_JIT_WAVES_PER_EU=$N timeout -k 10 200 python -u bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/wpe_${W}_$N.json 2> gpurun_out/wpe_${W}_$N.err || { tail -5 gpurun_out/wpe_${W}_$N.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/wpe_${W}_$N.json')); print('$W wpe=$N', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
