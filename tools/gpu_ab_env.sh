#!/bin/bash
# Decode time of bench workloads under environment settings (tuning A/B in one GPU call).
# Usage: tools/gpu_ab_env.sh "ENV=V ..." "ENV=V ..." -- WORKLOAD...   ("-" = no setting; "lib:NAME" = CBX_LIB_VARIANT)
set -u
SETS=()
while [ "$1" != "--" ]; do SETS+=("$1"); shift; done
shift
mkdir -p gpurun_out
for W in "$@"; do
  for round in 1 2; do
    for S in "${SETS[@]}"; do
      E=""; [ "$S" != "-" ] && E="$S"
      E=${E/lib:/CBX_LIB_VARIANT=}
      env $E timeout -k 10 200 python -u bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/abe.json 2>gpurun_out/abe.err || { echo "bench $W [$S] failed"; tail -5 gpurun_out/abe.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/abe.json')); print('$W', '[$S]', $round, d['ms_per_step'], round(d['kernel_ms']['decode_kernel'],3), d['roofline']['kernel'][:22])"
    done
  done
done
