#!/bin/bash
# GPU parity tests + short bench lines (no CPU baseline / end-to-end).  Usage: tools/gpu_quick.sh TAG [workloads...]
set -u
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests -m gpu ${GPU_X--x} -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests_$TAG.log | head; exit $rc; }
for W in "$@"; do
  timeout -k 10 200 python -u bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/bq_${TAG}_$W.json 2> gpurun_out/bq_${TAG}_$W.err || { tail -5 gpurun_out/bq_${TAG}_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bq_${TAG}_$W.json')); print('$W', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
