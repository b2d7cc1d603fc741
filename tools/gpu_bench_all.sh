#!/bin/bash
# GPU parity tests + one bench line per BASELINE workload.  Usage: tools/gpu_bench_all.sh TAG
set -u
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error" gpurun_out/gpu_tests_$TAG.log | head -20; exit $rc; }
for W in syn200 synstr200 rdw_narrow wide_odo; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err
  rc=$?; cat gpurun_out/bench_${TAG}_$W.json
  [ $rc -eq 0 ] || { echo "bench $W failed rc=$rc"; tail -20 gpurun_out/bench_${TAG}_$W.err; exit $rc; }
done
echo ALL_OK
