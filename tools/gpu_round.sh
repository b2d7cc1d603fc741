#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprof profile.  Usage: tools/gpu_round.sh TAG [bench args...]
set -u
TAG=${1:-r01}; shift || true
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || { echo "bench failed rc=$rc"; tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
bash tools/gpu_profile.sh $TAG 50000000
