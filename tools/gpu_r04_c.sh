#!/bin/bash
# Round-4: C3 bench lines first (views, Utf8; optional env A/B via $1), then string parity tests.
set -u
mkdir -p gpurun_out
for S in views offsets; do
  timeout -k 10 300 python -u bench.py --workload synstr200 --records 50000000 --strings $S --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/c3_$S.json 2> gpurun_out/c3_$S.err || { tail -5 gpurun_out/c3_$S.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c3_$S.json')); print('$S', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_rdw.py tests/test_gpu_arrow_device.py -x -q --timeout 300 --timeout-method thread \
  -k "two_byte or synstr200 or var_span or fuzz or test10 or test1b or test24 or test9 or device_export or utf8 or string" > gpurun_out/t_r04c.log 2>&1
rc=$?; tail -3 gpurun_out/t_r04c.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/t_r04c.log | head -20; exit $rc; }
