#!/bin/bash
# Round-4: C2 (SYN200) cooperative-tile check: dump the specialised sources, parity tests, bench A/B.
set -u
mkdir -p gpurun_out/jit2
CBX_JIT_DUMP=gpurun_out/jit2 timeout -k 10 300 python -u bench.py --records 2000000 --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/jit2/b.log 2>&1 || { tail -5 gpurun_out/jit2/b.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "syn200 or fuzz or specialised or synstr200" > gpurun_out/t_f.log 2>&1
rc=$?; tail -3 gpurun_out/t_f.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/t_f.log | head; exit $rc; }
for V in X=0 CBX_NO_COOP=1; do
  env $V timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -5 gpurun_out/c2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c2.json')); print('$V', d['ms_per_step'], d['roofline']['frac'])"
done
