set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/jit_check.py syn200 views && timeout -k 10 120 python tools/jit_check.py synstr200 views && timeout -k 10 120 python tools/jit_check.py syn200 && \
timeout -k 10 200 python -u bench.py --workload syn200 --strings offsets --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/b_off.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --workload syn200 --strings views --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/b_view.json 2>/dev/null && \
python3 -c "
import json
for f in ['gpurun_out/b_off.json','gpurun_out/b_view.json']:
    d=json.load(open(f)); print(f, d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
