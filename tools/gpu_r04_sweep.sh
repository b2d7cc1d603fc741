#!/bin/bash
# Same-box knob sweep: each spec "workload|bench args|ENV=V" -> decode ms, frac, step ms.
set -u
mkdir -p gpurun_out/r04_sweep
i=0
for spec in "$@"; do
  i=$((i+1))
  W=$(echo "$spec" | cut -d'|' -f1); A=$(echo "$spec" | cut -d'|' -f2); E=$(echo "$spec" | cut -d'|' -f3)
  env $E timeout -k 10 300 python3 bench.py --workload $W $A --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/r04_sweep/$i.json 2> gpurun_out/r04_sweep/$i.err || { echo "$spec failed"; tail -5 gpurun_out/r04_sweep/$i.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r04_sweep/$i.json') if l.startswith('{')][-1]); print('$spec', d['kernel_ms']['decode_kernel'], d['roofline']['frac'], d['ms_per_step'])"
done
