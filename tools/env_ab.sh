#!/bin/bash
# Same-box A/B of an environment knob: tools/env_ab.sh TAG VAR "W ..." -- each workload once with VAR
# unset and once with VAR=1, twice over (the second pass in reverse order); bench lines under gpurun_out/TAG.
set -u
TAG=$1; VAR=$2; WL=$3
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for W in $WL; do
    VS="off on"; [ $rep -eq 2 ] && VS="on off"
    for V in $VS; do
      if [ $V = on ]; then export $VAR=1; else unset $VAR; fi
      F=$OUT/${W}_${V}_$rep
      timeout -k 10 400 python -u bench.py --workload $W --steps 8 --warmup 2 --no-cpu-baseline --no-end-to-end > $F.json 2> $F.err || { tail -5 $F.err; exit 1; }
      python3 -c "import json; d=json.load(open('$F.json')); k=d['kernel_ms']; fr=[v for kk,v in k.items() if 'framing' in kk]; print('$W', '$V', $rep, d['ms_per_step'], round(fr[0],3) if fr else None, round(k['decode_kernel'],3))"
    done
  done
done
unset $VAR
echo AB_OK
