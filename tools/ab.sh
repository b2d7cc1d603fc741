#!/bin/bash
# Same-box A/B of library variants (tools/build_variant.py builds libcobrix_hip_<name>.so).  Usage:
#   tools/ab.sh TAG "W[:args] ..." VARIANT...      (VARIANT "-" = the product library)
# Every workload runs once per variant, variants interleaved, twice over (the second pass in reverse
# variant order: the first run of a pair tends to be slower); one bench line each
# (5 steps, no CPU baseline / end-to-end).  Each GPU step has its own time limit; stops at a failure.
set -u
TAG=$1; WL=$2; shift 2
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOTDIR
for rep in 1 2; do
  for S in $WL; do
    W=${S%%:*}; EXTRA=""; NAME=$W
    if [ "$S" != "$W" ]; then EXTRA=$(echo ${S#*:} | tr ',' ' '); NAME=${W}$(echo ${S#*:} | tr -d '-' | tr ', ' '__'); fi
    VS=("$@"); [ $rep -eq 2 ] && VS=($(printf '%s\n' "$@" | tac))
    for V in "${VS[@]}"; do
      if [ "$V" = "-" ]; then unset CBX_LIB_VARIANT; else export CBX_LIB_VARIANT=$V; fi
      F=$OUT/${NAME}_${V/-/prod}_$rep
      timeout -k 10 400 python -u bench.py --workload $W $EXTRA --steps 8 --warmup 2 --no-cpu-baseline --no-end-to-end > $F.json 2> $F.err || { tail -8 $F.err; exit 1; }
      python3 -c "import json; d=json.load(open('$F.json')); print('$NAME', '$V', $rep, d['ms_per_step'], d.get('kernel_ms'), d['roofline']['frac'])"
    done
  done
done
echo AB_OK
