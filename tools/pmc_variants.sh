#!/bin/bash
# PMC passes (VALU/SALU/LDS/SMEM/waits) over tools/prof_variants.py variants; gpurun_out/pmcv_<tag>/
set -u
TAG=${1:-v}
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcv_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for V in no_string string_only one_field; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/$V -o run -- python3 tools/prof_variants.py --records 2000000 --iters 1 --only $V > $OUT/$V.log 2>&1 || { echo "pmc $V failed"; exit 1; }
done
echo pmc ok
