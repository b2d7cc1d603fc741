#!/bin/bash
# rocprofv3 passes over tools/prof_decode.py (the bench's SYN200 config); outputs under
# gpurun_out/prof_<tag>/ plus traffic_<records>.json (HBM bytes per decode-kernel launch from
# FETCH_SIZE / WRITE_SIZE, gfx950 FETCH_SIZE doubled for 16-byte loads -- MI355X_MICROARCH.md HBM).
set -u
TAG=${1:-r01}
REC=${2:-50000000}
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_decode.py --records $REC > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc1 -o run -- python3 tools/prof_decode.py --records $REC --iters 1 > $OUT/pmc1.log 2>&1 || { echo "pmc1 failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- python3 tools/prof_decode.py --records $REC --iters 1 > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 tools/prof_decode.py --records $REC --iters 1 > $OUT/pmc3.log 2>&1 || { echo "pmc3 failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o run -- python3 tools/prof_decode.py --records $REC --iters 1 > $OUT/pmc4.log 2>&1 || { echo "pmc4 failed"; exit 1; }
python3 tools/traffic.py $OUT $REC > $OUT/traffic_$REC.json || { echo "traffic summary failed"; exit 1; }
echo "profile ok"
