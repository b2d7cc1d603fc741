#!/bin/bash
# One GPU session (run through gpurun).  Usage:
#   tools/gpu.sh TAG
# with the steps chosen by environment variables (each optional, in this order):
#   TESTS="all" | "<pytest -k expression>"   the -m gpu suite (all) or a selection of it
#   SMOKE=1                                   __graft_entry__.smoke()
#   BENCH="W[:args] ..."                      short bench lines (5 steps, no CPU baseline / end-to-end);
#                                             args comma-separated, e.g. synstr200:--records,50000000
#   PROF="W[:args] ..."                       the bench under rocprofv3 --kernel-trace --stats (10 steps)
#   PMC="W[:args] ..."                        FETCH/WRITE + SQ counter passes of a 1-step run (tools/evidence.sh groups)
#   ENVS="K=V ..."                            exported before every step (A/B knobs)
# Every GPU step has its own time limit and the script stops at the first failure.
set -u
TAG=$1
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOTDIR
for kv in ${ENVS:-}; do export "$kv"; done
if [ -n "${TESTS:-}" ]; then
  if [ "$TESTS" = "all" ]; then K=(); else K=(-k "$TESTS"); fi
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "${K[@]}" > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -2 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; exit $rc; }
fi
if [ -n "${SMOKE:-}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
spec() { W=${1%%:*}; EXTRA=""; NAME=$W; if [ "$1" != "$W" ]; then EXTRA=$(echo ${1#*:} | tr ',' ' '); NAME=${W}$(echo ${1#*:} | tr -d '-' | tr ', ' '__'); fi; }
for S in ${BENCH:-}; do
  spec "$S"
  timeout -k 10 400 python -u bench.py --workload $W $EXTRA --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > $OUT/b_$NAME.json 2> $OUT/b_$NAME.err || { tail -8 $OUT/b_$NAME.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$NAME.json')); print('$NAME', d['ms_per_step'], d.get('kernel_ms'), d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
for S in ${PROF:-}; do
  spec "$S"
  D=$OUT/p_$NAME; mkdir -p $D
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 -u $ROOTDIR/bench.py --workload $W $EXTRA --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $D/bench.json 2> $D/bench.err
  rc=$?; [ $rc -eq 0 ] || { echo "prof $NAME failed rc=$rc"; tail -8 $D/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench.json')); print('$NAME', d['ms_per_step'], d.get('kernel_ms'), d['roofline']['frac'])"
  f=$(find $D/trace -name "*kernel_stats.csv" | head -1); head -8 $f | cut -d, -f1-5
done
for S in ${PMC:-}; do
  spec "$S"
  D=$OUT/p_$NAME; mkdir -p $D
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
             "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o run -- python3 $ROOTDIR/bench.py --workload $W $EXTRA --steps 1 --warmup 1 --no-cpu-baseline --no-end-to-end > $D/pmc$i.log 2>&1 || { echo "pmc pass $i ($NAME) failed"; tail -3 $D/pmc$i.log; exit 1; }
  done
  cd $ROOTDIR && python3 tools/prof_summary.py $D > $D/summary.json && python3 -c "import json; d=json.load(open('$D/summary.json')); print('$NAME', json.dumps(d.get('check')))"; cd /tmp
  find $D -name "run_kernel_trace.csv" -o -name "run_counter_collection.csv" | xargs -r gzip -f
done
echo GPU_SH_OK
