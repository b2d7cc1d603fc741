#!/bin/bash
# A round's GPU evidence for the bench configurations.  Usage: tools/evidence.sh TAG [--no-tests] WORKLOAD[:extra bench args,comma-separated]...
# 1. the -m gpu suite (unless --no-tests);
# 2. per workload: the bench command itself under rocprofv3 --kernel-trace --stats (the JSON line and the
#    kernel trace come from ONE process, so roofline.frac can be recomputed from the trace), then PMC
#    passes of a 1-step run, one counter group per pass (FETCH_SIZE; WRITE_SIZE; two SQ groups);
# 3. tools/prof_summary.py -> gpurun_out/TAG/<workload>/summary.json (copied into profiles/TAG/).
set -u
TAG=$1; shift
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $ROOTDIR
if [ "${1:-}" = "--no-tests" ]; then shift; else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -2 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
fi
for SPEC in "$@"; do
  W=${SPEC%%:*}; EXTRA=""; NAME=$W
  if [ "$SPEC" != "$W" ]; then EXTRA=$(echo ${SPEC#*:} | tr ',' ' '); NAME=${W}$(echo ${SPEC#*:} | tr -d '-' | tr ', ' '__'); fi
  D=$OUT/$NAME; mkdir -p $D
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 -u bench.py --workload $W $EXTRA --steps 10 --warmup 3 > $D/bench.json 2> $D/bench.err
  rc=$?; cat $D/bench.json
  [ $rc -eq 0 ] || { echo "bench $NAME failed rc=$rc"; tail -20 $D/bench.err; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
             "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o run -- python3 bench.py --workload $W $EXTRA --steps 1 --warmup 1 --no-cpu-baseline --no-end-to-end > $D/pmc$i.log 2>&1 || { echo "pmc pass $i ($NAME) failed"; tail -3 $D/pmc$i.log; exit 1; }
  done
  python3 tools/prof_summary.py $D > $D/summary.json && python3 -c "import json; d=json.load(open('$D/summary.json')); print('$NAME', json.dumps(d['check']))"
  # the raw per-dispatch CSVs compressed (gpurun copies back at most 64 MiB of gpurun_out/)
  find $D -name "run_kernel_trace.csv" -o -name "run_counter_collection.csv" | xargs -r gzip -f
done
echo ALL_OK
