#!/bin/bash
# Selected GPU tests then short bench lines.  Usage: tools/gpu_tests_sel.sh TAG "pytest -k expr or ''" [workload[:args]]...
set -u
TAG=$1; K=$2; shift 2
OUT=gpurun_out/sel_$TAG; mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/tests.log | head -30; exit $rc; }
fi
for SPEC in "$@"; do
  W=${SPEC%%:*}; EXTRA=""; [ "$SPEC" != "$W" ] && EXTRA=$(echo ${SPEC#*:} | tr ',' ' ')
  N=$(echo "$SPEC" | tr ':, ' '___')
  timeout -k 10 300 python -u bench.py --workload $W $EXTRA --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $OUT/b_$N.json 2> $OUT/b_$N.err || { tail -20 $OUT/b_$N.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$N.json')); print('$SPEC', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['roofline']['layout_overhead'])"
done
echo SEL_OK
