#!/bin/bash
# Selected GPU tests, then per workload one bench line under rocprofv3 --kernel-trace --stats
# (kernel split of the step).  Usage: tools/gpu_sel_prof.sh TAG "pytest -k expr or ''" [workload[:args]]...
set -u
TAG=$1; K=$2; shift 2
OUT=gpurun_out/selp_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp; cd - > /dev/null
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/tests.log | head -30; exit $rc; }
fi
for SPEC in "$@"; do
  W=${SPEC%%:*}; EXTRA=""; [ "$SPEC" != "$W" ] && EXTRA=$(echo ${SPEC#*:} | tr ',' ' ')
  N=$(echo "$SPEC" | tr ':, ' '___')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$N -o run -- python3 -u bench.py --workload $W $EXTRA --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $OUT/b_$N.json 2> $OUT/b_$N.err || { tail -20 $OUT/b_$N.err; exit 1; }
  python3 - <<PY
import csv, glob, json
d = json.load(open('$OUT/b_$N.json'))
print('$SPEC', 'step', d['ms_per_step'], 'frac', d['roofline']['frac'], d['kernel_ms'])
for f in glob.glob('$OUT/$N/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'cbx' in r['Name']:
            print('   %-60s %6s %9.4f ms' % (r['Name'].split('(')[0][:60], r['Calls'], float(r['AverageNs']) / 1e6))
PY
done
echo SELP_OK
