#!/bin/bash
# Round-4 final evidence, part A: the -m gpu suite, smoke(), the record-walk profile.
set -u
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/r04_z
mkdir -p $OUT
cd $ROOTDIR
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 bash tools/gpu_walkprof.sh r04_z || exit 1
timeout -k 10 300 python tools/bench_walk.py > $OUT/walk_jit.json 2> $OUT/walk.err && cat $OUT/walk_jit.json
timeout -k 10 300 python tools/bench_walk.py --table > $OUT/walk_table.json 2>> $OUT/walk.err && cat $OUT/walk_table.json
echo PART_A_OK
