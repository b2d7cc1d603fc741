#!/bin/bash
# rocprofv3 evidence for one bench workload: kernel-trace stats of a bench run, then FETCH_SIZE and
# WRITE_SIZE passes (one counter per run) -> traffic_<tag>.json (HBM bytes per decode launch).
# Usage: tools/gpu_profile_workload.sh ROUNDTAG WORKLOAD [STRINGS: views|offsets]
set -u
TAG=$1; W=$2; S=${3:-views}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$W
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 -u bench.py --workload $W --strings $S --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > $OUT/bench.json 2> $OUT/bench.err || { echo "trace failed"; tail -3 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
N=$(python3 -c "import json; print(json.load(open('$OUT/bench.json'))['config']['records_per_gpu'])")
TAGN=${W}_${S}_$N
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 bench.py --workload $W --strings $S --steps 1 --warmup 1 --no-cpu-baseline --no-end-to-end > $OUT/pmc3.log 2>&1 || { echo "pmc3 failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o run -- python3 bench.py --workload $W --strings $S --steps 1 --warmup 1 --no-cpu-baseline --no-end-to-end > $OUT/pmc4.log 2>&1 || { echo "pmc4 failed"; exit 1; }
for d in pmc3 pmc4; do f=$(find $OUT/$d -name run_counter_collection.csv | head -1); cp $f $OUT/$d/run_counter_collection.csv 2>/dev/null || true; done
python3 tools/traffic.py $OUT $N > $OUT/traffic_$TAGN.json && cat $OUT/traffic_$TAGN.json
