set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -x -q -k "golden_rows or wide_odo or arrow or odo or occurs" --timeout 120 --timeout-method thread > gpurun_out/t_list.log 2>&1; rc=$?; tail -3 gpurun_out/t_list.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/t_list.log | head -8; exit $rc; }
for o in lists slots; do
  timeout -k 10 300 python -u bench.py --workload wide_odo --occurs $o --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/c5_$o.json 2> gpurun_out/c5_$o.err || { tail -5 gpurun_out/c5_$o.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c5_$o.json')); print('$o', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5l -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wide_odo --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > $GRAFT_REPO_ROOT/gpurun_out/prof_c5l.log 2>&1; find $GRAFT_REPO_ROOT/gpurun_out/prof_c5l -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -8
