set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "list or wide_odo" --timeout 120 --timeout-method thread > gpurun_out/t_list.log 2>&1; rc=$?; tail -3 gpurun_out/t_list.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/t_list.log | head -8; exit $rc; }
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5x -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wide_odo --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > $GRAFT_REPO_ROOT/gpurun_out/prof_c5x.log 2>&1; cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/prof_c5x -name "*kernel_stats.csv" | head -1); grep -E "list_kernel|jit_decode" $f | cut -d, -f1-4
