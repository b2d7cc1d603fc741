mkdir -p gpurun_out/r06_lw
timeout -k 10 500 python -u -m pytest tests/test_gpu_rdw.py tests/test_gpu_shards.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r06_lw/tests.log 2>&1
tail -2 gpurun_out/r06_lw/tests.log; grep -E "FAILED|Error" gpurun_out/r06_lw/tests.log | head -5
CBX_RDW_DEBUG=1 timeout -k 10 100 python -u tools/rdw_probe.py 20000 2>&1 | grep -v amdgpu.ids | grep -v "chunk " || exit 1
for rep in 1 2; do for L in 0 1; do
  CBX_RDW_LANE_WALK=$L timeout -k 10 300 python -u bench.py --workload wide_odo --steps 8 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/r06_lw/c5_${L}_${rep}.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06_lw/c5_${L}_${rep}.json')); k=d['kernel_ms']; print('C5 lane=${L}', ${rep}, d['ms_per_step'], round(k['rdw_framing (cbx_frame_rdw_async, count on the device)'],3), d['roofline'].get('frac_moved_bytes'))"
done; done
for L in 0 1; do
  CBX_RDW_LANE_WALK=$L timeout -k 10 300 python -u bench.py --workload rdw_narrow --steps 8 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/r06_lw/c4_${L}.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06_lw/c4_${L}.json')); k=d['kernel_ms']; print('C4 lane=${L}', d['ms_per_step'], round(k['rdw_framing (cbx_frame_rdw_async, count on the device)'],3))"
done
