set -u
mkdir -p gpurun_out
for b in 3 4 5 6 16; do
  CBX_MAX_BLOCKS_PER_CU=$b timeout -k 10 300 python -u bench.py --workload rdw_narrow --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/sb_$b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sb_$b.json')); print('blocks $b', d['ms_per_step'], d['kernel_ms']['decode_kernel'])"
done
