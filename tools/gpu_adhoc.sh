set -u
mkdir -p gpurun_out
for W in synstr200 syn200 rdw_narrow wide_odo; do
for b in 3 4 5 16; do
  CBX_MAX_BLOCKS_PER_CU=$b timeout -k 10 200 python -u bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/occ_${W}_$b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/occ_${W}_$b.json')); print('$W blocks $b', d['ms_per_step'], d['kernel_ms']['decode_kernel'])"
done
done
