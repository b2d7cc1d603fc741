# Same-box A/B of records per Utf8 decode call on C3 (bench.py --batch-records); usage: bash tools/batch_ab.sh TAG N...
set -u
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for B in "$@"; do
  timeout -k 10 400 python -u bench.py --workload synstr200 --batch-records $B --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > "$OUT/b_$B.json" 2> "$OUT/b_$B.err" || { tail -5 "$OUT/b_$B.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$B.json')); print('batch=$B', d['ms_per_step'], d['roofline']['frac'])"
done
