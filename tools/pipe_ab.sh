# A/B of the pipelined fixed-length Utf8 job (bench.py --pipeline C,D) on C3; usage: bash tools/pipe_ab.sh TAG "" "0,0" ...
set -u
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for P in "$@"; do
  A=""; [ "$P" != "-" ] && A="--pipeline $P"
  timeout -k 10 300 python -u bench.py --workload synstr200 $A --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > "$OUT/b_$P.json" 2> "$OUT/b_$P.err" || { tail -5 "$OUT/b_$P.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$P.json')); print('pipe=$P', d['ms_per_step'], d['roofline']['frac'])"
done
