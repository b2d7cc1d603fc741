# Same-box A/B of copybook-specialised kernel variants on one workload: each variant is a
# CBX_JIT_DEFINES value ('-' = none) for a short bench run.
# usage: bash tools/jit_ab.sh TAG WORKLOAD "DEF=1" - "DEF=1" - ...
set -u
OUT=gpurun_out/$1; WL=$2; shift 2; mkdir -p $OUT
i=0
for V in "$@"; do
  i=$((i + 1))
  if [ "$V" = "-" ]; then unset CBX_JIT_DEFINES; else export CBX_JIT_DEFINES="$V"; fi
  timeout -k 10 400 python -u bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > "$OUT/b_${WL}_$i.json" 2> "$OUT/b_${WL}_$i.err" || { tail -5 "$OUT/b_${WL}_$i.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${WL}_$i.json')); print('$WL', 'defines=$V', d['ms_per_step'], d['kernel_ms']['decode_kernel'], d['roofline']['frac'])"
done
unset CBX_JIT_DEFINES
