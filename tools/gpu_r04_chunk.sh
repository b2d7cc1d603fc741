set -u
mkdir -p gpurun_out/r04_chunk
for spec in ${SPECS:-"wide_odo:65536" "wide_odo:262144" "rdw_narrow:65536" "rdw_narrow:131072"}; do
  W=${spec%%:*}; C=${spec#*:}
  CBX_RDW_CHUNK_BYTES=$C timeout -k 10 300 python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/r04_chunk/${W}_$C.json 2> gpurun_out/r04_chunk/${W}_$C.err || { tail -5 gpurun_out/r04_chunk/${W}_$C.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r04_chunk/${W}_$C.json') if l.startswith('{')][-1]); k=d['kernel_ms']; print('$W $C', d['ms_per_step'], k['decode_kernel'], [v for kk,v in k.items() if kk.startswith('rdw_framing')])"
done
