#!/bin/bash
# SYN200 decode time of diagnostic library variants (tools/build_variant.py) next to the product build.
# Usage: tools/gpu_diag_variants.sh VARIANT...
set -u
mkdir -p gpurun_out
for V in cur "$@"; do
  if [ "$V" = cur ]; then unset CBX_LIB_VARIANT; else export CBX_LIB_VARIANT=$V; fi
  timeout -k 10 120 python tools/prof_variants.py --records 50000000 --views --only full > gpurun_out/diag_$V.txt 2>&1 || { echo "variant $V failed"; tail -5 gpurun_out/diag_$V.txt; exit 1; }
  echo "$V $(cat gpurun_out/diag_$V.txt | grep full)"
done
