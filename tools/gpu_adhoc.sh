set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/stamps.py --records 50000000 --views > gpurun_out/stamps_r02k.txt 2>&1 && cat gpurun_out/stamps_r02k.txt && \
bash tools/pmc_workload.sh r02k syn200 50000000
