# Record-walk evidence: kernel trace + two PMC passes of tools/bench_walk.py (3 M records).
set -e
cd /root/repo
D=gpurun_out/${1:-r04_w}/prof
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/bench_walk.py --records 3000000 --steps 3 > $D/b.json 2> $D/b.err
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $D/p1 -o run -- python3 tools/bench_walk.py --records 3000000 --steps 1 --warmup 1 > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_FLAT --output-format csv -d $D/p2 -o run -- python3 tools/bench_walk.py --records 3000000 --steps 1 --warmup 1 > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
echo done
