"""Probe: can two ranks share the box's one GPU over RCCL (backend "nccl")?  If so, bench.py's N > 1
path (its all-gather of the run's record count on the device) can run over RCCL on a 1-GPU box.

usage: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
       --master-port 29533 tools/rccl_probe.py
"""
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    x = torch.full((4,), rank + 1, dtype=torch.int64, device="cuda")
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_gather -> {[int(t[0]) for t in out]}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
