"""Multi-GPU sharding of a decode job.

One process per GPU.  Records are independent, so every rank decodes its own record range with no
data-path collective.  The only cross-shard quantities are global positions:

* ``Record_Id`` of a variable-length shard depends on how many records the shards before it framed
  (`VarLenNestedIterator` numbers records from the index entry's ``recordIndex`` on,
  VarLenNestedIterator.scala:80-147);
* a consumer that wants one global Arrow string array per column needs each shard's byte base.

Both come from ONE all-gather of ``int64[1 + S]`` per rank (record count + S string-column payload
sizes) over RCCL (``torch.distributed`` backend "nccl") -- a few hundred bytes at 8 GPUs, so it is
latency-bound and sized for point-to-point xGMI as a single small message.  The counts stay on the
device (no host sync inside a step).  CPU tests run the same code over gloo.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple


def shard_range(n_records: int, world: int, rank: int) -> Tuple[int, int]:
    """Record index range [start, end) of `rank` when n_records are split evenly over `world`."""
    if world <= 0 or not 0 <= rank < world or n_records < 0:
        raise ValueError("bad shard arguments")
    return n_records * rank // world, n_records * (rank + 1) // world


def byte_shard(n_bytes: int, record_size: int, world: int, rank: int) -> Tuple[int, int]:
    """Byte range of a fixed-length file shard: whole records only (CobolScanners.scala:77-94)."""
    if record_size <= 0:
        raise ValueError("record_size must be positive")
    r0, r1 = shard_range(n_bytes // record_size, world, rank)
    return r0 * record_size, r1 * record_size


def global_bases(local_rows, local_string_bytes: Sequence = (), group=None):
    """All-gather of (rows, string bytes per column) -> this rank's global bases and the totals.

    `local_rows` is an int or a 0-d / 1-element int64 tensor; `local_string_bytes` a sequence of
    ints or int64 tensors (e.g. the `sizes` tensors the decoder writes).  Returns
    (row_base, string_bases [S], totals [1 + S]) as int64 tensors on the communication device
    (the current CUDA device for nccl, CPU for gloo).
    """
    import torch
    import torch.distributed as dist

    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    def _t(x):
        if isinstance(x, torch.Tensor):
            return x.reshape(-1)[:1].to(device=dev, dtype=torch.int64)
        return torch.tensor([int(x)], dtype=torch.int64, device=dev)

    mine = torch.cat([_t(local_rows)] + [_t(x) for x in local_string_bytes])
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts: List = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    allv = torch.stack(parts)                       # [world, 1 + S]
    excl = torch.cumsum(allv, 0) - allv             # exclusive prefix over ranks
    return excl[rank, 0], excl[rank, 1:], allv.sum(0)


def record_bases(local_records, group=None) -> Tuple[int, int]:
    """Record_Id base of this rank's shard of one variable-length file and the file's record total.

    Each rank frames a contiguous run of the file's index entries and knows only its own record
    count; the reference numbers records from the entry's recordIndex on (IndexGenerator counts every
    record before it, VRLRecordReader.scala:55, 71).  The exclusive prefix of the ranks' counts is
    that number for the shard's first record: one all-gather, no sequential index pass."""
    rb, _, tot = global_bases(local_records, (), group)
    return int(rb), int(tot[0])


def entry_shards(entries, n_bytes: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous runs of sparse-index entries per rank, balanced by bytes: [first, end) entry index
    ranges.  An entry goes to the rank whose byte share holds its first byte (offset_from), so the
    runs are contiguous and in file order; a rank may get none when entries are large."""
    if world <= 0 or n_bytes < 0:
        raise ValueError("bad shard arguments")
    owner = [min(world - 1, e.offset_from * world // max(n_bytes, 1)) for e in entries]
    out = []
    for r in range(world):
        ks = [k for k, o in enumerate(owner) if o == r]
        first = ks[0] if ks else (out[-1][1] if out else 0)
        out.append((first, ks[-1] + 1 if ks else first))
    return out


def init_from_env(backend: Optional[str] = None):
    """torch.distributed init from torchrun's environment (RANK / WORLD_SIZE / MASTER_*);
    no-op for a single process.  Returns (world, rank, local_rank)."""
    import os

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return world, rank, local
