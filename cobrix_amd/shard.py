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


def index_chain(buf, tail_room: int, index_fn, group=None, split_bytes: Optional[int] = None) -> dict:
    """Sparse index of ONE variable-length file whose blocks are spread over the ranks (rank r holds
    block r, the blocks in rank order, each starting at a record header), with every rank holding
    only its own block plus, in front of it, the tail of the file before it that belongs to its run.

    IndexGenerator.sparseIndexGenerator (CP/reader/index/IndexGenerator.scala:33-127) with the
    default entry size resets its byte count at every cut, so the cuts after an entry start depend
    only on the records from that start on: the file's index is a chain.  Rank r receives from rank
    r - 1 the start of the last entry found so far (file offset, record index) and the bytes from
    there to the end of block r - 1 (at most one entry), indexes that tail + its block as a file of
    its own -- index_fn(region, start_bytes) -> ([(offset_from, record_index)] region-relative, the
    first (0, 0); record count) -- keeps every entry but the last, and sends the last one on.  The last
    rank keeps all of its entries.  Rank r's run = its entries: a contiguous, balanced (one block, give
    or take an entry) share of the file in file order; the union over the ranks is the whole file's index.
    The subtracting split-size rule (split_bytes: an explicit input_split_size_mb or the HDFS block size,
    VarLenNestedReader.scala:237-243) does not reset the byte count at a cut, it subtracts the split size:
    the count at entry k is its offset minus k split sizes, so the link also carries that residual of
    the entry it hands on, and the next rank indexes its region starting from it (start_bytes; 0 with
    the resetting default, whose count is 0 at every entry).

    buf: uint8 tensor [tail_room + block bytes], the block at buf[tail_room:]; the received tail
    lands right in front of it.  Point-to-point send/recv of int64[3] + the tail bytes (device
    tensors over RCCL, CPU tensors over gloo), N - 1 hops in sequence (setup, not the step).
    Returns {"run": uint8 view of buf, "run_start": file offset of the run, "seeds": entry offsets
    relative to the run, "entries": [(offset_from, record_index)] absolute, "record_base": record
    index of the run's first record, "n_records": records in the run}."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    # gloo moves host tensors only: device buffers then go through host copies
    host = buf.is_cuda and dist.is_initialized() and dist.get_backend(group) == "gloo"
    cdev = "cpu" if host else buf.device

    def recv_into(t, src):
        if host:
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src=src, group=group)
            t.copy_(h)
        else:
            dist.recv(t, src=src, group=group)

    meta = torch.zeros(4, dtype=torch.int64, device=cdev)   # file offset, record index, tail bytes, residual
    if rank > 0:
        dist.recv(meta, src=rank - 1, group=group)
    r_off, r_rec, tail, r_res = (int(x) for x in meta.tolist())
    if tail < 0:
        raise RuntimeError(f"index_chain: rank {rank - 1} had a tail larger than the {tail_room}-byte room")
    if tail > 0:
        recv_into(buf[tail_room - tail:tail_room], rank - 1)
    res, fwd = chain_step(buf[tail_room - tail:], index_fn, r_off, r_rec, rank == world - 1, r_res, split_bytes)
    if fwd is not None:
        f_off, f_rec, f_bytes, f_res = fwd
        ok = f_bytes.numel() <= tail_room
        out = torch.tensor([f_off, f_rec, f_bytes.numel() if ok else -1, f_res], dtype=torch.int64, device=cdev)
        dist.send(out, dst=rank + 1, group=group)
        if not ok:
            raise RuntimeError(f"index_chain: {f_bytes.numel()}-byte tail for rank {rank + 1} exceeds the "
                               f"{tail_room}-byte room")
        if f_bytes.numel() > 0:
            dist.send(f_bytes.cpu() if host else f_bytes.contiguous(), dst=rank + 1, group=group)
    return res


def chain_step(region, index_fn, r_off: int, r_rec: int, last: bool, r_res: int = 0,
               split_bytes: Optional[int] = None):
    """One link of index_chain: `region` starts at the file offset r_off (record index r_rec) at an
    entry start, whose byte count is r_res (subtracting split), and runs to the end of this rank's
    block.  Returns (result, forward): the result dict of index_chain, and (file offset, record index,
    bytes, residual) of the entry handed to the next rank (None for the last rank)."""
    ents, n_rec = index_fn(region, r_res)
    if not ents or ents[0][0] != 0:
        raise RuntimeError("index_chain: index_fn must return the region's entries, the first at offset 0")
    fwd = None
    if not last:
        last_off, last_rec = ents[-1]
        # IndexGenerator.scala:110-116: the count at the region's k-th entry = r_res + its offset - k S
        res_last = r_res + last_off - (len(ents) - 1) * split_bytes if split_bytes else 0
        fwd = (r_off + last_off, r_rec + last_rec, region[last_off:], res_last)
        keep, run_end, n_run = ents[:-1], last_off, last_rec
    else:
        keep, run_end, n_run = ents, int(region.numel()), n_rec
    return ({"run": region[:run_end], "run_start": r_off, "seeds": [o for o, _ in keep],
             "entries": [(r_off + o, r_rec + k) for o, k in keep], "record_base": r_rec, "n_records": n_run}, fwd)


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
