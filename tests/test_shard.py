"""Sharding helpers (cobrix_amd/shard.py) on CPU: ranges, and the count all-gather over gloo with
world_size 2 and 3 (the same code runs over RCCL on the GPUs)."""
from __future__ import annotations

import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

from cobrix_amd.shard import byte_shard, global_bases, shard_range  # noqa: E402


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 64, 1000, 50_000_001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    assert byte_shard(10 * 200 + 13, 200, 3, 2) == (6 * 200, 10 * 200)
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = 10 * (rank + 1)
    sizes = [torch.tensor([100 + rank], dtype=torch.int64), 7 * rank]
    rb, sb, tot = global_bases(rows, sizes)
    q.put((rank, int(rb), [int(x) for x in sb], [int(x) for x in tot]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_bases_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = [10 * (r + 1) for r in range(world)]
    s0 = [100 + r for r in range(world)]
    s1 = [7 * r for r in range(world)]
    for rank, rb, sb, tot in res:
        assert rb == sum(rows[:rank])
        assert sb == [sum(s0[:rank]), sum(s1[:rank])]
        assert tot == [sum(rows), sum(s0), sum(s1)]


def _varlen_worker(rank, world, port, q):
    """One rank of a 2-way split of ONE variable-length file (test5, Test5MultisegmentSpec.scala:95-148
    options): the rank frames only its run of index entries, learns its Record_Id base from the
    count all-gather (shard.record_bases) and numbers its entries from it."""
    import torch.distributed as dist
    import goldens as G
    import numpy as np
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import parse_copybook_for
    from cobrix_amd.shard import entry_shards, record_bases
    from oracle import oracle as O
    from oracle import reader_oracle as RO
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    p, _ = parse_options({"is_record_sequence": "true", "input_split_records": "100", "segment_field": "SEGMENT_ID",
                          "segment_id_root": "C", "segment_id_prefix": "B", "generate_record_id": "true"})
    cb = parse_copybook_for(G.read("test5_copybook.cob").decode("latin-1"), p)
    entries = RO.sparse_index(cb, raw, p)          # entry byte offsets (the split plan)
    k0, k1 = entry_shards(entries, len(raw), world)[rank]
    mine = entries[k0:k1]
    lo = mine[0].offset_from if mine else len(raw)
    hi = (mine[-1].offset_to if mine[-1].offset_to > 0 else len(raw)) if mine else len(raw)
    off, _ = O.frame_rdw(raw[lo:hi])               # this rank's records only
    base, total = record_bases(len(off))
    local = [RO.Entry(e.offset_from, e.offset_to, e.file_id,
                      base + int(np.searchsorted(off + lo, e.offset_from))) for e in mine]
    recs = RO.var_len_records(cb, raw, p, entries=local) if local else []
    q.put((rank, total, [(r.record_id, r.seg_ids) for r in recs]))
    dist.destroy_process_group()


def test_varlen_shards_record_ids_gloo():
    """Record_Id and Seg_Id of a file split over 2 ranks (each framing only its entries) equal the
    single-rank read of the whole file."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_varlen_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import goldens as G
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import parse_copybook_for
    from oracle import reader_oracle as RO
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    p, _ = parse_options({"is_record_sequence": "true", "input_split_records": "100", "segment_field": "SEGMENT_ID",
                          "segment_id_root": "C", "segment_id_prefix": "B", "generate_record_id": "true"})
    cb = parse_copybook_for(G.read("test5_copybook.cob").decode("latin-1"), p)
    whole = [(r.record_id, r.seg_ids) for r in RO.var_len_records(cb, raw, p)]
    split = res[0][2] + res[1][2]
    assert res[0][1] == res[1][1] == 1000
    assert len(res[0][2]) > 100 and len(res[1][2]) > 100
    assert split == whole


def test_bench_launcher_two_ranks_gloo():
    """`bench.py --gpus 2` with no torchrun environment starts its own 2 ranks (torch.distributed.run,
    127.0.0.1); --dry-run keeps them on the CPU (gloo): process group, the per-step record-count
    all-gather (exclusive prefix = each rank's Record_Id base), barrier + max-over-ranks timing, and
    ONE JSON line from rank 0 reporting both ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                        "--warmup", "0"], capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"]
    assert sorted((g["rank"], g["base"], g["ok"]) for g in out["ranks"]) == [(0, 0, True), (1, 1000, True)]


def test_bench_rejects_world_mismatch():
    """Under a torchrun environment whose WORLD_SIZE differs from --gpus, bench.py exits non-zero."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert r.returncode == 2 and "WORLD_SIZE 1 != --gpus 2" in r.stderr


def _chain_worker(rank, world, port, q, entry_bytes, subtract=False):
    """One rank of a chained index (shard.index_chain): it holds only its own block of the file and
    the tail the rank before it sends; index_fn = the oracle restatement of IndexGenerator."""
    import torch.distributed as dist
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import parse_copybook_for
    from cobrix_amd.shard import index_chain
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    from oracle import oracle as O
    from oracle import reader_oracle as RO
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    block = rdw_narrow(2500 + 700 * rank, seed=40 + rank)[0]
    room = entry_bytes + 4096
    buf = torch.zeros(room + block.numel(), dtype=torch.uint8)
    buf[room:] = block
    p, _ = parse_options({**_CHAIN_OPTS})
    cb = parse_copybook_for(RDW_NARROW_COPYBOOK, p)

    def index_fn(region, start_bytes):
        raw = region.numpy().tobytes()
        ents = (RO.sparse_index(cb, raw, p, 0, split_bytes=entry_bytes, start_bytes=start_bytes) if subtract
                else RO.sparse_index(cb, raw, p, 0, entry_bytes))
        return [(e.offset_from, e.record_index) for e in ents], len(O.frame_rdw(raw)[0])

    r = index_chain(buf, room, index_fn, split_bytes=entry_bytes if subtract else None)
    q.put((rank, r["entries"], r["record_base"], r["n_records"], r["run_start"], r["seeds"],
           r["run"].numpy().tobytes()))
    dist.destroy_process_group()


_CHAIN_OPTS = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID", "segment_id_root": "C"}


@pytest.mark.parametrize("subtract", [False, True], ids=["reset", "subtract"])
@pytest.mark.parametrize("world,entry_bytes", [(2, 20_000), (3, 7_000), (3, 100_000)])
def test_index_chain_equals_whole_file_index_gloo(world, entry_bytes, subtract):
    """A file's index computed as a chain over ranks that each hold one block (+ one entry of tail)
    equals the oracle's index of the whole file: same entries, the runs tile the file in order, the
    record bases are the record counts before each run.  At 100 kB entries over ~200 kB blocks
    some ranks get one entry or none.  subtract: the split size subtracted at each cut (an explicit
    split size / the HDFS block size, IndexGenerator.scala:110-116), the links carrying the residual."""
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import parse_copybook_for
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    from oracle import oracle as O
    from oracle import reader_oracle as RO
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, q, entry_bytes, subtract)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    whole = b"".join(rdw_narrow(2500 + 700 * b, seed=40 + b)[0].numpy().tobytes() for b in range(world))
    p, _ = parse_options({**_CHAIN_OPTS})
    cb = parse_copybook_for(RDW_NARROW_COPYBOOK, p)
    ents = (RO.sparse_index(cb, whole, p, 0, split_bytes=entry_bytes) if subtract
            else RO.sparse_index(cb, whole, p, 0, entry_bytes))
    exp = [(e.offset_from, e.record_index) for e in ents]
    assert len(exp) > world
    assert [e for r in res for e in r[1]] == exp
    assert b"".join(r[6] for r in res) == whole
    n_before = 0
    for rank, ents, base, n_rec, start, seeds, run in res:
        assert base == n_before and start == sum(len(x[6]) for x in res[:rank])
        assert [start + s for s in seeds] == [o for o, _ in ents]
        assert n_rec == len(O.frame_rdw(run)[0])
        n_before += n_rec
    assert n_before == len(O.frame_rdw(whole)[0])
