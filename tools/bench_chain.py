"""Timing of the chunk-parallel chain framings (cbx_chain.h) on >= 1 GB streams (GPU).

* record_length_field: records of a 2-byte big-endian COMP length (20..400 bytes, the whole record's)
  and random bodies -- a block generated on the host, repeated on the GPU to the stream size (every
  block ends on a record boundary, so the repeats are one valid stream);
* variable_size_occurs framing (VarOccursRecordExtractor): the record walk's nested-ODO records
  (synth.walk_nested_record), a block repeated the same way.

Each framing is timed (HIP events around the C-ABI call, which includes its host reads of the fix
rounds' flags) at the default chunk size and with ONE chunk (CBX_CHAIN_CHUNK above the stream size:
the sequential walk of one lane, the round-4 form); the length-field record count is checked against the
blocks', the var-occurs framing against the sequential one on the same prefix.
Prints one JSON line per (framing, chunking).

usage: python tools/bench_chain.py [GB] [--seq-mb MB]   (sequential runs on the first MB only: a lane
       walks ~1-2 M records/s, so the whole stream would take minutes)"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _time(fn, reps=3):
    import torch
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("gb", type=float, nargs="?", default=1.0)
    ap.add_argument("--seq-mb", type=float, default=16.0)
    a = ap.parse_args()
    import torch
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from cobrix_amd import synth

    def repeated(block: bytes, n_bytes: int):
        reps = max(1, n_bytes // len(block))
        t = torch.frombuffer(bytearray(block), dtype=torch.uint8).cuda()
        return t.repeat(reps), reps

    # record_length_field
    rng = np.random.default_rng(1)
    out, n_blk = bytearray(), 0
    while len(out) < (8 << 20):
        total = int(rng.integers(20, 401))
        out += total.to_bytes(2, "big") + bytes(rng.integers(0, 256, total - 2, dtype=np.uint8))
        n_blk += 1
    p, _ = parse_options({"record_length_field": "REC-LEN"})
    rd = VarLenNestedReader("""
       01  REC.
           05  REC-LEN     PIC 9(4) COMP.
           05  BODY        PIC X(400).
""", p)
    big, reps = repeated(bytes(out), int(a.gb * 1e9))
    for label, chunk, n in (("chunked", None, big.numel()), ("one chunk (sequential)", str(1 << 40), int(a.seq_mb * 1e6))):
        if chunk:
            os.environ["CBX_CHAIN_CHUNK"] = chunk
        else:
            os.environ.pop("CBX_CHAIN_CHUNK", None)
        n = min(n, big.numel())
        dt, (off, ln) = _time(lambda: rd.frame_length_field(big, n), reps=3 if chunk is None else 1)
        rec = int(off.numel())
        if n == big.numel():
            assert rec == n_blk * reps, (rec, n_blk * reps)
        print(json.dumps({"framing": "record_length_field", "form": label, "bytes": n, "records": rec,
                          "ms": round(dt * 1e3, 3), "GB_s": round(n / dt / 1e9, 2), "Mrec_s": round(rec / dt / 1e6, 2)}),
              flush=True)
        del off, ln
    del big
    torch.cuda.empty_cache()

    # variable_size_occurs framing
    rnd = random.Random(3)
    recs = []
    size = 0
    while size < (8 << 20):
        r = synth.walk_nested_record(rnd, True)
        recs.append(r)
        size += len(r)
    p2, _ = parse_options({"variable_size_occurs": "true"})
    rd2 = VarLenNestedReader(synth.WALK_NESTED_COPYBOOK, p2)
    import dataclasses
    rd_jit = VarLenNestedReader(synth.WALK_NESTED_COPYBOOK, dataclasses.replace(p2, jit_min_records=1))
    big, reps = repeated(b"".join(recs), int(a.gb * 1e9))
    # forms: the step is walk_length (the node-table walk) or its copybook-specialised form
    # (jit_chain_source, the default from jit_min_records records).  Checks: every prefix form against
    # the sequential walk, the whole stream's specialised framing against the table step's.
    seq = full = None
    pre = int(a.seq_mb * 1e6)
    forms = (("one chunk (sequential), table step", str(1 << 40), pre, rd2, True),
             ("chunked, same prefix, table step", None, pre, rd2, True),
             ("chunked, same prefix, specialised step", None, pre, rd_jit, False),
             ("chunked, table step", None, big.numel(), rd2, True),
             ("chunked", None, big.numel(), rd2, False))
    for label, chunk, n, rd, table in forms:
        if chunk:
            os.environ["CBX_CHAIN_CHUNK"] = chunk
        else:
            os.environ.pop("CBX_CHAIN_CHUNK", None)
        if table:
            os.environ["CBX_NO_JIT_WALK"] = "1"
        else:
            os.environ.pop("CBX_NO_JIT_WALK", None)
        n = min(n, big.numel())
        dt, res = _time(lambda: rd.frame_var_occurs(big, n), reps=3 if chunk is None else 1)
        rec = int(res[0].numel())
        kind = _frame_kind(rd)
        assert kind == (0 if table else 1), (label, kind)
        got = (res[0].cpu(), res[1].cpu(), res[2])
        ref = None
        if n == pre:
            if seq is None:
                seq = got
            else:
                ref = seq
        elif full is None:
            full = got
        else:
            ref = full
        if ref is not None:
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]) and got[2] == ref[2], label
        print(json.dumps({"framing": "variable_size_occurs", "form": label, "bytes": n, "records": rec,
                          "ms": round(dt * 1e3, 3), "GB_s": round(n / dt / 1e9, 2), "Mrec_s": round(rec / dt / 1e6, 2),
                          "checked": ref is not None}),
              flush=True)
        del res
    os.environ.pop("CBX_NO_JIT_WALK", None)


def _frame_kind(rd) -> int:
    import ctypes
    from cobrix_amd import native as N
    k = ctypes.c_int32()
    N.check(N.load().cbx_plan_frame_kind(rd.native.handle, ctypes.byref(k)))
    return k.value


if __name__ == "__main__":
    main()
