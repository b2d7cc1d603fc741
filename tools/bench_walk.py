"""Timing line for the record walk (cbx_walk.h: extractRecord with data-dependent offsets, a tile of
64 records walked in step -- the copybook-specialised cbx_jit_walk, or with --table the table-driven
walk_kernel; SURVEY.md 8(f)4 -- RecordExtractors.scala:66-134 with variable_size_occurs = true).

The layout is cobrix_amd/synth.py's WALK_NESTED copybook (an OCCURS 0 TO 3 DEPENDING ON holding an
OCCURS 1 TO 4 DEPENDING ON, COMP-3 / zoned / strings around them), records laid out as
variable_size_occurs = true writes them, in an RDW file.  A block of 3,000 generated records is
repeated to the requested size (synthetic data; parity of this layout against the oracle is
tests/test_gpu_walk.py).  A step = one cbx_decode_var call over the resident file (framed once);
time = HIP events around the walk kernel (cbx_plan_kernel_times).  Bytes = SURVEY.md 8(d) as in
bench.py (input + Arrow output bytes; nested-ODO columns at every slot).

Usage: python tools/bench_walk.py [--records N] [--steps K] -> one JSON line."""
import argparse
import ctypes
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=30_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--table", action="store_true", help="the table-driven walk (no copybook-specialised kernel)")
    args = ap.parse_args()
    import torch
    import bench
    from cobrix_amd import native as N
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from cobrix_amd.synth import WALK_NESTED_COPYBOOK as NESTED, rdw_file, walk_nested_record

    rnd = random.Random(20261017)
    block = rdw_file([walk_nested_record(rnd, True) for _ in range(3000)])
    reps = max(1, args.records // 3000)
    raw = block * reps
    n_rec = 3000 * reps
    dev = torch.device("cuda", 0)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    p, _ = parse_options({"is_record_sequence": "true", "variable_size_occurs": "true", "generate_record_id": "true"})
    if args.table:
        import dataclasses
        p = dataclasses.replace(p, jit_min_records=-1)
    rd = VarLenNestedReader(NESTED, p)
    assert rd.walk
    off, ln = rd.frame(t, len(raw))
    assert int(off.numel()) >= n_rec
    L, h = N.load(), rd.native.handle
    for _ in range(args.warmup):
        b = rd.decode_device(t, len(raw), off[:n_rec], ln[:n_rec])
    torch.cuda.synchronize()
    N.check(L.cbx_plan_set_profiling(h, 1))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        del b
        b = rd.decode_device(t, len(raw), off[:n_rec], ln[:n_rec])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    dec = (ctypes.c_float * args.steps)()
    post = (ctypes.c_float * args.steps)()
    nc = ctypes.c_int32()
    N.check(L.cbx_plan_kernel_times(h, dec, post, args.steps, ctypes.byref(nc)))
    N.check(L.cbx_plan_set_profiling(h, 0))
    kind = ctypes.c_int32()
    N.check(L.cbx_plan_kernel_kind(h, ctypes.byref(kind)))
    ms = sum(dec[i] for i in range(nc.value)) / max(1, nc.value)
    in_bytes = len(raw)
    payload = bench.string_payload(rd.plan, b.cols, n_rec)
    present = bench.present_elements(rd.plan, b.cols, n_rec)
    alg = bench.algorithmic_bytes(rd.plan, n_rec, in_bytes, payload, present)
    achieved = alg / (ms * 1e-3) / 1e9
    print(json.dumps({
        "metric": "record walk (variable_size_occurs) decode: input GB/s + records/s", "kernel": {2: "cbx::walk_kernel (table-driven)", 3: "cbx_jit_walk (copybook-specialised, hipRTC)"}.get(kind.value, "?"),
        "kernel_kind": kind.value, "records": n_rec, "input_bytes": in_bytes,
        "value": round(in_bytes / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "records_per_s": round(n_rec / (ms * 1e-3), 1),
        "walk_kernel_ms": round(ms, 4), "call_ms_wall": round(wall * 1e3, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / bench.HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg},
        "data": "synth.WALK_NESTED records (variable_size_occurs = true, 5 % non-numeric / out-of-range "
                "counts, 15 % short records) in an RDW file, a 3,000-record block repeated",
    }), flush=True)


if __name__ == "__main__":
    main()
