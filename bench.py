"""Benchmark: GPU decode of the SYN200 fixed-length numeric mix (BASELINE.json config C2).

`python bench.py --gpus N --steps K --warmup W` -- one rank per GPU (torchrun for N > 1); each
rank decodes its own shard of records already resident in HBM (weak scaling: records are
independent, shards need no data-path collective).  A step = one full decode of the shard
through the C ABI (`cbx_decode_fixed`): the decode kernel (numerics + tile-local strings), the
fixup kernel for deferred values and the string scan + placement kernels, into Arrow-style columns.
Rank 0 prints ONE JSON line.

roofline: algorithmic bytes (input record bytes + every output buffer byte)
of one decode-kernel launch / its average duration, measured with HIP events recorded by the
library on the launch stream over the timed steps (cbx_plan_kernel_times).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(plan, n_rec: int, record_bytes: int, payload_bytes: int) -> int:
    """input bytes + every output buffer byte one decode writes."""
    from cobrix_amd import native as N
    total = n_rec * record_bytes + payload_bytes
    for info in plan.columns:
        n = n_rec * info.n_slots
        total += (n + 7) // 8                                   # validity bits
        if info.out_type in (N.O_STRING, N.O_BINARY):
            total += 8 * (n + info.n_slots)                     # int64 offsets (n_rec + 1 per slot)
        else:
            total += n * N.OUT_WIDTH[info.out_type]
    return total


def measured_traffic(n_rec: int):
    """HBM bytes per decode-kernel launch from the newest committed rocprofv3 FETCH_SIZE/WRITE_SIZE
    passes of this configuration (tools/gpu_profile.sh -> profiles/<round tag>/traffic_<n_rec>.json)."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"traffic_{n_rec}.json")))
    if not found:
        return None, None
    with open(found[-1]) as f:
        t = json.load(f)
    return int(t["traffic_bytes"]), os.path.relpath(found[-1], ROOT)


def _cpu_baseline(seconds: float = 12.0):
    """Oracle (scalar C restatement of the reference decoders) on a bounded SYN200 sample, 1 core."""
    from cobrix_amd.copybook import parse_copybook
    from cobrix_amd.synth import SYN200_COPYBOOK, syn200
    from oracle import oracle as O
    cb = parse_copybook(SYN200_COPYBOOK)
    ast = O.OracleAst(cb)
    n = 2000
    data = syn200(n, seed=99).numpy().tobytes()
    t0 = time.perf_counter()
    O.decode_fixed(cb, data, ast=ast)
    dt = time.perf_counter() - t0
    rate = n / max(dt, 1e-9)
    n2 = int(min(max(rate * seconds, 2000), 6_000_000))
    data = syn200(n2, seed=100).numpy().tobytes()
    t0 = time.perf_counter()
    O.decode_fixed(cb, data, ast=ast)
    dt = time.perf_counter() - t0
    return {"value": round(n2 * 200 / dt / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
            "records_per_s": round(n2 / dt, 1),
            "sample": f"{n2} SYN200 records ({n2 * 200 / 1e6:.1f} MB) through oracle/cobrix_oracle.c "
                      f"(restatement of extractRecord + decoders), 1 thread, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=50_000_000, help="records per GPU (200 B each)")
    ap.add_argument("--window", type=int, default=0, help="LDS window bytes (0 = plan default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from cobrix_amd import native as N
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, _alloc_columns, string_capacity
    from cobrix_amd.synth import SYN200_COPYBOOK, SYN200_RECORD_SIZE, syn200

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    n_rec = args.records
    rec = syn200(n_rec, seed=20261015 + rank, device=dev).view(-1)
    torch.cuda.synchronize()

    rd = FixedLenNestedReader(SYN200_COPYBOOK, ReaderParameters(window_bytes=args.window))
    L = N.load()
    h = rd.native.handle
    st = torch.cuda.current_stream()
    cols, cs = _alloc_columns(rd.plan, n_rec, string_capacity(rd.native, n_rec), dev)
    stream = ctypes.c_void_p(st.cuda_stream)

    def step():
        N.check(L.cbx_decode_fixed(h, rec.data_ptr(), n_rec, SYN200_RECORD_SIZE, 0, 0, cs, stream))

    for _ in range(args.warmup):
        step()
    N.check(L.cbx_plan_check(h, stream))
    N.check(L.cbx_plan_set_profiling(h, 1))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    N.check(L.cbx_plan_check(h, stream))
    dec = (ctypes.c_float * args.steps)()
    fix = (ctypes.c_float * args.steps)()
    nc = ctypes.c_int32()
    N.check(L.cbx_plan_kernel_times(h, dec, fix, args.steps, ctypes.byref(nc)))
    N.check(L.cbx_plan_set_profiling(h, 0))
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    payload = sum(int(c["sizes"].sum().item()) for c in cols if "sizes" in c)
    steps = args.steps
    ms_per_step = elapsed / steps * 1e3
    in_bytes_total = n_rec * SYN200_RECORD_SIZE * world
    gbs = in_bytes_total / (elapsed / steps) / 1e9
    recs_per_s = n_rec * world / (elapsed / steps)
    alg = algorithmic_bytes(rd.plan, n_rec, SYN200_RECORD_SIZE, payload)
    dec_avg_ms = sum(dec[: nc.value]) / max(1, nc.value)
    fix_avg_ms = sum(fix[: nc.value]) / max(1, nc.value)
    achieved = alg / (dec_avg_ms * 1e-3) / 1e9
    kind = ctypes.c_int32(0)
    N.check(L.cbx_plan_kernel_kind(h, ctypes.byref(kind)))
    kname = "cbx_jit_decode (copybook-specialised, hipRTC)" if kind.value == 1 else "cbx::decode_kernel (table-driven)"
    traffic, traffic_src = measured_traffic(n_rec)
    if rank == 0:
        out = {
            "metric": "decoded input GB/s + records/s, fixed-len COMP-3 mix, 1-8 MI355X; % HBM peak",
            "value": round(gbs, 3),
            "unit": "GB/s",
            "records_per_s": round(recs_per_s, 1),
            "hbm_frac_step": round(alg * world / (elapsed / steps) / 1e9 / (HBM_PEAK_GBS * world), 4),
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (cobrix_amd/synth.py SYN200, seed 20261015+rank, 0.5% malformed numerics)",
            "config": {"workload": "SYN200: fixed-length 200-byte EBCDIC records, numeric mix "
                                   "(COMP, COMP-3, zoned DISPLAY overpunch, IBM COMP-2, cp037 X(18)) -- BASELINE config C2",
                       "records_per_gpu": n_rec, "record_bytes": SYN200_RECORD_SIZE,
                       "input_gb_per_gpu": round(n_rec * SYN200_RECORD_SIZE / 1e9, 3),
                       "output_columns": rd.plan.n_columns, "parallelism": f"dp{world}",
                       "inputs_resident_in_hbm": True},
            "kernel_ms": {"decode_kernel": round(dec_avg_ms, 4),
                          "post_kernels (deferred-value fixup, string scan + placement)": round(fix_avg_ms, 4)},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": alg, "traffic": traffic,
                         "traffic_source": traffic_src},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = _cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
