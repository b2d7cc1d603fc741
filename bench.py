"""Benchmark: GPU decode of the BASELINE.json configs (default: config C2, SYN200 numeric mix).

`python bench.py --gpus N --steps K --warmup W [--workload syn200|synstr200|rdw_narrow|wide_odo]`
-- one rank per GPU (torchrun for N > 1); each rank decodes its own shard of records already
resident in HBM (weak scaling: records are independent, shards need no data-path collective;
fixed-length shards know their Record_Id base statically, variable-length shards get it from one
RCCL all-gather of their framed record counts per step).  Rank 0 prints ONE JSON line.

A step = one full decode of the shard through the C ABI:
  fixed-length (C2 syn200, C3 synstr200): `cbx_decode_fixed` -- decode kernel (numerics and
      strings; with the default --strings views every string value is written once, into an Arrow
      string view + its tile's data region) + fixup kernel for deferred values (--strings offsets:
      Arrow large-string offsets, + string scan and placement kernels);
  variable-length (C4 rdw_narrow, C5 wide_odo): `cbx_frame_rdw` (GPU RDW offset discovery seeded
      by the sparse-index entries cbx_sparse_index cut at setup, 100 MB at root segments) +
      `cbx_decode_var` (segment redefines, ODO); for N > 1 one all-gather of the shard's record count
      between framing and decode gives its Record_Id base.

roofline: algorithmic bytes (input record bytes + every output buffer byte of the
layout produced -- validity bits, values, 16-byte string views + the payload of views longer than
12 bytes, or int64 offsets + payload) of one decode-kernel launch / its average duration, measured
with HIP events recorded by the library on the launch stream over the timed steps
(cbx_plan_kernel_times).

end_to_end (fixed-length workloads, N = 1 view per rank): the same shard streamed from pinned host
memory -- H2D copies of 2.5M-record chunks on a copy stream overlapped with the decode of the
previous chunk on the decode stream (double-buffered) -- reported beside `value`, never as it.
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
METRIC = "decoded input GB/s + records/s, fixed-len COMP-3 mix, 1-8 MI355X; % HBM peak"


def algorithmic_bytes(plan, n_rec: int, in_bytes: int, payload_bytes: int, present=None) -> int:
    """input bytes + every output buffer byte one decode writes (payload_bytes: the
    string payload written to data buffers -- all of it in the offsets layout, the values longer
    than 12 bytes in the view layout).  present[column]: elements that exist (OCCURS DEPENDING ON:
    the records' element counts) -- absent elements are not algorithmic output, whatever the
    slot-major layout writes for them."""
    from cobrix_amd import native as N
    total = in_bytes + payload_bytes
    views = bool(plan.options.string_views)
    present = present or {}
    for info in plan.columns:
        n = present.get(info.index, n_rec * info.n_slots)
        total += (n + 7) // 8                                   # validity bits
        if info.out_type in (N.O_STRING, N.O_BINARY):
            total += 16 * n if views else 8 * (n + info.n_slots)   # views / int64 offsets (n_rec + 1 per slot)
        else:
            total += n * N.OUT_WIDTH[info.out_type]
    return total


def _round_key(path: str):
    """Natural order of profiles/<round>_<variant> directories (r02_b after r02_a, r01_v10 after r01_v9)."""
    import re
    d = os.path.basename(os.path.dirname(path))
    return [int(x) if x.isdigit() else x for x in re.split(r"(\d+)", d)]


def measured_traffic(tag: str):
    """HBM bytes per decode-kernel launch from the newest committed rocprofv3 FETCH_SIZE/WRITE_SIZE
    passes of this configuration (tools/gpu_profile.sh -> profiles/<round tag>/traffic_<tag>.json)."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"traffic_{tag}.json")), key=_round_key)
    if not found:
        return None, None
    with open(found[-1]) as f:
        t = json.load(f)
    return int(t["traffic_bytes"]), os.path.relpath(found[-1], ROOT)


# ------------------------------------------------------------------------------------------------
# workloads
# ------------------------------------------------------------------------------------------------
WORKLOADS = {
    "syn200": dict(records=50_000_000, config="C2",
                   desc="SYN200: fixed-length 200-byte EBCDIC records, numeric mix (COMP, COMP-3, zoned DISPLAY "
                        "overpunch, IBM COMP-2, cp037 X(18)) -- BASELINE config C2",
                   data="synthetic (cobrix_amd/synth.py SYN200, seed 20261015+rank, 0.5% malformed numerics)"),
    "synstr200": dict(records=50_000_000, config="C3",
                      desc="SYNSTR200: fixed-length 200-byte records, 10 x PIC X(20) cp037 -> UTF-8, trim both, "
                           "Arrow string offsets -- BASELINE config C3",
                      data="synthetic (cobrix_amd/synth.py SYNSTR200: lengths 0-20, 25% accented, 10% leading "
                           "spaces, 1% control bytes)"),
    "rdw_narrow": dict(records=150_000_000, config="C4",
                       desc="RDW multisegment file, exp2/test5 layout (C 68 B / P 64 B records, segment redefines), "
                            "GPU RDW offset discovery seeded every 100 MB + var-len decode -- BASELINE config C4",
                       data="synthetic (cobrix_amd/synth.py rdw_narrow, 35% root segments)"),
    "wide_odo": dict(records=770_000, config="C5",
                     desc="Wide multisegment RDW file (exp3 layout + OCCURS 0 TO 2000 DEPENDING ON, 16,070 B roots, "
                          "64 B children) -- BASELINE config C5 (per-GPU shard of the 8-GPU job)",
                     data="synthetic (cobrix_amd/synth.py wide_odo, element counts uniform 0-2000, 0-4 children)"),
}


class _Fixed:
    def __init__(self, name, n_rec, dev, rank, window, views):
        import torch
        from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters
        from cobrix_amd import synth
        if name == "syn200":
            cb, self.stride = synth.SYN200_COPYBOOK, synth.SYN200_RECORD_SIZE
            self.rec = synth.syn200(n_rec, seed=20261015 + rank, device=dev).view(-1)
            params = ReaderParameters(window_bytes=window, string_views=views)
        else:
            cb, self.stride = synth.SYNSTR200_COPYBOOK, synth.SYNSTR200_RECORD_SIZE
            self.rec = synth.synstr200(n_rec, seed=20261017 + rank, device=dev).view(-1)
            params = ReaderParameters(window_bytes=window, ebcdic_code_page="cp037", string_views=views)
        torch.cuda.synchronize()
        self.rd = FixedLenNestedReader(cb, params)
        self.n_rec, self.in_bytes, self.dev = n_rec, n_rec * self.stride, dev
        self.record_base = rank * n_rec

    def prepare(self, stream):
        from cobrix_amd import native as N
        from cobrix_amd.reader import _alloc_columns, string_capacity
        self.L, self.h, self.stream = N.load(), self.rd.native.handle, ctypes.c_void_p(stream.cuda_stream)
        self.cols, self.cs = _alloc_columns(self.rd.plan, self.n_rec, string_capacity(self.rd.native, self.n_rec),
                                            self.dev)

    def step(self, world=1):
        from cobrix_amd import native as N
        # fixed-length shards: rank r holds records [r n, (r + 1) n) -- the Record_Id base is static
        N.check(self.L.cbx_decode_fixed(self.h, self.rec.data_ptr(), self.n_rec, self.stride, 0, self.record_base,
                                        self.cs, self.stream))
        return None

    def end_to_end(self, chunk_rec: int = 2_500_000, passes: int = 2):
        """H2D (pinned host) + decode, chunked and double-buffered over two streams."""
        import torch
        from cobrix_amd import native as N
        from cobrix_amd.reader import _alloc_columns, string_capacity
        host = torch.empty(self.in_bytes, dtype=torch.uint8, pin_memory=True)
        host.copy_(self.rec)
        chunk_rec = min(chunk_rec, self.n_rec)
        cb = chunk_rec * self.stride
        bufs = [torch.empty(cb, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        outs = [_alloc_columns(self.rd.plan, chunk_rec, string_capacity(self.rd.native, chunk_rec), self.dev)
                for _ in range(2)]
        cp, dc = torch.cuda.Stream(self.dev), torch.cuda.Stream(self.dev)
        done = [torch.cuda.Event() for _ in range(2)]
        copied = [torch.cuda.Event() for _ in range(2)]
        for e in done:
            e.record(dc)
        dstream = ctypes.c_void_p(dc.cuda_stream)
        n_chunks = (self.n_rec + chunk_rec - 1) // chunk_rec

        def run():
            for i in range(n_chunks):
                b = i % 2
                r0 = i * chunk_rec
                m = min(chunk_rec, self.n_rec - r0)
                cp.wait_event(done[b])
                with torch.cuda.stream(cp):
                    bufs[b][: m * self.stride].copy_(host[r0 * self.stride:(r0 + m) * self.stride], non_blocking=True)
                copied[b].record(cp)
                dc.wait_event(copied[b])
                N.check(self.L.cbx_decode_fixed(self.h, bufs[b].data_ptr(), m, self.stride, 0, r0, outs[b][1],
                                                dstream))
                done[b].record(dc)

        run()                          # warm-up pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(passes):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / passes
        N.check(self.L.cbx_plan_check(self.h, dstream))
        del host
        return {"value": round(self.in_bytes / dt / 1e9, 3), "unit": "GB/s", "records_per_s": round(self.n_rec / dt, 1),
                "ms_per_pass": round(dt * 1e3, 3),
                "how": f"{n_chunks} chunks of {chunk_rec} records: pinned-host H2D on a copy stream overlapped with "
                       "cbx_decode_fixed of the previous chunk (double-buffered), per rank"}

    def payload(self):
        return _payload(self.cols, self.n_rec)


def present_elements(plan, cols, n_rec: int):
    """Per value column under one OCCURS DEPENDING ON level: the elements the records hold (the sum
    of the array's count column); columns under fixed OCCURS or deeper nesting keep every slot."""
    import torch
    out = {}
    for f in plan.fields:
        if f.n_dims != 1:
            continue
        ar = plan.arrays[f.dim_array[0]]
        if ar.dependee < 0 or ar.count_column < 0:
            continue
        cnt = cols[ar.count_column]["values"][:n_rec].to(dtype=torch.int64)
        if ar.segment >= 0 and plan.segment_column >= 0:   # arrays of an inactive segment redefine are absent
            seg = cols[plan.segment_column]["values"][:n_rec]
            cnt = cnt * (seg == ar.segment)
        out[f.column] = int(cnt.sum().item())
    return out


def _payload(cols, n_rec: int) -> int:
    """String payload bytes the last decode wrote to data buffers: per-slot sizes (offsets layout)
    or the lengths of views longer than 12 bytes (view layout)."""
    import torch
    tot = 0
    for c in cols:
        if "sizes" in c:
            tot += int(c["sizes"].sum().item())
        elif "views" in c:
            pitch = 64 * ((n_rec + 63) // 64)
            ln = c["views"].view(-1, pitch, 16)[:, :n_rec].reshape(-1, 16)[:, :4].contiguous().view(torch.int32).view(-1)
            tot += int(torch.where(ln > 12, ln, 0).to(torch.int64).sum().item())
    return tot


class _VarLen:
    """C4 / C5: one file (per rank: its shard, a contiguous run of the global file's index entries).

    Setup (untimed, as the reference's index pass is a separate Spark job): the shard is framed
    once on the GPU from its start and cut into sparse-index entries by cbx_sparse_index (100 MB
    entries at root segments); the entries' offsets seed every step's framing.  A step = RDW framing
    seeded by the entries + (N > 1) one all-gather of the shard's record count, whose exclusive
    prefix is the shard's Record_Id base (cobrix_amd/shard.py record_bases) + decode."""

    def __init__(self, name, n_rec, dev, rank, window, views, lists=True):
        import torch
        from cobrix_amd import synth
        from cobrix_amd.reader import ReaderParameters, VarLenNestedReader
        if name == "rdw_narrow":
            self.raw, hdr = synth.rdw_narrow_large(n_rec, seed=20261016 + rank, device=dev)
            cb, segs = synth.RDW_NARROW_COPYBOOK, synth.RDW_NARROW_SEGMENTS
        else:
            self.raw, hdr = synth.wide_odo(n_rec, seed=20261018 + rank, device=dev)
            cb, segs = synth.WIDE_ODO_COPYBOOK, synth.WIDE_ODO_SEGMENTS
        self.in_bytes = int(self.raw.numel())
        self.n_expected = int(hdr.numel())
        del hdr
        torch.cuda.synchronize()
        # segment_id_root only shapes the index (cuts at roots); the decode plan is the C4/C5 one
        self.rd = VarLenNestedReader(cb, ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                                                          segment_id_redefine_map=segs, window_bytes=window,
                                                          string_views=views, occurs_lists=lists))
        idx_rd = VarLenNestedReader(cb, ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                                                         segment_id_levels=["C"], input_split_size_mb=100))
        t0 = time.perf_counter()
        off, ln = idx_rd.frame(self.raw, self.in_bytes)
        self.entries = idx_rd.generate_index(self.raw, self.in_bytes, off, ln)
        torch.cuda.synchronize()
        self.index_ms = (time.perf_counter() - t0) * 1e3
        self.seeds = [e.offset_from for e in self.entries]
        del off, ln, idx_rd
        self.dev = dev

    def prepare(self, stream):
        import torch
        from cobrix_amd import native as N
        from cobrix_amd.reader import _alloc_columns, string_capacity
        self.L, self.h, self.stream = N.load(), self.rd.native.handle, ctypes.c_void_p(stream.cuda_stream)
        self.cap = self.n_expected + 1
        self.off = torch.empty(self.cap, dtype=torch.int64, device=self.dev)
        self.ln = torch.empty(self.cap, dtype=torch.int32, device=self.dev)
        self.sd = (ctypes.c_int64 * len(self.seeds))(*self.seeds)
        self.prm = self.rd.rdw_params()
        self.nfr = ctypes.c_int64(0)
        self.n_rec = self.n_expected
        self.cols, self.cs = _alloc_columns(self.rd.plan, self.n_rec, string_capacity(self.rd.native, self.n_rec),
                                            self.dev)
        self.fr0, self.fr1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.record_base = 0

    def step(self, world=1):
        from cobrix_amd import native as N
        from cobrix_amd.shard import record_bases
        self.fr0.record()
        N.check(self.L.cbx_frame_rdw(self.raw.data_ptr(), self.in_bytes, self.sd, len(self.seeds),
                                     ctypes.byref(self.prm), self.off.data_ptr(), self.ln.data_ptr(), self.cap,
                                     ctypes.byref(self.nfr), self.stream))
        self.fr1.record()
        if self.nfr.value != self.n_expected:
            raise RuntimeError(f"framing found {self.nfr.value} records, generator wrote {self.n_expected}")
        if world > 1:
            self.record_base, _ = record_bases(self.nfr.value)     # Record_Id base of this shard
        N.check(self.L.cbx_decode_var(self.h, self.raw.data_ptr(), self.in_bytes, self.off.data_ptr(),
                                      self.ln.data_ptr(), self.n_rec, 0, self.record_base, self.cs, self.stream))
        return (self.fr0, self.fr1)

    def end_to_end(self):
        return None

    def payload(self):
        return _payload(self.cols, self.n_rec)


def _probe_reference_jvm():
    """the reference CPU path runs only where a JVM + Spark + a Cobrix jar exist."""
    import shutil
    found = {t: shutil.which(t) for t in ("java", "spark-submit")}
    if all(found.values()):
        return "java and spark-submit present (reference run not wired into this bench)"
    return "probed on this host: " + ", ".join(f"{t} {'found' if v else 'absent'}" for t, v in found.items()) + \
        " -- the reference Cobrix/Spark CPU path cannot run here; the oracle restatement is timed instead"


def _cpu_threads() -> int:
    """Host cores of this GPU's share: a 1-GPU box exposes the whole machine in nproc but allots 16
    CPUs per GPU (CBX_CPU_THREADS overrides)."""
    return int(os.environ.get("CBX_CPU_THREADS", str(min(16, os.cpu_count() or 1))))


def _cpu_baseline(workload: str, seconds: float = 10.0):
    """The oracle (scalar C restatement of the reference decoders) on a bounded sample of the same
    workload, at 1 thread and at the GPU's host-core share (threads over record chunks: ctypes
    releases the GIL inside the C calls).  For RDW workloads the header walk stays sequential, as
    the reference's index pass is per file (IndexGenerator.scala:61-120); decode is split."""
    import threading
    import numpy as np
    from cobrix_amd.copybook import parse_copybook
    from cobrix_amd import synth
    from oracle import oracle as O
    fixed = workload in ("syn200", "synstr200")
    if fixed:
        text, gen, size = ((synth.SYN200_COPYBOOK, synth.syn200, 200) if workload == "syn200"
                           else (synth.SYNSTR200_COPYBOOK, synth.synstr200, 200))
        cb = parse_copybook(text, code_page="common" if workload == "syn200" else "cp037")
    else:
        text, gen = ((synth.RDW_NARROW_COPYBOOK, synth.rdw_narrow) if workload == "rdw_narrow"
                     else (synth.WIDE_ODO_COPYBOOK, synth.wide_odo))
        cb = parse_copybook(text, segment_redefines=["STATIC-DETAILS", "CONTACTS"])
    ast = O.OracleAst(cb)
    lib = O.lib()
    chunk = 20_000 if workload != "wide_odo" else 50

    def make(n, seed):
        if fixed:
            data = gen(n, seed=seed).numpy().tobytes()
            return data, None, None, None
        raw = gen(n, seed=seed)[0].numpy().tobytes()
        t0 = time.perf_counter()
        off, ln = O.frame_rdw(raw)                          # sequential header walk (timed below)
        t_frame = time.perf_counter() - t0
        act = np.array([ast.names.get("STATIC_DETAILS" if raw[o] == 0xC3 else "CONTACTS") for o in off], np.int32)
        return raw, (off, ln, act), t_frame, None

    def decode_range(data, fr, r0, r1):
        ev = np.zeros(chunk * ast.max_events_per_record(), dtype=O.EVENT_DTYPE)
        heap = np.zeros(chunk * ast.max_heap_per_record() + 64, dtype=np.uint8)
        n_ev, hl = ctypes.c_int64(0), ctypes.c_int64(0)
        buf = np.frombuffer(data, dtype=np.uint8)
        for c0 in range(r0, r1, chunk):
            c1 = min(r1, c0 + chunk)
            n_ev.value = hl.value = 0
            if fixed:
                r = lib.ora_decode_fixed(ctypes.addressof(ast.nodes), 0, ctypes.addressof(ast.handlers),
                                         ctypes.addressof(ast.opts), buf[c0 * size:].ctypes.data, c1 - c0, size, 0, -1, 0,
                                         None, 0, ev.ctypes.data, len(ev), ctypes.byref(n_ev), heap.ctypes.data,
                                         len(heap), ctypes.byref(hl))
            else:
                off, ln, act = fr
                r = lib.ora_extract_var(ctypes.addressof(ast.nodes), 0, ctypes.addressof(ast.handlers),
                                        ctypes.addressof(ast.opts), buf.ctypes.data, off[c0:].ctypes.data,
                                        ln[c0:].ctypes.data, act[c0:].ctypes.data, c1 - c0, 0, ev.ctypes.data, len(ev),
                                        ctypes.byref(n_ev), heap.ctypes.data, len(heap), ctypes.byref(hl))
            if r != 0:
                raise RuntimeError(f"oracle decode failed {r}")

    def timed(data, fr, t_frame, threads):
        n = (len(data) // size) if fixed else len(fr[0])
        bounds = [n * t // threads for t in range(threads + 1)]
        ths = [threading.Thread(target=decode_range, args=(data, fr, bounds[t], bounds[t + 1])) for t in range(threads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0 + (t_frame or 0.0), n

    n0 = 4000 if workload != "wide_odo" else 40
    d0, f0, tf0, _ = make(n0, 99)
    dt, _ = timed(d0, f0, tf0, 1)
    n = int(min(max(n0 / max(dt, 1e-9) * seconds, n0), 6_000_000 if workload != "wide_odo" else 60_000))
    data, fr, t_frame, _ = make(n, 100)
    dt1, nrec = timed(data, fr, t_frame, 1)
    T = _cpu_threads()
    dtT, _ = timed(data, fr, t_frame, T)
    unit_n = {"syn200": "SYN200 records", "synstr200": "SYNSTR200 records", "rdw_narrow": "RDW records",
              "wide_odo": "root records (+ children)"}[workload]
    return {"value": round(len(data) / dtT / 1e9, 6), "unit": "GB/s", "cores": T, "kind": "port",
            "value_1_core": round(len(data) / dt1 / 1e9, 6),
            "sample": f"{n} {unit_n} ({len(data) / 1e6:.1f} MB, {nrec} records) through oracle/cobrix_oracle.c "
                      f"(restatement of extractRecord + decoders{'' if fixed else '; RDW header walk sequential'}): "
                      f"{dt1:.1f} s at 1 thread, {dtT:.2f} s at {T} threads",
            "reference_jvm": _probe_reference_jvm()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="syn200", choices=sorted(WORKLOADS))
    ap.add_argument("--records", type=int, default=0, help="records per GPU (root records for wide_odo); "
                                                           "0 = the workload's default")
    ap.add_argument("--window", type=int, default=0, help="LDS window bytes (0 = plan default)")
    ap.add_argument("--strings", default="views", choices=["views", "offsets"],
                    help="string column layout: Arrow string views (one pass) or Arrow large-string offsets")
    ap.add_argument("--occurs", default="lists", choices=["lists", "slots"],
                    help="OCCURS DEPENDING ON layout: Arrow lists (present elements) or one slot row per element")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from cobrix_amd import native as N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    W = WORKLOADS[args.workload]
    n_req = args.records or W["records"]

    def progress(msg):
        if rank == 0:
            print(f"[bench {args.workload}] {msg}", file=sys.stderr, flush=True)

    progress(f"generating {n_req} records on {dev}")
    views = args.strings == "views"
    if args.workload in ("syn200", "synstr200"):
        job = _Fixed(args.workload, n_req, dev, rank, args.window, views)
    else:
        job = _VarLen(args.workload, n_req, dev, rank, args.window, views, args.occurs == "lists")
    st = torch.cuda.current_stream()
    progress(f"{job.in_bytes / 1e9:.2f} GB generated; allocating columns")
    job.prepare(st)
    progress("warm-up")
    L, h = job.L, job.h

    def step():
        return job.step(world)

    for _ in range(args.warmup):
        step()
    N.check(L.cbx_plan_check(h, job.stream))
    N.check(L.cbx_plan_set_profiling(h, 1))
    frame_ev = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fr = step()
        if fr is not None:
            frame_ev.append(fr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    N.check(L.cbx_plan_check(h, job.stream))
    dec = (ctypes.c_float * args.steps)()
    fix = (ctypes.c_float * args.steps)()
    nc = ctypes.c_int32()
    N.check(L.cbx_plan_kernel_times(h, dec, fix, args.steps, ctypes.byref(nc)))
    N.check(L.cbx_plan_set_profiling(h, 0))
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    n_rec = job.n_rec
    payload = job.payload()
    steps = args.steps
    ms_per_step = elapsed / steps * 1e3
    gbs = job.in_bytes * world / (elapsed / steps) / 1e9
    recs_per_s = n_rec * world / (elapsed / steps)
    alg = algorithmic_bytes(job.rd.plan, n_rec, job.in_bytes, payload, present_elements(job.rd.plan, job.cols, n_rec))
    dec_avg_ms = sum(dec[: nc.value]) / max(1, nc.value)
    fix_avg_ms = sum(fix[: nc.value]) / max(1, nc.value)
    achieved = alg / (dec_avg_ms * 1e-3) / 1e9
    kind = ctypes.c_int32(0)
    N.check(L.cbx_plan_kernel_kind(h, ctypes.byref(kind)))
    kname = "cbx_jit_decode (copybook-specialised, hipRTC)" if kind.value == 1 else "cbx::decode_kernel (table-driven)"
    lists = any(c.list_array >= 0 for c in job.rd.plan.columns)
    if lists:   # the OCCURS list elements: the element-parallel kernel launched right after the decode kernel
        kname += " + cbx::list_kernel (OCCURS lists; decode_kernel time covers both)"
    tag = f"{args.workload}_{args.strings}{'' if args.occurs == 'lists' else '_slots'}_{n_rec}"
    traffic, traffic_src = measured_traffic(tag)
    kernel_ms = {"decode_kernel": round(dec_avg_ms, 4),
                 ("post_kernels (deferred-value fixup)" if views else
                  "post_kernels (deferred-value fixup, string scan + placement)"): round(fix_avg_ms, 4)}
    if frame_ev:
        fms = sum(a.elapsed_time(b) for a, b in frame_ev) / len(frame_ev)
        kernel_ms["rdw_framing (cbx_frame_rdw incl. count readback)"] = round(fms, 4)
    if hasattr(job, "entries"):
        kernel_ms["sparse_index_setup (untimed: frame + cbx_sparse_index, once)"] = round(job.index_ms, 3)
    e2e = None
    if not args.no_end_to_end and world == 1:
        progress("end-to-end (pinned host -> HBM) pass")
        e2e = job.end_to_end()
    progress("cpu baseline" if not args.no_cpu_baseline and world == 1 else "done")
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(gbs, 3),
            "unit": "GB/s",
            "records_per_s": round(recs_per_s, 1),
            "hbm_frac_step": round(alg / (elapsed / steps) / 1e9 / HBM_PEAK_GBS, 4),
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": W["data"],
            "config": {"workload": W["desc"], "baseline_config": W["config"],
                       "records_per_gpu": n_rec, "input_bytes_per_gpu": job.in_bytes,
                       "input_gb_per_gpu": round(job.in_bytes / 1e9, 3),
                       "output_columns": job.rd.plan.n_columns, "parallelism": f"dp{world}",
                       "string_layout": "Arrow string views (16 B views + long payloads, one pass)" if views
                       else "Arrow large-string (int64 offsets + payload, scan + placement)",
                       "occurs_layout": "Arrow lists (present elements only)" if args.occurs == "lists"
                       else "one slot row per element",
                       "inputs_resident_in_hbm": True},
            "kernel_ms": kernel_ms,
            **({"seeds": f"{len(job.entries)} sparse-index entries from cbx_sparse_index (100 MB, root segments)"}
               if hasattr(job, "entries") else {}),
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": alg, "traffic": traffic,
                         "traffic_source": traffic_src},
        }
        if e2e is not None:
            out["end_to_end"] = e2e
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = _cpu_baseline(args.workload)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
