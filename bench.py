"""Benchmark: GPU decode of the BASELINE.json configs (default: config C2, SYN200 numeric mix).

`python bench.py --gpus N --steps K --warmup W [--workload syn200|synstr200|rdw_narrow|wide_odo]`
-- one rank per GPU.  With N > 1 and no torchrun environment, bench.py starts the N ranks itself
(`python -m torch.distributed.run --nproc-per-node N ... bench.py`, before anything touches a GPU)
and exits with their status; under torchrun (the driver's launch) it checks WORLD_SIZE == N.
Rank 0 prints ONE JSON line.

Shards, weak scaling -- the per-GPU work is fixed as N grows:
  fixed-length (C2, C3): rank r decodes records [r n, (r + 1) n) of an N n-record job; the
      Record_Id base r n is static, there is no collective on the data path;
  variable-length (C4, C5): ONE RDW file of N blocks (block b generated with seed + b) is indexed
      once at setup (GPU framing + cbx_sparse_index, untimed like the reference's index job); rank r
      takes the contiguous run of index entries shard.entry_shards gives it (balanced by bytes) and
      keeps only those bytes.  A step frames the run from its entries' offsets, all-gathers the
      run's record count on the device (RCCL, int64 per rank), and decodes with the exclusive
      prefix as its Record_Id base -- a device pointer (cbx_plan_set_record_base), no host read.

A step = one full decode of the shard through the C ABI:
  fixed-length: `cbx_decode_fixed` -- decode kernel + fixup of deferred values (+ string scan and
      placement in the large-string layout);
  variable-length: `cbx_frame_rdw` (RDW offset discovery seeded by the shard's index entries) +
      `cbx_decode_var`.

roofline: algorithmic bytes = input bytes + for every output value its Arrow
width (int32 4, int64 8, decimal <= 18 digits 8, <= 38 16, float 4, double 8), 1 validity bit per
value, strings as UTF-8 payload + a 4-byte offset per value, OCCURS DEPENDING ON lists as a 4-byte
offset per list; absent ODO elements count nothing.  The layout actually written (16-byte string
views, int64 offsets, count / segment columns) is reported as `layout_overhead` beside it, never in
`achieved`.  achieved = algorithmic bytes / the decode kernel's average duration (HIP events recorded
by the library on the launch stream over the timed steps, cbx_plan_kernel_times); the rocprofv3
summary of the same command is committed under profiles/ (tools/evidence.sh).

end_to_end (N = 1): the same shard streamed from pinned host memory -- fixed-length: 2.5 M-record
chunks; variable-length: pieces of whole index entries (their offsets seed the framing of the
piece) -- H2D on a copy stream overlapped with the framing / decode of the previous piece on the
decode stream (double-buffered); reported beside `value`, never as it.
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
HBM_MEASURED_GBS = 6300.0  # achievable (MI355X_MICROARCH.md, HBM)
METRIC = "decoded input GB/s + records/s, fixed-len COMP-3 mix, 1-8 MI355X; % HBM peak"


# ------------------------------------------------------------------------------------------------
# SURVEY.md 8(d) byte counts
# ------------------------------------------------------------------------------------------------
def _valid_mask(c, n_slots: int, n_rec: int):
    """Validity bits of the n_rec records of every slot row as a bool tensor [n_slots, n_rec]."""
    import torch
    pw = (n_rec + 63) // 64
    b = c["validity"][: n_slots * pw].view(torch.uint8).view(n_slots, pw * 8)
    bits = (b.unsqueeze(-1) >> torch.arange(8, device=b.device, dtype=torch.uint8)) & 1
    return bits.view(n_slots, pw * 64)[:, :n_rec].bool()


def string_payload(plan, cols, n_rec: int) -> dict:
    """Per string column: UTF-8 payload bytes of the batch's values (all of them, whatever the layout:
    the view lengths, or the offsets layout's per-slot sizes)."""
    import torch
    from cobrix_amd import native as N
    out = {}
    pitch = 64 * ((n_rec + 63) // 64)
    for ci, info in enumerate(plan.columns):
        if info.out_type not in (N.O_STRING, N.O_BINARY):
            continue
        c = cols[ci]
        if "sizes" in c:
            out[ci] = int(c["sizes"].sum().item())
        elif "views" in c:
            ln = c["views"].view(-1, pitch, 16)[:, :n_rec, :4].contiguous().view(torch.int32).view(info.n_slots, n_rec)
            out[ci] = int((ln.to(torch.int64) * _valid_mask(c, info.n_slots, n_rec)).sum().item())
        elif "offsets32" in c:
            offs = c["offsets32"].view(info.n_slots, pitch + 1)
            out[ci] = int((offs[:, n_rec].to(torch.int64) - offs[:, 0].to(torch.int64)).sum().item())
    return out


def present_elements(plan, cols, n_rec: int):
    """Per value column under one OCCURS DEPENDING ON level: the elements the records hold (the sum
    of the array's valid counts); columns under fixed OCCURS or deeper nesting keep every slot."""
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


def absent_element_bytes(plan, cols, n_rec: int) -> int:
    """Input bytes of OCCURS DEPENDING ON elements past each record's count (records keep every
    element's bytes at max size: variable_size_occurs = false): the list layout's kernels never read
    them, so they are part of the 8(d) input term but not of the bytes the decode must move."""
    import torch
    total, seen = 0, set()
    for f in plan.fields:
        if f.n_dims != 1:
            continue
        ai = f.dim_array[0]
        ar = plan.arrays[ai]
        if ai in seen or ar.dependee < 0 or ar.count_column < 0:
            continue
        seen.add(ai)
        cnt = cols[ar.count_column]["values"][:n_rec].to(dtype=torch.int64)
        hold = torch.ones_like(cnt, dtype=torch.bool)
        if ar.segment >= 0 and plan.segment_column >= 0:
            hold = cols[plan.segment_column]["values"][:n_rec] == ar.segment
        total += int(((f.dim_count[0] - cnt) * hold).sum().item()) * int(f.dim_stride[0])
    return total


def algorithmic_bytes(plan, n_rec: int, in_bytes: int, payload: dict, present: dict) -> int:
    """input + Arrow output bytes (see the module docstring), independent of the layout
    the library writes."""
    from cobrix_amd import native as N
    total = in_bytes
    for ci, info in enumerate(plan.columns):
        n = present.get(ci, n_rec * info.n_slots)
        if info.kind == "count":
            # one list per (record, enclosing slot): a 4-byte offset + a validity bit
            total += 4 * n + (n + 7) // 8
        elif info.kind in ("list_offsets", "segment"):
            continue                     # the list offsets are the count's; the segment index is the structs' bit
        elif info.out_type in (N.O_STRING, N.O_BINARY):
            total += 4 * n + payload.get(ci, 0) + (n + 7) // 8
        else:
            total += n * N.OUT_WIDTH[info.out_type] + (n + 7) // 8
    total += len(plan.segment_groups) * ((n_rec + 7) // 8)   # validity of each segment-redefine struct
    return total


def layout_bytes(plan, cols, n_rec: int, in_bytes: int, payload: dict, present: dict) -> int:
    """Bytes the chosen layout writes for the same batch (views / int64 offsets / count, list-offset
    and segment columns, padded list runs): the algorithmic count plus the layout's overhead."""
    from cobrix_amd import native as N
    total = in_bytes
    pitch = 64 * ((n_rec + 63) // 64)
    for ci, info in enumerate(plan.columns):
        c = cols[ci]
        n = n_rec * info.n_slots if info.list_array < 0 else present.get(ci, n_rec * info.n_slots)
        total += (n + 7) // 8
        if "views" in c:
            total += 16 * n + _long_view_payload(c, info.n_slots, n_rec, pitch)
        elif "offsets" in c:
            total += 8 * (n + info.n_slots) + payload.get(ci, 0)
        elif "offsets32" in c:
            total += 4 * (n + info.n_slots) + payload.get(ci, 0)
        else:
            total += n * N.OUT_WIDTH[info.out_type]
    return total


def _long_view_payload(c, n_slots: int, n_rec: int, pitch: int) -> int:
    import torch
    ln = c["views"].view(-1, pitch, 16)[:, :n_rec, :4].contiguous().view(torch.int32).view(n_slots, n_rec)
    ln = ln * _valid_mask(c, n_slots, n_rec)
    return int(torch.where(ln > 12, ln, 0).to(torch.int64).sum().item())


def _round_key(path: str):
    """Natural order of profiles/<round>_<variant> directories (r02_b after r02_a, r01_v10 after r01_v9)."""
    import re
    d = os.path.basename(os.path.dirname(path))
    return [int(x) if x.isdigit() else x for x in re.split(r"(\d+)", d)]


def measured_traffic(tag: str):
    """HBM bytes per decode-kernel launch from the newest committed rocprofv3 FETCH_SIZE/WRITE_SIZE
    passes of this configuration (tools/evidence.sh -> profiles/<round tag>/traffic_<tag>.json)."""
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
    "syn200": dict(records=50_000_000, config="C2", strings="views",
                   desc="SYN200: fixed-length 200-byte EBCDIC records, numeric mix (COMP, COMP-3, zoned DISPLAY "
                        "overpunch, IBM COMP-2, cp037 X(18)) -- BASELINE config C2",
                   data="synthetic (cobrix_amd/synth.py SYN200, seed 20261015+rank, 0.5% malformed numerics)"),
    # C3 is quoted on 64 GB strong-scaled: 320 M records over the job, decoded in
    # batches whose int32 Utf8 offsets fit (an Arrow chunked array: one chunk per batch and column)
    "synstr200": dict(records=320_000_000, config="C3", strings="offsets", strong=True,
                      batch_records=50_000_000, pipeline="0,0",
                      desc="SYNSTR200: fixed-length 200-byte records, 10 x PIC X(20) cp037 -> UTF-8, trim both "
                           "-- BASELINE config C3 (64 GB strong-scaled over the job)",
                      data="synthetic (cobrix_amd/synth.py SYNSTR200: lengths 0-20, 25% accented, 10% leading "
                           "spaces, 1% control bytes)"),
    # C4 in the Utf8 layout (--strings offsets): batches whose int32 offsets fit the widest column's worst
    # case (X(28) -> <= 56 UTF-8 bytes per value)
    "rdw_narrow": dict(records=150_000_000, config="C4", strings="views", batch_records=37_500_000,
                       desc="RDW multisegment file, exp2/test5 layout (C 68 B / P 64 B records, segment redefines, "
                            "File_Id + Record_Id), GPU RDW offset discovery seeded by sparse-index entries + var-len "
                            "decode -- BASELINE config C4",
                       data="synthetic (cobrix_amd/synth.py rdw_narrow, 35% root segments; one file of N blocks)"),
    "wide_odo": dict(records=770_000, config="C5", strings="views",
                     desc="Wide multisegment RDW file (exp3 layout + OCCURS 0 TO 2000 DEPENDING ON, 16,070 B roots, "
                          "64 B children, File_Id + Record_Id) -- BASELINE config C5 (per-GPU shard of the 8-GPU job)",
                     data="synthetic (cobrix_amd/synth.py wide_odo, element counts uniform 0-2000, 0-4 children; "
                          "one file of N blocks)"),
}

STRING_LAYOUTS = {
    "views": "Arrow string views (16 B views + long payloads, one pass)",
    "offsets": "Arrow Utf8 (int32 offsets + payload: count pass, device scan, written once in place)",
    "large": "Arrow large-string (int64 offsets + payload: scratch, scan, placement pass)",
}


def _layout_params(strings: str) -> dict:
    return {"string_views": strings == "views", "string_utf8": strings == "offsets"}


class _Fixed:
    """A fixed-length shard resident in HBM, decoded as one call per batch of at most batch_records
    records (every batch its own output columns: for the Utf8 layout one Arrow array per batch and
    column -- a chunked array -- whose int32 offsets fit its slot region)."""

    def __init__(self, name, n_rec, dev, rank, window, strings, batch_records=0, record_base=None, pipeline=""):
        import torch
        from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters
        from cobrix_amd import synth
        lay = _layout_params(strings)
        self.batch = batch_records if batch_records > 0 else n_rec
        if name == "syn200":
            cb, self.stride = synth.SYN200_COPYBOOK, synth.SYN200_RECORD_SIZE
            self.rec = synth.syn200(n_rec, seed=20261015 + rank, device=dev).view(-1)
            params = ReaderParameters(window_bytes=window, **lay)
        else:
            cb, self.stride = synth.SYNSTR200_COPYBOOK, synth.SYNSTR200_RECORD_SIZE
            self.rec = synth.synstr200(n_rec, seed=20261017 + rank, device=dev).view(-1)
            params = ReaderParameters(window_bytes=window, ebcdic_code_page="cp037", **lay)
        torch.cuda.synchronize()
        self.rd = FixedLenNestedReader(cb, params)
        # --pipeline C,D: odd batches on a second plan and stream (cbx_plan_pipeline)
        self.pipe = tuple(int(x) for x in pipeline.split(",")) if pipeline else None
        self.rdB = FixedLenNestedReader(cb, params) if self.pipe and self.batch < n_rec else None
        self.n_rec, self.in_bytes, self.dev = n_rec, n_rec * self.stride, dev
        self.record_base = rank * n_rec if record_base is None else record_base
        self.shard_note = f"records [{self.record_base}, {self.record_base + n_rec}) of the job, Record_Id base static"
        if self.batch < n_rec:
            self.shard_note += f"; {(n_rec + self.batch - 1) // self.batch} batches of <= {self.batch} records"

    def prepare(self, stream):
        from cobrix_amd import native as N
        from cobrix_amd.reader import _alloc_columns, string_capacity
        self.L, self.h, self.stream = N.load(), self.rd.native.handle, ctypes.c_void_p(stream.cuda_stream)
        self.targets = [(self.h, self.stream)]
        if self.rdB is not None:
            import torch
            self.streamB = torch.cuda.Stream(self.dev)
            hB = self.rdB.native.handle
            N.check(self.L.cbx_plan_pipeline(self.h, hB, self.pipe[0], self.pipe[1]))
            self.targets.append((hB, ctypes.c_void_p(self.streamB.cuda_stream)))
            self.shard_note += (f"; batches alternating between two plans on two streams (cbx_plan_pipeline: count pass "
                                f"beside the other plan's decode, {self.pipe[0]} / {self.pipe[1]} workgroups per CU)")
        # parts: (first record, records, columns, cbx_column table) per batch
        self.parts = []
        for r0 in range(0, self.n_rec, self.batch):
            m = min(self.batch, self.n_rec - r0)
            cols, cs = _alloc_columns(self.rd.plan, m, string_capacity(self.rd.native, m), self.dev)
            self.parts.append((r0, m, cols, cs))
        self.cols, self.cs = self.parts[0][2], self.parts[0][3]

    def calls_per_step(self) -> int:
        return (len(self.parts) + len(self.targets) - 1) // len(self.targets)   # (the profiled plan's calls)

    def pipelined(self) -> bool:
        return len(self.targets) > 1

    def step(self, world=1):
        from cobrix_amd import native as N
        # fixed-length shards: rank r holds records [r n, (r + 1) n) -- the Record_Id base is static
        for i, (r0, m, _, cs) in enumerate(self.parts):
            h, st = self.targets[i % len(self.targets)]
            N.check(self.L.cbx_decode_fixed(h, self.rec.data_ptr() + r0 * self.stride, m, self.stride, 0,
                                            self.record_base + r0, cs, st))
        return None

    def verify(self, world):
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


def _host_staged() -> bool:
    """gloo backend (--dist-backend gloo): collectives on device tensors go through host copies."""
    import torch.distributed as dist
    return dist.is_initialized() and dist.get_backend() == "gloo"


def _all_reduce(t, op=None):
    import torch.distributed as dist
    op = op if op is not None else dist.ReduceOp.SUM
    if _host_staged() and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def _all_gather_into(out, inp):
    import torch
    import torch.distributed as dist
    if _host_staged() and inp.is_cuda:
        parts = [torch.empty_like(inp, device="cpu") for _ in range(dist.get_world_size())]
        dist.all_gather(parts, inp.cpu())
        out.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(out, inp)


def _frame_rdw(L, data, n_bytes, seeds, prm, cap, dev, stream):
    """cbx_frame_rdw into fresh (offsets, lengths) tensors of `cap` records -> (off, len, n)."""
    import torch
    from cobrix_amd import native as N
    off = torch.empty(max(1, cap), dtype=torch.int64, device=dev)
    ln = torch.empty(max(1, cap), dtype=torch.int32, device=dev)
    sd = (ctypes.c_int64 * len(seeds))(*seeds)
    n = ctypes.c_int64(0)
    N.check(L.cbx_frame_rdw(data.data_ptr(), n_bytes, sd, len(seeds), ctypes.byref(prm), off.data_ptr(),
                            ln.data_ptr(), cap, ctypes.byref(n), stream))
    return off, ln, n.value


class _VarLen:
    """C4 / C5: one RDW file of `world` blocks; this rank keeps the bytes of its run of index entries.

    Setup (untimed, as the reference's index pass is a separate Spark job): the file is framed on the
    GPU (the block starts are known record boundaries and seed the walk with the file start) and cut
    into sparse-index entries by cbx_sparse_index (`seed_mb`: the 100 MB default, reset at each entry,
    or a 32 MB block size, subtracted -- VarLenNestedReader.scala:237-243) at root segments.  A step =
    RDW framing of the run seeded by its entries + (N > 1) one device all-gather of the run's record
    count, whose exclusive prefix is the run's Record_Id base + decode."""

    def __init__(self, name, n_rec, dev, rank, world, window, strings, lists=True, seed_mb=100, batch_records=0,
                 pieces=1):
        import torch
        import torch.distributed as dist
        from cobrix_amd import native as N
        from cobrix_amd import synth
        from cobrix_amd.reader import ReaderParameters, VarLenNestedReader
        from cobrix_amd.shard import entry_shards, index_chain
        if name == "rdw_narrow":
            gen = lambda b, out=None: synth.rdw_narrow_large(n_rec, seed=20261016 + b, device=dev, out=out)  # noqa: E731
            size = lambda b: synth.rdw_narrow_large_size(n_rec, seed=20261016 + b, device=dev)  # noqa: E731
            cb, segs = synth.RDW_NARROW_COPYBOOK, synth.RDW_NARROW_SEGMENTS
        else:
            gen = lambda b, out=None: synth.wide_odo(n_rec, seed=20261018 + b, device=dev, out=out)  # noqa: E731
            size = lambda b: synth.wide_odo_size(n_rec, seed=20261018 + b, device=dev)  # noqa: E731
            cb, segs = synth.WIDE_ODO_COPYBOOK, synth.WIDE_ODO_SEGMENTS
        self.dev, self.world, self.rank = dev, world, rank
        self.batch = batch_records
        self.n_pieces = pieces
        self.seed_recs = None   # records of the run before each seed (the setup framing), for pieces
        L = N.load()
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        opts = dict(is_record_sequence=True, segment_field="SEGMENT-ID", segment_id_redefine_map=segs,
                    window_bytes=window, occurs_lists=lists, generate_record_id=True, **_layout_params(strings))
        self.rd = VarLenNestedReader(cb, ReaderParameters(**opts))
        # segment_id_root only shapes the index (cuts at roots); the decode plan is the C4/C5 one
        ip = dict(is_record_sequence=True, segment_field="SEGMENT-ID", segment_id_levels=["C"])
        if seed_mb != 100:
            ip["hdfs_default_block_size_mb"] = seed_mb     # a block size: subtracted (VarLenNestedReader.scala:237-243)
        idx_rd = VarLenNestedReader(cb, ReaderParameters(**ip))
        self.prm = self.rd.rdw_params()
        self.seed_mb = seed_mb
        t0 = time.perf_counter()
        if world > 1:
            # O(shard) setup: rank r generates block r only (its size first, then in place behind a
            # room for one index entry of tail), and the file's index is built as a chain over the
            # ranks (shard.index_chain: the 100 MB default resets at every cut; a 32 MB block size is
            # subtracted, and the link carries the residual) -- each rank holds its block + the tail of
            # the file before it that its run starts in
            S = seed_mb * 1024 * 1024
            room = (S + (16 << 20) + 255) & ~255
            blen = size(rank)
            buf = torch.empty(room + blen, dtype=torch.uint8, device=dev)
            _, hdr = gen(rank, out=buf[room:])
            n_block = int(hdr.numel())
            del hdr

            def index_fn(region, start_bytes):
                n = int(region.numel())
                off, ln, nf = _frame_rdw(L, region, n, [0], self.prm, n_block + (n - blen) // 8 + 2, dev, st)
                ents = idx_rd.generate_index(region, n, off[:nf], ln[:nf], start_bytes=start_bytes)
                del off, ln
                return [(e.offset_from, e.record_index) for e in ents], nf

            res = index_chain(buf, room, index_fn, split_bytes=idx_rd.split_residual_bytes())
            torch.cuda.synchronize()
            self.index_ms = (time.perf_counter() - t0) * 1e3
            self.raw = res["run"]
            self.in_bytes = int(self.raw.numel())
            self.seeds = res["seeds"] or [0]
            self.expected_base, self.n_expected = res["record_base"], res["n_records"]
            counts = [None] * world
            dist.all_gather_object(counts, (len(res["entries"]), blen))
            k0 = sum(c[0] for c in counts[:rank])
            self.n_entries_file, self.entry_run = sum(c[0] for c in counts), (k0, k0 + len(res["entries"]))
            total_bytes, lo = sum(c[1] for c in counts), res["run_start"]
            self.setup_bytes_held = int(buf.numel())
            torch.cuda.empty_cache()
            self.shard_note = (f"entries [{k0}, {k0 + len(res['entries'])}) of the file's {self.n_entries_file} "
                               f"({seed_mb} MB index built as a chain over the ranks, shard.index_chain), bytes "
                               f"[{lo}, {lo + self.in_bytes}) of {total_bytes}; this rank generated and holds "
                               f"only its block + {room} bytes of room for the tail before it "
                               f"({self.setup_bytes_held / max(1, self.in_bytes):.3f} x its run); Record_Id base "
                               f"from a device all-gather of record counts")
            return
        # one GPU: the whole file, framed and indexed here
        full, hdr = gen(0)
        starts, n_total = [0], int(hdr.numel())
        del hdr
        torch.cuda.synchronize()
        total_bytes = int(full.numel())
        off, ln, nf = _frame_rdw(L, full, total_bytes, starts, self.prm, n_total + 1, dev, st)
        if nf != n_total:
            raise RuntimeError(f"setup framing found {nf} records, the generator wrote {n_total}")
        entries = idx_rd.generate_index(full, total_bytes, off[:nf], ln[:nf])
        torch.cuda.synchronize()
        self.index_ms = (time.perf_counter() - t0) * 1e3
        k0, k1 = entry_shards(entries, total_bytes, world)[rank]
        lo = entries[k0].offset_from if k0 < len(entries) else total_bytes
        hi = entries[k1].offset_from if k1 < len(entries) else total_bytes
        hdr_off = off[:nf] - 4                               # RDW header offsets of the framed records
        self.expected_base = int(torch.searchsorted(hdr_off, torch.tensor([lo], device=dev)).item())
        self.n_expected = int(torch.searchsorted(hdr_off, torch.tensor([hi], device=dev)).item()) - self.expected_base
        self.raw = full[lo:hi].clone() if world > 1 else full
        self.in_bytes = hi - lo
        self.seeds = [e.offset_from - lo for e in entries[k0:k1]] or [0]
        sd_abs = torch.tensor([lo + x for x in self.seeds], dtype=hdr_off.dtype, device=dev)
        self.seed_recs = [int(v) - self.expected_base for v in torch.searchsorted(hdr_off, sd_abs).tolist()]
        self.n_entries_file, self.entry_run = len(entries), (k0, k1)
        self.setup_bytes_held = int(self.raw.numel())
        del full, off, ln, hdr_off, idx_rd
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        self.shard_note = (f"entries [{k0}, {k1}) of the file's {len(entries)} ({seed_mb} MB index), bytes "
                           f"[{lo}, {hi}) of {total_bytes}; Record_Id base from a device all-gather of record counts")

    def prepare(self, stream):
        import torch
        from cobrix_amd import native as N
        from cobrix_amd.reader import _alloc_columns, string_capacity
        self.L, self.h, self.stream = N.load(), self.rd.native.handle, ctypes.c_void_p(stream.cuda_stream)
        self.cap = self.n_expected + 1
        self.off = torch.empty(self.cap, dtype=torch.int64, device=self.dev)
        self.ln = torch.empty(self.cap, dtype=torch.int32, device=self.dev)
        self.sd = (ctypes.c_int64 * len(self.seeds))(*self.seeds)
        self.state = torch.zeros(3, dtype=torch.int64, device=self.dev)   # cbx_frame_rdw_async outcome
        self.n_rec = self.n_expected
        # parts: (first record, records, columns, cbx_column table) per decode call -- the Utf8 layout
        # decodes the run in batches whose int32 offsets fit (one Arrow array per batch and column)
        self.batch = self.batch if 0 < self.batch < self.n_rec else max(1, self.n_rec)
        self.parts = []
        self.pieces = []
        if self.n_pieces > 1 and self.seed_recs is not None and len(self.seeds) > 1:
            # pieces: runs of whole index entries, each framed from its own entries and decoded as its
            # own batch (as the reference reads one partition per index entry), the framing of the
            # next pieces on a second stream beside the decode of this one
            # consecutive entries to a piece while it stays within n_rec / pieces records (and the batch)
            target = min(self.batch, -(-self.n_rec // self.n_pieces))
            ends = self.seed_recs[1:] + [self.n_rec]
            cuts = [0]
            for j in range(1, len(self.seeds)):
                if ends[j] - self.seed_recs[cuts[-1]] > target:
                    cuts.append(j)
            cuts.append(len(self.seeds))
            for i in range(len(cuts) - 1):
                a = self.seeds[cuts[i]]
                b = self.seeds[cuts[i + 1]] if cuts[i + 1] < len(self.seeds) else self.in_bytes
                r0 = self.seed_recs[cuts[i]]
                r1 = self.seed_recs[cuts[i + 1]] if cuts[i + 1] < len(self.seeds) else self.n_rec
                if r1 - r0 > self.batch and self.batch < self.n_rec:
                    raise RuntimeError(f"piece of {r1 - r0} records exceeds the batch of {self.batch}")
                sd = (ctypes.c_int64 * (cuts[i + 1] - cuts[i]))(*[x - a for x in self.seeds[cuts[i]:cuts[i + 1]]])
                cols, cs = _alloc_columns(self.rd.plan, r1 - r0, string_capacity(self.rd.native, r1 - r0), self.dev)
                self.parts.append((r0, r1 - r0, cols, cs))
                self.pieces.append(dict(a=a, b=b, sd=sd, r0=r0, m=r1 - r0,
                                        state=torch.zeros(3, dtype=torch.int64, device=self.dev),
                                        framed=torch.cuda.Event(), decoded=torch.cuda.Event()))
            self.fstream = torch.cuda.Stream(self.dev)
            self.fstream_p = ctypes.c_void_p(self.fstream.cuda_stream)
            self.shard_note += (f"; {len(self.pieces)} pieces of whole index entries, each framed (second stream) "
                                f"and decoded as its own batch, the framing beside the previous piece's decode")
        else:
            for r0 in range(0, max(1, self.n_rec), self.batch):
                m = min(self.batch, self.n_rec - r0)
                cols, cs = _alloc_columns(self.rd.plan, m, string_capacity(self.rd.native, m), self.dev)
                self.parts.append((r0, m, cols, cs))
            if len(self.parts) > 1:
                self.shard_note += f"; decoded in {len(self.parts)} batches of <= {self.batch} records"
        self.cols, self.cs = self.parts[0][2], self.parts[0][3]
        self.fr0, self.fr1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the run's Record_Id base lives on the device: the decode kernels read it (cbx_plan_set_record_base)
        self.base = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.gathered = torch.zeros(self.world, dtype=torch.int64, device=self.dev)
        N.check(self.L.cbx_plan_set_record_base(self.h, self.base.data_ptr()))

    def step(self, world=1):
        import torch.distributed as dist
        from cobrix_amd import native as N
        # no host wait inside the step: the framing's count stays on the device (cbx_frame_rdw_async),
        # is all-gathered there, and the decode runs over the count the index run predicts (checked
        # against the framing's after the timed steps, cbx_frame_rdw_state)
        if self.pieces:
            return self._step_pieces()
        self.fr0.record()
        N.check(self.L.cbx_frame_rdw_async(self.raw.data_ptr(), self.in_bytes, self.sd, len(self.seeds),
                                           ctypes.byref(self.prm), self.off.data_ptr(), self.ln.data_ptr(), self.cap,
                                           self.state.data_ptr(), 0, self.stream))
        self.fr1.record()
        if world > 1:   # Record_Id base = exclusive prefix of the ranks' counts, computed on the device
            _all_gather_into(self.gathered, self.state[:1])
            self.base.copy_(self.gathered[: self.rank].sum().view(1))
        for r0, m, _, cs in self.parts:
            N.check(self.L.cbx_decode_var(self.h, self.raw.data_ptr(), self.in_bytes, self.off.data_ptr() + 8 * r0,
                                          self.ln.data_ptr() + 4 * r0, m, 0, r0, cs, self.stream))
        return (self.fr0, self.fr1)

    def _step_pieces(self):
        """The run as pieces of index entries: piece k's framing on the second stream (after the previous
        step's decode of piece k read its offsets), piece k's decode on the launch stream after it."""
        import torch
        from cobrix_amd import native as N
        cur = torch.cuda.current_stream()
        base = self.raw.data_ptr()
        for i, pc in enumerate(self.pieces):
            self.fstream.wait_event(pc["decoded"])
            if i == 0:
                self.fr0.record(self.fstream)
            N.check(self.L.cbx_frame_rdw_async(base + pc["a"], pc["b"] - pc["a"], pc["sd"], len(pc["sd"]),
                                               ctypes.byref(self.prm), self.off.data_ptr() + 8 * pc["r0"],
                                               self.ln.data_ptr() + 4 * pc["r0"], pc["m"], pc["state"].data_ptr(), 0,
                                               self.fstream_p))
            pc["framed"].record(self.fstream)
        self.fr1.record(self.fstream)
        for pc, (r0, m, _, cs) in zip(self.pieces, self.parts):
            cur.wait_event(pc["framed"])
            N.check(self.L.cbx_decode_var(self.h, base + pc["a"], pc["b"] - pc["a"], self.off.data_ptr() + 8 * r0,
                                          self.ln.data_ptr() + 4 * r0, m, 0, r0, cs, self.stream))
            pc["decoded"].record(cur)
        return (self.fr0, self.fr1)

    def pieces_check(self) -> bool:
        """After timing: every piece's framing found the records the index run puts in it."""
        from cobrix_amd import native as N
        nfr = ctypes.c_int64(0)
        for pc in self.pieces:
            N.check(self.L.cbx_frame_rdw_state(pc["state"].data_ptr(), ctypes.byref(nfr), self.stream))
            if nfr.value != pc["m"]:
                raise RuntimeError(f"piece framing found {nfr.value} records, the index run holds {pc['m']}")
        return True

    def calls_per_step(self) -> int:
        return len(self.parts)

    def part_bytes(self, i: int) -> int:
        """Input bytes of part i's records (payloads + their 4-byte RDW headers), from the framing."""
        r0, m, _, _ = self.parts[i]
        if len(self.parts) == 1:
            return self.in_bytes
        return int(self.ln[r0:r0 + m].to(dtype=self.off.dtype).sum().item()) + 4 * m

    def verify(self, world):
        """After timing: the device base equals the records before this run in the setup framing, and
        the Record_Id column starts there."""
        import torch
        from cobrix_amd import native as N
        nfr = ctypes.c_int64(0)
        if self.pieces:
            self.pieces_check()
        else:
            N.check(self.L.cbx_frame_rdw_state(self.state.data_ptr(), ctypes.byref(nfr), self.stream))
            if nfr.value != self.n_expected:
                raise RuntimeError(f"framing found {nfr.value} records, the index run holds {self.n_expected}")
        got = int(self.base.item()) if world > 1 else 0
        rid0 = self.parts[0][2][self.rd.plan.record_id_column]["values"]
        r0, m, cols, _ = self.parts[-1]
        rid1 = cols[self.rd.plan.record_id_column]["values"]
        first = int(rid0[0].item()) if self.n_rec else got
        last = int(rid1[m - 1].item()) if self.n_rec else got - 1
        torch.cuda.synchronize()
        ok = got == self.expected_base and first == got and last == got + self.n_rec - 1
        return {"record_id_base": got, "expected": self.expected_base, "ok": ok}

    def end_to_end(self, entries_per_piece: int = 4, passes: int = 2):
        """H2D of the run in pieces of whole index entries (pinned host), each framed from its entries'
        offsets and decoded while the next piece is copied (two streams, double-buffered)."""
        import torch
        from cobrix_amd import native as N
        from cobrix_amd.reader import _alloc_columns, string_capacity
        host = torch.empty(self.in_bytes, dtype=torch.uint8, pin_memory=True)
        host.copy_(self.raw)
        bounds = self.seeds[::entries_per_piece] + [self.in_bytes]
        pieces = [(bounds[i], bounds[i + 1], [s - bounds[i] for s in self.seeds if bounds[i] <= s < bounds[i + 1]])
                  for i in range(len(bounds) - 1)]
        # records per piece from the timed framing (the same seeds give the same boundaries)
        if self.seed_recs is not None:   # (pieces leave piece-relative offsets in self.off)
            cnt = self.seed_recs[::entries_per_piece] + [self.n_rec]
        else:
            offs = self.off[: self.n_rec] - 4
            cnt = [int(torch.searchsorted(offs, torch.tensor([b], device=self.dev)).item()) for b in bounds]
        max_rec = max(cnt[i + 1] - cnt[i] for i in range(len(pieces)))
        max_bytes = max(b - a for a, b, _ in pieces)
        bufs = [torch.empty(max_bytes, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        outs = [_alloc_columns(self.rd.plan, max_rec, string_capacity(self.rd.native, max_rec), self.dev)
                for _ in range(2)]
        fo = [(torch.empty(max_rec + 1, dtype=torch.int64, device=self.dev),
               torch.empty(max_rec + 1, dtype=torch.int32, device=self.dev)) for _ in range(2)]
        cp, dc = torch.cuda.Stream(self.dev), torch.cuda.Stream(self.dev)
        done = [torch.cuda.Event() for _ in range(2)]
        copied = [torch.cuda.Event() for _ in range(2)]
        for e in done:
            e.record(dc)
        dstream = ctypes.c_void_p(dc.cuda_stream)
        N.check(self.L.cbx_plan_set_record_base(self.h, None))
        nfr = ctypes.c_int64(0)

        def run():
            rbase = 0
            for i, (a, b, sd) in enumerate(pieces):
                k = i % 2
                cp.wait_event(done[k])
                with torch.cuda.stream(cp):
                    bufs[k][: b - a].copy_(host[a:b], non_blocking=True)
                copied[k].record(cp)
                dc.wait_event(copied[k])
                seeds = (ctypes.c_int64 * len(sd))(*sd)
                N.check(self.L.cbx_frame_rdw(bufs[k].data_ptr(), b - a, seeds, len(sd), ctypes.byref(self.prm),
                                             fo[k][0].data_ptr(), fo[k][1].data_ptr(), max_rec + 1, ctypes.byref(nfr),
                                             dstream))
                N.check(self.L.cbx_decode_var(self.h, bufs[k].data_ptr(), b - a, fo[k][0].data_ptr(),
                                              fo[k][1].data_ptr(), nfr.value, 0, rbase, outs[k][1], dstream))
                rbase += nfr.value
                done[k].record(dc)
            return rbase

        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(passes):
            n = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / passes
        N.check(self.L.cbx_plan_check(self.h, dstream))
        N.check(self.L.cbx_plan_set_record_base(self.h, self.base.data_ptr()))
        if n != self.n_rec:
            raise RuntimeError(f"end-to-end pieces framed {n} records, expected {self.n_rec}")
        del host
        return {"value": round(self.in_bytes / dt / 1e9, 3), "unit": "GB/s", "records_per_s": round(self.n_rec / dt, 1),
                "ms_per_pass": round(dt * 1e3, 3),
                "how": f"{len(pieces)} pieces of {entries_per_piece} index entries ({self.seed_mb} MB): pinned-host "
                       "H2D on a copy stream overlapped with cbx_frame_rdw (seeded by the piece's entries) + "
                       "cbx_decode_var of the previous piece (double-buffered), per rank"}


# ------------------------------------------------------------------------------------------------
# CPU baseline (the oracle restatement; the reference's JVM path is not runnable here)
# ------------------------------------------------------------------------------------------------
def _probe_reference_jvm():
    """the reference CPU path runs only where a JVM + Spark + a Cobrix jar exist."""
    import shutil
    found = {t: shutil.which(t) for t in ("java", "spark-submit")}
    if all(found.values()):
        return "java and spark-submit present (reference run not wired into this bench)"
    return "probed on this host: " + ", ".join(f"{t} {'found' if v else 'absent'}" for t, v in found.items()) + \
        " -- the reference Cobrix/Spark CPU path cannot run here; the oracle restatement is timed instead"


def _cpu_counts():
    """(nproc = CPUs this process may run on, the cgroup CPU quota or None)."""
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    return nproc, quota


def _cpu_baseline(workload: str, seconds: float = 10.0):
    """The oracle (scalar C restatement of the reference decoders) on a bounded sample of the same
    workload, at 1 thread and at N = nproc threads (capped at 64; threads over record chunks: ctypes
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
    nproc, quota = _cpu_counts()
    # threads = the CPUs this process can actually use: nproc, capped by the cgroup quota (a quota of
    # 16 CPUs runs 64 threads on at most 16 CPUs) and at 64
    usable = min(64, nproc, max(1, int(quota)) if quota else nproc)
    T = int(os.environ.get("CBX_CPU_THREADS", str(usable)))
    dtT, _ = timed(data, fr, t_frame, T)
    unit_n = {"syn200": "SYN200 records", "synstr200": "SYNSTR200 records", "rdw_narrow": "RDW records",
              "wide_odo": "root records (+ children)"}[workload]
    return {"value": round(len(data) / dtT / 1e9, 6), "unit": "GB/s", "cores": min(T, usable), "threads": T,
            "kind": "port",
            "value_1_core": round(len(data) / dt1 / 1e9, 6),
            "nproc": nproc, "cgroup_cpu_quota": quota,
            "sample": f"{n} {unit_n} ({len(data) / 1e6:.1f} MB, {nrec} records) through oracle/cobrix_oracle.c "
                      f"(restatement of extractRecord + decoders{'' if fixed else '; RDW header walk sequential'}): "
                      f"{dt1:.1f} s at 1 thread, {dtT:.2f} s at N = {T} threads (nproc {nproc}"
                      f"{'' if quota is None else f', cgroup quota {quota:g} CPUs'})",
            "reference_jvm": _probe_reference_jvm()}


# ------------------------------------------------------------------------------------------------
# launcher
# ------------------------------------------------------------------------------------------------
def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start n ranks of this script under torch.distributed.run (one process per GPU) and return
    their exit status.  Called before anything initialises a GPU in this process."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def _dry_run(args, world, rank):
    """CPU plumbing of the multi-rank job (gloo): launcher, process group, the per-step count
    all-gather and the barrier + max-over-ranks timing -- no decode (the product path needs a GPU)."""
    import torch
    import torch.distributed as dist
    from cobrix_amd.shard import global_bases
    if world > 1:
        dist.init_process_group("gloo")
    n_local = 1000 + 7 * rank
    bases = []
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rb, _, tot = global_bases(n_local) if world > 1 else (torch.tensor(0), None, torch.tensor([n_local]))
        bases.append(int(rb))
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    expect = sum(1000 + 7 * r for r in range(rank))
    ok = all(b == expect for b in bases)
    gathered = [None] * world
    if world > 1:
        dist.all_gather_object(gathered, {"rank": rank, "ok": ok, "base": bases[-1] if bases else None})
    else:
        gathered = [{"rank": 0, "ok": ok, "base": 0}]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": float(t.item()) / max(1, args.steps) * 1e3,
                          "dry_run": True, "ranks": gathered}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if all(g["ok"] for g in gathered) else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="syn200", choices=sorted(WORKLOADS))
    ap.add_argument("--records", type=int, default=0, help="records per GPU (root records for wide_odo); "
                                                           "0 = the workload's default")
    ap.add_argument("--window", type=int, default=0, help="LDS window bytes (0 = plan default)")
    ap.add_argument("--strings", default="", choices=["", "views", "offsets", "large"],
                    help="string column layout (default per workload): Arrow string views, Arrow Utf8 offsets "
                         "(in place after a count pass) or Arrow large-string offsets (placement pass)")
    ap.add_argument("--pipeline", default="",
                    help="C,D: a fixed-length Utf8 job's batches alternate between two plans on two streams "
                         "(cbx_plan_pipeline), one plan's count pass beside the other's decode, the count / decode "
                         "kernels capped at C / D resident workgroups per CU (0: default occupancy); default per "
                         "workload (C3: 0,0 -- 53.3 -> 51.3 ms per 64 GB step; capped forms were slower), '-': off")
    ap.add_argument("--batch-records", type=int, default=0,
                    help="Utf8 layout: records per decode call (0 = the workload's batch; int32 offsets must fit)")
    ap.add_argument("--pieces", type=int, default=0,
                    help="rdw_narrow / wide_odo on one GPU: the run framed and decoded as this many pieces of "
                         "whole index entries, a piece's framing beside the previous piece's decode (0 = workload "
                         "default, 1 = one framing + one decode)")
    ap.add_argument("--occurs", default="lists", choices=["lists", "slots"],
                    help="OCCURS DEPENDING ON layout: Arrow lists (present elements) or one slot row per element")
    ap.add_argument("--seed-mb", type=int, default=100, choices=[100, 32],
                    help="var-len index entry size: 100 MB default (reset) or a 32 MB block size (subtracted)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="CPU plumbing only (gloo): launcher, all-gather, timing")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL, the measured path) or gloo: ranks may then share one GPU and collectives "
                         "go through host copies -- a correctness run of the multi-rank path on a one-GPU box, "
                         "not a measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE {world} != --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        sys.exit(_dry_run(args, world, rank))

    import torch
    import torch.distributed as dist

    from cobrix_amd import native as N

    if args.dist_backend == "gloo":   # ranks may share the box's GPUs (correctness runs of the N > 1 path)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    W = WORKLOADS[args.workload]
    n_req = args.records or W["records"]
    strings = args.strings or W["strings"]
    strong = bool(W.get("strong"))
    rec_base = None
    if strong:   # the job's records split over the ranks (strong scaling): rank r takes a contiguous range
        rec_base = n_req * rank // world
        n_req = n_req * (rank + 1) // world - rec_base
    # a batch per call: Utf8 int32 offsets must fit each slot region (<= 40 UTF-8 bytes per X(20) value)
    batch = (args.batch_records or W.get("batch_records", 0)) if strings == "offsets" else 0

    def progress(msg):
        if rank == 0:
            print(f"[bench {args.workload}] {msg}", file=sys.stderr, flush=True)

    progress(f"generating {n_req} records per GPU on {dev} (world {world})")
    if args.workload in ("syn200", "synstr200"):
        pipe = args.pipeline or W.get("pipeline", "")
        job = _Fixed(args.workload, n_req, dev, rank, args.window, strings, batch, rec_base,
                     pipeline=pipe if strings == "offsets" and pipe != "-" else "")
    else:
        pieces = args.pieces if args.pieces > 0 else W.get("pieces", 1)
        job = _VarLen(args.workload, n_req, dev, rank, world, args.window, strings, args.occurs == "lists",
                      args.seed_mb, batch, pieces=pieces if world == 1 else 1)
    st = torch.cuda.current_stream()
    progress(f"{job.in_bytes / 1e9:.2f} GB on this rank; allocating columns")
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
    for hx, sx in getattr(job, "targets", [])[1:]:   # the pipelined second plan's calls
        N.check(L.cbx_plan_check(hx, sx))
    calls = args.steps * (job.calls_per_step() if hasattr(job, "calls_per_step") else 1)
    dec = (ctypes.c_float * calls)()
    fix = (ctypes.c_float * calls)()
    nc = ctypes.c_int32()
    N.check(L.cbx_plan_kernel_times(h, dec, fix, calls, ctypes.byref(nc)))
    N.check(L.cbx_plan_set_profiling(h, 0))
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        _all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    check = job.verify(world)

    n_rec = job.n_rec
    plan = job.rd.plan
    # job totals: every rank's input bytes and records (var-len runs differ in size)
    tot = torch.tensor([job.in_bytes, n_rec], dtype=torch.float64, device=dev)
    if world > 1:
        _all_reduce(tot)
    job_bytes, job_recs = float(tot[0].item()), float(tot[1].item())
    steps = args.steps
    ms_per_step = elapsed / steps * 1e3
    gbs = job_bytes / (elapsed / steps) / 1e9
    recs_per_s = job_recs / (elapsed / steps)
    # per batch (a fixed-length job decodes its shard in batches; the others in one call), summed
    parts = getattr(job, "parts", None) or [(0, n_rec, job.cols, None)]
    alg = lay = absent = 0
    has_lists = any(c.list_array >= 0 for c in plan.columns)
    for i, (_, m, cols, _) in enumerate(parts):
        present = present_elements(plan, cols, m)
        payload = string_payload(plan, cols, m)
        in_b = job.part_bytes(i) if hasattr(job, "part_bytes") else m * job.stride if len(parts) > 1 else job.in_bytes
        alg += algorithmic_bytes(plan, m, in_b, payload, present)
        lay += layout_bytes(plan, cols, m, in_b, payload, present)
        # OCCURS lists: the 8(d) input term counts every record byte, absent ODO elements included;
        # the bytes the kernels must move leave those out (reported beside, never as `frac`)
        absent += absent_element_bytes(plan, cols, m) if has_lists else 0
    dec_avg_ms = sum(dec[: nc.value]) / max(1, args.steps)     # per step: every call of the step
    fix_avg_ms = sum(fix[: nc.value]) / max(1, args.steps)
    # the decode chain: the record kernel (+ its Utf8 count pass and scan, list kernels) and the fixup
    # pass of the values it deferred -- all of cbx_decode_*'s device work
    chain_ms = dec_avg_ms + fix_avg_ms
    piped = hasattr(job, "pipelined") and job.pipelined()
    if piped:   # two plans' chains overlap on two streams: the step's wall time is the chain
        chain_ms = ms_per_step
    achieved = alg / (chain_ms * 1e-3) / 1e9
    kind = ctypes.c_int32(0)
    N.check(L.cbx_plan_kernel_kind(h, ctypes.byref(kind)))
    kname = {1: "cbx_jit_decode (copybook-specialised, hipRTC)", 2: "cbx::walk_kernel (record walk)"}.get(
        kind.value, "cbx::decode_kernel (table-driven)")
    if strings == "offsets" and any(c.out_type in (N.O_STRING, N.O_BINARY) for c in plan.columns):
        kname = "Utf8 count pass (cbx_jit_count) + device scan + " + kname + " (decode_kernel time covers all three)"
    lists = any(c.list_array >= 0 for c in plan.columns)
    if lists:   # the OCCURS list elements: the element-parallel kernel launched right after the decode kernel
        kname += " + cbx::list_kernel (OCCURS lists; decode_kernel time covers both)"
    kname += " + cbx::fixup_kernel (deferred values; post_kernels time)"
    tag = f"{args.workload}_{strings}{'' if args.occurs == 'lists' else '_slots'}_{n_rec}"
    traffic, traffic_src = measured_traffic(tag)
    kernel_ms = {"decode_kernel": round(dec_avg_ms, 4), "post_kernels": round(fix_avg_ms, 4)}
    fms = None
    if frame_ev:
        fms = sum(a.elapsed_time(b) for a, b in frame_ev) / len(frame_ev)
        kernel_ms["rdw_framing (cbx_frame_rdw_async, count on the device)"] = round(fms, 4)
    if hasattr(job, "index_ms"):
        kernel_ms["sparse_index_setup (untimed, once: frame + cbx_sparse_index of the whole file, or of this "
                  "rank's block + tail in the N > 1 chain)"] = round(job.index_ms, 3)
    e2e = None
    if not args.no_end_to_end and world == 1:
        progress("end-to-end (pinned host -> HBM) pass")
        e2e = job.end_to_end()
    progress("cpu baseline" if not args.no_cpu_baseline and world == 1 else "done")
    kernels_sum = dec_avg_ms + fix_avg_ms + (fms or 0.0)
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
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": W["data"],
            "config": {"workload": W["desc"], "baseline_config": W["config"],
                       "records_per_gpu": n_rec, "input_bytes_per_gpu": job.in_bytes,
                       **({"job_records": int(W["records"] if not args.records else args.records),
                           "batches_per_gpu": len(parts), "batch_records": job.batch} if len(parts) > 1 or strong else {}),
                       "input_gb_per_gpu": round(job.in_bytes / 1e9, 3), "job_input_bytes": int(job_bytes),
                       "output_columns": plan.n_columns, "parallelism": f"dp{world}",
                       "shard": job.shard_note,
                       **({"setup_bytes_held_per_rank": job.setup_bytes_held} if hasattr(job, "setup_bytes_held") else {}),
                       "string_layout": STRING_LAYOUTS[strings],
                       "occurs_layout": "Arrow lists (present elements only)" if args.occurs == "lists"
                       else "one slot row per element",
                       "inputs_resident_in_hbm": True},
            "kernel_ms": kernel_ms,
            "step_vs_kernels": round(ms_per_step / kernels_sum, 3) if kernels_sum > 0 else None,
            **({"seeds": f"{len(job.seeds)} sparse-index entries of this rank's run ({args.seed_mb} MB, root segments)",
                "record_id_check": check} if hasattr(job, "seeds") else {}),
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "frac_of_measured_peak": round(achieved / HBM_MEASURED_GBS, 4),
                         "algorithmic_bytes_per_launch": alg,
                         **({"absent_element_bytes": absent, "moved_bytes_per_launch": alg - absent,
                             "frac_moved_bytes": round((alg - absent) / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "note": "8(d) counts the input records whole (absent ODO elements included); "
                                     "frac_moved_bytes counts what the kernels must read and write"}
                            if absent else {}),
                         "layout_bytes_per_launch": lay, "layout_overhead": lay - alg,
                         "timing": ("wall time of the step: two plans' count + decode chains overlapped on two streams "
                                    "(cbx_plan_pipeline)") if piped else
                                   ("HIP events on the launch stream (cbx_plan_kernel_times): decode_kernel + post_kernels "
                                    "(the fixup pass), average of the timed steps"),
                         "traffic": traffic, "traffic_source": traffic_src},
        }
        if e2e is not None:
            out["end_to_end"] = e2e
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = _cpu_baseline(args.workload)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if check is not None and not check["ok"]:
        print(f"[bench] Record_Id base check failed on rank {rank}: {check}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
