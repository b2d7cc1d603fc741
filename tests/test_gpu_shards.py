"""Multi-GPU sharding of one variable-length file on one GPU: the file's sparse
index is cut into contiguous entry runs (shard.entry_shards), each run is framed and decoded on its
own from its entries' offsets, and the Record_Id base of a run is the exclusive prefix of the runs'
framed record counts -- computed on the device, as bench.py does over RCCL.  The concatenated
shards must equal the single-shot read of the whole file (Record_Id, Seg_IdN, every column)."""
from __future__ import annotations

import ctypes

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _file(name):
    import goldens as G
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    if name == "test5":
        return (G.read("test5_copybook.cob").decode("latin-1"), G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat"),
                {"is_record_sequence": "true", "segment_field": "SEGMENT_ID", "segment_id_root": "C",
                 "input_split_records": "100", "segment_id_prefix": "B", "generate_record_id": "true"})
    raw = rdw_narrow(20_000, seed=77)[0].numpy().tobytes()
    return (RDW_NARROW_COPYBOOK, raw,
            {"is_record_sequence": "true", "segment_field": "SEGMENT_ID", "segment_id_level0": "C",
             "segment_id_level1": "P", "input_split_records": "1500", "generate_record_id": "true",
             "redefine_segment_id_map:0": "STATIC-DETAILS => C", "redefine-segment-id-map:1": "CONTACTS => P"})


def _reader(cb, opts, **kw):
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    p, var_len = parse_options(opts)
    assert var_len
    return VarLenNestedReader(cb, dataclasses.replace(p, **kw))


def _runs(rd, raw, world):
    """Index of the whole file on the GPU, cut into `world` entry runs -> [(lo, hi, entries)]."""
    from cobrix_amd.shard import entry_shards
    t = rd._device_file(raw)
    off, ln, _ = rd.frame_file(t, len(raw))
    entries = rd.generate_index(t, len(raw), off, ln)
    out = []
    for k0, k1 in entry_shards(entries, len(raw), world):
        lo = entries[k0].offset_from if k0 < len(entries) else len(raw)
        hi = entries[k1].offset_from if k1 < len(entries) else len(raw)
        out.append((lo, hi, entries[k0:k1]))
    return entries, out


def _frame_run(rd, raw, lo, hi, ents):
    t = rd._device_file(raw[lo:hi])
    off, ln = rd.frame(t, hi - lo, [e.offset_from - lo for e in ents] or [0])
    return t, off, ln


def _device_bases(counts):
    """Exclusive prefix of the runs' record counts on the device (the all-gather's result)."""
    c = torch.tensor(counts, dtype=torch.int64, device="cuda")
    return torch.cumsum(c, 0) - c


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["test5", "rdw_narrow"])
def test_entry_run_shards_selection_equal_single_read(name, world):
    """cbx_frame_rdw + cbx_select_records + cbx_decode_selected per run, each run's entries numbered
    from its device base: the rows equal rd.read() of the whole file."""
    from cobrix_amd.reader import SparseIndexEntry
    cb, raw, opts = _file(name)
    rd = _reader(cb, opts)
    whole = rd.read(raw).to_rows()
    entries, runs = _runs(rd, raw, world)
    assert len(entries) > world
    framed = [_frame_run(rd, raw, lo, hi, ents) for lo, hi, ents in runs]
    bases = _device_bases([int(f[1].numel()) for f in framed])
    rows = []
    for (lo, hi, ents), (t, off, ln), base in zip(runs, framed, bases):
        if not ents:
            continue
        hdr = (off - 4).cpu()
        local = []
        for e in ents:
            ri = int(base.item()) + int(torch.searchsorted(hdr, torch.tensor([e.offset_from - lo])).item())
            assert ri == e.record_index          # the device prefix reproduces the index's numbering
            local.append(SparseIndexEntry(e.offset_from - lo, e.offset_to - lo if e.offset_to >= 0 else -1,
                                          e.file_id, ri))
        sel = rd.select(t, hi - lo, off, ln, local)
        rows += rd.decode_selected(t, hi - lo, sel).to_rows()
    assert len(rows) == len(whole)
    bad = [i for i, (a, b) in enumerate(zip(rows, whole)) if a != b]
    assert not bad, (bad[:5], rows[bad[0]], whole[bad[0]])


@pytest.mark.parametrize("views", [True, False])
@pytest.mark.parametrize("name", ["test5", "rdw_narrow"])
def test_entry_run_shards_device_record_base(name, views):
    """bench.py's step: cbx_frame_rdw + cbx_decode_var per run with the Record_Id base read by the
    kernel from device memory (cbx_plan_set_record_base); the runs equal one cbx_decode_var of the
    whole file (specialised and table-driven kernels)."""
    from cobrix_amd import native as N
    cb, raw, opts = _file(name)
    for jit in (-1, 1):
        rd = _reader(cb, opts, string_views=views, jit_min_records=jit)
        t = rd._device_file(raw)
        off, ln = rd.frame(t, len(raw))
        whole = rd.decode_device(t, len(raw), off, ln).to_rows()
        _, runs = _runs(rd, raw, 2)
        framed = [_frame_run(rd, raw, lo, hi, ents) for lo, hi, ents in runs]
        bases = _device_bases([int(f[1].numel()) for f in framed])
        rows = []
        L = N.load()
        try:
            for (lo, hi, _), (tt, o, ln_), k in zip(runs, framed, range(len(runs))):
                N.check(L.cbx_plan_set_record_base(rd.native.handle, ctypes.c_void_p(bases[k:k + 1].data_ptr())))
                rows += rd.decode_device(tt, hi - lo, o, ln_).to_rows()
        finally:
            N.check(L.cbx_plan_set_record_base(rd.native.handle, None))
        assert len(rows) == len(whole)
        bad = [i for i, (a, b) in enumerate(zip(rows, whole)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], whole[bad[0]])
