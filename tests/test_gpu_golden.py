"""The reference's integration specs (tests/golden_cases.py) through the HIP path: rows decoded by
libcobrix_hip.so against the reference's golden rows, and column by column against the oracle.

Run on an MI355X: python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
from __future__ import annotations

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import golden_cases as GC  # noqa: E402

from oracle import reader_oracle as RO  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _replace(p, **kw):
    import dataclasses
    return dataclasses.replace(p, **kw)


def gpu_rows(case, **extra):
    from cobrix_amd.reader import FixedLenNestedReader, VarLenNestedReader
    p, var_len = GC.params(case)
    for k, v in extra.items():
        setattr(p, k, v)
    data = GC.data_bytes(case)
    if var_len:
        rd = VarLenNestedReader(GC.copybook_text(case), p)
        return rd, rd.read(data).to_rows()
    rd = FixedLenNestedReader(GC.copybook_text(case), p)
    return rd, rd.decode(data).to_rows()


@pytest.mark.parametrize("name", sorted(GC.CASES))
@pytest.mark.parametrize("jit,views,lists", [(-1, False, False), (1, False, False), (-1, True, True), (1, True, True),
                                             (-1, "utf8", True), (1, "utf8", False)])
def test_gpu_golden_rows(name, jit, views, lists):
    """Both decode kernels (table-driven: jit=-1; copybook-specialised: jit=1), in the three string
    layouts (Arrow large-string offsets / Arrow string views / Arrow Utf8 written in place after a count
    pass) and both OCCURS DEPENDING ON layouts (slot rows / lists), reproduce the reference's golden
    rows and the oracle's full row set."""
    case = GC.CASES[name]
    rd, rows = gpu_rows(case, jit_min_records=jit, string_views=views is True, string_utf8=views == "utf8",
                        occurs_lists=lists)
    errs = GC.compare(case, rows)
    assert not errs, errs[:10]
    p, var_len = GC.params(case)
    cb = rd.copybook
    exp = RO.var_len_rows(cb, GC.data_bytes(case), p) if var_len else RO.fixed_len_rows(cb, GC.data_bytes(case), p)
    assert len(rows) == len(exp)
    bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
    assert not bad, (bad[:5], rows[bad[0]], exp[bad[0]])


# ---- sparse index (IndexGenerator) and record selection (VarLenNestedIterator) on the GPU

def _var_reader(copybook_text, options):
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    p, var_len = parse_options(options)
    assert var_len
    return VarLenNestedReader(copybook_text, p), p


def _gpu_index(rd, data: bytes, file_id=0, prm_override=None):
    import ctypes
    from cobrix_amd import native as N
    t = rd._device_file(data)
    off, ln, _ = rd.frame_file(t, len(data))
    if prm_override is None:
        return [(e.offset_from, e.offset_to, e.record_index) for e in rd.generate_index(t, len(data), off, ln, file_id)]
    prm = rd.index_params(file_id)
    for k, v in prm_override.items():
        setattr(prm, k, v)
    ents = (N.CbxIndexEntry * 100000)()
    n = ctypes.c_int64(0)
    N.check(N.load().cbx_sparse_index(rd.native.handle, t.data_ptr(), len(data), off.data_ptr(), ln.data_ptr(),
                                      int(off.numel()), ctypes.byref(prm), ents, 100000, ctypes.byref(n), None))
    return [(e.offset_from, e.offset_to, e.record_index) for e in ents[: n.value]]


def test_gpu_sparse_index_known_answer():
    """Test5MultisegmentSpec.scala:205-218: 10 records per entry cut at root 'C' -> 88 entries,
    each equal to the IndexGenerator restatement's."""
    import goldens as G
    opts = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID", "segment_id_root": "C",
            "input_split_records": "10"}
    rd, p = _var_reader(G.read("test5_copybook.cob").decode("latin-1"), opts)
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    got = _gpu_index(rd, raw)
    assert len(got) == 88
    exp = [(e.offset_from, e.offset_to, e.record_index) for e in RO.sparse_index(rd.copybook, raw, p)]
    assert got == exp


_SYN_OPTS = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID"}


@pytest.mark.parametrize("extra,override,n", [
    ({"input_split_records": "1000"}, None, 40_000),                                   # records, closed form
    ({"input_split_records": "777", "segment_id_level0": "C", "segment_id_level1": "P"}, None, 40_000),  # chain walk
    ({"input_split_records": "3", "segment_id_root": "C"}, None, 3_000),               # many short entries
    ({"input_split_size_mb": "1"}, None, 40_000),                                      # size, subtract
    ({"input_split_size_mb": "1", "segment_id_root": "C"}, None, 40_000),
    ({}, {"bytes_per_entry": 300_000, "subtract_size": 0}, 40_000),                     # size, reset
    ({"segment_id_root": "C"}, {"bytes_per_entry": 300_000, "subtract_size": 0}, 40_000),
    ({"input_split_records": "100", "segment_id_root": "C", "file_start_offset": "100", "file_end_offset": "120"},
     None, 5_000),                                                                     # file header / footer
    # split gaps of ~4,100-4,160 candidates: the galloping walk's second probe round (step 64) must
    # resume right after its last probe (lo + 63 step + 1), not 64 step further on
    ({"input_split_records": "11770", "segment_id_root": "C"}, None, 90_000),
    ({"segment_id_root": "C"}, {"bytes_per_entry": 780_000, "subtract_size": 0}, 90_000),
])
def test_gpu_sparse_index_modes(extra, override, n):
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    raw_t, _ = rdw_narrow(n, seed=n + len(extra))
    raw = raw_t.numpy().tobytes()
    if "file_start_offset" in extra:
        raw = bytes(range(100)) + raw + bytes(120)
    rd, p = _var_reader(RDW_NARROW_COPYBOOK, {**_SYN_OPTS, **extra})
    got = _gpu_index(rd, raw, file_id=3, prm_override=override)
    dflt = override["bytes_per_entry"] if override else None
    exp = [(e.offset_from, e.offset_to, e.record_index) for e in RO.sparse_index(rd.copybook, raw, p, 3, dflt)]
    assert len(exp) > 2
    assert got == exp


@pytest.mark.parametrize("views", [False, True])
@pytest.mark.parametrize("extra", [
    {"segment_id_level0": "C", "segment_id_level1": "P", "segment_id_prefix": "XYZ", "input_split_records": "1000",
     "generate_record_id": "true"},
    {"segment_id_root": "C", "segment_filter": "P", "segment_id_prefix": "Q", "input_split_records": "250",
     "generate_record_id": "true", "redefine_segment_id_map:0": "STATIC-DETAILS => C",
     "redefine-segment-id-map:1": "CONTACTS => P", "schema_retention_policy": "collapse_root"},
    {"segment_id_level0": "P", "segment_id_level1": "C", "segment_filter": "C,P", "input_split_size_mb": "1",
     "file_start_offset": "100", "file_end_offset": "120", "generate_record_id": "true"},
])
def test_gpu_selection_vs_oracle(extra, views):
    """Record_Id per entry, Seg_IdN, segment_filter and root-reached filtering on 20 k records
    (both decode kernels, both string layouts)."""
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    raw = rdw_narrow(20_000, seed=11)[0].numpy().tobytes()
    if "file_start_offset" in extra:
        raw = bytes(range(100)) + raw + bytes(120)
    for jit in (-1, 1):
        rd, p = _var_reader(RDW_NARROW_COPYBOOK, {**_SYN_OPTS, **extra})
        rd.params.jit_min_records = jit
        if views:
            rd = type(rd)(RDW_NARROW_COPYBOOK, _replace(rd.params, string_views=True))
        rows = rd.read(raw, file_id=2).to_rows()
        exp = RO.var_len_rows(rd.copybook, raw, p, file_id=2)
        assert len(rows) == len(exp)
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


@pytest.mark.parametrize("per", [1, 3])
@pytest.mark.parametrize("extra", [
    {"segment_id_root": "C", "input_split_records": "700", "generate_record_id": "true"},
    {"segment_id_level0": "C", "segment_id_level1": "P", "segment_id_prefix": "XYZ", "input_split_records": "1000",
     "generate_record_id": "true"},
    {"segment_id_root": "C", "segment_filter": "P", "input_split_records": "250", "generate_record_id": "true",
     "redefine_segment_id_map:0": "STATIC-DETAILS => C", "redefine-segment-id-map:1": "CONTACTS => P"},
    {"segment_id_level0": "P", "segment_id_level1": "C", "input_split_records": "900",
     "file_start_offset": "100", "file_end_offset": "120", "generate_record_id": "true"},
])
def test_gpu_read_entries_pieces_vs_oracle(extra, per):
    """read_entries: the file as pieces of index entries (each framed from its entries on a second
    stream, selected and decoded as its own batch) -> the rows of the whole-file oracle, in order."""
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    raw = rdw_narrow(20_000, seed=12)[0].numpy().tobytes()
    if "file_start_offset" in extra:
        raw = bytes(range(100)) + raw + bytes(120)
    rd, p = _var_reader(RDW_NARROW_COPYBOOK, {**_SYN_OPTS, **extra})
    t = rd._device_file(raw)
    off, ln, _ = rd.frame_file(t, len(raw))
    ents = rd.generate_index(t, len(raw), off, ln, file_id=2)
    assert len(ents) > 4
    exp_ents = [(e.offset_from, e.offset_to, e.record_index) for e in RO.sparse_index(rd.copybook, raw, p, 2)]
    assert [(e.offset_from, e.offset_to, e.record_index) for e in ents] == exp_ents
    whole = rd.read(raw, file_id=2).to_rows()
    batches = rd.read_entries(t, len(raw), ents, entries_per_piece=per, file_id=2)
    assert len(batches) == -(-len(ents) // per)
    rows = [r for b in batches for r in b.to_rows()]
    exp = RO.var_len_rows(rd.copybook, raw, p, file_id=2)
    assert len(whole) == len(exp)
    assert len(rows) == len(exp), (len(rows), len(exp), [len(b.to_rows()) for b in batches][:6], ents[:3])
    bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
    assert not bad, (bad[:5], rows[bad[0]], exp[bad[0]])


def _norm(v):
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, (np.floating, float)):
        f = float(v)
        return "nan" if f != f else f
    if isinstance(v, np.integer):
        return int(v)
    return v


@pytest.mark.parametrize("views", [False, True, "utf8"])
@pytest.mark.parametrize("name", ["test1", "test5", "test6", "test9_cp037", "test19", "test17a", "test17c", "test17d", "test17e", "test17f"])
def test_gpu_arrow_export_matches_rows(name, views):
    _arrow_vs_rows(name, views)


def _arrow_vs_rows(name, views):
    """DecodedBatch.to_arrow (structs, OCCURS DEPENDING ON lists, segment-redefine nulls, views or
    large strings, decimal128) holds exactly the rows to_rows rebuilds."""
    pytest.importorskip("pyarrow")
    from cobrix_amd.reader import FixedLenNestedReader, VarLenNestedReader
    case = GC.CASES[name]
    p, var_len = GC.params(case)
    p.string_views = views is True
    p.string_utf8 = views == "utf8"
    p.occurs_lists = bool(views)
    data = GC.data_bytes(case)
    rd = (VarLenNestedReader if var_len else FixedLenNestedReader)(GC.copybook_text(case), p)
    batch = rd.read(data) if var_len else rd.decode(data)
    table = batch.to_arrow()
    table.validate(full=True)
    assert _norm(table.to_pylist()) == _norm(batch.to_rows())


@pytest.mark.parametrize("name,lengths", [("test21", [1, 2, 4, 6, 5]), ("test25", [3, 5])])
def test_gpu_var_occurs_framing(name, lengths):
    """cbx_frame_var_occurs against the reference's VarOccursRecordExtractor unit tests
    (Test21VariableOccurs.scala:38-60, Test25OccursMappings.scala:52-79)."""
    from cobrix_amd.reader import VarLenNestedReader
    case = GC.CASES[name]
    p, _ = GC.params(case)
    data = GC.data_bytes(case)
    rd = VarLenNestedReader(GC.copybook_text(case), p)
    assert rd.walk
    t = rd._device_file(data)
    off, ln, vb = rd.frame_file(t, len(data))
    assert ln.cpu().tolist() == lengths
    assert off.cpu().tolist() == [sum(lengths[:i]) for i in range(len(lengths))]
    assert vb == max(len(data), sum(lengths))


@pytest.mark.parametrize("n,entry_bytes", [(600_000, 1_500_000), (600_000, 2_000_000)])
def test_gpu_sparse_index_reset_long_gaps(n, entry_bytes):
    """Size splits with the reset rule at root segments over gaps of thousands of candidates: the
    one-wave walk's galloping reaches step 64 and its 64-ary search spans of 4,095 candidates, where a
    match in the last stride once left the ballot empty."""
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    raw = rdw_narrow(n, seed=5)[0].numpy().tobytes()
    rd, p = _var_reader(RDW_NARROW_COPYBOOK, {**_SYN_OPTS, "segment_id_root": "C"})
    got = _gpu_index(rd, raw, prm_override={"bytes_per_entry": entry_bytes, "subtract_size": 0})
    exp = [(e.offset_from, e.offset_to, e.record_index) for e in RO.sparse_index(rd.copybook, raw, p, 0, entry_bytes)]
    assert len(exp) >= 15   # (~39 MB of records: 20 / 26 entries)
    assert got == exp


def test_gpu_sparse_index_reset_bench_scale():
    """The bench's index at scale: 100 MB entries (the default, reset) cut at roots over a 5 M-record
    file with 16 MB entries (gaps of ~90 k candidates: galloping at step 4,096); expected entries
    from the rule itself (next root whose header offset is >= the last entry's + the entry size),
    which the oracle restatement pins on the smaller cases above."""
    import bisect
    import numpy as np
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow_large
    t, hdr = rdw_narrow_large(5_000_000, seed=9, device="cuda")
    n_bytes = int(t.numel())
    rd, p = _var_reader(RDW_NARROW_COPYBOOK, {**_SYN_OPTS, "segment_id_root": "C"})
    off, ln = rd.frame(t, n_bytes)
    h = hdr.cpu().numpy()
    assert off.numel() == h.size
    S = 16 * 1024 * 1024
    ents = rd.generate_index(t, n_bytes, off, ln)
    raw = t.cpu().numpy()
    lens = ln.cpu().numpy().astype(np.int64)
    root = (raw[h + 4] == 0xC3) & (h + 4 + lens < n_bytes)
    cand = h[root].tolist()
    exp, pp = [0], 0
    while True:
        r = bisect.bisect_left(cand, pp + S)
        if r >= len(cand):
            break
        pp = cand[r]
        exp.append(pp)
    assert len(exp) >= 15   # (~325 MB of records: 20 entries)
    # the reader's index uses the 100 MB default: cut this file with 16 MB entries instead
    prm = rd.index_params()
    prm.bytes_per_entry, prm.subtract_size = S, 0
    import ctypes
    from cobrix_amd import native as N
    arr = (N.CbxIndexEntry * 1000)()
    ne = ctypes.c_int64(0)
    N.check(N.load().cbx_sparse_index(rd.native.handle, t.data_ptr(), n_bytes, off.data_ptr(), ln.data_ptr(),
                                      int(off.numel()), ctypes.byref(prm), arr, 1000, ctypes.byref(ne), None))
    assert [arr[k].offset_from for k in range(ne.value)] == exp
    exp100, pp = [0], 0
    while True:
        r = bisect.bisect_left(cand, pp + 100 * 1024 * 1024)
        if r >= len(cand):
            break
        pp = cand[r]
        exp100.append(pp)
    assert [e.offset_from for e in ents] == exp100 and len(exp100) == 4
