"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference goldens.

Run on an MI355X: python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
from __future__ import annotations

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import goldens as G  # noqa: E402
from parity import compare_batch  # noqa: E402

from cobrix_amd import copybook as cbk  # noqa: E402
from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, VarLenNestedReader  # noqa: E402
from cobrix_amd.synth import SYN200_COPYBOOK, syn200  # noqa: E402
from oracle import oracle as O  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


LAYOUTS = ["large", "views", "utf8"]   # Arrow large-string offsets, string views, Arrow Utf8 (in place)


def _layout(name):
    return {"string_views": name == "views", "string_utf8": name == "utf8"}


def _fixed(copybook_text, data: bytes, **kw):
    params = ReaderParameters(**kw)
    rd = FixedLenNestedReader(copybook_text, params)
    return rd, rd.decode(data)


def test_test1_golden_and_oracle():
    cb_text = G.read("test1_copybook.cob").decode()
    data = G.read("test1_data", "example.bin")
    rd, batch = _fixed(cb_text, data, schema_policy="collapse_root")
    rows = batch.to_rows()
    assert not G.compare_rows(rows, G.load_lines("test1_expected", "test1.txt"))
    res = O.decode_fixed(rd.copybook, data)
    assert not compare_batch(batch, res)


def test_test6_golden_ieee754():
    cb_text = G.read("test6_copybook.cob").decode()
    data = G.read("test6_data", "INTEGR.TYPES.NOV28.DATA.dat")
    rd, batch = _fixed(cb_text, data, schema_policy="collapse_root", floating_point_format="IEEE754")
    rows = batch.to_rows()
    rows.sort(key=lambda r: (r["ID"] is None, r["ID"]))
    assert not G.compare_rows(rows, G.load_lines("test6_expected", "test6.txt"), na_fill=True)
    res = O.decode_fixed(rd.copybook, data)
    assert not compare_batch(batch, res)


@pytest.mark.parametrize("fmt", ["IBM", "IEEE754"])
def test_test6_all_fields_vs_oracle(fmt):
    cb_text = G.read("test6_copybook.cob").decode()
    data = G.read("test6_data", "INTEGR.TYPES.NOV28.DATA.dat")
    rd, batch = _fixed(cb_text, data, floating_point_format=fmt)
    assert not compare_batch(batch, O.decode_fixed(rd.copybook, data))


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1000, 100_003])
def test_syn200_vs_oracle(n):
    rec = syn200(n, seed=7 + n) if n else torch.zeros((0, 200), dtype=torch.uint8)
    data = rec.numpy().tobytes()
    rd, batch = _fixed(SYN200_COPYBOOK, data) if n else (None, None)
    if n == 0:
        rd = FixedLenNestedReader(SYN200_COPYBOOK, ReaderParameters())
        b = rd.decode_device(torch.zeros(16, dtype=torch.uint8, device="cuda"), 0)
        assert b.n_rec == 0
        return
    res = O.decode_fixed(rd.copybook, data)
    errs = compare_batch(batch, res)
    assert not errs, errs


def test_fuzz_copybook_vs_oracle():
    from test_decode_fuzz import FUZZ_COPYBOOK, _random_bytes
    for code_page, trim, fmt in [("common", "both", "IBM"), ("cp037", "left", "IEEE754"), ("cp875", "none", "IBM_LE")]:
        cb = cbk.parse_copybook(FUZZ_COPYBOOK, code_page=code_page, string_trimming=trim, floating_point_format=fmt)
        rng = np.random.default_rng(5)
        n = 3000
        recs = bytearray()
        leaves = list(O._iter_leaves(cb.ast))
        for _ in range(n):
            for p in leaves:
                recs += _random_bytes(rng, p, p.data_size)
        assert len(recs) == n * cb.record_size
        rd, batch = _fixed(FUZZ_COPYBOOK, bytes(recs), ebcdic_code_page=code_page, string_trimming_policy=trim,
                           floating_point_format=fmt)
        errs = compare_batch(batch, O.decode_fixed(rd.copybook, bytes(recs)))
        assert not errs, (code_page, errs)


@pytest.mark.parametrize("big_endian,charset,n", [(True, "", 3000), (False, "windows-1252", 3000),
                                                   (True, "ISO-8859-1", 70_001)])
def test_ascii_file_vs_oracle(big_endian, charset, n):
    """ASCII data: DISPLAY numbers (decodeAsciiNumber, deferred to the fixup kernel), ASCII / charset
    strings and UTF-16 PIC N through the decode kernel (A15)."""
    from test_decode_fuzz import ASCII_COPYBOOK, _random_ascii_bytes
    cb = cbk.parse_copybook(ASCII_COPYBOOK, data_encoding=cbk.ASCII, is_utf16_big_endian=big_endian,
                            ascii_charset=charset)
    rng = np.random.default_rng(11)
    leaves = list(O._iter_leaves(cb.ast))
    pool = [b"".join(_random_ascii_bytes(rng, p, p.data_size, big_endian) for p in leaves) for _ in range(997)]
    recs = b"".join(pool[i % 997] if i % 5 else pool[(i * 7) % 997] for i in range(n))
    assert len(recs) == n * cb.record_size
    rd, batch = _fixed(ASCII_COPYBOOK, recs, is_ebcdic=False, is_utf16_big_endian=big_endian, ascii_charset=charset)
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, recs))
    assert not errs, errs


@pytest.mark.parametrize("start,end,rl", [(3, 2, None), (0, 0, 2000), (5, 0, 2300)])
def test_record_offsets_and_length(start, end, rl):
    """record_start_offset / record_end_offset / record_length (FixedLenNestedReader.scala:60-94)."""
    cb_text = G.read("test1_copybook.cob").decode()
    base = G.read("test1_data", "example.bin")
    L = 2202
    inner = rl if rl is not None else L
    recs = bytearray()
    rng = np.random.default_rng(1)
    for i in range(10):
        r = base[i * L:(i + 1) * L]
        r = (r + bytes(rng.integers(0, 256, max(0, inner - L), dtype=np.uint8)))[:inner]
        recs += bytes(rng.integers(0, 256, start, dtype=np.uint8)) + r + bytes(rng.integers(0, 256, end, dtype=np.uint8))
    rd, batch = _fixed(cb_text, bytes(recs), start_offset=start, end_offset=end, record_length=rl)
    res = O.decode_fixed(rd.copybook, bytes(recs), record_size=inner, start_offset=start, end_offset=end)
    assert not compare_batch(batch, res)


def test_segment_redefines_fixed():
    """Segment-redefine selection on fixed-length records (test5 layout, FixedLenNestedRowIterator)."""
    cb_text = G.read("test5_copybook.cob").decode()
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    off, ln = O.frame_rdw(raw)
    cb = cbk.parse_copybook(cb_text)
    L = cb.record_size
    recs = b"".join((raw[o:o + l] + b"\x40" * L)[:L] for o, l in zip(off, ln))
    seg_map = {"C": "STATIC-DETAILS", "P": "CONTACTS"}
    rd, batch = _fixed(cb_text, recs, segment_field="SEGMENT-ID", segment_id_redefine_map=seg_map)
    res = O.decode_fixed(rd.copybook, recs, segment_field="SEGMENT-ID", segment_redefine_map=seg_map)
    assert not compare_batch(batch, res)
    rows = batch.to_rows()
    assert rows == O.rows(res, collapse_root=False)


def test_rdw_framing_and_var_decode():
    """test5 RDW file: GPU framing == oracle framing; var-len decode == oracle (short records)."""
    cb_text = G.read("test5_copybook.cob").decode()
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map={"C": "STATIC-DETAILS", "P": "CONTACTS"})
    rd = VarLenNestedReader(cb_text, params)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    off, ln = rd.frame(t, len(raw))
    eo, el = O.frame_rdw(raw)
    assert np.array_equal(off.cpu().numpy(), eo) and np.array_equal(ln.cpu().numpy(), el)
    # seeded from sparse-index entries: same result
    idx = O.sparse_index(raw, records_per_entry=10)
    off2, ln2 = rd.frame(t, len(raw), seeds=[e[0] for e in idx])
    assert np.array_equal(off2.cpu().numpy(), eo)
    batch = rd.decode_device(t, len(raw), off, ln)
    segs = []
    for o, l in zip(eo, el):
        sid = raw[o:o + 5]
        segs.append({"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(sid.decode("cp037"))))
    res = O.decode_records(rd.copybook, [raw[o:o + l] for o, l in zip(eo, el)], active_segments=segs)
    assert not compare_batch(batch, res)


def test_rdw_errors():
    """Zero-length RDW raises (RecordHeaderParserRDW.scala:74-83)."""
    from cobrix_amd.native import CbxError
    cb_text = G.read("test5_copybook.cob").decode()
    rd = VarLenNestedReader(cb_text, ReaderParameters(is_record_sequence=True))
    bad = bytes([0, 0, 0, 0]) + b"\x40" * 10
    t = torch.frombuffer(bytearray(bad), dtype=torch.uint8).cuda()
    with pytest.raises(CbxError):
        rd.frame(t, len(bad))


def _kernel_kind(rd) -> int:
    import ctypes
    from cobrix_amd import native as N
    k = ctypes.c_int32(-1)
    N.check(N.load().cbx_plan_kernel_kind(rd.native.handle, ctypes.byref(k)))
    return k.value


def _jit_cases():
    from test_decode_fuzz import FUZZ_COPYBOOK, _random_bytes
    t1 = (G.read("test1_copybook.cob").decode(), G.read("test1_data", "example.bin"), {}, {})
    t6 = (G.read("test6_copybook.cob").decode(), G.read("test6_data", "INTEGR.TYPES.NOV28.DATA.dat"), {}, {})
    syn = (SYN200_COPYBOOK, syn200(100_003, seed=11).numpy().tobytes(), {}, {})
    cb = cbk.parse_copybook(FUZZ_COPYBOOK, code_page="cp037", string_trimming="left", floating_point_format="IEEE754")
    rng = np.random.default_rng(9)
    leaves = list(O._iter_leaves(cb.ast))
    recs = bytearray()
    for _ in range(2000):
        for p in leaves:
            recs += _random_bytes(rng, p, p.data_size)
    fz = (FUZZ_COPYBOOK, bytes(recs),
          dict(ebcdic_code_page="cp037", string_trimming_policy="left", floating_point_format="IEEE754"), {})
    return {"test1": t1, "test6": t6, "syn200": syn, "fuzz_cp037": fz}


@pytest.mark.parametrize("views", LAYOUTS)
@pytest.mark.parametrize("case", ["test1", "test6", "syn200", "fuzz_cp037"])
def test_specialised_kernel_vs_oracle(case, views):
    """The copybook-specialised kernel (hipRTC, cbx_jit.h) gives the oracle's results bit for bit,
    in the three string layouts (Arrow large-string offsets / string views / Utf8)."""
    cb_text, data, kw, okw = _jit_cases()[case]
    rd, batch = _fixed(cb_text, data, jit_min_records=1, **_layout(views), **kw)
    assert _kernel_kind(rd) == 1, "specialised kernel did not run"
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data, **okw))
    assert not errs, errs
    # the table-driven kernel on the same plan layout agrees as well
    rd2, batch2 = _fixed(cb_text, data, jit_min_records=-1, **_layout(views), **kw)
    assert _kernel_kind(rd2) == 0
    assert not compare_batch(batch2, O.decode_fixed(rd2.copybook, data, **okw))


def test_specialised_kernel_segments_and_offsets():
    cb_text = G.read("test5_copybook.cob").decode()
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    off, ln = O.frame_rdw(raw)
    cb = cbk.parse_copybook(cb_text)
    L = cb.record_size
    recs = b"".join(b"\x00\x11\x22" + (raw[o:o + l] + b"\x40" * L)[:L] + b"\x33" for o, l in zip(off, ln))
    seg_map = {"C": "STATIC-DETAILS", "P": "CONTACTS"}
    rd, batch = _fixed(cb_text, recs, segment_field="SEGMENT-ID", segment_id_redefine_map=seg_map,
                       start_offset=3, end_offset=1, jit_min_records=1)
    assert _kernel_kind(rd) == 1
    res = O.decode_fixed(rd.copybook, recs, segment_field="SEGMENT-ID", segment_redefine_map=seg_map,
                         record_size=L, start_offset=3, end_offset=1)
    assert not compare_batch(batch, res)


@pytest.mark.parametrize("views", LAYOUTS)
@pytest.mark.parametrize("n,jit", [(1, 0), (4097, 0), (50_000, 0), (50_000, 1), (300_001, 0)])
def test_synstr200_vs_oracle(n, jit, views):
    """Config C3 (string-heavy cp037, trim both): UTF-8 payloads bit-exact in the three string
    layouts, on both kernels (jit=1 forces the copybook-specialised kernel the bench runs; 300,001
    records pass the default specialisation threshold)."""
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    data = synstr200(n, seed=3 + n).numpy().tobytes()
    rd, batch = _fixed(SYNSTR200_COPYBOOK, data, ebcdic_code_page="cp037", jit_min_records=jit, **_layout(views))
    if n >= 262_144 or jit == 1:
        assert _kernel_kind(rd) == 1
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data))
    assert not errs, errs


@pytest.mark.parametrize("lists,jit", [(False, 0), (True, 0), (True, 1)])
def test_wide_odo_vs_oracle(lists, jit):
    """Config C5 (exp3 wide layout, OCCURS 0 TO 2000 DEPENDING ON, segment redefines, RDW), the
    array in slot rows or in the list layout (child elements packed per record)."""
    from cobrix_amd.synth import WIDE_ODO_COPYBOOK, WIDE_ODO_SEGMENTS, wide_odo
    raw_t, hdr = wide_odo(40, seed=5)
    raw = raw_t.numpy().tobytes()
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map=WIDE_ODO_SEGMENTS, occurs_lists=lists, jit_min_records=jit)
    rd = VarLenNestedReader(WIDE_ODO_COPYBOOK, params)
    t = raw_t.cuda()
    off, ln = rd.frame(t, len(raw))
    eo, el = O.frame_rdw(raw)
    assert np.array_equal(off.cpu().numpy(), eo) and np.array_equal(ln.cpu().numpy(), el)
    assert np.array_equal(eo - 4, hdr.numpy())
    batch = rd.decode_device(t, len(raw), off, ln)
    segs = [{"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(raw[o:o + 5].decode("cp037")))
            for o in eo]
    res = O.decode_records(rd.copybook, [raw[o:o + l] for o, l in zip(eo, el)], active_segments=segs)
    errs = compare_batch(batch, res)
    assert not errs, errs


LIST_COPYBOOK = """
       01  REC.
           05  CNT-A         PIC 9(3).
           05  CNT-B         PIC S9(4) COMP.
           05  ARR-A OCCURS 0 TO 150 TIMES DEPENDING ON CNT-A.
               10  A-BCD     PIC S9(5) COMP-3.
               10  A-BIN     PIC 9(4) COMP.
               10  A-ZON     PIC S9(3).
           05  ARR-B OCCURS 1 TO 5 TIMES DEPENDING ON CNT-B.
               10  B-ZON     PIC S9(18).
               10  B-WIDE    PIC 9(20)V9(5).
               10  B-BCD     PIC S9(17)V9(10) COMP-3.
               10  B-DBL     COMP-2.
"""


@pytest.mark.parametrize("n,jit", [(1, 0), (3001, 0), (3001, 1)])
def test_list_layout_fixed_vs_oracle(n, jit):
    """List layout on a fixed-length file: an 8-byte element array (list kernel, LDS-staged element
    groups, counts 0-170 incl. out-of-range ones) and a 65-byte element array (per-lane loads;
    zoned, wide DISPLAY, 14-byte COMP-3 and COMP-2 elements) against the oracle."""
    from test_decode_fuzz import _random_bytes
    cb = cbk.parse_copybook(LIST_COPYBOOK)
    leaves = {nm: cb.get_field_by_name(nm) for nm in ("A-BCD", "A-BIN", "A-ZON", "B-ZON", "B-WIDE", "B-BCD", "B-DBL")}
    rng = np.random.default_rng(n)
    pool_a = [b"".join(_random_bytes(rng, leaves[k], leaves[k].data_size) for k in ("A-BCD", "A-BIN", "A-ZON"))
              for _ in range(301)]
    pool_b = [b"".join(_random_bytes(rng, leaves[k], leaves[k].data_size) for k in ("B-ZON", "B-WIDE", "B-BCD", "B-DBL"))
              for _ in range(97)]
    recs = bytearray()
    for i in range(n):
        ca = int(rng.integers(0, 171))
        cb_ = int(rng.integers(0, 8))
        r = bytearray(("%03d" % ca).encode("cp037")) + cb_.to_bytes(2, "big")
        r += b"".join(pool_a[(i * 7 + j) % 301] for j in range(150))
        r += b"".join(pool_b[(i * 3 + j) % 97] for j in range(5))
        recs += r
    assert len(recs) == n * cb.record_size
    rd, batch = _fixed(LIST_COPYBOOK, bytes(recs), occurs_lists=True, jit_min_records=jit)
    assert sum(c.list_array >= 0 for c in rd.plan.columns) == 7
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, bytes(recs)))
    assert not errs, errs


@pytest.mark.parametrize("views", LAYOUTS)
def test_syn200_full_size_sampled_parity(views):
    """The bench's own configuration (C2: 50 M SYN200 records = 10 GB resident in HBM, the
    copybook-specialised kernel): 6,000 records sampled across the whole batch (random, plus the
    first and last tiles) are bit-exact against the oracle, and every string offset row is monotone."""
    from parity import compare_sample
    n = 50_000_000
    rec = syn200(n, seed=20261015, device="cuda")
    rd = FixedLenNestedReader(SYN200_COPYBOOK, ReaderParameters(**_layout(views)))
    batch = rd.decode_device(rec.view(-1), n * 200)
    assert _kernel_kind(rd) == 1
    rng = np.random.default_rng(2)
    idx = np.unique(np.concatenate([np.arange(128), n - 128 + np.arange(128), rng.integers(0, n, 5744)]))
    sample = rec[torch.as_tensor(idx, device="cuda")].cpu().numpy().tobytes()
    errs = compare_sample(batch, idx, O.decode_fixed(rd.copybook, sample))
    assert not errs, errs
    for ci, info in enumerate(rd.plan.columns):
        if info.out_type == 7 and views != "views":   # O_STRING: offsets non-decreasing over all 50 M records
            offs = batch.cols[ci]["offsets" if views == "large" else "offsets32"][: n + 1]
            assert bool((offs[1:] >= offs[:-1]).all())
    del batch, rec
    torch.cuda.empty_cache()


def test_synstr200_full_size_sampled_views():
    """Config C3 at the bench's size (50 M SYNSTR200 records, string views, the specialised
    kernel): a sample across the batch is bit-exact; every view is well-formed (inline bytes past
    the length are zero, long views point inside their tile's region)."""
    from parity import compare_sample
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    n = 50_000_000
    rec = synstr200(n, seed=20261017, device="cuda")
    rd = FixedLenNestedReader(SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_views=True))
    batch = rd.decode_device(rec.view(-1), n * 200)
    assert _kernel_kind(rd) == 1
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([np.arange(128), n - 128 + np.arange(128), rng.integers(0, n, 3744)]))
    sample = rec[torch.as_tensor(idx, device="cuda")].cpu().numpy().tobytes()
    errs = compare_sample(batch, idx, O.decode_fixed(rd.copybook, sample))
    assert not errs, errs
    c = batch.cols[0]
    v = c["views"].view(-1, 16)[:n].view(torch.int32)
    ln = v[:, 0]
    assert int(ln.min()) >= 0 and int(ln.max()) <= 40
    short = ln <= 12
    # inline padding is zero: the bytes of word k of a short view past its length
    for k in (1, 2, 3):
        w = v[:, k].to(torch.int64) & 0xFFFFFFFF
        keep = (ln - 4 * (k - 1)).clamp(0, 4)
        mask = torch.where(keep >= 4, torch.full_like(w, 0xFFFFFFFF), (1 << (8 * keep.to(torch.int64))) - 1)
        assert bool(((w & ~mask)[short] == 0).all())
    tiles = torch.arange(n, device="cuda") // 64
    pos = v[:, 2].to(torch.int64) * c["buffer_bytes"] + v[:, 3].to(torch.int64)
    lo = tiles * c["tile_bytes"]
    assert bool(((pos >= lo) & (pos + ln.to(torch.int64) <= lo + c["tile_bytes"]))[~short].all())
    del batch, rec
    torch.cuda.empty_cache()


def _var_decode_vs_oracle(raw: bytes, views: str, **kw):
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, RDW_NARROW_SEGMENTS
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map=RDW_NARROW_SEGMENTS, **_layout(views), **kw)
    rd = VarLenNestedReader(RDW_NARROW_COPYBOOK, params)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    off, ln = rd.frame(t, len(raw))
    eo, el = O.frame_rdw(raw)
    assert np.array_equal(off.cpu().numpy(), eo) and np.array_equal(ln.cpu().numpy(), el)
    batch = rd.decode_device(t, len(raw), off, ln)
    segs = [{"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(raw[o:o + min(5, l)].decode("cp037")))
            for o, l in zip(eo, el)]
    res = O.decode_records(rd.copybook, [raw[o:o + l] for o, l in zip(eo, el)], active_segments=segs)
    return rd, compare_batch(batch, res)


@pytest.mark.parametrize("views", LAYOUTS)
def test_var_span_kernel_vs_oracle(views):
    """The specialised span kernel (variable-length tiles staged by byte span, span_loop) on the C4
    layout, and on records of 1-3,000 bytes where many tiles overflow the span staging and fall
    back to record-by-record windows (short records: trailing fields null / truncated).  In the
    view layout the C and P string fields are decoded in pairs (str_view_pair): lanes of either
    segment, of neither, and short records in one pass."""
    from cobrix_amd.synth import rdw_narrow
    raw = rdw_narrow(20_000, seed=21)[0].numpy().tobytes()
    rd, errs = _var_decode_vs_oracle(raw, views, jit_min_records=1)
    assert _kernel_kind(rd) == 1 and not errs, errs
    rng = np.random.default_rng(4)
    body = bytearray()
    for i in range(5000):
        ln = int(rng.integers(1, 3000)) if rng.random() < 0.2 else int(rng.integers(1, 90))
        payload = bytearray(rng.integers(0x40, 0xFA, ln, dtype=np.uint8).tobytes())
        # segment id C / P (cp037), or X: a segment with no redefine (all its redefine fields null)
        payload[:5] = (b"\xE7" if i % 7 == 0 else b"\xC3" if i % 3 else b"\xD7") + b"\x40" * 4
        payload = payload[:ln]
        body += bytes([0, 0, ln & 0xFF, ln >> 8]) + bytes(payload)
    rd, errs = _var_decode_vs_oracle(bytes(body), views, jit_min_records=1)
    assert _kernel_kind(rd) == 1 and not errs, errs


@pytest.mark.parametrize("n", [1, 63, 4097, 20_011, 300_001])
def test_utf8_chain_vs_oracle(n):
    """The Arrow Utf8 chain of the specialised kernels (count pass, scan of the tile totals, decode
    writing every payload byte at its final place): bit-exact against the oracle across tile and grid
    round boundaries."""
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    data = synstr200(n, seed=5 + n).numpy().tobytes()
    rd, batch = _fixed(SYNSTR200_COPYBOOK, data, ebcdic_code_page="cp037", jit_min_records=1, string_utf8=True)
    assert _kernel_kind(rd) == 1, "specialised kernel did not run"
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data))
    assert not errs, errs


@pytest.mark.parametrize("trim", ["none", "left", "right", "both"])
@pytest.mark.parametrize("cp", ["cp037", "common", "ascii"])
def test_utf8_code_pages_and_trim(cp, trim):
    """The Utf8 decode's width-pattern compose (characters of 0 / 1 / 2 UTF-8 bytes, those outside
    the trimmed range dropped) on every trim policy, single- and two-byte code pages and ASCII, with
    fields of 1..32 bytes (groups of 4 characters cut at every phase) and values full of trimmable
    bytes: bit-exact against the oracle."""
    sizes = [1, 2, 3, 4, 5, 7, 8, 9, 13, 16, 17, 20, 31, 32]
    cb_text = "       01  R.\n" + "".join(f"          05  F{i}  PIC X({s}).\n" for i, s in enumerate(sizes))
    rec = sum(sizes)
    rng = np.random.default_rng(17)
    n = 70_000
    raw = rng.integers(0, 256, (n, rec), dtype=np.uint8)
    # a third of the bytes trimmable in runs at either end, spaces inside
    pad = 0x40 if cp != "ascii" else 0x20
    sp = rng.random((n, rec)) < 0.33
    raw[sp] = pad
    raw[:, ::5][rng.random((n, (rec + 4) // 5)) < 0.2] = 0x05 if cp != "ascii" else 0x09
    data = raw.tobytes()
    kw = dict(string_trimming_policy=trim, jit_min_records=1, string_utf8=True)
    if cp == "ascii":
        kw["is_ebcdic"] = False
    else:
        kw["ebcdic_code_page"] = cp
    rd, batch = _fixed(cb_text, data, **kw)
    assert _kernel_kind(rd) == 1
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data))
    assert not errs, errs


@pytest.mark.parametrize("staged", [False, True])
@pytest.mark.parametrize("trim", ["none", "left", "right", "both"])
@pytest.mark.parametrize("cp", ["cp037", "common", "ascii"])
def test_utf8_decode_code_pages_and_trim(cp, trim, staged, monkeypatch):
    """The count + scan + decode Arrow Utf8 path on fields of 1..32 bytes full of trimmable bytes, every
    trim policy, single- / two-byte code pages and ASCII; staged (the default): the tile-staged payload
    store (kept bytes OR-ed into a zeroed tile-contiguous LDS staging, copied out in aligned 16-byte
    chunks, byte stores at the ends), else each lane's own stores (CBX_U8_DIRECT).  Bit-exact against
    the oracle."""
    sizes = [1, 2, 3, 4, 5, 7, 8, 9, 13, 16, 17, 20, 31, 32]
    cb_text = "       01  R.\n" + "".join(f"          05  F{i}  PIC X({s}).\n" for i, s in enumerate(sizes))
    rec = sum(sizes)
    rng = np.random.default_rng(19)
    n = 70_003
    raw = rng.integers(0, 256, (n, rec), dtype=np.uint8)
    pad = 0x40 if cp != "ascii" else 0x20
    raw[rng.random((n, rec)) < 0.33] = pad
    raw[:, ::5][rng.random((n, (rec + 4) // 5)) < 0.2] = 0x05 if cp != "ascii" else 0x09
    data = raw.tobytes()
    if not staged:
        monkeypatch.setenv("CBX_JIT_DEFINES", "CBX_U8_DIRECT=1")
    kw = dict(string_trimming_policy=trim, jit_min_records=1, string_utf8=True)
    if cp == "ascii":
        kw["is_ebcdic"] = False
    else:
        kw["ebcdic_code_page"] = cp
    rd, batch = _fixed(cb_text, data, **kw)
    assert _kernel_kind(rd) == 1
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data))
    assert not errs, errs


def test_synstr200_full_size_sampled_utf8():
    """Config C3 as the bench runs it (50 M SYNSTR200 records, Arrow Utf8 layout: count pass, device
    scan, every offset and payload byte written once by the specialised decode kernel): a sample
    across the batch is bit-exact; every slot's int32 offsets start at 0, never decrease, end at the
    slot's size, and the payload bytes equal the sum of the view-layout lengths of the same input."""
    from parity import compare_sample
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    n = 50_000_000
    rec = synstr200(n, seed=20261017, device="cuda")
    rd = FixedLenNestedReader(SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_utf8=True))
    batch = rd.decode_device(rec.view(-1), n * 200)
    assert _kernel_kind(rd) == 1
    rng = np.random.default_rng(6)
    idx = np.unique(np.concatenate([np.arange(128), n - 128 + np.arange(128), rng.integers(0, n, 3744)]))
    sample = rec[torch.as_tensor(idx, device="cuda")].cpu().numpy().tobytes()
    errs = compare_sample(batch, idx, O.decode_fixed(rd.copybook, sample))
    assert not errs, errs
    for c in batch.cols:
        o = c["offsets32"][: n + 1]
        assert int(o[0]) == 0 and bool((o[1:] >= o[:-1]).all())
        assert int(o[n]) == int(c["sizes"][0]) and 0 < int(o[n]) <= c["capacity"]
    del batch, rec
    torch.cuda.empty_cache()


def test_utf8_layout_capacity_overflow_reported():
    """A Utf8 region smaller than the batch's payload: nothing is written past it, and the plan's
    check reports CBX_E_CAPACITY (as the large-string layout does)."""
    import ctypes
    from cobrix_amd import native as N
    from cobrix_amd.reader import _alloc_columns
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    n = 10_000
    data = synstr200(n, seed=8, device="cuda").view(-1)
    rd = FixedLenNestedReader(SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_utf8=True))
    cols, cs = _alloc_columns(rd.plan, n, [1000] * rd.plan.n_columns, "cuda")
    guard = [c["data"].clone() for c in cols]
    L = N.load()
    N.check(L.cbx_decode_fixed(rd.native.handle, data.data_ptr(), n, 200, 0, 0, cs, None))
    with pytest.raises(N.CbxError) as e:
        N.check(L.cbx_plan_check(rd.native.handle, None))
    assert e.value.code == N.CBX_E_CAPACITY
    assert all(c["data"].numel() == g.numel() for c, g in zip(cols, guard))
    N.check(L.cbx_plan_check(rd.native.handle, None))   # the flag is cleared


COMPOSE_COPYBOOK = """
       01  REC.
           05  S01   PIC X(1).
           05  S03   PIC X(3).
           05  S04   PIC X(4).
           05  S05   PIC X(5).
           05  S07   PIC X(7).
           05  S08   PIC X(8).
           05  S13   PIC X(13).
           05  S20   PIC X(20).
           05  S31   PIC X(31).
           05  S32   PIC X(32).
"""


def _compose_records(n: int, size: int, seed: int) -> bytes:
    """Record bytes that exercise the string compose: any byte value (cp037 maps half of them to
    2-byte UTF-8, and 0x00-0x3F to C0/C1 controls, some trimmable), text with runs of EBCDIC
    spaces at either end, all-space and all-wide values."""
    rng = np.random.default_rng(seed)
    out = np.empty((n, size), dtype=np.uint8)
    kind = rng.integers(0, 5, n)
    out[:] = rng.integers(0, 256, (n, size), dtype=np.uint8)
    text = rng.integers(0x40, 0xFF, (n, size), dtype=np.uint8)
    out[kind == 1] = text[kind == 1]
    pad = rng.random((n, size)) < 0.3
    out[(kind == 2)[:, None] & pad] = 0x40
    out[kind == 3] = 0x40
    out[kind == 4] = rng.integers(0x80, 0x100, (int((kind == 4).sum()), size), dtype=np.uint8)
    return out.tobytes()


@pytest.mark.parametrize("views", ["views", "utf8"])
@pytest.mark.parametrize("trim", ["none", "left", "right", "both"])
@pytest.mark.parametrize("jit", [-1, 1])
def test_two_byte_page_compose_vs_oracle(views, trim, jit):
    """Register-path strings of a 2-byte code page (cp037: str_lane_group2 composes 4 characters at a
    time and places them with dword LDS stores) -- fields of 1-32 bytes at every dword phase, every
    trimming policy, both kernels, the view and Utf8 layouts -- against the oracle's
    StringDecoders.decodeEbcdicString + StringTools.trim* restatement."""
    cb = cbk.parse_copybook(COMPOSE_COPYBOOK, code_page="cp037", string_trimming=trim)
    data = _compose_records(4097, cb.record_size, seed=len(trim) + 7 * (jit + 2))
    rd, batch = _fixed(COMPOSE_COPYBOOK, data, ebcdic_code_page="cp037", string_trimming_policy=trim,
                       jit_min_records=jit, **_layout(views))
    if jit == 1:
        assert _kernel_kind(rd) == 1
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data))
    assert not errs, errs[:10]


@pytest.mark.parametrize("views", ["views", "utf8"])
@pytest.mark.parametrize("trim", ["none", "both", "left"])
@pytest.mark.parametrize("jit", [-1, 1])
def test_one_byte_waves_compose_vs_oracle(views, trim, jit):
    """cp037 fields whose characters all map to 1-byte UTF-8 (letters, digits, EBCDIC spaces and
    trimmable controls) in most tiles, every third tile with one accented character in one record:
    the 2-byte group compose on waves of (almost) only 1-byte characters, fields of 1-32 bytes at
    every dword phase, against the oracle."""
    from cobrix_amd.synth import _CP037_ALNUM, _CP037_ACCENTED
    cb = cbk.parse_copybook(COMPOSE_COPYBOOK, code_page="cp037", string_trimming=trim)
    n, size = 64 * 97 + 13, cb.record_size
    rng = np.random.default_rng(len(trim) + 3 * (jit + 2))
    narrow = np.array(_CP037_ALNUM + [0x40] * 12 + [0x05, 0x25, 0x4B, 0x6B], dtype=np.uint8)
    out = narrow[rng.integers(0, len(narrow), (n, size))]
    lead = rng.random(n) < 0.2
    out[lead, : size // 3] = 0x40
    for t in range(0, (n + 63) // 64, 3):   # one accented character in every third tile
        r = min(n - 1, 64 * t + int(rng.integers(0, 64)))
        out[r, int(rng.integers(0, size))] = _CP037_ACCENTED[t % len(_CP037_ACCENTED)]
    data = out.tobytes()
    rd, batch = _fixed(COMPOSE_COPYBOOK, data, ebcdic_code_page="cp037", string_trimming_policy=trim,
                       jit_min_records=jit, **_layout(views))
    errs = compare_batch(batch, O.decode_fixed(rd.copybook, data))
    assert not errs, errs[:10]


def _wide_odo_forced(n_roots: int, seed: int):
    """C5 records (wide_odo) with the NUM-STRAT dependee forced, root by root, to 0, 1, 2000, out of
    range (2001, 65535) or random, and a share of C records cut before NUM-STRAT (a null dependee:
    decodeTypeValue past the record end, so the array takes its maximum) or inside the elements."""
    from cobrix_amd.synth import wide_odo
    raw_t, hdr = wide_odo(n_roots, seed=seed)
    raw = raw_t.numpy()
    hdr = hdr.numpy()
    rng = np.random.default_rng(seed)
    out = bytearray()
    forced = [0, 1, 2000, 2001, 65535]
    ci = 0
    for i, h in enumerate(hdr):
        ln = int(raw[h + 2]) | int(raw[h + 3]) << 8
        payload = bytearray(raw[h + 4:h + 4 + ln].tobytes())
        if payload[0] == 0xC3:
            cnt = forced[ci % 6] if ci % 6 < 5 else int(rng.integers(0, 2001))
            payload[64:66] = cnt.to_bytes(2, "big")
            ci += 1
            u = rng.random()
            if u < 0.03:
                payload = payload[:int(rng.integers(1, 66))]            # NUM-STRAT missing: null
            elif u < 0.06:
                payload = payload[:int(rng.integers(66, len(payload)))]  # elements cut short
        out += bytes([0, 0, len(payload) & 0xFF, len(payload) >> 8]) + bytes(payload)
    return bytes(out)


@pytest.mark.parametrize("jit", [0, 1])
def test_wide_odo_forced_counts_vs_oracle(jit):
    """C5 at 2,000 roots (+ ~4,000 children): element counts 0, 1, 2000, out of range and null
    (RecordExtractors.scala:66-114 extractArray: a dependee outside [min, max] or unset -> max), short
    records, both kernels, the list layout -- every value bit-exact against the oracle."""
    from cobrix_amd.synth import WIDE_ODO_COPYBOOK, WIDE_ODO_SEGMENTS
    raw = _wide_odo_forced(2000, seed=31 + jit)
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map=WIDE_ODO_SEGMENTS, occurs_lists=True, jit_min_records=jit)
    rd = VarLenNestedReader(WIDE_ODO_COPYBOOK, params)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    off, ln = rd.frame(t, len(raw))
    eo, el = O.frame_rdw(raw)
    assert np.array_equal(off.cpu().numpy(), eo) and np.array_equal(ln.cpu().numpy(), el)
    batch = rd.decode_device(t, len(raw), off, ln)
    segs = [{"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(raw[o:o + min(5, l)].decode("cp037")))
            for o, l in zip(eo, el)]
    res = O.decode_records(rd.copybook, [raw[o:o + l] for o, l in zip(eo, el)], active_segments=segs)
    errs = compare_batch(batch, res)
    assert not errs, errs
    # every forced count class is present
    cnt_ci = rd.plan.arrays[0].count_column
    cnts = batch.host_column(cnt_ci)["values"][:batch.n_rec]
    for c in (0, 1, 2000):
        assert (cnts == c).any()


def _check_framing(off, ln, hdr, n_bytes):
    """Every framed record against the generator's RDW header list: payload at header + 4, length up to
    the next header (the file end for the last)."""
    hdr = hdr.to(off.device)
    assert off.numel() == hdr.numel(), (off.numel(), hdr.numel())
    assert torch.equal(off, hdr + 4)
    nxt = torch.cat([hdr[1:], torch.tensor([n_bytes], dtype=hdr.dtype, device=hdr.device)])
    assert torch.equal(ln.to(torch.int64), nxt - hdr - 4)


def test_rdw_narrow_full_size_framing_and_sample():
    """C4 as the bench runs it: 150 M RDW records (9.8 GB) framed by cbx_frame_rdw from seeds at the
    100 MB index spacing -- every record's offset and length equal to the generator's header list --
    then decoded (string views, the bench's layout); 2,000 records sampled across the batch are
    bit-exact against the oracle's decode of the same records."""
    from parity import compare_sample
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, RDW_NARROW_SEGMENTS, rdw_narrow_large
    n = 150_000_000
    raw_t, hdr = rdw_narrow_large(n, device="cuda")
    n_bytes = int(raw_t.numel())
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map=RDW_NARROW_SEGMENTS, string_views=True)
    rd = VarLenNestedReader(RDW_NARROW_COPYBOOK, params)
    marks = torch.arange(0, n_bytes, 100 * 1024 * 1024, device="cuda")
    seeds = torch.unique(hdr[torch.searchsorted(hdr, marks).clamp(max=n - 1)]).tolist()
    off, ln = rd.frame(raw_t, n_bytes, seeds=seeds)
    _check_framing(off, ln, hdr, n_bytes)
    del hdr
    torch.cuda.empty_cache()
    batch = rd.decode_device(raw_t, n_bytes, off, ln)
    assert batch.n_rec == n
    rng = np.random.default_rng(13)
    idx = np.unique(np.concatenate([np.arange(64), n - 64 + np.arange(64), rng.integers(0, n, 1872)]))
    offs = off[torch.as_tensor(idx, device="cuda")].cpu().numpy()
    lens = ln[torch.as_tensor(idx, device="cuda")].cpu().numpy()
    recs = [raw_t[o:o + l].cpu().numpy().tobytes() for o, l in zip(offs, lens)]
    segs = [{"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(r[:5].decode("cp037"))) for r in recs]
    res = O.decode_records(rd.copybook, recs, active_segments=segs)
    errs = compare_sample(batch, idx, res)
    assert not errs, errs
    del batch, raw_t, off, ln
    torch.cuda.empty_cache()


def test_wide_odo_full_size_sampled_parity():
    """C5 as the bench runs it (770,000 roots + children = 2.31 M records, 12.5 GB, list layout, the
    specialised kernels): the framing against the generator's header list, then 2,000 records sampled
    across the batch -- counts, list offsets and every present element -- bit-exact against the
    oracle's decode of the same records."""
    from parity import compare_sample_lists, compare_sample
    from cobrix_amd.synth import WIDE_ODO_COPYBOOK, WIDE_ODO_SEGMENTS, wide_odo
    raw_t, hdr = wide_odo(770_000, seed=20261018, device="cuda")
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map=WIDE_ODO_SEGMENTS, occurs_lists=True, string_views=True)
    rd = VarLenNestedReader(WIDE_ODO_COPYBOOK, params)
    n_bytes = int(raw_t.numel())
    off, ln = rd.frame(raw_t, n_bytes)
    _check_framing(off, ln, hdr, n_bytes)
    batch = rd.decode_device(raw_t, n_bytes, off, ln)
    assert batch.n_rec > 2_000_000 and _kernel_kind(rd) in (1, 4)
    rng = np.random.default_rng(12)
    n = batch.n_rec
    idx = np.unique(np.concatenate([np.arange(64), n - 64 + np.arange(64), rng.integers(0, n, 1872)]))
    offs = off[torch.as_tensor(idx, device="cuda")].cpu().numpy()
    lens = ln[torch.as_tensor(idx, device="cuda")].cpu().numpy()
    recs = [raw_t[o:o + l].cpu().numpy().tobytes() for o, l in zip(offs, lens)]
    segs = [{"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(r[:5].decode("cp037"))) for r in recs]
    res = O.decode_records(rd.copybook, recs, active_segments=segs)
    errs = compare_sample(batch, idx, res) + compare_sample_lists(batch, idx, res)
    assert not errs, errs
    del batch, raw_t
    torch.cuda.empty_cache()


def test_var_utf8_batches_vs_oracle():
    """C4 in the Arrow Utf8 layout decoded in batches whose int32 offsets fit (bench.py --strings
    offsets: one Arrow array per batch and column): each batch of framed records -- cut mid-run, at
    ragged sizes -- is bit-exact against the oracle, and its Record_Id continues from the batch's
    first record."""
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, RDW_NARROW_SEGMENTS, rdw_narrow
    raw_t, _ = rdw_narrow(200_003, seed=31)
    raw = raw_t.numpy().tobytes()
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID", generate_record_id=True,
                              segment_id_redefine_map=RDW_NARROW_SEGMENTS, string_utf8=True)
    rd = VarLenNestedReader(RDW_NARROW_COPYBOOK, params)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    off, ln = rd.frame(t, len(raw))
    eo, el = O.frame_rdw(raw)
    assert np.array_equal(off.cpu().numpy(), eo)
    n = len(eo)
    cuts = [0, 64_000, 64_001, 131_072 + 37, n]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        batch = rd.decode_device(t, len(raw), off[r0:r1], ln[r0:r1], first_record_id=r0)
        recs = [raw[o:o + l] for o, l in zip(eo[r0:r1], el[r0:r1])]
        segs = [{"C": "STATIC_DETAILS", "P": "CONTACTS"}.get(G.java_trim(r[:5].decode("cp037"))) for r in recs]
        errs = compare_batch(batch, O.decode_records(rd.copybook, recs, active_segments=segs))
        assert not errs, (r0, errs)
        rid = batch.cols[rd.plan.record_id_column]["values"][: r1 - r0].cpu().numpy()
        assert np.array_equal(rid, np.arange(r0, r1)), r0


@pytest.mark.parametrize("caps", [(0, 0), (1, 7)])
def test_utf8_pipelined_plans_vs_single(caps):
    """cbx_plan_pipeline: batches alternating between two linked plans on two streams (each call's count
    pass after the peer's, beside the peer's decode; the kernels' workgroups per CU capped) give the same
    columns as one plan decoding the batches in turn, and as the oracle on a sample."""
    import ctypes
    from cobrix_amd import native as N
    from cobrix_amd.reader import _alloc_columns, string_capacity, DecodedBatch
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    from parity import compare_sample
    n, nb = 2_000_000, 5
    rec = synstr200(n, seed=31, device="cuda").view(-1)
    prm = ReaderParameters(ebcdic_code_page="cp037", string_utf8=True)
    A, B, S = (FixedLenNestedReader(SYNSTR200_COPYBOOK, prm) for _ in range(3))
    L = N.load()
    N.check(L.cbx_plan_pipeline(A.native.handle, B.native.handle, caps[0], caps[1]))
    s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream()
    s2.wait_stream(s1)   # (the generated input)
    m = n // nb
    outs, refs = [], []
    for i in range(nb):
        h, st = (A.native.handle, s1) if i % 2 == 0 else (B.native.handle, s2)
        with torch.cuda.stream(st):   # (zero-filled on the stream that decodes the batch)
            cols, cs = _alloc_columns(A.plan, m, string_capacity(A.native, m), rec.device)
        N.check(L.cbx_decode_fixed(h, rec.data_ptr() + i * m * 200, m, 200, 0, i * m, cs, ctypes.c_void_p(st.cuda_stream)))
        outs.append(cols)
    torch.cuda.synchronize()
    for rd in (A, B):
        N.check(L.cbx_plan_check(rd.native.handle, ctypes.c_void_p(s1.cuda_stream)))
    for i in range(nb):
        cols, cs = _alloc_columns(S.plan, m, string_capacity(S.native, m), rec.device)
        N.check(L.cbx_decode_fixed(S.native.handle, rec.data_ptr() + i * m * 200, m, 200, 0, i * m, cs,
                                   ctypes.c_void_p(s1.cuda_stream)))
        refs.append(cols)
    torch.cuda.synchronize()
    for i in range(nb):
        for a, b in zip(outs[i], refs[i]):
            assert torch.equal(a["offsets32"], b["offsets32"]) and torch.equal(a["validity"], b["validity"])
            assert torch.equal(a["data"][: int(b["sizes"][0])], b["data"][: int(b["sizes"][0])])
    batch = DecodedBatch(A.plan, m, outs[3], 3 * m, False, False)
    idx = np.unique(np.random.default_rng(2).integers(0, m, 2000))
    sample = rec.view(n, 200)[torch.as_tensor(3 * m + idx, device="cuda")].cpu().numpy().tobytes()
    assert not compare_sample(batch, idx, O.decode_fixed(A.copybook, sample))
    N.check(L.cbx_plan_pipeline(A.native.handle, None, 0, 0))


def test_decode_batches_pipelined_utf8():
    """FixedLenNestedReader.decode_batches in the Utf8 layout: batches alternate between the reader's
    plan and a pipelined peer (cbx_plan_pipeline) on two streams; every batch equals decode_device of
    the same records, and the views layout decodes the same batches in turn."""
    from cobrix_amd.synth import SYNSTR200_COPYBOOK, synstr200
    n, bs = 700_003, 150_000
    rec = synstr200(n, seed=41, device="cuda").view(-1)
    rd = FixedLenNestedReader(SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_utf8=True))
    batches = rd.decode_batches(rec, n * 200, bs, first_record_id=10)
    assert [b.n_rec for b in batches] == [bs] * 4 + [n - 4 * bs]
    ref = FixedLenNestedReader(SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_utf8=True))
    for k, b in enumerate(batches):
        r = ref.decode_device(rec[k * bs * 200: min(n, (k + 1) * bs) * 200], b.n_rec * 200, first_record_id=10 + k * bs)
        for x, y in zip(b.cols, r.cols):
            assert torch.equal(x["offsets32"], y["offsets32"]) and torch.equal(x["validity"], y["validity"])
            assert torch.equal(x["data"][: int(y["sizes"][0])], y["data"][: int(y["sizes"][0])])
    assert batches[4].to_rows()[:50] == ref.decode_device(rec[4 * bs * 200:], (n - 4 * bs) * 200).to_rows()[:50]
    rd.close()
    vw = FixedLenNestedReader(SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_views=True))
    vb = vw.decode_batches(rec, n * 200, bs)
    assert sum(b.n_rec for b in vb) == n and vb[1].to_rows()[:20] == batches[1].to_rows()[:20]
