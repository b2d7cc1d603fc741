"""GPU RDW offset discovery (cbx_frame_rdw, chunk-parallel speculate / verify / repair) against the
oracle's sequential walk (RecordHeaderParserRDW.scala:44-85, VRLRecordReader.scala:151-186).

Small CBX_RDW_CHUNK_BYTES values force thousands of chunks per file, so most chunks start inside
a record and their speculated entries must be checked and repaired.
"""
from __future__ import annotations

import re

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from cobrix_amd.native import CbxError  # noqa: E402
from cobrix_amd.reader import ReaderParameters, VarLenNestedReader  # noqa: E402
from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import reader_oracle as RO  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _frame(raw: bytes, seeds=None, **kw):
    rd = VarLenNestedReader(RDW_NARROW_COPYBOOK, ReaderParameters(is_record_sequence=True, **kw))
    t = torch.frombuffer(bytearray(raw) if raw else bytearray(16), dtype=torch.uint8).cuda()
    off, ln = rd.frame(t, len(raw), seeds=seeds)
    return off.cpu().numpy(), ln.cpu().numpy()


def _oracle(raw: bytes, **kw):
    return O.frame_rdw(raw, **kw)


def _adversarial(n: int, seed: int, big_endian=False, adjust=0, max_len=3000, p_long=0.3) -> bytes:
    """Records of 1..max_len bytes whose payloads are full of zeros and fake plausible headers."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    for _ in range(n):
        ln = int(rng.integers(1, max_len)) if rng.random() < p_long else int(rng.integers(1, 80))
        hl = ln - adjust
        h = bytes([hl >> 8, hl & 0xFF, 0, 0]) if big_endian else bytes([0, 0, hl & 0xFF, hl >> 8])
        body = bytearray(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
        for _ in range(ln // 16):   # fake headers inside the payload
            p = int(rng.integers(0, max(1, ln - 4)))
            fl = int(rng.integers(1, 200))
            body[p:p + 4] = bytes([fl >> 8, fl & 0xFF, 0, 0]) if big_endian else bytes([0, 0, fl & 0xFF, fl >> 8])
        if rng.random() < 0.2:
            body[:] = bytes(len(body))
        out += h + bytes(body[:ln])
    return bytes(out)


@pytest.mark.parametrize("chunk", [8, 37, 256, 4096, None])
@pytest.mark.parametrize("big_endian", [False, True])
def test_c4_layout_vs_oracle(monkeypatch, chunk, big_endian):
    if chunk:
        monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", str(chunk))
    d, _ = rdw_narrow(20_000, seed=3, big_endian=big_endian)
    raw = d.numpy().tobytes()
    eo, el = _oracle(raw, big_endian=big_endian)
    off, ln = _frame(raw, is_rdw_big_endian=big_endian)
    assert np.array_equal(off, eo) and np.array_equal(ln, el)
    seeds = [e[0] for e in O.sparse_index(raw, big_endian=big_endian, records_per_entry=997)]
    off2, ln2 = _frame(raw, seeds=seeds, is_rdw_big_endian=big_endian)
    assert np.array_equal(off2, eo) and np.array_equal(ln2, el)


@pytest.mark.parametrize("chunk", [8, 64, 1000])
@pytest.mark.parametrize("case", [dict(), dict(big_endian=True), dict(adjust=-4), dict(header=10, footer=7)])
def test_adversarial_payloads(monkeypatch, chunk, case):
    monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", str(chunk))
    be, adj = case.get("big_endian", False), case.get("adjust", 0)
    body = _adversarial(800, seed=chunk + 7 * len(case), big_endian=be, adjust=adj)
    hb, fb = case.get("header", 0), case.get("footer", 0)
    raw = (bytes([0, 0, 0, 0]) + b"\x11" * (hb - 4) if hb else b"") + body + b"\x22" * fb
    eo, el = _oracle(raw, big_endian=be, adjustment=adj, file_header_bytes=hb, file_footer_bytes=fb)
    kw = dict(is_rdw_big_endian=be, rdw_adjustment=adj, file_start_offset=hb, file_end_offset=fb)
    off, ln = _frame(raw, **kw)
    assert len(off) == len(eo)
    assert np.array_equal(off, eo) and np.array_equal(ln, el)


@pytest.mark.parametrize("lane_walk", ["1", "0"])
@pytest.mark.parametrize("chunk", [4096, 65536, None])
@pytest.mark.parametrize("case", [dict(), dict(big_endian=True), dict(adjust=-4), dict(header=10, footer=7)])
def test_long_records_lane_walk(monkeypatch, lane_walk, chunk, case):
    """Records of ~1-20 KB (C5-like) with fake headers in their payloads: chunks of long records are
    walked one lane per chunk (rdw_lane_walk_kernel) after the speculation pass, dense stretches handed
    back to the wave walk -- the same offsets as the sequential walk, with (1) and without (0) the lane
    walk; small chunks make most speculated entries wrong."""
    monkeypatch.setenv("CBX_RDW_LANE_WALK", lane_walk)
    if chunk:
        monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", str(chunk))
    be, adj = case.get("big_endian", False), case.get("adjust", 0)
    body = _adversarial(600, seed=(chunk or 1) + 11 * len(case), big_endian=be, adjust=adj, max_len=20000, p_long=0.8)
    hb, fb = case.get("header", 0), case.get("footer", 0)
    raw = (bytes([0, 0, 0, 0]) + b"\x11" * (hb - 4) if hb else b"") + body + b"\x22" * fb
    eo, el = _oracle(raw, big_endian=be, adjustment=adj, file_header_bytes=hb, file_footer_bytes=fb)
    kw = dict(is_rdw_big_endian=be, rdw_adjustment=adj, file_start_offset=hb, file_end_offset=fb)
    off, ln = _frame(raw, **kw)
    assert len(off) == len(eo)
    assert np.array_equal(off, eo) and np.array_equal(ln, el)
    seeds = [e[0] for e in O.sparse_index(raw, big_endian=be, records_per_entry=97, adjustment=adj,
                                          file_header_bytes=hb, file_footer_bytes=fb)]
    off2, ln2 = _frame(raw, seeds=seeds, **kw)
    assert np.array_equal(off2, eo) and np.array_equal(ln2, el)


@pytest.mark.parametrize("lane_walk", ["1", "0"])
def test_long_records_error_position(monkeypatch, lane_walk):
    """A zero-length header among long records: the first one on the chain is reported, lane walk or not."""
    monkeypatch.setenv("CBX_RDW_LANE_WALK", lane_walk)
    monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", "65536")
    rng = np.random.default_rng(4)
    raw = bytearray()
    hdrs = []
    for _ in range(300):
        ln = int(rng.integers(4000, 16000))
        hdrs.append(len(raw))
        raw += bytes([0, 0, ln & 0xFF, ln >> 8]) + bytes(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
    for k in (150, 250):
        raw[hdrs[k]:hdrs[k] + 4] = bytes(4)
    raw = bytes(raw)
    with pytest.raises(RuntimeError) as oe:
        _oracle(raw)
    with pytest.raises(CbxError) as ge:
        _frame(raw)
    want = int(re.search(r"offset (\d+)", str(oe.value)).group(1))
    assert f"at {want}." in str(ge.value), (str(ge.value), want)


def test_record_spanning_many_chunks(monkeypatch):
    monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", "512")
    rng = np.random.default_rng(2)
    raw = bytearray()
    for ln in (10, 60000, 3, 64000, 5, 17):
        raw += bytes([0, 0, ln & 0xFF, ln >> 8]) + bytes(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
    raw = bytes(raw)
    eo, el = _oracle(raw)
    off, ln = _frame(raw)
    assert np.array_equal(off, eo) and np.array_equal(ln, el)


def test_truncated_last_record_and_tiny_inputs():
    d, _ = rdw_narrow(50, seed=5)
    raw = d.numpy().tobytes()
    for cut in (len(raw) - 1, len(raw) - 30, len(raw) - 66, 3, 2, 0):
        part = raw[:cut]
        eo, el = _oracle(part)
        off, ln = _frame(part)
        assert np.array_equal(off, eo) and np.array_equal(ln, el), cut


@pytest.mark.parametrize("chunk", [16, None])
def test_zero_length_header_is_an_error_at_the_first_occurrence(monkeypatch, chunk):
    if chunk:
        monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", str(chunk))
    d, hdr = rdw_narrow(400, seed=9)
    raw = bytearray(d.numpy().tobytes())
    for k in (123, 300):   # two zero-length headers: the first one is reported
        h = int(hdr[k])
        raw[h:h + 4] = bytes(4)
    raw = bytes(raw)
    with pytest.raises(RuntimeError) as oe:
        _oracle(raw)
    with pytest.raises(CbxError) as ge:
        _frame(raw)
    want = int(re.search(r"offset (\d+)", str(oe.value)).group(1))
    assert f"at {want}." in str(ge.value), (str(ge.value), want)


LENFIELD_COPYBOOK = """
       01  REC.
           05  HDR         PIC X(2).
           05  REC-LEN     PIC 9(3).
           05  KIND        PIC X(1).
           05  BODY        PIC X(40).
"""


def _lenfield_file(rng, n, bad_at=None):
    out = bytearray()
    for i in range(n):
        body_len = int(rng.integers(0, 40))
        total = 6 + body_len
        ln = f"{total:03d}" if i != bad_at else "x1y"
        out += b"\x40\x40" + ln.encode("cp037") + ("C" if i % 3 else "P").encode("cp037")
        out += bytes(rng.integers(0xC1, 0xCA, body_len, dtype=np.uint8))
    return bytes(out)


@pytest.mark.parametrize("chunk", [None, "64"])
@pytest.mark.parametrize("start,end,adj", [(0, 0, 0), (3, 0, 3), (0, 2, -2), (2, 1, 1)])
def test_record_length_field_framing_vs_oracle(start, end, adj, chunk, monkeypatch):
    """record_length_field (VRLRecordReader.fetchRecordUsingRecordLengthField) on the GPU: records
    whose DISPLAY length field gives the record size (+ rdw_adjustment), record_start/end_offset
    bytes around each record, a truncated last record -- framing and rows equal the oracle's, at the
    default chunking and with 64-byte chunks (cbx_chain.h: every record chain crosses chunks)."""
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    if chunk is not None:
        monkeypatch.setenv("CBX_CHAIN_CHUNK", chunk)
    rng = np.random.default_rng(start * 7 + end)
    recs = []
    for i in range(3000):
        body_len = int(rng.integers(0, 40))
        total = 6 + body_len
        head = bytes(rng.integers(0, 256, start, dtype=np.uint8))
        rec = b"\x40\x40" + f"{total - adj:03d}".encode("cp037") + ("C" if i % 3 else "P").encode("cp037")
        rec += bytes(rng.integers(0xC1, 0xCA, body_len, dtype=np.uint8)) + bytes(rng.integers(0, 256, end, dtype=np.uint8))
        recs.append(head + rec)
    raw = b"".join(recs)[:-5]     # the last record is cut short
    p, var_len = parse_options({"record_length_field": "REC-LEN", "rdw_adjustment": str(adj), "record_start_offset": str(start),
                                "record_end_offset": str(end), "segment_field": "KIND", "generate_record_id": "true"})
    assert var_len
    rd = VarLenNestedReader(LENFIELD_COPYBOOK, p)
    t = rd._device_file(raw)
    off, ln, _ = rd.frame_file(t, len(raw))
    lens = [len(r) for r in recs]
    lens[-1] -= 5
    assert ln.cpu().tolist() == lens
    assert off.cpu().tolist() == [sum(lens[:i]) for i in range(len(lens))]
    rows = rd.read(raw).to_rows()
    exp = RO.var_len_rows(rd.copybook, raw, p)
    assert len(rows) == len(exp) == 3000
    assert rows == exp
    # decode() (frame + decode as one entry, no selection stage) frames by the length field too
    rows_d = rd.decode(raw).to_rows()
    assert rows_d == exp


def test_record_length_field_errors():
    """A length field that does not decode (non-digits) fails like the reference's
    IllegalStateException; a non-integral length field is rejected when the reader frames."""
    from cobrix_amd import native as N
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    rng = np.random.default_rng(3)
    raw = _lenfield_file(rng, 50, bad_at=20)
    p, _ = parse_options({"record_length_field": "REC-LEN"})
    rd = VarLenNestedReader(LENFIELD_COPYBOOK, p)
    with pytest.raises(N.CbxError) as e:
        rd.read(raw)
    assert e.value.code == N.CBX_E_STATE
    # the reference's message names the field (VRLRecordReader.scala:131-134)
    assert "Record length value of the field REC-LEN must be an integral type." in str(e.value)
    with pytest.raises(RuntimeError):
        RO.var_len_rows(rd.copybook, raw, p)
    p2, _ = parse_options({"record_length_field": "KIND"})
    rd2 = VarLenNestedReader(LENFIELD_COPYBOOK, p2)
    with pytest.raises(ValueError):
        rd2.read(_lenfield_file(rng, 5))


LENFIELD_BIN_COPYBOOK = """
       01  REC.
           05  REC-LEN     PIC 9(4) COMP.
           05  BODY        PIC X(400).
"""


def _lenfield_bin_file(rng, n, lo=2, hi=400, digits=False):
    """n records of a 2-byte big-endian COMP length (the whole record's) + body.  digits: bodies of
    cp037 digits and record-like bytes (every position a plausible-looking start); else random bytes."""
    out, offs = bytearray(), []
    for _ in range(n):
        total = int(rng.integers(lo, hi + 1))
        offs.append(len(out))
        out += total.to_bytes(2, "big")
        if digits:
            body = rng.integers(0, 3, total - 2, dtype=np.uint8)   # 0x00 0x01 0x02: lengths of 1, 2 or 258+ bytes
        else:
            body = rng.integers(0, 256, total - 2, dtype=np.uint8)
        out += bytes(body)
    return bytes(out), offs


@pytest.mark.parametrize("chunk", ["32", "96", "1024", None])
@pytest.mark.parametrize("kind", ["display", "binary", "adversarial"])
def test_record_length_field_chunked_framing(kind, chunk, monkeypatch):
    """The chunk-parallel length-field framing (cbx_chain.h: speculated chunk entries, fix rounds that
    stop where the true chain meets the speculated one, the settle pass) gives the sequential walk's
    records for chunks from 32 bytes (chains crossing thousands of chunks) to the default, on streams
    whose bodies look like record starts everywhere ("adversarial": 2-byte lengths of 0..2, so every
    speculation walks a wrong chain) -- offsets / lengths equal the generator's."""
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    if chunk is not None:
        monkeypatch.setenv("CBX_CHAIN_CHUNK", chunk)
    rng = np.random.default_rng({"display": 5, "binary": 6, "adversarial": 7}[kind])
    if kind == "display":
        raw = _lenfield_file(rng, 20_000)
        p, _ = parse_options({"record_length_field": "REC-LEN"})
        rd = VarLenNestedReader(LENFIELD_COPYBOOK, p)
        off = [0]
        for _ in range(20_000 - 1):
            off.append(off[-1] + int(raw[off[-1] + 2:off[-1] + 5].decode("cp037")))
    else:
        raw, off = _lenfield_bin_file(rng, 20_000, digits=kind == "adversarial")
        p, _ = parse_options({"record_length_field": "REC-LEN", "rdw_adjustment": "0"})
        rd = VarLenNestedReader(LENFIELD_BIN_COPYBOOK, p)
    t = rd._device_file(raw)
    o, ln, _ = rd.frame_file(t, len(raw))
    assert o.cpu().tolist() == off
    assert ln.cpu().tolist() == [b - a for a, b in zip(off, off[1:] + [len(raw)])]


@pytest.mark.parametrize("chunk", ["32", None])
def test_record_length_field_chunked_error_position(chunk, monkeypatch):
    """With chunks of 32 bytes the first undecodable length ON the record chain fails the framing,
    as the reference's walk does; undecodable bytes the speculated chains meet elsewhere do not."""
    from cobrix_amd import native as N
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    if chunk is not None:
        monkeypatch.setenv("CBX_CHAIN_CHUNK", chunk)
    rng = np.random.default_rng(11)
    raw = _lenfield_file(rng, 2000, bad_at=1500)
    p, _ = parse_options({"record_length_field": "REC-LEN"})
    rd = VarLenNestedReader(LENFIELD_COPYBOOK, p)
    with pytest.raises(N.CbxError) as e:
        rd.read(raw)
    assert e.value.code == N.CBX_E_STATE
    good = _lenfield_file(np.random.default_rng(11), 2000)
    rows = rd.read(good).to_rows()
    assert rows == RO.var_len_rows(rd.copybook, good, p)


def _frame_async(raw: bytes, seeds=None, cap=None, max_rounds=0):
    """cbx_frame_rdw_async + cbx_frame_rdw_state -> (offsets, lengths, state) or CbxError."""
    import ctypes
    from cobrix_amd import native as N
    rd = VarLenNestedReader(RDW_NARROW_COPYBOOK, ReaderParameters(is_record_sequence=True))
    t = torch.frombuffer(bytearray(raw) if raw else bytearray(16), dtype=torch.uint8).cuda()
    cap = cap if cap is not None else len(raw) // 4 + 2
    off = torch.empty(max(1, cap), dtype=torch.int64, device="cuda")
    ln = torch.empty(max(1, cap), dtype=torch.int32, device="cuda")
    state = torch.full((3,), -7, dtype=torch.int64, device="cuda")
    sd = seeds or [0]
    arr = (ctypes.c_int64 * len(sd))(*sd)
    prm = rd.rdw_params()
    st = torch.cuda.current_stream().cuda_stream
    L = N.load()
    N.check(L.cbx_frame_rdw_async(t.data_ptr(), len(raw), arr, len(sd), ctypes.byref(prm), off.data_ptr(),
                                  ln.data_ptr(), cap, state.data_ptr(), max_rounds, ctypes.c_void_p(st)))
    n = ctypes.c_int64(-1)
    rc = L.cbx_frame_rdw_state(state.data_ptr(), ctypes.byref(n), ctypes.c_void_p(st))
    s = state.cpu().tolist()
    N.check(rc)
    return off[: n.value].cpu().numpy(), ln[: n.value].cpu().numpy(), s


@pytest.mark.parametrize("chunk", [37, 4096, None])
def test_async_framing_equals_sync(monkeypatch, chunk):
    """cbx_frame_rdw_async (no host wait; count and errors left on the device) frames exactly what
    cbx_frame_rdw does, seeded or not; its state row is (count, -1, 0)."""
    if chunk:
        monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", str(chunk))
    d, _ = rdw_narrow(20_000, seed=11)
    raw = d.numpy().tobytes()
    eo, el = _oracle(raw)
    seeds = [e[0] for e in O.sparse_index(raw, records_per_entry=997)]
    for sd in (None, seeds):
        off, ln, s = _frame_async(raw, seeds=sd)
        assert np.array_equal(off, eo) and np.array_equal(ln, el)
        assert s == [len(eo), -1, 0]
    off, ln, s = _frame_async(_adversarial(600, seed=5))
    eo2, el2 = _oracle(_adversarial(600, seed=5))
    assert np.array_equal(off, eo2) and np.array_equal(ln, el2)


def test_async_framing_reports_errors_on_the_device(monkeypatch):
    """A zero-length header and a capacity below the record count surface from cbx_frame_rdw_state
    with the codes cbx_frame_rdw returns; fix rounds cut short are settled on the device."""
    from cobrix_amd import native as N
    d, hdr = rdw_narrow(400, seed=9)
    raw = bytearray(d.numpy().tobytes())
    h = int(hdr[123])
    raw[h:h + 4] = bytes(4)
    with pytest.raises(CbxError) as e:
        _frame_async(bytes(raw))
    with pytest.raises(CbxError) as e_sync:
        _frame(bytes(raw))
    assert e.value.code == N.CBX_E_STATE and str(e.value) == str(e_sync.value)
    with pytest.raises(CbxError) as e:
        _frame_async(d.numpy().tobytes(), cap=100)
    assert e.value.code == N.CBX_E_CAPACITY
    # 8-byte chunks over adversarial payloads, one parallel fix round: the device settle pass finishes
    # the chains of failed speculations it leaves
    monkeypatch.setenv("CBX_RDW_CHUNK_BYTES", "8")
    adv = _adversarial(300, seed=3)
    eo, el = _oracle(adv)
    for rounds in (1, 2, 0):
        off, ln, s = _frame_async(adv, max_rounds=rounds)
        assert np.array_equal(off, eo) and np.array_equal(ln, el) and s == [len(eo), -1, 0]


@pytest.mark.parametrize("subtract", [0, 1])
def test_index_chain_on_the_device_equals_whole_file_index(subtract):
    """shard.chain_step links run in sequence on the GPU (framing + cbx_sparse_index of each rank's
    tail + block, 64 kB entries at roots; resetting or subtracting the split size, the subtracting links
    starting from the residual the previous link hands on): the union of the runs' entries is the GPU
    index of the whole file, the runs tile it, and the record bases are the counts before each run."""
    import ctypes
    from cobrix_amd import native as N
    from cobrix_amd.shard import chain_step
    from cobrix_amd.synth import rdw_narrow_large
    blocks = [rdw_narrow_large(9000 + 2000 * b, seed=70 + b, device="cuda")[0] for b in range(4)]
    rd = VarLenNestedReader(RDW_NARROW_COPYBOOK, ReaderParameters(
        is_record_sequence=True, segment_field="SEGMENT-ID", segment_id_levels=["C"]))
    S = 64 * 1024

    def index_fn(region, start_bytes=0):
        n = int(region.numel())
        off, ln = rd.frame(region, n)
        prm = rd.index_params()
        prm.bytes_per_entry, prm.subtract_size, prm.start_bytes = S, subtract, start_bytes
        arr = (N.CbxIndexEntry * 4096)()
        ne = ctypes.c_int64(0)
        N.check(N.load().cbx_sparse_index(rd.native.handle, region.data_ptr(), n, off.data_ptr(), ln.data_ptr(),
                                          int(off.numel()), ctypes.byref(prm), arr, 4096, ctypes.byref(ne), None))
        return [(arr[k].offset_from, arr[k].record_index) for k in range(ne.value)], int(off.numel())

    whole = torch.cat(blocks)
    exp, n_all = index_fn(whole)
    got, runs, r_off, r_rec, r_res, tail = [], [], 0, 0, 0, None
    for b, blk in enumerate(blocks):
        region = blk if tail is None else torch.cat([tail, blk])
        res, fwd = chain_step(region, index_fn, r_off, r_rec, b == len(blocks) - 1, r_res, S if subtract else None)
        assert res["record_base"] == sum(r["n_records"] for r in runs)
        got += res["entries"]
        runs.append(res)
        if fwd is not None:
            r_off, r_rec, tail, r_res = fwd[0], fwd[1], fwd[2].clone(), fwd[3]
            # the residual is the whole file's bytesInChunk at that entry: its offset minus the cuts so far
            assert not subtract or r_res == r_off - len(got) * S
    assert len(exp) > 8 and got == exp
    assert torch.equal(torch.cat([r["run"] for r in runs]), whole)
    assert sum(r["n_records"] for r in runs) == n_all
