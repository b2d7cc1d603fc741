"""The record walk (cbx_walk.h: extractRecord with data-dependent offsets, one lane per record)
against the oracle: variable_size_occurs = true over RDW records and over VarOccursRecordExtractor
framing, DEPENDING ON inside an OCCURS, string dependees through occurs_mappings, short records.
The reference's own goldens for these layouts (test21, test25) run in test_gpu_golden.py."""
from __future__ import annotations

import random

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import reader_oracle as RO  # noqa: E402
from cobrix_amd.synth import WALK_NESTED_COPYBOOK as NESTED, _ebcdic, rdw_file  # noqa: E402
from cobrix_amd.synth import walk_nested_record as nested_record  # noqa: E402

MAPPED = """
       01  REC.
           05  ID          PIC 9(2).
           05  CODE        PIC X(2).
           05  ITEMS       OCCURS 0 TO 3 TIMES DEPENDING ON CODE.
               10  V       PIC X(3).
           05  AFTER       PIC 9(3).
"""


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


_JIT_MIN = -1


@pytest.fixture(autouse=True, params=["table", "jit"])
def _walk_kernel(request):
    """Every test runs on both walks: the table-driven walk_kernel and the copybook-specialised
    cbx_jit_walk (hipRTC), which a decode call uses from jit_min_records records on."""
    global _JIT_MIN
    _JIT_MIN = -1 if request.param == "table" else 1
    yield request.param


def _reader(copybook: str, options: dict, **params):
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    p, var_len = parse_options(options)
    assert var_len
    p = dataclasses.replace(p, **{"jit_min_records": _JIT_MIN, **params})
    return VarLenNestedReader(copybook, p), p


def _walk_kind(rd) -> int:
    import ctypes
    from cobrix_amd import native as N
    k = ctypes.c_int32()
    N.check(N.load().cbx_plan_kernel_kind(rd.native.handle, ctypes.byref(k)))
    return k.value


def _frame_kind(rd) -> int:
    """1: the last var-occurs framing ran its copybook-specialised step (jit_chain_source), 0: walk_length."""
    import ctypes
    from cobrix_amd import native as N
    k = ctypes.c_int32()
    N.check(N.load().cbx_plan_frame_kind(rd.native.handle, ctypes.byref(k)))
    return k.value


@pytest.mark.parametrize("utf8", [False, True])
@pytest.mark.parametrize("var_size", [True, False])
def test_walk_nested_odo_rdw_vs_oracle(var_size, utf8):
    """utf8: string_utf8 on the walk, which writes views -- its string columns handed out as Arrow Utf8
    (cbx_views_to_utf8), the same rows and a Utf8 ("u") Arrow export."""
    rnd = random.Random(5 + var_size)
    raw = rdw_file([nested_record(rnd, var_size) for _ in range(3000)])
    opts = {"is_record_sequence": "true", "variable_size_occurs": str(var_size).lower(), "generate_record_id": "true"}
    rd, p = _reader(NESTED, opts, **({"string_utf8": True} if utf8 else {}))
    assert rd.walk
    batch = rd.read(raw, file_id=1)
    if utf8:
        strs = [c for c in batch.cols if "offsets32" in c or "views" in c]
        assert strs and all("offsets32" in c for c in strs)
        from cobrix_amd.arrow_device import export_device
        _, _, nodes = export_device(batch)

        def fmts(ns):
            for n in ns:
                yield n.fmt
                yield from fmts(n.children)
        f = set(fmts(nodes))
        assert "u" in f and "vu" not in f, f
    rows = batch.to_rows()
    assert _walk_kind(rd) == (3 if _JIT_MIN > 0 else 2)
    exp = RO.var_len_rows(rd.copybook, raw, p, file_id=1)
    assert len(rows) == len(exp) == 3000
    bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
    assert not bad, (bad[:5], rows[bad[0]], exp[bad[0]])


@pytest.mark.parametrize("chunk", [None, "32", "128"])
def test_walk_var_occurs_extractor_vs_oracle(chunk, monkeypatch):
    """No RDW: VarOccursRecordExtractor framing on the GPU (chunk-parallel, cbx_chain.h: chunks of 32 /
    128 bytes make every record chain cross many speculated chunk entries), then the walk decode."""
    if chunk is not None:
        monkeypatch.setenv("CBX_CHAIN_CHUNK", chunk)
    rnd = random.Random(11)
    raw = b"".join(nested_record(rnd, True) for _ in range(400 if chunk is None else 3000))
    rd, p = _reader(NESTED, {"variable_size_occurs": "true"})
    rows = rd.read(raw).to_rows()
    assert _frame_kind(rd) == (1 if _JIT_MIN > 0 else 0)
    exp = RO.var_len_rows(rd.copybook, raw, p)
    assert len(rows) == len(exp) > 200
    bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
    assert not bad, (bad[:5], rows[bad[0]], exp[bad[0]])


@pytest.mark.parametrize("var_size,rdw", [(True, True), (False, True), (True, False)])
def test_walk_string_dependee_occurs_mappings(var_size, rdw, monkeypatch):
    """rdw False: the records back to back, framed by VarOccursRecordExtractor -- a string dependee
    through occurs_mappings decides each record's length (both framing steps; 64-byte chunks so the
    chains cross many speculated entries)."""
    if not rdw:
        monkeypatch.setenv("CBX_CHAIN_CHUNK", "64")
    rnd = random.Random(3)
    recs = []
    for i in range(2000):
        code = rnd.choice(["A ", "B ", "C ", "ZZ", "  "])
        n = {"A ": 0, "B ": 1, "C ": 3}.get(code, 3)
        body = f"{i % 100:02d}{code}" + "".join(rnd.choice(["abc", "XYZ", "   "]) for _ in range(n if var_size else 3)) + f"{i % 1000:03d}"
        recs.append(body.encode("cp037"))
    raw = rdw_file(recs) if rdw else b"".join(recs)
    opts = {"variable_size_occurs": str(var_size).lower(), "occurs_mappings": '{"ITEMS":{"A":0,"B":1,"C":3}}'}
    if rdw:
        opts["is_record_sequence"] = "true"
    rd, p = _reader(MAPPED, opts)
    assert rd.walk
    rows = rd.read(raw).to_rows()
    if not rdw:
        assert _frame_kind(rd) == (1 if _JIT_MIN > 0 else 0)
    exp = RO.var_len_rows(rd.copybook, raw, p)
    assert len(rows) == len(exp) == 2000
    assert rows == exp


@pytest.mark.parametrize("policy", ["hex", "raw"])
def test_debug_fields_vs_oracle(policy):
    """HEX / RAW debug fields (debug = true | raw, CopybookParser.addDebugFields) on the test1 layout."""
    import goldens as G
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters
    from oracle import oracle as O
    from parity import compare_batch
    cb_text = G.read("test1_copybook.cob").decode("latin-1")
    data = G.read("test1_data", "example.bin")
    # table-driven kernel only: test1's OCCURS slots doubled by the debug twins make a specialised
    # kernel that takes hipRTC minutes (the specialised path is exercised on debug fields by test17f)
    for jit in (-1,):
        rd = FixedLenNestedReader(cb_text, ReaderParameters(schema_policy="collapse_root", debug_fields_policy=policy,
                                                            jit_min_records=jit))
        b = rd.decode(data)
        errs = compare_batch(b, O.decode_fixed(rd.copybook, data))
        assert not errs, errs[:5]
        rows = b.to_rows()
        assert rows == RO.fixed_len_rows(rd.copybook, data, rd.params)


LONGSTR = """
       01  REC.
           05  N-OUT       PIC 9(1).
           05  OUTER       OCCURS 0 TO 3 TIMES DEPENDING ON N-OUT.
               10  NAME    PIC X(24).
           05  TAIL-TXT    PIC X(30).
"""


def test_walk_long_strings_multi_buffer(monkeypatch):
    """Long (> 12 byte) strings of the record walk land in Arrow data buffers of a power-of-two
    number of tiles, like the other view writers: with a 64 KiB buffer cap every slot region spans
    several buffers (view index = tile >> log2(tiles per buffer))."""
    monkeypatch.setenv("CBX_VIEW_BUFFER_BYTES", str(65536))
    rnd = random.Random(17)
    recs = []
    for _ in range(6000):
        n = rnd.choice([0, 1, 2, 3])
        b = bytes([0xF0 + n])
        for _ in range(n):
            b += _ebcdic("".join(rnd.choice("ABCDEFGHIJ KLMNOP") for _ in range(24)))
        b += _ebcdic(("TAIL" + "x" * rnd.randrange(26)).ljust(30))
        recs.append(b)
    raw = rdw_file(recs)
    opts = {"is_record_sequence": "true", "variable_size_occurs": "true"}
    rd, p = _reader(LONGSTR, opts)
    assert rd.walk
    batch = rd.read(raw)
    ci = next(i for i, c in enumerate(batch.cols) if "buffer_bytes" in c)
    assert batch.cols[ci]["capacity"] > 2 * batch.cols[ci]["buffer_bytes"]
    rows = batch.to_rows()
    exp = RO.var_len_rows(rd.copybook, raw, p)
    assert len(rows) == len(exp) == 6000
    bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
    assert not bad, (bad[:5], rows[bad[0]], exp[bad[0]])


SEGODO = """
       01  REC.
           05  SEG         PIC X(1).
           05  A-PART.
               10  NA      PIC 9(1).
               10  AITEMS  OCCURS 0 TO 4 TIMES DEPENDING ON NA.
                   15  AV  PIC S9(3) COMP-3.
           05  B-PART REDEFINES A-PART.
               10  NB      PIC 9(1).
               10  BITEMS  OCCURS 0 TO 2 TIMES DEPENDING ON NB.
                   15  BV  PIC X(4).
"""


def test_walk_segment_redefine_odo_to_arrow():
    """to_arrow of a record-walk batch whose OCCURS DEPENDING ON arrays sit inside segment
    redefines: the walk leaves the inactive redefine's count cells unwritten (invalid), which must
    give no list elements rather than garbage counts."""
    pytest.importorskip("pyarrow")
    rnd = random.Random(23)
    recs = []
    for _ in range(3000):
        if rnd.random() < 0.5:
            n = rnd.randrange(5)
            b = _ebcdic("A") + bytes([0xF0 + n]) + b"".join(bytes([rnd.randrange(10) << 4 | rnd.randrange(10),
                                                                  rnd.randrange(10) << 4 | 0x0C]) for _ in range(n))
        else:
            n = rnd.randrange(3)
            b = _ebcdic("B") + bytes([0xF0 + n]) + b"".join(_ebcdic(rnd.choice(["ab  ", "WXYZ", "    "])) for _ in range(n))
        recs.append(b)
    raw = rdw_file(recs)
    opts = {"is_record_sequence": "true", "variable_size_occurs": "true", "segment_field": "SEG",
            "redefine_segment_id_map:0": "A-PART => A", "redefine_segment_id_map:1": "B-PART => B"}
    rd, p = _reader(SEGODO, opts)
    assert rd.walk
    batch = rd.read(raw)
    # count cells the walk does not write hold whatever the allocator left: make that visible
    for ar in batch.plan.arrays:
        c = batch.cols[ar.count_column]
        if ar.segment >= 0:
            vb = c["validity"].cpu().numpy().view("uint8")
            import numpy as np
            bits = np.unpackbits(vb, bitorder="little")[: batch.n_rec].astype(bool)
            c["values"][: batch.n_rec][torch.from_numpy(~bits).to(c["values"].device)] = 1_000_000
    table = batch.to_arrow()
    table.validate(full=True)
    rows = batch.to_rows()
    from test_gpu_golden import _norm
    assert _norm(table.to_pylist()) == _norm(rows)
    assert rows == RO.var_len_rows(rd.copybook, raw, p)


ELEMDEP = """
       01  REC.
           05  CNT         PIC 9(1) OCCURS 2 TIMES.
           05  ITEMS       OCCURS 0 TO 3 TIMES DEPENDING ON CNT.
               10  V       PIC X(2).
           05  AFTER       PIC 9(2).
"""


@pytest.mark.parametrize("var_size", [True, False])
def test_walk_primitive_array_element_is_no_dependee(var_size):
    """A DEPENDING ON name that is an element of a primitive OCCURS: extractArray decodes those
    elements with decodeTypeValue and never records them in dependFields (RecordExtractors.scala:96-107),
    so the array keeps its maximum size."""
    rnd = random.Random(31)
    recs = []
    for i in range(500):
        body = f"{rnd.randrange(4)}{rnd.randrange(4)}" + "".join(rnd.choice(["ab", "XY", "  "]) for _ in range(3)) + f"{i % 100:02d}"
        recs.append(body.encode("cp037"))
    raw = rdw_file(recs)
    rd, p = _reader(ELEMDEP, {"is_record_sequence": "true", "variable_size_occurs": str(var_size).lower()})
    assert rd.walk
    rows = rd.read(raw).to_rows()
    exp = RO.var_len_rows(rd.copybook, raw, p)
    assert rows == exp
