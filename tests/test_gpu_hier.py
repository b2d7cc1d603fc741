"""Hierarchical records (`segment-children`, VarLenHierarchicalIterator + extractHierarchicalRecord)
through the HIP path (cbx_hier_select / cbx_decode_selected / cbx_hier_list_offsets) against the
oracle's literal restatement (oracle/reader_oracle.py hier_rows), on synthetic streams that break
every rule of the tree walk: children before the first root, grandchildren whose parent is missing,
siblings interleaved with cousins, unknown segment ids, short records.  The reference's own
hierarchical goldens (test17c-f) run in test_gpu_golden.py.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import goldens as G  # noqa: E402

from oracle import reader_oracle as RO  # noqa: E402

OPTS = {"is_record_sequence": "true", "generate_record_id": "true", "schema_retention_policy": "collapse_root",
        "segment_field": "SEGMENT_ID",
        "redefine_segment_id_map:1": "COMPANY => 1", "redefine-segment-id-map:2": "DEPT => 2",
        "redefine-segment-id-map:3": "EMPLOYEE => 3", "redefine-segment-id-map:4": "OFFICE => 4",
        "redefine-segment-id-map:5": "CUSTOMER => 5", "redefine-segment-id-map:6": "CONTACT => 6",
        "redefine-segment-id-map:7": "CONTRACT => 7",
        "segment-children:1": "COMPANY => DEPT,CUSTOMER", "segment-children:2": "DEPT => EMPLOYEE,OFFICE",
        "segment-children:3": "CUSTOMER => CONTACT,CONTRACT"}

_EBCDIC_TEXT = bytes([0x40] * 4) + bytes(range(0xC1, 0xCA)) + bytes(range(0xD1, 0xDA)) + bytes(range(0xF0, 0xFA))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def hier_stream(n: int, seed: int, tree_like: float = 0.8) -> bytes:
    """n RDW records of the test17 layout: mostly tree-ordered segments (company, departments with
    employees / offices, customers with contacts / contracts), with a share of random ids (0-9,
    incl. ids no redefine maps) and lengths from 1 byte to the full record."""
    rnd = random.Random(seed)
    seq = []
    while len(seq) < n:
        if rnd.random() < tree_like:
            seq.append(1)
            for _ in range(rnd.randint(0, 3)):
                if rnd.random() < 0.5:
                    seq.append(2)
                    seq += [rnd.choice((3, 4)) for _ in range(rnd.randint(0, 4))]
                else:
                    seq.append(5)
                    seq += [rnd.choice((6, 7)) for _ in range(rnd.randint(0, 4))]
        else:
            seq += [rnd.randint(0, 9) for _ in range(rnd.randint(1, 6))]
    out = bytearray()
    for sid in seq[:n]:
        ln = 108 if rnd.random() < 0.8 else rnd.randint(1, 108)
        body = bytes([0xF0 + sid]) + bytes(rnd.choice(_EBCDIC_TEXT) if rnd.random() < 0.9 else rnd.randrange(256)
                                            for _ in range(ln - 1))
        out += bytes([0, 0, ln & 0xFF, ln >> 8]) + body[:ln]
    return bytes(out)


def _reader(extra=None, **params):
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    p, var_len = parse_options({**OPTS, **(extra or {})})
    assert var_len
    p = dataclasses.replace(p, **params)
    return VarLenNestedReader(G.read("test17_hierarchical.cob").decode("latin-1"), p), p


@pytest.mark.parametrize("seed,n,tree_like", [(1, 200, 1.0), (2, 3000, 0.8), (3, 3000, 0.3), (4, 20000, 0.9)])
@pytest.mark.parametrize("views", [False, True])
def test_hier_synthetic_vs_oracle(seed, n, tree_like, views):
    raw = hier_stream(n, seed, tree_like)
    for jit in (-1, 1):
        rd, p = _reader(string_views=views, jit_min_records=jit)
        rows = rd.read(raw, file_id=4).to_rows()
        exp = RO.var_len_rows(rd.copybook, raw, p, file_id=4)
        assert len(rows) == len(exp)
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


def test_hier_entries_cut_at_roots():
    """With input_split_records the reference reads each index entry (cut at root records) with its
    own iterator; the GPU reads the stream once -- same rows, same Record_Ids."""
    raw = hier_stream(5000, 7, 0.7)
    rd, p = _reader({"input_split_records": "37"})
    t = rd._device_file(raw)
    off, ln, _ = rd.frame_file(t, len(raw))
    ents = rd.generate_index(t, len(raw), off, ln)
    exp_ents = RO.sparse_index(rd.copybook, raw, p)
    assert [(e.offset_from, e.offset_to, e.record_index) for e in ents] == \
        [(e.offset_from, e.offset_to, e.record_index) for e in exp_ents]
    assert len(ents) > 10
    rows = rd.read(raw).to_rows()
    assert rows == RO.var_len_rows(rd.copybook, raw, p)


def test_hier_arrow_matches_rows():
    pytest.importorskip("pyarrow")
    raw = hier_stream(3000, 9, 0.8)
    rd, _ = _reader(string_views=True)
    batch = rd.read(raw)
    table = batch.to_arrow()
    table.validate(full=True)
    assert table.num_rows == len(batch.to_rows())
    from test_gpu_golden import _norm
    assert _norm(table.to_pylist()) == _norm(batch.to_rows())


def test_hier_empty_and_rootless():
    rd, p = _reader()
    assert rd.read(b"").to_rows() == []
    recs = bytearray()   # no root record: every record is dropped
    for sid in (2, 3, 5, 6, 9, 0):
        recs += bytes([0, 0, 10, 0]) + bytes([0xF0 + sid]) + b"\x40" * 9
    assert rd.read(bytes(recs)).to_rows() == RO.var_len_rows(rd.copybook, bytes(recs), p) == []


MULTI_IDS = {"redefine_segment_id_map:1": "COMPANY => 1,0", "redefine-segment-id-map:2": "DEPT => 2,8",
             "redefine-segment-id-map:5": "CUSTOMER => 5,9"}


def _multi_id_stream(n: int, seed: int, tree_like: float) -> bytes:
    """hier_stream with the parent segments' records under either of their two ids (company 1 / 0,
    department 2 / 8, customer 5 / 9), so a department under id 8 does not end the children of one
    under id 2 (extractChildren's break compares ids): records then sit under several parents."""
    rnd = random.Random(seed + 1000)
    swap = {1: 0, 2: 8, 5: 9}
    raw = bytearray(hier_stream(n, seed, tree_like))
    i = 0
    while i < len(raw):
        ln = raw[i + 2] | (raw[i + 3] << 8)
        sid = raw[i + 4] - 0xF0 if ln else -1
        if sid in swap and rnd.random() < 0.5:
            raw[i + 4] = 0xF0 + swap[sid]
        i += 4 + ln
    return bytes(raw)


@pytest.mark.parametrize("seed,n,tree_like", [(11, 300, 1.0), (12, 4000, 0.8), (13, 4000, 0.3)])
@pytest.mark.parametrize("views", [False, True])
def test_hier_multi_id_parents_vs_oracle(seed, n, tree_like, views):
    """Parent segments mapped from several segment ids (CobolParametersParser.scala:389-404 splits the
    comma list): the general walk (cbx_hier_params.flags) breaks a parent's children only at its own
    id or an ancestor's (RecordExtractors.scala:306-316), so a child record can appear under several
    parents -- rows equal the oracle's literal walk, with more rows than records."""
    raw = _multi_id_stream(n, seed, tree_like)
    for jit in (-1, 1):
        rd, p = _reader(MULTI_IDS, string_views=views, jit_min_records=jit)
        rows = rd.read(raw, file_id=2).to_rows()
        exp = RO.var_len_rows(rd.copybook, raw, p, file_id=2)
        assert len(rows) == len(exp)
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


@pytest.mark.parametrize("start", [3, 8])
def test_hier_record_start_offset_vs_oracle(start):
    """record_start_offset on hierarchical records: the root record is decoded from the start offset
    (VarLenHierarchicalIterator.scala:139-144 -> RecordExtractors.scala:379-381), each child segment at
    its group's offset in its own data, without it (extractChildren, RecordExtractors.scala:308-310).
    Every record carries `start` leading bytes; segment ids are read after them (VRLRecordReader)."""
    rnd = np.random.default_rng(start)
    raw = hier_stream(4000, 11 + start, 0.8)
    out, pos = bytearray(), 0
    while pos < len(raw):   # insert the leading bytes into every RDW record
        ln = raw[pos + 2] | raw[pos + 3] << 8
        body = bytes(rnd.integers(0, 256, start, dtype=np.uint8)) + raw[pos + 4:pos + 4 + ln]
        out += bytes([0, 0, len(body) & 0xFF, len(body) >> 8]) + body
        pos += 4 + ln
    for jit in (-1, 1):
        rd, p = _reader({"record_start_offset": str(start)}, jit_min_records=jit)
        rows = rd.read(bytes(out), file_id=2).to_rows()
        exp = RO.var_len_rows(rd.copybook, bytes(out), p, file_id=2)
        assert len(rows) == len(exp) > 100
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


def test_hier_record_id_is_next_root():
    """Record_Id of a hierarchical record = the index of the next root record (or the record count
    for the last one): VarLenHierarchicalIterator.scala:107-133."""
    recs = bytearray()
    for sid in (3, 1, 2, 3, 1, 5, 1):
        recs += bytes([0, 0, 20, 0]) + bytes([0xF0 + sid]) + b"\xC1" * 19
    rd, p = _reader()
    rows = rd.read(bytes(recs)).to_rows()
    assert [r["Record_Id"] for r in rows] == [4, 6, 7]
    assert rows == RO.var_len_rows(rd.copybook, bytes(recs), p)
    assert [len(r["COMPANY"]["DEPT"]) for r in rows] == [1, 0, 0]
    assert len(rows[0]["COMPANY"]["DEPT"][0]["EMPLOYEE"]) == 1


def _hier_odo_stream(n: int, seed: int, start: int = 0) -> bytes:
    """Records of tests/test_hier_oracle.py's layout: parents, children and grandchildren in tree
    order (with strays), count digits often invalid (null dependees), every length."""
    rnd = random.Random(seed)
    out = bytearray()
    digits = "0123456789X "
    while n > 0:
        kind = rnd.choice("PPCCCGGGZ")
        if kind == "P":
            body = "P" + rnd.choice(digits) + "NAME" + rnd.choice(digits) + "AB" * 5
        elif kind == "C":
            body = "C" + rnd.choice(digits) + "ABC" + rnd.choice(digits) + "aa" * 5 + "bb" * 5 + "hhhhh"
        elif kind == "G":
            body = "G" + rnd.choice(digits) + rnd.choice(digits) + "xyzuv"
        else:
            body = rnd.choice("QZ") + "9" * 10
        if rnd.random() < 0.15:
            body = body[:rnd.randint(1, len(body))]
        b = bytes(rnd.randrange(256) for _ in range(start)) + body.encode("cp037")
        out += bytes([0, 0, len(b) & 0xFF, len(b) >> 8]) + b
        n -= 1
    return bytes(out)


@pytest.mark.parametrize("start", [0, 3])
@pytest.mark.parametrize("views", [False, True])
def test_hier_shared_dependees_vs_oracle(start, views):
    """Arrays of child segments DEPENDING ON a field of the parent segment, of the common header
    (registered by the root only) and of their own segment when that field is null (the previous
    registration stays): the GPU resolves the counts the shared dependFields map gives
    (RecordExtractors.scala:224-245) and decodes the rows with them (cbx_plan_set_odo_counts); rows
    equal the oracle's ora_extract_hier walk."""
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from test_hier_oracle import HIER_ODO_COPYBOOK, HIER_ODO_OPTS
    raw = _hier_odo_stream(6000, 17 + start, start)
    for jit in (-1, 1):
        p, _ = parse_options({**HIER_ODO_OPTS, "generate_record_id": "true", "record_start_offset": str(start)})
        p = dataclasses.replace(p, string_views=views, jit_min_records=jit)
        rd = VarLenNestedReader(HIER_ODO_COPYBOOK, p)
        rows = rd.read(raw).to_rows()
        exp = RO.var_len_rows(rd.copybook, raw, p)
        assert len(rows) == len(exp) > 100
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


def _sibling_stream(n: int, seed: int) -> bytes:
    """Records of tests/test_hier_oracle.py's sibling layout in random order (B before A often), count
    digits sometimes invalid (null dependees), some records cut short."""
    rnd = random.Random(seed)
    out = bytearray()
    digits = "0123456789X"
    for _ in range(n):
        kind = rnd.choice("PAABBBZ")
        if kind == "P":
            body = "P" + rnd.choice(digits) + "ABC"
        elif kind == "A":
            body = "A" + rnd.choice(digits) + "yy" * 5
        elif kind == "B":
            body = "B" + rnd.choice(digits) + "x" * 5 + "p" * 5
        else:
            body = "Z" + "9" * 6
        if rnd.random() < 0.1:
            body = body[:rnd.randint(1, len(body))]
        b = body.encode("cp037")
        out += bytes([0, 0, len(b) & 0xFF, len(b) >> 8]) + b
    return bytes(out)


@pytest.mark.parametrize("views", [False, True])
def test_hier_sibling_dependees_vs_oracle(views):
    """An array of one child type DEPENDING ON a field of its sibling type, the siblings' records
    interleaved in the file: the counts follow the reference's walk (child types in copybook order,
    each instance's subtree after it), not the file order; rows equal the oracle's."""
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from test_hier_oracle import SIBLING_COPYBOOK, SIBLING_OPTS
    raw = _sibling_stream(5000, 23)
    for jit in (-1, 1):
        p, _ = parse_options({**SIBLING_OPTS, "generate_record_id": "true"})
        p = dataclasses.replace(p, string_views=views, jit_min_records=jit)
        rd = VarLenNestedReader(SIBLING_COPYBOOK, p)
        rows = rd.read(raw).to_rows()
        exp = RO.var_len_rows(rd.copybook, raw, p)
        assert len(rows) == len(exp) > 100
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


def _before_root_stream(n: int, seed: int) -> bytes:
    """Records of tests/test_hier_oracle.py's BEFORE_ROOT layout (a child segment's group placed before
    the root segment's) in random order, digits sometimes invalid (null dependees), some cut short."""
    rnd = random.Random(seed)
    out = bytearray()
    digits = "0123456789X"
    for _ in range(n):
        kind = rnd.choice("PAABBZ")
        if kind == "P":
            body = "P" + rnd.choice(digits) + "ABC" + "xyzwv"
        elif kind == "A":
            body = "A" + rnd.choice(digits) + "aa" * 5
        elif kind == "B":
            body = "B" + rnd.choice(digits) + "q" * 5
        else:
            body = "Z" + "9" * 6
        if rnd.random() < 0.1:
            body = body[:rnd.randint(1, len(body))]
        b = body.encode("cp037")
        out += bytes([0, 0, len(b) & 0xFF, len(b) >> 8]) + b
    return bytes(out)


@pytest.mark.parametrize("views", [False, True])
def test_hier_group_before_root_vs_oracle(views, monkeypatch):
    """A child segment's group placed before the root segment's in the copybook, its DEPENDING ON field
    used by the root's array and by a sibling's: the root's walk registers that field from the ROOT's
    bytes before the root's own group (RecordExtractors.scala:365-372) -- a layout round 5 reported as
    unsupported.  Counts resolved before the one decode (cbx_hier_dependee_values +
    cbx_hier_dependee_counts); rows equal the oracle's ora_extract_hier walk."""
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from test_hier_oracle import BEFORE_ROOT_COPYBOOK, BEFORE_ROOT_OPTS
    raw = _before_root_stream(6000, 29)
    calls = []
    orig = VarLenNestedReader.decode_selected
    monkeypatch.setattr(VarLenNestedReader, "decode_selected", lambda self, *a, **k: calls.append(1) or orig(self, *a, **k))
    for jit in (-1, 1):
        p, _ = parse_options({**BEFORE_ROOT_OPTS, "generate_record_id": "true"})
        p = dataclasses.replace(p, string_views=views, jit_min_records=jit)
        rd = VarLenNestedReader(BEFORE_ROOT_COPYBOOK, p)
        calls.clear()
        rows = rd.read(raw).to_rows()
        assert len(calls) == 1   # one decode of the rows
        exp = RO.var_len_rows(rd.copybook, raw, p)
        assert len(rows) == len(exp) > 100
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])


def test_hier_child_within_record_start_offset():
    """A child row whose bytes start within record_start_offset of the data (rows handed to
    read_hierarchical in record order, the child's bytes stored first): the child is decoded at its
    group's offset in its own data (RecordExtractors.scala:308-310) from a copy with the start offset in
    front -- round 5 reported this as unsupported.  Rows equal the oracle's on the RDW stream of the
    same records in record order."""
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from test_hier_oracle import HIER_ODO_COPYBOOK, HIER_ODO_OPTS
    s0 = 6
    root = b"\x11" * s0 + "P3NAME2AABBCCDDEE".encode("cp037")
    kid = b"\x22" * s0 + ("C9ABC1" + "aa" * 5 + "bb" * 5 + "hhhhh").encode("cp037")
    p, _ = parse_options({**HIER_ODO_OPTS, "record_start_offset": str(s0)})
    p = dataclasses.replace(p, jit_min_records=-1)
    rd = VarLenNestedReader(HIER_ODO_COPYBOOK, p)
    data = kid + root
    d = torch.tensor(list(data), dtype=torch.uint8, device="cuda")
    off = torch.tensor([len(kid), 0], dtype=torch.int64, device="cuda")
    ln = torch.tensor([len(root), len(kid)], dtype=torch.int32, device="cuda")
    rows = rd.read_hierarchical(d, len(data), off, ln).to_rows()
    stream = b"".join(bytes([0, 0, len(r) & 0xFF, len(r) >> 8]) + r for r in (root, kid))
    exp = RO.var_len_rows(rd.copybook, stream, p)
    for r in exp:
        r.pop("Record_Id", None), r.pop("File_Id", None)
    for r in rows:
        r.pop("Record_Id", None), r.pop("File_Id", None)
    assert rows == exp and len(rows) == 1 and len(rows[0]["REC"]["PARENT_SEG"]["CHILD_SEG"]) == 1


def _strdep_stream(n: int, seed: int) -> bytes:
    """Records of tests/test_hier_oracle.py's STRDEP layout: parents with a code A / B / C (listed by
    occurs_mappings) or another letter, children with their own code and up to three items, strays
    and records cut short."""
    rnd = random.Random(seed)
    out = bytearray()
    for _ in range(n):
        kind = rnd.choice("PCCCZ")
        if kind == "P":
            body = "P" + "NAME" + rnd.choice("ABCXB")
        elif kind == "C":
            body = "C" + "ABC" + rnd.choice("ABCQ") + "".join(rnd.choice(["aa", "bb", "cc"]) for _ in range(3))
        else:
            body = "Z" + "9" * 6
        if rnd.random() < 0.1:
            body = body[:rnd.randint(1, len(body))]
        b = body.encode("cp037")
        out += bytes([0, 0, len(b) & 0xFF, len(b) >> 8]) + b
    return bytes(out)


@pytest.mark.parametrize("dep", ["P-CODE", "C-CODE"])
@pytest.mark.parametrize("var_size", [False, True])
def test_hier_walk_cross_segment_dependee_vs_oracle(dep, var_size):
    """Record-walk plans (a string DEPENDING ON through occurs_mappings; variable_size_occurs) whose
    child array depends on its PARENT's field: each row's walk starts from the dependee map the
    hierarchical walk left before it (cbx_hier_dependee_values decodes the registrations, the resolver
    emits per-row seeds, cbx_plan_set_dep_seed hands them to the walk), and a child registers no common
    field -- round 5 reported these layouts as unsupported.  The own-segment dependee (C-CODE) is
    seeded too: a child whose own code is null (cut short) counts with the code an earlier child
    registered.  Rows equal the oracle's ora_extract_hier walk, both walks (table / specialised)."""
    import dataclasses
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    from test_hier_oracle import STRDEP_COPYBOOK, STRDEP_OPTS
    raw = _strdep_stream(5000, 31 + var_size)
    for jit in (-1, 1):
        opts = {**STRDEP_OPTS, "generate_record_id": "true", "variable_size_occurs": str(var_size).lower()}
        p, _ = parse_options(opts)
        p = dataclasses.replace(p, jit_min_records=jit)
        rd = VarLenNestedReader(STRDEP_COPYBOOK.format(dep=dep), p)
        assert rd.walk and rd.walk_seeds
        rows = rd.read(raw).to_rows()
        exp = RO.var_len_rows(rd.copybook, raw, p)
        assert len(rows) == len(exp) > 100
        bad = [i for i, (a, b) in enumerate(zip(rows, exp)) if a != b]
        assert not bad, (jit, bad[:5], rows[bad[0]], exp[bad[0]])
