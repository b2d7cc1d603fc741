"""The reference's integration specs (tests/golden_cases.py) on the CPU: the oracle against every
golden row file, and the host front-end (copybook layout, Spark schema) against the layout and
schema goldens.  These pin the checker before it is trusted with the GPU path, and pin the
front-end the oracle and the GPU share (a layout error there would be common-mode)."""
from __future__ import annotations

import json

import pytest

import goldens as G
import golden_cases as GC

from cobrix_amd.copybook import parse_copybook
from cobrix_amd.reader import parse_copybook_for, reader_schema
from cobrix_amd.schema import schema_json
from oracle import reader_oracle as RO


@pytest.mark.parametrize("name", sorted(GC.LAYOUTS))
def test_layout_golden(name):
    cb_file, kw, expected = GC.LAYOUTS[name]
    cb = parse_copybook(G.read(cb_file).decode("latin-1"), **kw)
    assert cb.generate_record_layout_positions() == G.read(*expected.split("/")).decode("latin-1")


SCHEMA_CASES = sorted(k for k, c in GC.CASES.items() if c.get("schema"))


@pytest.mark.parametrize("name", SCHEMA_CASES)
def test_schema_golden(name):
    case = GC.CASES[name]
    p, var_len = GC.params(case)
    cb = parse_copybook_for(GC.copybook_text(case), p)
    got = schema_json(reader_schema(cb, p, var_len))
    exp = json.loads(G.read(*case["schema"].split("/")).decode("latin-1"))
    assert got == exp


def oracle_rows(case):
    p, var_len = GC.params(case)
    cb = parse_copybook_for(GC.copybook_text(case), p)
    data = GC.data_bytes(case)
    if var_len:
        return RO.var_len_rows(cb, data, p)
    return RO.fixed_len_rows(cb, data, p)


@pytest.mark.parametrize("name", sorted(GC.CASES))
def test_oracle_golden_rows(name):
    case = GC.CASES[name]
    errs = GC.compare(case, oracle_rows(case))
    assert not errs, errs[:10]


def test_sparse_index_known_answer_python_restatement():
    """Test5MultisegmentSpec.scala:205-218 through the Python IndexGenerator restatement: 10 records
    per entry, cut at root 'C' -> 88 entries; the C restatement agrees entry for entry."""
    from cobrix_amd.options import parse_options
    from oracle import oracle as O
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    p, _ = parse_options({"is_record_sequence": "true", "segment_field": "SEGMENT_ID", "segment_id_root": "C",
                          "input_split_records": "10"})
    cb = parse_copybook_for(G.read("test5_copybook.cob").decode("latin-1"), p)
    idx = RO.sparse_index(cb, raw, p)
    assert len(idx) == 88
    off, _ = O.frame_rdw(raw)
    is_root = [1 if G.java_trim(raw[o:o + 5].decode("cp037")) == "C" else 0 for o in off]
    c_idx = O.sparse_index(raw, records_per_entry=10, is_root=is_root)
    assert [(e.offset_from, e.offset_to, e.record_index) for e in idx] == c_idx


@pytest.mark.parametrize("name,records", [
    ("test21", [b"0", b"10", b"12AB", b"21A2BC", b"21A1B"]),   # Test21VariableOccurs.scala:38-60
    ("test25", [b"1AX", b"2BXYZ"]),                            # Test25OccursMappings.scala:52-79
])
def test_var_occurs_record_extractor_known_answer(name, records):
    """VarOccursRecordExtractor splits the stream into the records the reference's unit tests list."""
    case = GC.CASES[name]
    p, _ = GC.params(case)
    cb = parse_copybook_for(GC.copybook_text(case), p)
    assert RO.var_occurs_records(cb, GC.data_bytes(case)) == records
