"""List layout of OCCURS DEPENDING ON arrays (cobrix_hip.h CBX_F_LIST) on the host: which arrays
qualify and what the plan hands to the library.  The device side is covered by the -m gpu tests
(every golden case and the C5 layout decoded with occurs_lists)."""
from __future__ import annotations

from cobrix_amd import native as N
from cobrix_amd.copybook import parse_copybook
from cobrix_amd.plan import build_plan
from cobrix_amd.synth import WIDE_ODO_COPYBOOK, WIDE_ODO_SEGMENTS


def _plan(text, **kw):
    return build_plan(parse_copybook(text, segment_redefines=sorted(set(WIDE_ODO_SEGMENTS.values()))),
                      segment_field="SEGMENT-ID", segment_redefine_map=WIDE_ODO_SEGMENTS, **kw)


def test_c5_array_becomes_a_list():
    plan = _plan(WIDE_ODO_COPYBOOK, occurs_lists=True)
    ars = [a for a in plan.arrays if a.dependee >= 0]
    assert len(ars) == 1 and ars[0].offsets_column >= 0
    assert plan.columns[ars[0].offsets_column].kind == "list_offsets"
    members = [f for f in plan.fields if f.n_dims == 1]
    assert members and all(f.flags & N.F_LIST for f in members)
    assert all(plan.columns[f.column].list_mpad == 2048 for f in members)
    # without the option: slot rows, no flag, no offsets column
    plan0 = _plan(WIDE_ODO_COPYBOOK)
    assert all(a.offsets_column == -1 for a in plan0.arrays)
    assert not any(f.flags & N.F_LIST for f in plan0.fields)


def test_string_elements_and_nested_arrays_stay_slot_rows():
    text = """
        01  R.
            05  SEGMENT-ID        PIC X(5).
            05  N                 PIC 9(2).
            05  A OCCURS 0 TO 5 DEPENDING ON N.
               10  S              PIC X(3).
               10  V              PIC 9(3) COMP-3.
            05  M                 PIC 9(2).
            05  B OCCURS 0 TO 4 DEPENDING ON M.
               10  C OCCURS 2.
                  15  W           PIC 9(2) COMP.
    """
    plan = build_plan(parse_copybook(text), occurs_lists=True)
    assert all(a.offsets_column == -1 for a in plan.arrays)
