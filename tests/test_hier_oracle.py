"""The oracle's restatement of extractHierarchicalRecord (oracle/cobrix_oracle.c ora_extract_hier) on
known answers read off the reference's code: ONE dependFields map shared by the segments of a
hierarchical record (RecordExtractors.scala:224-245), registrations in the walk's order -- the root
record's groups, then each segment's children (extractChildren, :300-322) -- and child segments
decoded at their group's offset without record_start_offset (:308-310).  CPU only."""
from __future__ import annotations

import pytest

from cobrix_amd.options import parse_options
from cobrix_amd.reader import parse_copybook_for
from oracle import reader_oracle as RO

HIER_ODO_COPYBOOK = """
       01  REC.
           05  SEGMENT-ID        PIC X(1).
           05  HDR-N             PIC 9(1).
           05  PARENT-SEG.
               10  P-NAME        PIC X(4).
               10  P-CNT         PIC 9(1).
               10  P-ITEMS OCCURS 0 TO 5 TIMES DEPENDING ON P-CNT.
                   15  P-V       PIC X(2).
           05  CHILD-SEG REDEFINES PARENT-SEG.
               10  C-NAME        PIC X(3).
               10  C-CNT         PIC 9(1).
               10  C-A OCCURS 0 TO 5 TIMES DEPENDING ON P-CNT.
                   15  C-AV      PIC X(2).
               10  C-B OCCURS 0 TO 5 TIMES DEPENDING ON C-CNT.
                   15  C-BV      PIC X(2).
               10  C-H OCCURS 0 TO 5 TIMES DEPENDING ON HDR-N.
                   15  C-HV      PIC X(1).
           05  GCHILD-SEG REDEFINES PARENT-SEG.
               10  G-CNT         PIC 9(1).
               10  G-X OCCURS 0 TO 5 TIMES DEPENDING ON C-CNT.
                   15  G-XV      PIC X(1).
"""

HIER_ODO_OPTS = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID",
                 "redefine_segment_id_map:1": "PARENT-SEG => P", "redefine-segment-id-map:2": "CHILD-SEG => C",
                 "redefine-segment-id-map:3": "GCHILD-SEG => G",
                 "segment-children:1": "PARENT-SEG => CHILD-SEG", "segment-children:2": "CHILD-SEG => GCHILD-SEG"}


def rdw(text: str) -> bytes:
    b = text.encode("cp037")
    return bytes([0, 0, len(b) & 0xFF, len(b) >> 8]) + b


def _rows(data: bytes, **extra):
    p, _ = parse_options({**HIER_ODO_OPTS, **{k: str(v) for k, v in extra.items()}})
    return RO.var_len_rows(parse_copybook_for(HIER_ODO_COPYBOOK, p), data, p)


def test_shared_dependee_map_known_answer():
    data = (rdw("P3NAME2AABBCCDDEE") + rdw("C9ABCX" + "aa" * 5 + "bb" * 5 + "hhhhh") + rdw("G7xxxxx") +
            rdw("C9DEF3" + "aa" * 5 + "bb" * 5 + "hhhhh") + rdw("GXyyyyy") +
            rdw("P1ROOTX") + rdw("C8GHI4" + "cc" * 5 + "dd" * 5 + "iiiii"))
    rows = _rows(data)
    assert len(rows) == 2
    r0, r1 = rows[0]["REC"], rows[1]["REC"]
    c0, c1 = r0["PARENT_SEG"]["CHILD_SEG"]
    # C-A depends on P-CNT of the parent segment (2); C-H on the root's header HDR-N (3, not the
    # child's own '9': children do not decode the header)
    assert len(c0["C_A"]) == 2 and len(c0["C_H"]) == 3 and len(c1["C_H"]) == 3
    # C-CNT null in the first child: nothing registered yet -> max; the second child's own 3
    assert c0["C_CNT"] is None and len(c0["C_B"]) == 5 and len(c1["C_B"]) == 3
    # the grandchild's G-X depends on C-CNT: unregistered under the first child (max), 3 under the second
    assert len(c0["GCHILD_SEG"][0]["G_X"]) == 5 and len(c1["GCHILD_SEG"][0]["G_X"]) == 3
    # a new hierarchical record starts a new map: P-CNT null in the second root -> C-A at max, and
    # C-CNT registered by the previous record is forgotten (own 4 here); HDR-N = 1 from this root
    c2 = r1["PARENT_SEG"]["CHILD_SEG"][0]
    assert r1["PARENT_SEG"]["P_CNT"] is None and len(c2["C_A"]) == 5 and len(c2["C_B"]) == 4 and len(c2["C_H"]) == 1


def test_null_dependee_takes_the_previous_registration():
    """A null C-CNT in the second child: the first child's value stays in the shared map."""
    data = (rdw("P2NAME1AA") + rdw("C0ABC2" + "aa" * 5 + "bb" * 5 + "hhhhh") + rdw("C0DEFX" + "aa" * 5 + "bb" * 5 + "hhhhh")
            + rdw("GXqqqqq"))
    c0, c1 = _rows(data)[0]["REC"]["PARENT_SEG"]["CHILD_SEG"]
    assert len(c0["C_B"]) == 2 and c1["C_CNT"] is None and len(c1["C_B"]) == 2
    assert len(c1["GCHILD_SEG"][0]["G_X"]) == 2


def test_children_skip_record_start_offset():
    """The root from record_start_offset, a child at its group's offset in its own data."""
    data = rdw("##P3NAME2AABB") + rdw("##C9ABC1" + "aa" * 5 + "bb" * 5 + "hhhhh")
    r = _rows(data, record_start_offset=2)[0]["REC"]
    assert r["SEGMENT_ID"] == "P" and r["PARENT_SEG"]["P_NAME"] == "NAME"
    # the child group (offset 2) read from the child's byte 2 -- the start offset is not applied
    assert r["PARENT_SEG"]["CHILD_SEG"][0]["C_NAME"] == "C9A"


SIBLING_COPYBOOK = """
       01  REC.
           05  SEGMENT-ID        PIC X(1).
           05  PARENT-SEG.
               10  P-CNT         PIC 9(1).
               10  P-NAME        PIC X(3).
           05  SIB-A REDEFINES PARENT-SEG.
               10  A-CNT         PIC 9(1).
               10  A-ITEMS OCCURS 0 TO 5 TIMES DEPENDING ON P-CNT.
                   15  A-V       PIC X(2).
           05  SIB-B REDEFINES PARENT-SEG.
               10  B-CNT         PIC 9(1).
               10  B-ITEMS OCCURS 0 TO 5 TIMES DEPENDING ON A-CNT.
                   15  B-V       PIC X(1).
               10  B-P OCCURS 0 TO 5 TIMES DEPENDING ON P-CNT.
                   15  B-PV      PIC X(1).
"""

SIBLING_OPTS = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID",
                "redefine_segment_id_map:1": "PARENT-SEG => P", "redefine-segment-id-map:2": "SIB-A => A",
                "redefine-segment-id-map:3": "SIB-B => B", "segment-children:1": "PARENT-SEG => SIB-A,SIB-B"}


def test_sibling_dependees_follow_the_walk_not_the_file():
    """Sibling segment types under one parent, B's array DEPENDING ON A's field, the B record placed
    before the A record in the file: extractHierarchicalRecord walks the child types in copybook order
    (RecordExtractors.scala:364-370, getParentToChildrenMap), so A is decoded first and B's B-ITEMS
    sees A-CNT = 3 (by file order nothing would be registered yet: the maximum, 5)."""
    p, _ = parse_options(SIBLING_OPTS)
    data = rdw("P1ABC") + rdw("B2" + "x" * 10) + rdw("A3" + "yy" * 5)
    rows = RO.var_len_rows(parse_copybook_for(SIBLING_COPYBOOK, p), data, p)
    assert len(rows) == 1
    par = rows[0]["REC"]["PARENT_SEG"]
    (a,), (b,) = par["SIB_A"], par["SIB_B"]
    assert a["A_CNT"] == 3 and len(a["A_ITEMS"]) == 1
    assert b["B_CNT"] == 2 and len(b["B_ITEMS"]) == 3 and len(b["B_P"]) == 1


STRDEP_COPYBOOK = """
       01  REC.
           05  SEGMENT-ID        PIC X(1).
           05  PARENT-SEG.
               10  P-NAME        PIC X(4).
               10  P-CODE        PIC X(1).
           05  CHILD-SEG REDEFINES PARENT-SEG.
               10  C-NAME        PIC X(3).
               10  C-CODE        PIC X(1).
               10  C-A OCCURS 0 TO 3 TIMES DEPENDING ON {dep}.
                   15  C-AV      PIC X(2).
"""
STRDEP_OPTS = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID",
               "redefine_segment_id_map:1": "PARENT-SEG => P", "redefine-segment-id-map:2": "CHILD-SEG => C",
               "segment-children:1": "PARENT-SEG => CHILD-SEG", "occurs_mappings": '{"C_A":{"A":1,"B":2,"C":3}}'}


def test_cross_segment_string_dependee_seeds_the_walk():
    """A child's OCCURS DEPENDING ON a string field of its parent (occurs_mappings) needs the record walk,
    which decodes each row from its own bytes: the reader seeds each row's dependee map with the
    hierarchical walk's state before it (check_hierarchical -> walk_seeds, cbx_plan_set_dep_seed) -- the
    oracle's walk resolves the parent's "B" to 2 elements.  The same array DEPENDING ON its own segment's
    field is seeded as well (a null own code leaves the earlier registration in force)."""
    import cobrix_amd.reader as R
    p, _ = parse_options(STRDEP_OPTS)
    cb = parse_copybook_for(STRDEP_COPYBOOK.format(dep="P-CODE"), p)
    rows = RO.var_len_rows(cb, rdw("PNAMEB") + rdw("CABCZaabbcc"), p)
    assert len(rows[0]["REC"]["PARENT_SEG"]["CHILD_SEG"][0]["C_A"]) == 2
    orig = R.NativePlan
    R.NativePlan = lambda plan: None   # (the check runs before any device allocation)
    try:
        rd = R.VarLenNestedReader(STRDEP_COPYBOOK.format(dep="P-CODE"), p)
        assert rd.walk and rd.walk_seeds
        rd = R.VarLenNestedReader(STRDEP_COPYBOOK.format(dep="C-CODE"), p)
        assert rd.walk and rd.walk_seeds
    finally:
        R.NativePlan = orig


BEFORE_ROOT_COPYBOOK = """
       01  REC.
           05  SEGMENT-ID        PIC X(1).
           05  SIB-A.
               10  A-CNT         PIC 9(1).
               10  A-ITEMS OCCURS 0 TO 5 TIMES DEPENDING ON A-CNT.
                   15  A-V       PIC X(2).
           05  PARENT-SEG REDEFINES SIB-A.
               10  P-CNT         PIC 9(1).
               10  P-NAME        PIC X(3).
               10  P-ITEMS OCCURS 0 TO 5 TIMES DEPENDING ON A-CNT.
                   15  P-V       PIC X(1).
           05  SIB-B REDEFINES SIB-A.
               10  B-CNT         PIC 9(1).
               10  B-ITEMS OCCURS 0 TO 5 TIMES DEPENDING ON A-CNT.
                   15  B-V       PIC X(1).
"""

BEFORE_ROOT_OPTS = {"is_record_sequence": "true", "segment_field": "SEGMENT_ID",
                    "redefine_segment_id_map:1": "PARENT-SEG => P", "redefine-segment-id-map:2": "SIB-A => A",
                    "redefine-segment-id-map:3": "SIB-B => B", "segment-children:1": "PARENT-SEG => SIB-A,SIB-B"}


def test_group_before_the_root_registers_from_the_root_bytes():
    """A child segment's group placed before the root segment's: the root record's walk decodes it from
    the ROOT's bytes first (getGroupValues over the record group, RecordExtractors.scala:365-372), so
    A-CNT is registered with the root's byte at that offset (its P-CNT digit) before the root's own
    P-ITEMS reads it; the A children then register their own A-CNT for B's B-ITEMS."""
    p, _ = parse_options(BEFORE_ROOT_OPTS)
    cb = parse_copybook_for(BEFORE_ROOT_COPYBOOK, p)
    data = rdw("P2ABCxyzw") + rdw("B4wxyz") + rdw("A3aabbcc") + rdw("B1qrst")
    r = RO.var_len_rows(cb, data, p)[0]["REC"]["PARENT_SEG"]
    # P-ITEMS: A-CNT from the root's bytes = '2'; the A child: A-ITEMS on its own A-CNT = 3
    assert r["P_CNT"] == 2 and len(r["P_ITEMS"]) == 2
    assert len(r["SIB_A"]) == 1 and len(r["SIB_A"][0]["A_ITEMS"]) == 3
    # the B children are walked after the A children (copybook order): A-CNT = 3 from the A record
    assert [len(b["B_ITEMS"]) for b in r["SIB_B"]] == [3, 3]
