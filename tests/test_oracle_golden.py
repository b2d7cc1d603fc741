"""The oracle (oracle/cobrix_oracle.c) against the reference's own golden outputs -- this is what
pins the parity checker before it is trusted with the GPU path."""
from __future__ import annotations

import goldens as G

from cobrix_amd.copybook import parse_copybook
from oracle import oracle as O


def test_test1_fixed_length_with_odo():
    # Test1FixedLengthRecordsSpec.scala:38-66: collapse_root, OCCURS 80 DEPENDING ON, REDEFINES
    cb = parse_copybook(G.read("test1_copybook.cob").decode())
    rows = O.rows(O.decode_fixed(cb, G.read("test1_data", "example.bin")))
    assert not G.compare_rows(rows, G.load_lines("test1_expected", "test1.txt"))


def test_test6_type_variety_ieee754():
    # Test6TypeVarietySpec.scala:60-100: every numeric encoding, IEEE754 floats, na.fill(0)
    cb = parse_copybook(G.read("test6_copybook.cob").decode(), floating_point_format="IEEE754")
    rows = O.rows(O.decode_fixed(cb, G.read("test6_data", "INTEGR.TYPES.NOV28.DATA.dat")))
    rows.sort(key=lambda r: (r["ID"] is None, r["ID"]))
    assert not G.compare_rows(rows, G.load_lines("test6_expected", "test6.txt"), na_fill=True)


def test_rdw_sparse_index_known_answer():
    # Test5MultisegmentSpec.scala:205-218: 10 records per entry, cut at root "C" -> 88 entries
    raw = G.read("test5_data", "COMP.DETAILS.SEP30.DATA.dat")
    off, ln = O.frame_rdw(raw)
    assert len(off) == 1000 and off[-1] + ln[-1] == len(raw)
    seg = [G.java_trim(raw[o:o + 5].decode("cp037")) for o in off]
    is_root = [1 if s == "C" else 0 for s in seg]
    idx = O.sparse_index(raw, records_per_entry=10, is_root=is_root)
    assert len(idx) == 88
    assert idx[0][0] == 0 and all(a[1] == b[0] for a, b in zip(idx, idx[1:]))


def test_oracle_batch_var_equals_per_record():
    """ora_extract_var (one C call per batch, used by bench.py's cpu_baseline) == per-record decode."""
    import numpy as np
    from cobrix_amd import copybook as cbk
    from cobrix_amd.synth import RDW_NARROW_COPYBOOK, rdw_narrow
    raw_t, _ = rdw_narrow(500, seed=3)
    raw = raw_t.numpy().tobytes()
    cb = cbk.parse_copybook(RDW_NARROW_COPYBOOK, segment_redefines=["STATIC-DETAILS", "CONTACTS"])
    off, ln = O.frame_rdw(raw)
    segs = ["STATIC_DETAILS" if raw[o] == 0xC3 else "CONTACTS" for o in off]
    a = O.decode_var(cb, raw, off, ln, active_segments=segs)
    b = O.decode_records(cb, [raw[o:o + n] for o, n in zip(off, ln)], active_segments=segs)
    assert a.n_rec == b.n_rec == 500
    assert np.array_equal(a.events, b.events) and a.heap == b.heap
