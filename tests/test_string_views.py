"""The string-view output layout (cobrix_hip.h, cbx_plan_options.string_views) on the host side:
the view decoder used by DecodedBatch agrees with Arrow's own reading of the same buffers, and the
buffer geometry matches the library's rule.  The device side is covered by the -m gpu tests
(test_gpu_golden.py / test_gpu_parity.py run every golden case in both layouts)."""
from __future__ import annotations

import numpy as np
import pytest

from cobrix_amd.reader import decode_views, view_geometry


def _views(values, tile_bytes, buffer_bytes):
    """Build views + data the way the decode kernel lays them out: per tile of 64 values the long
    payloads packed in the tile's region."""
    n = len(values)
    n_tiles = (n + 63) // 64
    data = bytearray(n_tiles * tile_bytes)
    tpb = buffer_bytes // tile_bytes
    views = np.zeros((n, 16), dtype=np.uint8)
    for t in range(n_tiles):
        ex = 0
        for r in range(64 * t, min(n, 64 * t + 64)):
            b = values[r]
            views[r, 0:4] = np.frombuffer(np.int32(len(b)).tobytes(), np.uint8)
            if len(b) <= 12:
                views[r, 4:4 + len(b)] = np.frombuffer(b, np.uint8) if b else []
                continue
            base = t * tile_bytes + ex
            data[base:base + len(b)] = b
            views[r, 4:8] = np.frombuffer(b[:4], np.uint8)
            views[r, 8:12] = np.frombuffer(np.int32(t // tpb).tobytes(), np.uint8)
            views[r, 12:16] = np.frombuffer(np.int32((t % tpb) * tile_bytes + ex).tobytes(), np.uint8)
            ex += len(b)
    return views, bytes(data)


def test_view_geometry_rule():
    # tile_bytes = capacity / tiles; buffers hold a power-of-two number of whole tiles (<= 1 GiB)
    # 2**30 // 2560 = 419,430 tiles fit; the buffer takes the largest power of two of them
    assert view_geometry(781_250 * 2560, 781_250) == (2560, 262_144 * 2560)
    assert view_geometry(64 * 4096, 64) == (4096, 2 ** 30)
    assert view_geometry(0, 10) == (0, 0)
    tb, bb = view_geometry(3 * (2 ** 30 + 16), 3)
    assert tb == 2 ** 30 + 16 and bb == tb   # a tile larger than 1 GiB is its own buffer


@pytest.mark.parametrize("seed", [1, 2])
def test_decode_views_matches_arrow(seed):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(seed)
    alphabet = "abcdefghijklmnopqrstuvwxyzÀÉÎõü€ 0123456789"
    vals = ["".join(rng.choice(list(alphabet), int(rng.integers(0, 30)))).encode() for _ in range(1000)]
    tile_bytes = 64 * 90
    buffer_bytes = 3 * tile_bytes   # small buffers: views spread over several Arrow data buffers
    views, data = _views(vals, tile_bytes, buffer_bytes)
    assert decode_views(views, data, buffer_bytes, 0) == vals
    nbuf = (len(data) + buffer_bytes - 1) // buffer_bytes
    bufs = [pa.py_buffer(data[k * buffer_bytes:(k + 1) * buffer_bytes]) for k in range(nbuf)]
    arr = pa.Array.from_buffers(pa.binary_view(), len(vals), [None, pa.py_buffer(views.tobytes())] + bufs)
    arr.validate(full=True)
    assert arr.to_pylist() == vals
    sv = pa.Array.from_buffers(pa.string_view(), len(vals), [None, pa.py_buffer(views.tobytes())] + bufs)
    assert sv.to_pylist() == [v.decode() for v in vals]


def test_alloc_columns_view_layout(monkeypatch):
    """Host allocation of the view layout (CPU tensors stand in for device memory): 16-byte views
    per value, regions of whole tiles, the column table pointing at them."""
    torch = pytest.importorskip("torch")
    import cobrix_amd.reader as R
    monkeypatch.setattr(R, "_torch", lambda: torch)
    from cobrix_amd.copybook import parse_copybook
    from cobrix_amd.plan import build_plan
    from cobrix_amd.reader import _alloc_columns
    from cobrix_amd.synth import SYNSTR200_COPYBOOK
    from bench import algorithmic_bytes
    plan = build_plan(parse_copybook(SYNSTR200_COPYBOOK, code_page="cp037"), string_views=True)
    assert plan.options.string_views == 1
    n = 1000
    tiles = (n + 63) // 64
    caps = [tiles * 64 * 20 for _ in plan.columns]     # cp037: 1 byte per char in this table
    cols, cs = _alloc_columns(plan, n, caps, "cpu")
    for c, s in zip(cols, cs):
        assert c["views"].numel() == 16 * 64 * tiles and "offsets" not in c
        assert s.values == c["views"].data_ptr() and s.offsets is None and s.data_capacity == caps[0]
        assert c["tile_bytes"] == 64 * 20
    # SURVEY.md 8(d) accounting, whatever the layout: input + validity + a 4-byte offset per value +
    # the whole UTF-8 payload
    pay = {ci: 1000 + ci for ci in range(10)}
    assert algorithmic_bytes(plan, n, 200 * n, pay, {}) == 200 * n + sum(pay.values()) + 10 * ((n + 7) // 8 + 4 * n)
    from bench import layout_bytes, string_payload
    # views: lengths of valid values only; the layout writes 16-byte views + payloads over 12 bytes
    ln = torch.tensor([5, 13, 0, 20], dtype=torch.int32)
    cols[0]["views"].view(-1, 16)[:4, :4] = ln.view(torch.uint8).view(4, 4)
    cols[0]["validity"][0] = 0b1011                      # value 2 null (length 0 anyway), value 3 valid
    got = string_payload(plan, cols, n)
    assert got[0] == 5 + 13 + 20 and all(got[ci] == 0 for ci in range(1, 10))
    lay = layout_bytes(plan, cols, n, 200 * n, got, {})
    assert lay == 200 * n + 10 * ((n + 7) // 8 + 16 * n) + 13 + 20


def test_present_elements_counts_only_live_odo_elements():
    """bench.algorithmic_bytes counts the elements records hold: the ODO counts of records whose
    segment redefine holds the array (C5 accounting)."""
    torch = pytest.importorskip("torch")
    from bench import algorithmic_bytes, present_elements
    from cobrix_amd.copybook import parse_copybook
    from cobrix_amd.plan import build_plan
    from cobrix_amd.synth import WIDE_ODO_COPYBOOK, WIDE_ODO_SEGMENTS
    cb = parse_copybook(WIDE_ODO_COPYBOOK, segment_redefines=sorted(set(WIDE_ODO_SEGMENTS.values())))
    plan = build_plan(cb, segment_field="SEGMENT-ID", segment_redefine_map=WIDE_ODO_SEGMENTS)
    n = 5
    cols = [{"values": torch.zeros(64 * c.n_slots, dtype=torch.int32)} for c in plan.columns]
    arr = [a for a in plan.arrays if a.dependee >= 0][0]
    cols[arr.count_column]["values"][:n] = torch.tensor([10, 2000, 7, 0, 3], dtype=torch.int32)
    seg = torch.tensor([arr.segment, -1, arr.segment, arr.segment, 1 - arr.segment], dtype=torch.int32)
    cols[plan.segment_column]["values"][:n] = seg
    pres = present_elements(plan, cols, n)
    odo_cols = {f.column for f in plan.fields if f.n_dims == 1}
    assert set(pres) == odo_cols and all(v == 10 + 7 + 0 for v in pres.values())
    full = algorithmic_bytes(plan, n, 0, {}, {})
    live = algorithmic_bytes(plan, n, 0, {}, pres)
    per = sum(4 * (n * plan.columns[c].n_slots - pres[c]) for c in odo_cols)
    assert full - live >= per
