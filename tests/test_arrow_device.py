"""Arrow C Device Data Interface export (cobrix_amd/arrow_device.py) on the CPU: columns allocated
as the decoder's caller allocates them (CPU tensors stand in for HBM), filled with known values,
exported, imported through pyarrow's C device importer (device type CPU) and compared with the
host Arrow builder's arrays; the structs' release callbacks free their keep-alive entries."""
from __future__ import annotations

import ctypes

import pytest

torch = pytest.importorskip("torch")
pa = pytest.importorskip("pyarrow")

import golden_cases as GC  # noqa: E402


def _fake_batch(monkeypatch, name, string_views):
    import cobrix_amd.reader as R
    monkeypatch.setattr(R, "_torch", lambda: torch)
    from cobrix_amd.copybook import parse_copybook
    from cobrix_amd.plan import build_plan
    from cobrix_amd.reader import DecodedBatch, _alloc_columns
    cb = parse_copybook(GC.copybook_text(GC.CASES[name]))
    plan = build_plan(cb, string_views=string_views)
    n = 77
    pw = (n + 63) // 64
    cols, _ = _alloc_columns(plan, n, [4096] * plan.n_columns, "cpu")
    g = torch.Generator().manual_seed(1)
    for c in cols:
        c["validity"].copy_(torch.randint(-2 ** 62, 2 ** 62, c["validity"].shape, generator=g))
        if "values" in c:
            v = c["values"]
            v.copy_(torch.randint(-1000, 1000, v.shape, generator=g, dtype=torch.int64).to(v.dtype))
        for key in ("offsets", "offsets32"):
            if key in c:
                o = c[key].view(-1, 64 * pw + 1)
                steps = torch.randint(0, 5, o.shape, generator=g)
                steps[:, 0] = 0
                o.copy_(torch.cumsum(steps, 1).to(o.dtype))
                if key == "offsets":   # absolute into data: slot s's region starts at s * capacity
                    o += (torch.arange(o.shape[0]) * c["capacity"]).view(-1, 1)
                c["data"].copy_(torch.randint(97, 123, c["data"].shape, generator=g, dtype=torch.uint8))
    return plan, DecodedBatch(plan, n, cols, 0, False, False)


@pytest.mark.parametrize("layout", [0, 2])
@pytest.mark.parametrize("name", ["test1", "test6"])
def test_export_import_roundtrip(monkeypatch, name, layout):
    from cobrix_amd import arrow_device as AD
    plan, batch = _fake_batch(monkeypatch, name, layout)
    live0 = len(AD._LIVE)
    da, sc, kids = AD.export_device(batch)
    assert da.device_type == AD.ARROW_DEVICE_CPU
    rb = pa.RecordBatch._import_from_c_device(ctypes.addressof(da), ctypes.addressof(sc))
    rb.validate()
    n_checked = 0
    for ci, info in enumerate(plan.columns):
        if info.kind != "value" or info.hidden:
            continue
        name0 = AD._column_name(plan, ci)
        for s, h in enumerate(batch._slot_arrays(ci)):
            nm = name0 if info.n_slots == 1 else f"{name0}[{s}]"
            got = rb.column(rb.schema.get_field_index(nm))
            assert got.type == h.type or (pa.types.is_decimal(got.type) and pa.types.is_decimal(h.type))
            norm = lambda xs: ["nan" if isinstance(x, float) and x != x else x for x in xs]  # noqa: E731
            assert norm(got.to_pylist()) == norm(h.to_pylist()), nm
            n_checked += 1
    assert n_checked > 3
    del rb, got
    import gc
    gc.collect()
    assert len(AD._LIVE) == live0   # every struct released its keep-alive entry
