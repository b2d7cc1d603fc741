"""Arrow C Device Data Interface export (cobrix_amd/arrow_device.py): the decoded
columns described in place -- every buffer pointer of the ArrowDeviceArray is the decode's own HBM
buffer (device type ROCm).  pyarrow has no ROCm memory manager, so the test plays the consumer: it
copies each described buffer to the host through the pointers (hipMemcpy), relabels the tree as
CPU memory, imports it with pyarrow's C Device Data importer and compares every column with the
batch's host Arrow export (itself checked against the reference's golden rows in
test_gpu_golden.py::test_gpu_arrow_export_matches_rows)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pa = pytest.importorskip("pyarrow")

pytestmark = pytest.mark.gpu

import golden_cases as GC  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


_hip = None


def _d2h(ptr: int, n: int) -> bytes:
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    buf = ctypes.create_string_buffer(max(1, n))
    if n:
        assert _hip.hipMemcpy(buf, ctypes.c_void_p(ptr), n, 2) == 0   # hipMemcpyDeviceToHost
    return buf.raw[:n]


def _host_copy(node, keep):
    """The consumer's side: a CPU ArrowArray with copies of the buffers the node's pointers describe."""
    from cobrix_amd import arrow_device as AD
    n, f = node.length, node.fmt
    bufs = []

    def take(ptr, size):
        b = ctypes.create_string_buffer(_d2h(ptr, size), max(1, size))
        keep.append(b)
        bufs.append(ctypes.addressof(b))

    v = node.buffers
    if f == "+s" or not v[0]:
        bufs.append(0)   # no validity bitmap (struct root, dictionary indices of a constant column)
    else:
        take(v[0], 8 * ((n + 63) // 64))
    if f in ("i", "f"):
        take(v[1], 4 * n)
    elif f in ("l", "g") or f.endswith(",64"):
        take(v[1], 8 * n)
    elif f.startswith("d:"):
        take(v[1], 16 * n)
    elif f in ("u", "z"):
        offs = np.frombuffer(_d2h(v[1], 4 * (n + 1)), dtype=np.int32)
        take(v[1], 4 * (n + 1))
        take(v[2], int(offs[n]))
    elif f in ("U", "Z"):
        offs = np.frombuffer(_d2h(v[1], 8 * (n + 1)), dtype=np.int64)
        take(v[1], 8 * (n + 1))
        take(v[2], int(offs[n]))
    elif f in ("vu", "vz"):
        take(v[1], 16 * n)
        k = len(v) - 3
        # the variadic buffer sizes are host memory: read in place, as an importer does
        sizes = np.frombuffer(ctypes.string_at(v[-1], 8 * k), dtype=np.int64).copy()
        for j in range(k):
            take(v[2 + j], int(sizes[j]))
        b = ctypes.create_string_buffer(sizes.tobytes(), 8 * k)
        keep.append(b)
        bufs.append(ctypes.addressof(b))
    elif f == "+vL":
        take(v[1], 8 * n)
        take(v[2], 8 * n)
    kids = [_host_copy(c, keep) for c in node.children]
    a = AD.ArrowArray()
    if node.dictionary is not None:
        dic = _host_copy(node.dictionary, keep)
        keep.append(dic)
        a.dictionary = ctypes.pointer(dic)
    karr = (ctypes.POINTER(AD.ArrowArray) * max(1, len(kids)))(*[ctypes.pointer(k) for k in kids])
    barr = (ctypes.c_void_p * max(1, len(bufs)))(*[b or None for b in bufs])
    keep += [kids, karr, barr]
    a.length, a.null_count, a.offset = n, -1, 0
    a.n_buffers, a.n_children = len(bufs), len(kids)
    a.buffers = ctypes.cast(barr, ctypes.POINTER(ctypes.c_void_p))
    a.children = ctypes.cast(karr, ctypes.POINTER(ctypes.POINTER(AD.ArrowArray)))
    a.release = AD._release_array
    return a


def _import_host(da, schema, kids):
    from cobrix_amd import arrow_device as AD
    from cobrix_amd.arrow_device import _Node
    keep = []
    root = _Node("+s", "", da.array.length, [0], kids, nullable=False)
    host = AD.ArrowDeviceArray()
    host.array = _host_copy(root, keep)
    host.device_type, host.device_id, host.sync_event = AD.ARROW_DEVICE_CPU, -1, None
    rb = pa.RecordBatch._import_from_c_device(ctypes.addressof(host), ctypes.addressof(schema))
    return rb, keep   # the import is zero-copy: the host copies must outlive rb


def _norm(v):
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, float):
        return "nan" if v != v else v
    if isinstance(v, bytes):
        return v
    return v


def _check(batch, device_type=None):
    from cobrix_amd import arrow_device as AD
    da, schema, kids = AD.export_device(batch)
    if device_type is None:
        assert da.device_type == AD.ARROW_DEVICE_ROCM and da.device_id == torch.cuda.current_device()
    assert da.array.length == batch.n_rec and da.array.n_children == len(kids)
    # zero copy: every pointer lies inside one of the batch's own device tensors
    spans = [(t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for c in batch.cols for t in c.values()
             if isinstance(t, torch.Tensor)]

    def inside(p):
        return any(a <= p < b for a, b in spans)

    host = [(t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for nd in kids for t in _tensors(nd)
            if isinstance(t, torch.Tensor) and not t.is_cuda]

    def walk(nd):
        for j, b in enumerate(nd.buffers):
            if nd.fmt in ("vu", "vz") and j == len(nd.buffers) - 1:
                # the variadic buffer sizes: host memory the importer can read (cpu tensor)
                assert any(a <= b < e for a, e in host), (nd.name, "buffer sizes not in host memory")
            elif b and not (nd.fmt == "+vL" and j == 2) and nd.dictionary is None:
                assert inside(b), (nd.name, nd.fmt, j)
        for c in nd.children:
            walk(c)
    for k in kids:
        walk(k)
    rb, keep = _import_host(da, schema, kids)
    try:
        _compare(batch, rb)
    finally:
        # the import holds our release callback: drop it here, not at interpreter exit (a failing
        # assertion's traceback would otherwise keep it alive until shutdown)
        del rb
        keep.clear()


def _tensors(nd):
    out = [t for t in nd.keep if isinstance(t, torch.Tensor)]
    for c in nd.children:
        out += _tensors(c)
    return out


def _compare(batch, rb):
    from cobrix_amd import arrow_device as AD
    assert rb.num_rows == batch.n_rec
    plan = batch.plan
    # by position within a name: copybooks repeat field names across segments (test17's ADDRESS)
    got = {}
    for i, f in enumerate(rb.schema):
        got.setdefault(f.name, []).append(rb.column(i))
    n_checked = 0
    for ci, info in enumerate(plan.columns):
        if info.kind != "value" or info.hidden:
            continue
        name = AD._column_name(plan, ci)
        if info.list_array >= 0:
            vals, valid = batch._list_dense(ci)
            cnt_ci = plan.arrays[info.list_array].count_column
            cnt = batch.cols[cnt_ci]["values"].cpu().numpy()[: batch.n_rec]
            cbits = np.unpackbits(batch.cols[cnt_ci]["validity"].cpu().numpy().view(np.uint8), bitorder="little")
            vals = vals.reshape(info.n_slots, batch.n_rec, -1) if vals.ndim > 1 else vals.reshape(info.n_slots, batch.n_rec)
            arr = got[name].pop(0).to_pylist()
            for r in range(batch.n_rec):
                if not cbits[r]:
                    assert arr[r] is None or arr[r] == []
                    continue
                exp_row = [(vals[j, r] if valid[j, r] else None) for j in range(int(cnt[r]))]
                got_row = arr[r]
                assert len(got_row) == len(exp_row)
                for x, y in zip(got_row, exp_row):
                    assert (x is None) == (y is None)
                    if x is not None and isinstance(x, int):
                        assert x == int(y)
            n_checked += 1
            continue
        parts = batch._slot_arrays(ci)
        for s, host_arr in enumerate(parts):
            nm = name if info.n_slots == 1 else f"{name}[{s}]"
            assert _norm(got[nm].pop(0).to_pylist()) == _norm(host_arr.to_pylist()), nm
            n_checked += 1
    assert n_checked > 0


@pytest.mark.parametrize("layout", ["large", "views", "utf8"])
@pytest.mark.parametrize("name", ["test1", "test5", "test6", "test9_cp037", "test17a"])
def test_device_export_golden_cases(name, layout):
    from cobrix_amd.reader import FixedLenNestedReader, VarLenNestedReader
    case = GC.CASES[name]
    p, var_len = GC.params(case)
    p.string_views = layout == "views"
    p.string_utf8 = layout == "utf8"
    data = GC.data_bytes(case)
    rd = (VarLenNestedReader if var_len else FixedLenNestedReader)(GC.copybook_text(case), p)
    batch = rd.read(data) if var_len else rd.decode(data)
    _check(batch)


def test_device_export_lists():
    """OCCURS DEPENDING ON arrays in the list layout as LargeListView columns (C5 layout)."""
    from cobrix_amd.reader import ReaderParameters, VarLenNestedReader
    from cobrix_amd.synth import WIDE_ODO_COPYBOOK, WIDE_ODO_SEGMENTS, wide_odo
    raw_t, _ = wide_odo(30, seed=7)
    params = ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                              segment_id_redefine_map=WIDE_ODO_SEGMENTS, occurs_lists=True, string_views=True)
    rd = VarLenNestedReader(WIDE_ODO_COPYBOOK, params)
    t = raw_t.cuda()
    off, ln = rd.frame(t, int(t.numel()))
    batch = rd.decode_device(t, int(t.numel()), off, ln)
    assert any(c.list_array >= 0 for c in rd.plan.columns)
    _check(batch)


@pytest.mark.parametrize("gen_id", [False, True])
def test_device_export_input_file_column(gen_id):
    """with_input_file_name_col (Test20InputFileNameSpec.scala:94-165): the file name column is a
    dictionary-encoded Utf8 on the device, in the schema position the reference gives it (first, or
    after File_Id / Record_Id)."""
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    opts = {"is_record_sequence": "true", "encoding": "ascii", "with_input_file_name_col": "F"}
    if gen_id:
        opts["generate_record_id"] = "true"
    p, var_len = parse_options(opts)
    assert var_len
    rd = VarLenNestedReader(GC.copybook_text({"copybook": "test4_copybook.cob"}), p)
    data = GC.data_bytes({"data": "test4_data/COMP.DETAILS.SEP30.DATA.dat"})
    with pytest.raises(ValueError, match="needs the input file's name"):
        rd.read(data)
    batch = rd.read(data, input_file_name="COMP.DETAILS.SEP30.DATA.dat")
    from cobrix_amd import arrow_device as AD
    da, schema, kids = AD.export_device(batch)
    rb, keep = _import_host(da, schema, kids)
    try:
        names = rb.schema.names
        assert names.index("F") == (2 if gen_id else 0)
        col = rb.column(names.index("F"))
        assert col.to_pylist() == ["COMP.DETAILS.SEP30.DATA.dat"] * batch.n_rec
        _compare(batch, rb)
    finally:
        del rb
        keep.clear()
