"""Arrow C Device Data Interface export of a decoded batch (the columnar bridge).

The reference hands Spark one `Row` per record (RowHandler / Row.fromSeq,
spark-cobol/.../reader/SparkCobolRowType.scala:24-28) out of a TableScan relation
(spark-cobol/.../source/CobolRelation.scala:66-99).  The GPU path instead leaves the decoded columns
in HBM and describes them to a columnar consumer (a ColumnarBatch built over Arrow vectors, or any
Arrow device consumer) as one ArrowDeviceArray + ArrowSchema pair: a struct array whose children are
the batch's output columns, every buffer pointer aimed at the decode's own device buffers -- no host
copy, no repacking:

* numeric columns: int32 "i" / int64 "l" / float "f" / double "g" (bit patterns as decoded),
  decimals as Arrow decimal64 "d:p,s,64" (precision <= 18, unscaled int64) or decimal128 "d:p,s";
  the validity bitmap of the slot row (Arrow bit order);
* string columns: Utf8View "vu" (string-view layout: views + the slot region cut into data buffers
  + the variadic buffer sizes), Utf8 "u" (int32 offsets relative to the slot's region), or
  LargeUtf8 "U" (int64 offsets absolute into the column's data);
* a column under a fixed OCCURS: one child per element slot ("NAME[3]");
* an OCCURS DEPENDING ON array in the list layout: a LargeListView "+vL" per field (offsets = the
  array's int64 offsets column, sizes = its element counts widened to int64 on the device, nulls
  where the array's segment is not the record's) over the packed child elements;
* generated File_Id / Record_Id / Seg_IdN columns first, as the reference's schema has them; the
  with_input_file_name_col column as a dictionary-encoded Utf8 (one entry, zero indices);
* a Utf8View's variadic buffer-sizes buffer is host memory (metadata the importer reads on the
  CPU); every other buffer is the decode's device memory.
device_type is ARROW_DEVICE_ROCM (10) with the tensors' device id; the export synchronises the
decode stream, so sync_event is NULL (the data is ready).  The export owns references to the
batch's tensors until both release callbacks ran.
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, List, Optional, Tuple

from . import native as N

ARROW_DEVICE_CPU = 1
ARROW_DEVICE_ROCM = 10
ARROW_FLAG_NULLABLE = 2


class ArrowSchema(ctypes.Structure):
    pass


class ArrowArray(ctypes.Structure):
    pass


_SCHEMA_RELEASE = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchema))
_ARRAY_RELEASE = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowArray))

ArrowSchema._fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
                        ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64),
                        ("children", ctypes.POINTER(ctypes.POINTER(ArrowSchema))),
                        ("dictionary", ctypes.POINTER(ArrowSchema)), ("release", _SCHEMA_RELEASE),
                        ("private_data", ctypes.c_void_p)]
ArrowArray._fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                       ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64),
                       ("buffers", ctypes.POINTER(ctypes.c_void_p)),
                       ("children", ctypes.POINTER(ctypes.POINTER(ArrowArray))),
                       ("dictionary", ctypes.POINTER(ArrowArray)), ("release", _ARRAY_RELEASE),
                       ("private_data", ctypes.c_void_p)]


class ArrowDeviceArray(ctypes.Structure):
    _fields_ = [("array", ArrowArray), ("device_id", ctypes.c_int64), ("device_type", ctypes.c_int32),
                ("sync_event", ctypes.c_void_p), ("reserved", ctypes.c_int64 * 3)]


# keep-alive registry: exported structs -> the Python objects their pointers reach (released by the
# consumer through the release callbacks; a struct moved by the consumer keeps its private_data key)
_LIVE: Dict[int, List[Any]] = {}
_NEXT_KEY = [1]


def _register(objs: List[Any]) -> int:
    k = _NEXT_KEY[0]
    _NEXT_KEY[0] += 1
    _LIVE[k] = objs
    return k


def _make_release_callbacks():
    """The release callbacks, closing over what they use: a consumer may release while the
    interpreter shuts down, when module globals already read as None."""
    live, SR, AR = _LIVE, _SCHEMA_RELEASE, _ARRAY_RELEASE
    null_schema_cb, null_array_cb = SR(), AR()

    def drop(key):
        if key:
            live.pop(int(key), None)

    @SR
    def release_schema(p):
        s = p.contents
        try:
            for i in range(s.n_children):
                c = s.children[i].contents
                if c.release:
                    c.release(s.children[i])
            drop(s.private_data)
        finally:
            s.release = null_schema_cb   # released: the callback slot is cleared

    @AR
    def release_array(p):
        a = p.contents
        try:
            for i in range(a.n_children):
                c = a.children[i].contents
                if c.release:
                    c.release(a.children[i])
            drop(a.private_data)
        finally:
            a.release = null_array_cb

    return release_schema, release_array


_release_schema, _release_array = _make_release_callbacks()


class _Node:
    """One exported array: its format, buffers (device pointers), length and children."""

    def __init__(self, fmt: str, name: str, length: int, buffers: List[int], children: List["_Node"] = (),
                 keep: List[Any] = (), nullable: bool = True, dictionary: Optional["_Node"] = None):
        self.fmt, self.name, self.length = fmt, name, length
        self.buffers, self.children, self.keep, self.nullable = list(buffers), list(children), list(keep), nullable
        self.dictionary = dictionary   # dictionary-encoded: fmt is the index type, this the values

    def schema(self) -> ArrowSchema:
        s = ArrowSchema()
        fmt, name = ctypes.create_string_buffer(self.fmt.encode()), ctypes.create_string_buffer(self.name.encode())
        kids = [c.schema() for c in self.children]
        arr = (ctypes.POINTER(ArrowSchema) * max(1, len(kids)))(*[ctypes.pointer(k) for k in kids])
        s.format = ctypes.cast(fmt, ctypes.c_char_p)
        s.name = ctypes.cast(name, ctypes.c_char_p)
        s.flags = ARROW_FLAG_NULLABLE if self.nullable else 0
        s.n_children = len(kids)
        s.children = ctypes.cast(arr, ctypes.POINTER(ctypes.POINTER(ArrowSchema)))
        dic = self.dictionary.schema() if self.dictionary is not None else None
        if dic is not None:
            s.dictionary = ctypes.pointer(dic)
        s.release = _release_schema
        s.private_data = _register([fmt, name, kids, arr, dic])
        return s

    def array(self) -> ArrowArray:
        a = ArrowArray()
        kids = [c.array() for c in self.children]
        karr = (ctypes.POINTER(ArrowArray) * max(1, len(kids)))(*[ctypes.pointer(k) for k in kids])
        bufs = (ctypes.c_void_p * max(1, len(self.buffers)))(*[b or None for b in self.buffers])
        a.length = self.length
        a.null_count = -1
        a.offset = 0
        a.n_buffers = len(self.buffers)
        a.n_children = len(kids)
        a.buffers = ctypes.cast(bufs, ctypes.POINTER(ctypes.c_void_p))
        a.children = ctypes.cast(karr, ctypes.POINTER(ctypes.POINTER(ArrowArray)))
        dic = self.dictionary.array() if self.dictionary is not None else None
        if dic is not None:
            a.dictionary = ctypes.pointer(dic)
        a.release = _release_array
        a.private_data = _register([kids, karr, bufs, self.keep, dic])
        return a


def _prim_format(info) -> Tuple[str, int]:
    ot = info.out_type
    if ot == N.O_DEC64:
        _, p, s = info.stype
        return f"d:{p},{s},64", 8
    if ot == N.O_DEC128:
        _, p, s = info.stype
        return f"d:{p},{s}", 16
    return {N.O_I32: ("i", 4), N.O_I64: ("l", 8), N.O_F32: ("f", 4), N.O_F64: ("g", 8)}[ot]


def _column_nodes(batch, ci: int, name: str) -> List[_Node]:
    """The exported arrays of output column ci: one per slot row (or one list view per field)."""
    import torch
    plan = batch.plan
    info = plan.columns[ci]
    c = batch.cols[ci]
    n = batch.n_rec
    pw = (n + 63) // 64
    pitch = 64 * pw
    ot = info.out_type
    out = []
    is_str = ot in (N.O_STRING, N.O_BINARY)
    if info.list_array >= 0:
        ar = plan.arrays[info.list_array]
        fmt, w = _prim_format(info)
        cnt_col = batch.cols[ar.count_column]
        # sizes: int64 counts, zero where the count is null (the array's segment is not the record's)
        bits = (cnt_col["validity"][:pw].view(torch.uint8).unsqueeze(-1) >> torch.arange(8, device=c["values"].device,
                                                                                            dtype=torch.uint8)) & 1
        valid = bits.reshape(-1)[:n].to(torch.int64)
        sizes = cnt_col["values"][:n].to(torch.int64) * valid
        offs = batch.cols[ar.offsets_column]["values"]
        n_child = c["values"].numel() // (2 if w == 16 else 1)
        child = _Node(fmt, "element", n_child, [c["validity"].data_ptr(), c["values"].data_ptr()], keep=[c])
        out.append(_Node("+vL", name, n, [cnt_col["validity"].data_ptr(), offs.data_ptr(), sizes.data_ptr()],
                         [child], keep=[sizes, offs, cnt_col]))
        return out
    for s in range(info.n_slots):
        nm = name if info.n_slots == 1 else f"{name}[{s}]"
        vptr = c["validity"].data_ptr() + 8 * s * pw
        if is_str and "views" in c:
            cap, bb = c["capacity"], max(1, c["buffer_bytes"])
            region = c["data"].data_ptr() + s * cap
            n_buf = max(1, (cap + bb - 1) // bb)
            # the variadic buffer sizes are metadata a consumer reads on the host while it imports the
            # array (to size the data buffers): host memory, unlike every data buffer
            sizes = torch.tensor([min(bb, cap - k * bb) for k in range(n_buf)], dtype=torch.int64)
            bufs = [vptr, c["views"].data_ptr() + 16 * s * pitch] + [region + k * bb for k in range(n_buf)] + \
                [sizes.data_ptr()]
            out.append(_Node("vu" if ot == N.O_STRING else "vz", nm, n, bufs, keep=[c, sizes]))
        elif is_str and "offsets32" in c:
            out.append(_Node("u" if ot == N.O_STRING else "z", nm, n,
                             [vptr, c["offsets32"].data_ptr() + 4 * s * (pitch + 1),
                              c["data"].data_ptr() + s * c["capacity"]], keep=[c]))
        elif is_str:
            out.append(_Node("U" if ot == N.O_STRING else "Z", nm, n,
                             [vptr, c["offsets"].data_ptr() + 8 * s * (pitch + 1), c["data"].data_ptr()], keep=[c]))
        else:
            fmt, w = _prim_format(info)
            out.append(_Node(fmt, nm, n, [vptr, c["values"].data_ptr() + w * s * pitch], keep=[c]))
    return out


def _file_name_node(input_file, n: int, dev) -> _Node:
    """The input-file-name column: int32 indices (all 0) over a one-entry Utf8 dictionary, both on
    the batch's device."""
    import torch
    name, value = input_file
    raw = value.encode("utf-8")
    idx = torch.zeros(max(1, n), dtype=torch.int32, device=dev)
    offs = torch.tensor([0, len(raw)], dtype=torch.int32, device=dev)
    data = torch.tensor(list(raw) or [0], dtype=torch.uint8, device=dev)
    dic = _Node("u", "", 1, [0, offs.data_ptr(), data.data_ptr()], keep=[offs, data])
    return _Node("i", name, n, [0, idx.data_ptr()], keep=[idx], dictionary=dic)


def _column_name(plan, ci: int) -> str:
    info = plan.columns[ci]
    if ci == plan.file_id_column:
        return "File_Id"
    if ci == plan.record_id_column:
        return "Record_Id"
    if ci in plan.seg_id_columns:
        return f"Seg_Id{plan.seg_id_columns.index(ci)}"
    return info.node.name if info.node is not None else f"_col{ci}"


def export_device(batch, generated_first: bool = True) -> Tuple[ArrowDeviceArray, ArrowSchema, List[_Node]]:
    """The batch as (ArrowDeviceArray, ArrowSchema) of a struct array over its output columns (value
    columns, generated columns; OCCURS counts, list offsets and the segment index are not separate
    output columns -- the lists and structs carry them).  Returns the two structs and the node tree
    (which buffer of which column each pointer is)."""
    import torch
    plan = batch.plan
    dev = None
    for c in batch.cols:
        for t in c.values():
            if isinstance(t, torch.Tensor):
                dev = t.device
                break
        if dev is not None:
            break
    gen = [ci for ci in (plan.file_id_column, plan.record_id_column) if ci >= 0 and batch.generate_record_id] + \
        list(plan.seg_id_columns)
    skip = set(gen) | {plan.segment_column}
    skip |= {ar.count_column for ar in plan.arrays} | {ar.offsets_column for ar in plan.arrays}
    order = (gen if generated_first else []) + [ci for ci, info in enumerate(plan.columns)
                                               if ci not in skip and info.kind == "value" and not info.hidden]
    kids: List[_Node] = []
    for ci in order:
        kids += _column_nodes(batch, ci, _column_name(plan, ci))
    if getattr(batch, "input_file", None) is not None and generated_first:
        # with_input_file_name_col: a dictionary-encoded Utf8 column (one entry, n zero indices), in
        # the position the batch's generated fields give it (DecodedBatch.generated)
        names = [nm for nm, _ in batch.generated(lambda ci: ci)]
        pos = names.index(batch.input_file[0])
        kids.insert(pos, _file_name_node(batch.input_file, batch.n_rec, dev))
    if dev is not None and dev.type == "cuda":
        torch.cuda.synchronize(dev)
    root = _Node("+s", "", batch.n_rec, [0], kids, nullable=False)
    da = ArrowDeviceArray()
    da.array = root.array()
    da.device_type = ARROW_DEVICE_ROCM if dev is not None and dev.type == "cuda" else ARROW_DEVICE_CPU
    da.device_id = dev.index if dev is not None and dev.type == "cuda" and dev.index is not None else -1
    da.sync_event = None
    return da, root.schema(), kids
