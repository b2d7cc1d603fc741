"""Flatten a Cobrix copybook AST into the descriptor tables of the HIP library.

This is what the JVM host does once per query before calling libcobrix_hip.so: walk the
`Copybook` AST in `extractRecord` order (CP/reader/extractors/record/RecordExtractors.scala:
139-172) and emit one `cbx_field` per decoded Primitive (every REDEFINES alternative, every
OCCURS element as a "slot"), one `cbx_array` per OCCURS node with its DEPENDING ON source, and
the segment-redefine selection map (FixedLenNestedRowIterator.scala:64-99).

Output columns: one per field, one int32 element-count column per OCCURS node, optionally one
int32 "active segment" column, plus generated File_Id / Record_Id.
"""
from __future__ import annotations

import ctypes
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import copybook as cbk
from . import native as N
from .codepages import ascii_charset_table, is_us_ascii, lut_for, utf8_lut
from .schema import (ST_BINARY, ST_DECIMAL, ST_DOUBLE, ST_FLOAT, ST_INT, ST_LONG, ST_STRING,
                     spark_type)


class UnsupportedLayout(ValueError):
    """The layout uses a feature outside the GPU path (reported, never silently degraded)."""


class NeedsWalk(UnsupportedLayout):
    """The static-offset kernels cannot express the layout; the record walk can (build_plan(walk=True))."""


@dataclass
class ColumnInfo:
    index: int
    kind: str                      # "value" | "count" | "segment" | "record_id" | "file_id"
    out_type: int
    n_slots: int = 1
    node: Optional[cbk.Statement] = None
    stype: Tuple[int, int, int] = (0, 0, 0)
    hidden: bool = False           # decoded for a dependency only (e.g. FILLER dependee)
    list_array: int = -1           # list layout: the OCCURS DEPENDING ON array (child elements)
    list_mpad: int = 0             # list layout: elements per record slot in a tile region (max rounded to 64)


@dataclass
class DecodePlan:
    copybook: cbk.Copybook
    fields: List[N.CbxField]
    arrays: List[N.CbxArray]
    columns: List[ColumnInfo]
    options: N.CbxPlanOptions
    field_of_node: Dict[int, int] = field(default_factory=dict)     # id(Primitive) -> field index
    array_of_node: Dict[int, int] = field(default_factory=dict)     # id(Statement) -> array index
    segment_groups: List[cbk.Group] = field(default_factory=list)
    segment_column: int = -1
    record_id_column: int = -1
    file_id_column: int = -1
    seg_id_columns: List[int] = field(default_factory=list)   # Seg_Id0.. string columns
    walk: Optional["WalkTables"] = None                          # record-walk tables (cbx_plan_set_walk)

    @property
    def n_columns(self) -> int:
        return len(self.columns)


def _out_type(st) -> int:
    t, p, _ = st
    if t == ST_INT:
        return N.O_I32
    if t == ST_LONG:
        return N.O_I64
    if t == ST_DECIMAL:
        return N.O_DEC64 if p <= 18 else N.O_DEC128
    if t == ST_FLOAT:
        return N.O_F32
    if t == ST_DOUBLE:
        return N.O_F64
    if t == ST_STRING:
        return N.O_STRING
    if t == ST_BINARY:
        return N.O_BINARY
    raise UnsupportedLayout(f"unknown spark type {t}")


def _charset_strings(cb: cbk.Copybook) -> bool:
    """ASCII strings decode through AsciiStringDecoderWrapper (a charset other than US-ASCII,
    DecoderSelector.scala:78-84): the plan's byte table becomes that charset's."""
    return not is_us_ascii(cb.ascii_charset)


def _kind_and_flags(p: cbk.Primitive, cb: cbk.Copybook) -> Tuple[int, int]:
    d = p.dtype
    flags = 0
    if isinstance(d, cbk.AlphaNumeric):
        if d.enc == cbk.ASCII and _charset_strings(cb):
            return N.K_STRING, 0   # an ASCII copybook has no EBCDIC strings to share the table with
        kind = {cbk.EBCDIC: N.K_STRING, cbk.ASCII: N.K_STRING_ASCII, cbk.HEX: N.K_HEX, cbk.RAW: N.K_RAW,
                cbk.UTF16: N.K_UTF16_BE if cb.is_utf16_big_endian else N.K_UTF16_LE}.get(d.enc)
        if kind is None:
            raise UnsupportedLayout(f"{p.name}: {d.enc} strings are not on the GPU path yet")
        return kind, 0
    if d.sign_position is not None:
        flags |= N.F_SIGNED
    if isinstance(d, cbk.Integral):
        flags |= N.F_INTEGRAL
    if isinstance(d, cbk.Decimal) and d.explicit_decimal:
        flags |= N.F_EXPLICIT_DOT
    if p.is_dependee:
        flags |= N.F_DEPENDEE
    if d.compact is None:
        if d.enc != cbk.EBCDIC:
            if p.data_size > 64:
                raise UnsupportedLayout(f"{p.name}: ASCII DISPLAY numbers wider than 64 bytes are not on the GPU path")
            return N.K_ASCII_NUM, flags
        return N.K_ZONED, flags
    if d.compact == cbk.COMP3:
        return N.K_BCD, flags
    if d.compact in (cbk.COMP4, cbk.COMP5):
        return N.K_BINARY, flags | N.F_BIG_ENDIAN
    if d.compact == cbk.COMP9:
        return N.K_BINARY, flags
    if d.compact in (cbk.COMP1, cbk.COMP2):
        if isinstance(d, cbk.Integral):
            raise UnsupportedLayout(f"{p.name}: COMP-1/COMP-2 is incorrect for an integral number")
        fp = cb.floating_point_format
        if fp in ("IBM", "IBM_LE"):
            flags |= N.F_IBM
        if fp in ("IBM_LE", "IEEE754_LE"):
            flags |= N.F_LITTLE_ENDIAN_FP
        return (N.K_FLOAT if d.compact == cbk.COMP1 else N.K_DOUBLE), flags
    raise UnsupportedLayout(f"{p.name}: usage {d.compact}")


_CANONICAL_INT = re.compile(r"^-?(0|[1-9][0-9]*)$")


def segment_keys(redefine_map: Dict[str, str], levels: List[str], seg_filter: Optional[List[str]]) -> List[str]:
    """Distinct segment ids named by the options, in a fixed order: levels, redefine map, filter."""
    keys: List[str] = []
    for lv in levels:
        for k in lv.split(","):
            if k not in keys:
                keys.append(k)
    for k in list(redefine_map) + list(seg_filter or []):
        if k not in keys:
            keys.append(k)
    return keys


def build_plan(cb: cbk.Copybook, *, segment_field: Optional[str] = None,
               segment_redefine_map: Optional[Dict[str, str]] = None, generate_record_id: bool = False,
               file_id: int = 0, window_bytes: int = 0, jit_min_records: int = 0,
               segment_levels: Sequence[str] = (), segment_filter: Optional[List[str]] = None,
               segment_prefix: str = "", string_views: int = 0, occurs_lists: bool = False,
               root_keys: Sequence[str] = (), walk: bool = False, variable_size_occurs: bool = False) -> DecodePlan:
    """root_keys: segment ids of a hierarchical file's root segment (sparse-index cuts at level-0
    keys, IndexGenerator.scala:89-113, without Seg_IdN columns).  walk: the plan decodes through the
    record walk (cbx_walk.h) -- count columns of nested OCCURS get one slot per enclosing element,
    dependees inside OCCURS and string dependees (occurs_mappings) are allowed, no list layout."""
    fields: List[N.CbxField] = []
    arrays: List[N.CbxArray] = []
    columns: List[ColumnInfo] = []
    field_of_node: Dict[int, int] = {}
    array_of_node: Dict[int, int] = {}
    seg_groups: List[cbk.Group] = cb.all_segment_redefines()
    seg_index = {id(g): i for i, g in enumerate(seg_groups)}
    trim = N.TRIM[cb.string_trimming]
    pending_arrays: List[Tuple[int, cbk.Statement]] = []
    walk_order: Dict[int, int] = {}
    counter = [0]

    def add_column(**kw) -> int:
        ci = ColumnInfo(index=len(columns), **kw)
        columns.append(ci)
        return ci.index

    def visit(st: cbk.Statement, dims: List[Tuple[int, int, int]], segment: int, in_array: bool):
        counter[0] += 1
        walk_order[id(st)] = counter[0]
        if isinstance(st, cbk.Group) and st.is_segment_redefine:
            segment = seg_index[id(st)]
        my_dims = list(dims)
        if st.is_array:
            ai = len(arrays)
            ar = N.CbxArray()
            ar.max_count = st.array_max_size
            ar.min_count = st.array_min_size
            ar.dependee = -1
            ar.segment = segment
            ar.n_dims = len(dims)
            ar.parent = dims[-1][2] if dims else -1
            arrays.append(ar)
            array_of_node[id(st)] = ai
            outer = 1
            for (cnt, _, _) in dims:
                outer *= cnt
            ar.count_column = add_column(kind="count", out_type=N.O_I32, node=st, n_slots=outer if walk else 1)
            ar.offsets_column = -1
            pending_arrays.append((ai, st))
            my_dims.append((st.array_max_size, st.data_size, ai))
            if len(my_dims) > N.CBX_MAX_DIMS:
                raise UnsupportedLayout(f"{st.name}: more than {N.CBX_MAX_DIMS} nested OCCURS levels")
        if isinstance(st, cbk.Group):
            for c in st.children:
                visit(c, my_dims, segment, in_array or st.is_array)
            return
        p: cbk.Primitive = st  # type: ignore[assignment]
        if p.is_filler and not p.is_dependee:
            return
        kind, flags = _kind_and_flags(p, cb)
        stp = spark_type(p)
        f = N.CbxField()
        f.kind, f.out_type, f.offset, f.size = kind, _out_type(stp), p.offset, p.data_size
        d = p.dtype
        if not isinstance(d, cbk.AlphaNumeric):
            f.precision = d.precision
            if isinstance(d, cbk.Decimal):
                f.scale, f.scale_factor = d.scale, d.scale_factor
        f.out_precision, f.out_scale = stp[1], stp[2]
        f.flags, f.trim = flags, trim
        f.n_dims = len(my_dims)
        n_slots = 1
        for k, (cnt, stride, ai) in enumerate(my_dims):
            f.dim_count[k], f.dim_stride[k], f.dim_array[k] = cnt, stride, ai
            n_slots *= cnt
        f.segment = segment
        f.column = add_column(kind="value", out_type=f.out_type, n_slots=n_slots, node=p, stype=stp,
                              hidden=p.is_filler)
        field_of_node[id(p)] = len(fields)
        fields.append(f)
        p_in_array = in_array or p.is_array
        if p.is_dependee:
            p.__dict__["_cbx_in_array"] = p_in_array

    for rec in cb.ast.children:
        visit(rec, [], -1, False)

    # DEPENDING ON sources (RecordExtractors.scala:64, 72, 126-134)
    prims = [st for st in _iter_prims(cb.ast)]
    for ai, st in pending_arrays:
        if st.depending_on is None:
            continue
        cand = [q for q in prims if q.is_dependee and q.name == st.depending_on]
        if not cand:
            continue  # the name never registers -> always arrayMaxSize
        q = cand[0]
        if walk_order[id(q)] > walk_order[id(st)]:
            continue  # decoded after the array -> not yet in dependFields -> arrayMaxSize
        if q.__dict__.get("_cbx_in_array") or not isinstance(q.dtype, cbk.Integral) or q.dtype.precision > 18:
            if not walk:   # a count per enclosing element / a string dependee: the record walk
                raise NeedsWalk(f"{st.name}: DEPENDING ON {q.name} (inside an OCCURS or not integral)")
            continue
        arrays[ai].dependee = field_of_node[id(q)]

    if occurs_lists and not walk:
        # list layout (cobrix_hip.h, CBX_F_LIST): a top-level OCCURS DEPENDING ON array whose elements
        # are numeric leaves of that one level -- child elements packed per record, absent ones unwritten
        for ai, ar in enumerate(arrays):
            if ar.dependee < 0 or ar.n_dims != 0 or any(b.parent == ai for b in arrays):
                continue
            members = [f for f in fields if f.n_dims >= 1 and ai in list(f.dim_array)[:f.n_dims]]
            if not members or any(f.n_dims != 1 or f.out_type in (N.O_STRING, N.O_BINARY) or f.segment != ar.segment
                                  for f in members):
                continue
            mpad = (ar.max_count + 63) // 64 * 64
            for f in members:
                f.flags |= N.F_LIST
                columns[f.column].list_array = ai
                columns[f.column].list_mpad = mpad
            ar.offsets_column = add_column(kind="list_offsets", out_type=N.O_I64, node=None)

    opts = N.CbxPlanOptions()
    seg_col = -1
    levels = list(segment_levels) if segment_field is not None else []
    seg_filter = segment_filter if segment_field is not None else None
    red = dict(segment_redefine_map or {}) if segment_field is not None else {}
    seg_id_cols: List[int] = []
    if segment_field is not None and (red or levels or seg_filter is not None):
        # the segment map (cobrix_hip.h cbx_segment_map): every key the options name, with what
        # each option says about it (redefine group, Seg_Id level, filter membership)
        sf = cb.get_field_by_name(segment_field)
        if not isinstance(sf, cbk.Primitive):
            raise UnsupportedLayout("segment field must be a primitive field")
        field_is_int = isinstance(sf.dtype, cbk.Integral) and sf.dtype.precision <= 18
        if not field_is_int and not (isinstance(sf.dtype, cbk.AlphaNumeric) and sf.dtype.enc in (cbk.EBCDIC, cbk.ASCII)):
            raise UnsupportedLayout("segment field must be an EBCDIC / ASCII string or an integral field")
        if sf.is_array:
            raise UnsupportedLayout("segment field must not be an OCCURS array")
        keys = segment_keys(red, levels, seg_filter)
        if len(keys) > N.CBX_MAX_SEG_KEYS:
            raise UnsupportedLayout("too many segment ids")
        if len(levels) > N.CBX_MAX_SEG_LEVELS:
            raise UnsupportedLayout("too many segment id levels")
        pre = segment_prefix.encode("utf-8")
        if len(pre) > N.CBX_MAX_SEG_PREFIX:
            raise UnsupportedLayout("segment_id_prefix too long")
        level_sets = [lv.split(",") for lv in levels]
        opts.has_segments = 1
        sm = opts.segments
        sm.field_offset, sm.field_size, sm.n_keys = sf.offset, sf.actual_size, len(keys)
        sm.field = field_of_node.get(id(sf), -1)
        sm.field_is_int = int(field_is_int)
        if field_is_int and sm.field < 0:
            raise UnsupportedLayout("integral segment field is not decoded (FILLER)")
        for k, key in enumerate(keys):
            u = [ord(c) for c in key]
            if len(u) > N.CBX_MAX_SEG_KEY_LEN:
                raise UnsupportedLayout("segment id too long")
            for j, x in enumerate(u):
                sm.key[k][j] = x
            sm.key_len[k] = len(u)
            sm.key_segment[k] = -1
            if key in red:
                gname = cbk._transform_identifier(red[key]).upper()
                matches = [i for i, g in enumerate(seg_groups) if g.name.upper() == gname]
                sm.key_segment[k] = matches[0] if matches else -1
            sm.key_level[k] = next((i for i, ids in enumerate(level_sets) if key in ids), 0 if key in root_keys else -1)
            sm.key_in_filter[k] = int(seg_filter is not None and key in seg_filter)
            if field_is_int and _CANONICAL_INT.match(key) and -(1 << 63) <= int(key) < (1 << 63):
                sm.key_is_int[k], sm.key_int[k] = 1, int(key)
        sm.n_levels = len(levels)
        sm.has_filter = int(seg_filter is not None)
        sm.prefix_len = len(pre)
        for j, b in enumerate(pre):
            sm.prefix[j] = b
        if red:
            seg_col = add_column(kind="segment", out_type=N.O_I32)
    rid_col = fid_col = -1
    if generate_record_id:
        fid_col = add_column(kind="file_id", out_type=N.O_I32)
        f = N.CbxField()
        f.kind, f.out_type, f.segment, f.column = N.K_FILE_ID, N.O_I32, -1, fid_col
        fields.append(f)
        rid_col = add_column(kind="record_id", out_type=N.O_I64)
        f = N.CbxField()
        f.kind, f.out_type, f.segment, f.column = N.K_RECORD_ID, N.O_I64, -1, rid_col
        fields.append(f)
    for lv in range(len(levels) if opts.has_segments else 0):
        c = add_column(kind="seg_id", out_type=N.O_STRING)
        opts.segments.level_column[lv] = c
        seg_id_cols.append(c)
    for lv in range(len(levels) if opts.has_segments else 0, N.CBX_MAX_SEG_LEVELS):
        opts.segments.level_column[lv] = -1
    opts.n_columns = len(columns)
    opts.file_id = file_id
    opts.window_bytes = window_bytes
    opts.segment_column = seg_col
    opts.jit_min_records = jit_min_records
    # 0 Arrow large-string, 1 string views, 2 Arrow Utf8 (int32 offsets, count pass + one decode pass)
    opts.string_views = int(string_views) if string_views in (0, 1, 2) else 1
    # the byte table: the code page (EBCDIC), the charset (ASCII wrapper), or for a US-ASCII copybook
    # decodeAsciiString's own mapping (bytes < 32 and >= 128 -> ' ') -- its strings decode through
    # ascii_lut on the device; the table serves the segment-id match (segment_key)
    if _charset_strings(cb):
        table = ascii_charset_table(cb.ascii_charset)
    elif cb.data_encoding == cbk.ASCII:
        table = [b if 32 <= b < 128 else 0x20 for b in range(256)]
    else:
        table = lut_for(cb.code_page)
    lut = utf8_lut(table)
    for i in range(256):
        opts.lut[i] = int(lut[i])
    plan = DecodePlan(cb, fields, arrays, columns, opts, field_of_node, array_of_node, seg_groups,
                      seg_col, rid_col, fid_col, seg_id_cols)
    if walk:
        plan.walk = walk_tables(plan, variable_size_occurs, has_segments=bool(red))
    return plan


@dataclass
class WalkTables:
    nodes: List[N.CbxWalkNode]
    arrays: List[N.CbxWalkArray]
    handlers: List[N.CbxWalkHandler]
    root: int
    variable_size_occurs: bool


def walk_tables(plan: DecodePlan, variable_size_occurs: bool, has_segments: bool) -> WalkTables:
    """The copybook as cbx_walk_node records (DFS, child / sibling links): what extractRecord walks
    (RecordExtractors.scala:49-183), with each DEPENDING ON name a dependee slot (dependFields) and
    each array's occurs_mappings handlers (dependingOnHandlers)."""
    cb = plan.copybook
    nodes: List[N.CbxWalkNode] = []
    dep_slots: Dict[str, int] = {}
    stmts: List[cbk.Statement] = []

    def slot_of(name: str) -> int:
        if name not in dep_slots:
            if len(dep_slots) >= 8:
                raise UnsupportedLayout("more than 8 DEPENDING ON names")
            dep_slots[name] = len(dep_slots)
        return dep_slots[name]

    def add(st: cbk.Statement) -> int:
        i = len(nodes)
        nd = N.CbxWalkNode()
        nodes.append(nd)
        stmts.append(st)
        is_group = isinstance(st, cbk.Group)
        nd.kind = N.W_GROUP if is_group else N.W_PRIM
        nd.next = nd.child = -1
        nd.field = -1 if is_group else plan.field_of_node.get(id(st), -1)
        nd.array = plan.array_of_node.get(id(st), -1) if st.is_array else -1
        nd.flags = (N.W_REDEFINED if st.is_redefined else 0) | (N.W_REDEFINES if st.redefines is not None else 0)
        nd.data_size, nd.actual_size = st.data_size, st.actual_size
        nd.segment = plan.segment_groups.index(st) if (is_group and st.is_segment_redefine and has_segments) else -1
        nd.dep_slot = slot_of(st.name) if (not is_group and st.is_dependee) else -1
        if is_group:
            prev = -1
            for c in st.children:
                ci = add(c)
                if prev < 0:
                    nodes[i].child = ci
                else:
                    nodes[prev].next = ci
                prev = ci
        return i

    root = add(cb.ast)
    arrays: List[N.CbxWalkArray] = []
    handlers: List[N.CbxWalkHandler] = []
    key_ids: Dict[str, int] = {}
    for ai in range(len(plan.arrays)):
        st = next(s for s in stmts if plan.array_of_node.get(id(s)) == ai)
        wa = N.CbxWalkArray()
        wa.dep_slot = dep_slots.get(st.depending_on, -1) if st.depending_on is not None else -1
        wa.h_begin = len(handlers)
        for key, value in st.depending_on_handlers.items():
            kb = key.encode("utf-8")
            if len(kb) > 64:
                raise UnsupportedLayout("occurs_mappings key longer than 64 bytes")
            h = N.CbxWalkHandler()
            h.key_id = key_ids.setdefault(key, len(key_ids))
            h.key_len, h.value = len(kb), int(value)
            for j, b in enumerate(kb):
                h.key[j] = b
            handlers.append(h)
        wa.h_end = len(handlers)
        arrays.append(wa)
    return WalkTables(nodes, arrays, handlers, root, variable_size_occurs)


def _iter_prims(g: cbk.Group):
    for c in g.children:
        if isinstance(c, cbk.Group):
            yield from _iter_prims(c)
        else:
            yield c


class NativePlan:
    """Owns a `cbx_plan*` built from a DecodePlan."""

    def __init__(self, plan: DecodePlan):
        L = N.load()
        self.plan = plan
        self._fields = (N.CbxField * len(plan.fields))(*plan.fields)
        self._arrays = (N.CbxArray * max(1, len(plan.arrays)))(*plan.arrays) if plan.arrays else None
        h = ctypes.c_void_p()
        rc = L.cbx_plan_create(ctypes.addressof(self._fields), len(plan.fields),
                               ctypes.addressof(self._arrays) if self._arrays is not None else None,
                               len(plan.arrays), ctypes.byref(plan.options), ctypes.byref(h))
        N.check(rc)
        self.handle = h
        w = plan.walk
        if w is not None:
            self._wnodes = (N.CbxWalkNode * len(w.nodes))(*w.nodes)
            self._warr = (N.CbxWalkArray * max(1, len(w.arrays)))(*w.arrays)
            self._whand = (N.CbxWalkHandler * max(1, len(w.handlers)))(*w.handlers)
            N.check(L.cbx_plan_set_walk(h, ctypes.addressof(self._wnodes), len(w.nodes), w.root,
                                        ctypes.addressof(self._warr), ctypes.addressof(self._whand), len(w.handlers),
                                        int(w.variable_size_occurs)))

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            N.load().cbx_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
