"""TEST INFRASTRUCTURE ONLY: ctypes harness around the C oracle (oracle/cobrix_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It serialises a parsed copybook AST into the oracle's node table, runs the restated
`extractRecord` walk and turns its event stream into nested rows (Spark `Row` shape, for
golden-JSON comparison) or into per-leaf columns (for GPU parity).
"""
from __future__ import annotations

import codecs
import ctypes
import os
import subprocess
from decimal import Context as _Ctx, Decimal as PyDecimal
_CTX = _Ctx(prec=200)
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from cobrix_amd import copybook as cbk
from cobrix_amd.codepages import lut_for
from cobrix_amd.schema import (ST_BINARY, ST_DECIMAL, ST_DOUBLE, ST_FLOAT, ST_INT, ST_LONG,
                               ST_STRING, spark_type)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libcobrix_oracle.so")


class OraNode(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "kind", "first_child", "next_sibling", "name_id", "name_upper_id", "depending_on_id",
        "is_array", "occurs_min", "occurs_max", "is_redefined", "has_redefines", "is_filler",
        "is_segment_redefine", "is_dependee", "data_size", "actual_size", "tclass", "enc",
        "compact", "precision", "scale", "scale_factor", "explicit_decimal", "is_signed",
        "sign_separate", "handlers_begin", "handlers_end")]


class OraHandler(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint16 * 64), ("key_len", ctypes.c_int32), ("value", ctypes.c_int32)]


class OraOptions(ctypes.Structure):
    _fields_ = [("trimming", ctypes.c_int32), ("float_format", ctypes.c_int32),
                ("variable_size_occurs", ctypes.c_int32), ("utf16_big_endian", ctypes.c_int32),
                ("lut", ctypes.POINTER(ctypes.c_uint16)), ("ascii_lut", ctypes.POINTER(ctypes.c_uint16))]


EVENT_DTYPE = np.dtype([("rec", "<u4"), ("node", "<i4"), ("kind", "<i4"), ("isnull", "<i4"),
                        ("slot", "<i4"), ("stype", "<i4"), ("lo", "<i8"), ("hi", "<i8")])
EV_VALUE, EV_ARRAY, EV_SEGNULL, EV_CHILDREN = 1, 2, 3, 4
ORA_ALL_SEGMENTS = -3   # cobrix_oracle.h

_TRIM = {"none": 1, "left": 2, "right": 3, "both": 4}
_FP = {"IBM": 0, "IBM_LE": 1, "IEEE754": 2, "IEEE754_LE": 3}
_ENC = {cbk.EBCDIC: 0, cbk.ASCII: 1, cbk.UTF16: 2, cbk.HEX: 3, cbk.RAW: 4}
_COMP = {None: 0, cbk.COMP1: 1, cbk.COMP2: 2, cbk.COMP3: 3, cbk.COMP4: 4, cbk.COMP5: 5, cbk.COMP9: 9}

_lib = None


def build() -> str:
    """Compile the oracle (TEST INFRASTRUCTURE)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        L.ora_decode_fixed.argtypes = [P, ctypes.c_int32, P, P, P, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P, ctypes.c_int32,
                                       P, ctypes.c_int64, P, P, ctypes.c_int64, P]
        L.ora_extract_var.argtypes = [P, ctypes.c_int32, P, P, P, P, P, P, ctypes.c_int64, ctypes.c_int32,
                                      P, ctypes.c_int64, P, P, ctypes.c_int64, P]
        L.ora_extract_record.argtypes = [P, ctypes.c_int32, P, P, P, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_uint32, P, ctypes.c_int64, P, P,
                                         ctypes.c_int64, P]
        L.ora_frame_rdw.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, P, P, ctypes.c_int64, P]
        L.ora_frame_rdw.restype = ctypes.c_int64
        L.ora_frame_text.argtypes = [P, ctypes.c_int64, ctypes.c_int32, P, P, ctypes.c_int64, P]
        L.ora_frame_text.restype = ctypes.c_int64
        L.ora_sparse_index.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, P, P, P, P,
                                       ctypes.c_int64]
        L.ora_sparse_index.restype = ctypes.c_int64
        L.ora_decode_field.argtypes = [P, P, P, ctypes.c_int32, P, P, ctypes.c_int64, P]
        L.ora_extract_hier.argtypes = [P, ctypes.c_int32, P, P, ctypes.c_int32, P, P, P, P, P, P, P, P, P, P,
                                       ctypes.c_int32, ctypes.c_uint32, P, ctypes.c_int64, P, P, ctypes.c_int64, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleAst:
    """Node table for one copybook (DFS order, index 0 = the root group)."""

    def __init__(self, cb: cbk.Copybook, occurs_handlers_keys=None):
        self.cb = cb
        self.stmts: List[cbk.Statement] = []
        self.names: Dict[str, int] = {}
        nodes: List[OraNode] = []
        handlers: List[OraHandler] = []

        def intern(s: str) -> int:
            if s not in self.names:
                self.names[s] = len(self.names)
            return self.names[s]

        def add(st: cbk.Statement) -> int:
            idx = len(nodes)
            nd = OraNode()
            nodes.append(nd)
            self.stmts.append(st)
            nd.kind = 0 if isinstance(st, cbk.Group) else 1
            nd.first_child = -1
            nd.next_sibling = -1
            nd.name_id = intern(st.name)
            nd.name_upper_id = intern(st.name.upper())
            nd.depending_on_id = intern(st.depending_on) if st.depending_on is not None else -1
            nd.is_array = int(st.is_array)
            nd.occurs_min = st.array_min_size
            nd.occurs_max = st.array_max_size
            nd.is_redefined = int(st.is_redefined)
            nd.has_redefines = int(st.redefines is not None)
            nd.is_filler = int(st.is_filler)
            nd.data_size = st.data_size
            nd.actual_size = st.actual_size
            nd.handlers_begin = len(handlers)
            for k, v in st.depending_on_handlers.items():
                h = OraHandler()
                u = [ord(ch) for ch in k][:64]
                for i, x in enumerate(u):
                    h.key[i] = x
                h.key_len = len(u)
                h.value = v
                handlers.append(h)
            nd.handlers_end = len(handlers)
            if isinstance(st, cbk.Group):
                nd.is_segment_redefine = int(st.is_segment_redefine)
                prev = -1
                for c in st.children:
                    ci = add(c)
                    if prev < 0:
                        nodes[idx].first_child = ci
                    else:
                        nodes[prev].next_sibling = ci
                    prev = ci
            else:
                d = st.dtype
                nd.is_dependee = int(st.is_dependee)
                if isinstance(d, cbk.AlphaNumeric):
                    nd.tclass, nd.enc = 1, _ENC[d.enc]
                else:
                    nd.tclass = 2 if isinstance(d, cbk.Integral) else 3
                    nd.enc = _ENC[d.enc]
                    nd.compact = _COMP[d.compact]
                    nd.precision = d.precision
                    nd.is_signed = int(d.sign_position is not None)
                    nd.sign_separate = int(d.is_sign_separate)
                    if isinstance(d, cbk.Decimal):
                        nd.scale, nd.scale_factor = d.scale, d.scale_factor
                        nd.explicit_decimal = int(d.explicit_decimal)
            return idx

        add(cb.ast)
        self.nodes = (OraNode * len(nodes))(*nodes)
        self.handlers = (OraHandler * max(1, len(handlers)))(*handlers) if handlers else (OraHandler * 1)()
        self.index = {id(s): i for i, s in enumerate(self.stmts)}
        self._lut = np.array(lut_for(cb.code_page), dtype=np.uint16)
        self.opts = OraOptions()
        self.opts.trimming = _TRIM[cb.string_trimming]
        self.opts.float_format = _FP[cb.floating_point_format]
        self.opts.utf16_big_endian = int(cb.is_utf16_big_endian)
        self.opts.lut = self._lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))
        if cb.ascii_charset and codecs.lookup(cb.ascii_charset).name != "ascii":
            # Java's single-byte charset tables, as Python's codec registry holds them
            whole = bytes(range(256)).decode(cb.ascii_charset, errors="replace")
            self._ascii_lut = np.array([ord(c) for c in whole], dtype=np.uint16)
            self.opts.ascii_lut = self._ascii_lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))

    def node_of(self, st: cbk.Statement) -> int:
        return self.index[id(st)]

    def max_events_per_record(self) -> int:
        def cnt(st):
            if isinstance(st, cbk.Group):
                inner = sum(cnt(c) for c in st.children) + 1
            else:
                inner = 1
            return inner * st.array_max_size + (1 if st.is_array else 0)
        return cnt(self.cb.ast) + 4

    def max_heap_per_record(self) -> int:
        return max(16, self.cb.record_size * 3 + 16)


class OracleResult:
    def __init__(self, ast: OracleAst, events: np.ndarray, heap: bytes, n_rec: int):
        self.ast, self.events, self.heap, self.n_rec = ast, events, heap, n_rec


def decode_fixed(cb: cbk.Copybook, data: bytes, record_size: Optional[int] = None,
                 start_offset: int = 0, end_offset: int = 0, variable_size_occurs: bool = False,
                 segment_field: Optional[str] = None, segment_redefine_map: Optional[Dict[str, str]] = None,
                 ast: Optional[OracleAst] = None) -> OracleResult:
    """Fixed-length file decode: one record per `stride` bytes (CobolScanners.scala:77-94)."""
    ast = ast or OracleAst(cb)
    rec_len = record_size if record_size is not None else cb.record_size
    stride = rec_len + start_offset + end_offset
    n_rec = len(data) // stride
    ast.opts.variable_size_occurs = int(variable_size_occurs)
    ev_cap = max(1, n_rec * ast.max_events_per_record())
    ev = np.zeros(ev_cap, dtype=EVENT_DTYPE)
    heap_cap = max(64, n_rec * ast.max_heap_per_record())
    heap = np.zeros(heap_cap, dtype=np.uint8)
    n_ev = ctypes.c_int64(0)
    hl = ctypes.c_int64(0)
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    seg_idx, seg_off, keys = -1, 0, (OraHandler * 1)()
    nkeys = 0
    if segment_field is not None:
        f = cb.get_field_by_name(segment_field)
        seg_idx, seg_off = ast.node_of(f), f.offset
        items = list((segment_redefine_map or {}).items())
        keys = (OraHandler * max(1, len(items)))()
        for i, (k, grp) in enumerate(items):
            u = [ord(ch) for ch in k][:64]
            for j, x in enumerate(u):
                keys[i].key[j] = x
            keys[i].key_len = len(u)
            keys[i].value = ast.names.get(cbk._transform_identifier(grp).upper(), -2)
        nkeys = len(items)
    r = lib().ora_decode_fixed(ctypes.addressof(ast.nodes), 0, ctypes.addressof(ast.handlers),
                               ctypes.addressof(ast.opts), _ptr(buf), n_rec, stride, start_offset,
                               seg_idx, seg_off, ctypes.addressof(keys), nkeys, _ptr(ev), ev_cap,
                               ctypes.byref(n_ev), _ptr(heap), heap_cap, ctypes.byref(hl))
    if r != 0:
        raise RuntimeError(f"oracle decode failed: {r}")
    return OracleResult(ast, ev[:n_ev.value].copy(), heap[:hl.value].tobytes(), n_rec)


def decode_records(cb: cbk.Copybook, records: Sequence[bytes], start_offset: int = 0,
                   variable_size_occurs: bool = False, active_segments: Optional[Sequence[Optional[str]]] = None,
                   ast: Optional[OracleAst] = None) -> OracleResult:
    """Decode a list of variable-length record payloads (VarLenNestedIterator.fetchNext).
    active_segments: per record the active segment redefine (others decode to null), or "*" for
    every segment redefine decoded (the hierarchical reader)."""
    ast = ast or OracleAst(cb)
    ast.opts.variable_size_occurs = int(variable_size_occurs)
    n_rec = len(records)
    ev_cap = max(1, n_rec * ast.max_events_per_record())
    ev = np.zeros(ev_cap, dtype=EVENT_DTYPE)
    alts = 1 + (len(cb.all_segment_redefines()) if active_segments == "*" else 0)   # every alternative decodes
    heap_cap = max(64, sum(len(r) for r in records) * 3 * alts + 64 * n_rec + 64)
    heap = np.zeros(heap_cap, dtype=np.uint8)
    n_ev = ctypes.c_int64(0)
    hl = ctypes.c_int64(0)
    L = lib()
    for i, rec in enumerate(records):
        buf = np.frombuffer(rec, dtype=np.uint8) if len(rec) else np.zeros(1, np.uint8)
        act = -1
        if active_segments == "*":
            act = ORA_ALL_SEGMENTS
        elif active_segments is not None and active_segments[i]:
            act = ast.names.get(active_segments[i].upper(), -2)
        r = L.ora_extract_record(ctypes.addressof(ast.nodes), 0, ctypes.addressof(ast.handlers),
                                 ctypes.addressof(ast.opts), _ptr(buf), len(rec), start_offset, act, i,
                                 _ptr(ev), ev_cap, ctypes.byref(n_ev), _ptr(heap), heap_cap,
                                 ctypes.byref(hl))
        if r != 0:
            raise RuntimeError(f"oracle decode failed: {r}")
    return OracleResult(ast, ev[:n_ev.value].copy(), heap[:hl.value].tobytes(), n_rec)


def decode_var(cb: cbk.Copybook, data: bytes, rec_off: np.ndarray, rec_len: np.ndarray,
               active_segments: Optional[Sequence[Optional[str]]] = None, start_offset: int = 0,
               ast: Optional[OracleAst] = None) -> OracleResult:
    """decode_records over framed payloads of one buffer, in one C call (no per-record ctypes)."""
    ast = ast or OracleAst(cb)
    n_rec = len(rec_off)
    ev_cap = max(1, n_rec * ast.max_events_per_record())
    ev = np.zeros(ev_cap, dtype=EVENT_DTYPE)
    heap_cap = max(64, int(np.sum(rec_len)) * 3 + 64 * n_rec + 64)
    heap = np.zeros(heap_cap, dtype=np.uint8)
    act = None
    if active_segments is not None:
        act = np.array([ast.names.get(s.upper(), -2) if s else -1 for s in active_segments], dtype=np.int32)
    off = np.ascontiguousarray(rec_off, dtype=np.int64)
    ln = np.ascontiguousarray(rec_len, dtype=np.int32)
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    n_ev, hl = ctypes.c_int64(0), ctypes.c_int64(0)
    r = lib().ora_extract_var(ctypes.addressof(ast.nodes), 0, ctypes.addressof(ast.handlers),
                              ctypes.addressof(ast.opts), _ptr(buf), _ptr(off), _ptr(ln),
                              _ptr(act) if act is not None else None, n_rec, start_offset, _ptr(ev), ev_cap,
                              ctypes.byref(n_ev), _ptr(heap), heap_cap, ctypes.byref(hl))
    if r != 0:
        raise RuntimeError(f"oracle decode failed: {r}")
    return OracleResult(ast, ev[:n_ev.value].copy(), heap[:hl.value].tobytes(), n_rec)


def frame_rdw(data: bytes, big_endian: bool = False, adjustment: int = 0, file_header_bytes: int = 0,
              file_footer_bytes: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    cap = len(data) // 1 + 1
    off = np.zeros(cap, np.int64)
    ln = np.zeros(cap, np.int32)
    eo = ctypes.c_int64(0)
    n = lib().ora_frame_rdw(_ptr(buf), len(data), int(big_endian), adjustment, file_header_bytes,
                            file_footer_bytes, _ptr(off), _ptr(ln), cap, ctypes.byref(eo))
    if n < 0:
        raise RuntimeError(f"RDW framing error {n} at offset {eo.value}")
    return off[:n].copy(), ln[:n].copy()


def frame_text(data: bytes, record_size: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """TextRecordExtractor restated (cobrix_oracle.c ora_frame_text): (offsets, payload lengths,
    virtual stream length -- records may reach past len(data) into the reference's zero fill)."""
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    cap = len(data) + 2
    off = np.zeros(cap, np.int64)
    ln = np.zeros(cap, np.int32)
    vb = ctypes.c_int64(0)
    n = lib().ora_frame_text(_ptr(buf), len(data), record_size, _ptr(off), _ptr(ln), cap, ctypes.byref(vb))
    assert n <= cap
    return off[:n].copy(), ln[:n].copy(), vb.value


def sparse_index(data: bytes, big_endian: bool = False, adjustment: int = 0,
                 file_header_bytes: int = 0, file_footer_bytes: int = 0,
                 records_per_entry: Optional[int] = None, size_per_entry_mb: Optional[int] = None,
                 is_root: Optional[np.ndarray] = None) -> List[Tuple[int, int, int]]:
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    cap = len(data) // 4 + 2
    f = np.zeros(cap, np.int64)
    t = np.zeros(cap, np.int64)
    r = np.zeros(cap, np.int64)
    roots = None if is_root is None else np.ascontiguousarray(is_root, dtype=np.int32)
    n = lib().ora_sparse_index(_ptr(buf), len(data), int(big_endian), adjustment, file_header_bytes,
                               file_footer_bytes, records_per_entry or 0, size_per_entry_mb or 0,
                               _ptr(roots) if roots is not None else None, _ptr(f), _ptr(t), _ptr(r), cap)
    if n < 0:
        raise RuntimeError(f"sparse index error {n}")
    return [(int(f[i]), int(t[i]), int(r[i])) for i in range(n)]


# --------------------------------------------------------------------------------------
# Event stream -> Python values
# --------------------------------------------------------------------------------------

def event_value(e, heap: bytes, stype_info=None):
    if e["isnull"]:
        return None
    st = int(e["stype"])
    lo, hi = int(e["lo"]), int(e["hi"])
    if st in (ST_INT, ST_LONG):
        return lo
    if st == ST_DECIMAL:
        u = (hi << 64) | (lo & 0xFFFFFFFFFFFFFFFF)
        return u
    if st == ST_FLOAT:
        return np.array([lo & 0xFFFFFFFF], dtype=np.uint32).view(np.float32)[0]
    if st == ST_DOUBLE:
        return np.array([lo & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64).view(np.float64)[0]
    if st == ST_STRING:
        return heap[lo:lo + hi].decode("utf-8")
    if st == ST_BINARY:
        return heap[lo:lo + hi]
    raise ValueError(st)


def rows(res: OracleResult, collapse_root: bool = True) -> List[dict]:
    """Rebuild nested rows from the event stream (RecordHandler.create + applyRecordPostProcessing)."""
    ast = res.ast
    ev = res.events
    heap = res.heap
    out: List[dict] = []
    pos = 0
    n = len(ev)

    def dec_value(st, e):
        v = event_value(e, heap)
        if v is not None and int(e["stype"]) == ST_DECIMAL:
            t, p, s = spark_type(st)
            v = PyDecimal(v).scaleb(-s, context=_CTX)
        return v

    def walk_group(g: cbk.Group) -> dict:
        nonlocal pos
        d = {}
        for c in g.children:
            if c.is_array:
                e = ev[pos]
                assert e["kind"] == EV_ARRAY and e["node"] == ast.node_of(c), (pos, c.name)
                pos += 1
                cnt = int(e["lo"])
                vals = []
                for _ in range(cnt):
                    if isinstance(c, cbk.Group):
                        vals.append(walk_group(c))
                    else:
                        vals.append(dec_value(c, ev[pos]))
                        pos += 1
                val = vals
            elif isinstance(c, cbk.Group):
                e = ev[pos] if pos < n else None
                if e is not None and e["kind"] == EV_SEGNULL and e["node"] == ast.node_of(c):
                    pos += 1
                    val = None
                else:
                    val = walk_group(c)
            else:
                e = ev[pos]
                assert e["kind"] == EV_VALUE and e["node"] == ast.node_of(c), (pos, c.name, e)
                pos += 1
                val = dec_value(c, e)
            if not c.is_filler and not c.is_child_segment:
                d[c.name] = val
        return d

    for _r in range(res.n_rec):
        recs = []
        for g in res.ast.cb.ast.children:
            recs.append((g.name, walk_group(g)))
        if collapse_root:
            row = {}
            for _, v in recs:
                row.update(v)
        else:
            row = {k: v for k, v in recs}
        out.append(row)
    return out


def _iter_leaves(g):
    """Primitive nodes in AST (walk) order."""
    for c in g.children:
        if isinstance(c, cbk.Group):
            yield from _iter_leaves(c)
        else:
            yield c


def columns(res: OracleResult) -> Dict[int, Dict[str, np.ndarray]]:
    """Per-leaf columnar view of the event stream (slot-major like the GPU output).

    Returns {node id: {"rec", "slot", "valid", "lo", "hi", "bytes"}} for every primitive node that
    emitted values, and {node id: {"rec", "slot", "count"}} for OCCURS nodes."""
    ev = res.events
    out: Dict[int, Dict[str, np.ndarray]] = {}
    vals = ev[ev["kind"] == EV_VALUE]
    arrs = ev[ev["kind"] == EV_ARRAY]
    order = np.argsort(vals["node"], kind="stable")
    vals = vals[order]
    nodes, starts = np.unique(vals["node"], return_index=True)
    ends = list(starts[1:]) + [len(vals)]
    for nid, s, e in zip(nodes, starts, ends):
        v = vals[s:e]
        d = {"rec": v["rec"].astype(np.int64), "slot": v["slot"].astype(np.int64),
             "valid": v["isnull"] == 0, "lo": v["lo"], "hi": v["hi"], "stype": v["stype"]}
        out[int(nid)] = d
    for nid in np.unique(arrs["node"]):
        a = arrs[arrs["node"] == nid]
        out[int(nid)] = {"rec": a["rec"].astype(np.int64), "slot": a["slot"].astype(np.int64),
                         "count": a["lo"]}
    return out
