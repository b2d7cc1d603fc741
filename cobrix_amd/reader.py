"""Reader facade mirroring Cobrix's `FixedLenNestedReader` / `VarLenNestedReader` over the GPU path.

Reference interfaces (CP = cobol-parser/src/main/scala/za/co/absa/cobrix/cobol/):
  * FixedLenNestedReader  CP/reader/FixedLenNestedReader.scala:43-144  (getRecordSize,
    checkBinaryDataValidity, getRecordIterator -> one extractRecord per record)
  * VarLenNestedReader    CP/reader/VarLenNestedReader.scala:46-310   (generateIndex,
    getRecordIterator over a SimpleStream with RDW headers)
  * ReaderParameters      CP/reader/parameters/ReaderParameters.scala:65-103
The GPU decodes a whole batch (split / partition) per call instead of one record per call;
`DecodedBatch` holds the columnar result and can rebuild the reference's nested rows.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from decimal import Context, Decimal
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import copybook as cbk
from . import native as N
from .plan import DecodePlan, NativePlan, NeedsWalk, build_plan
from .schema import ST_DECIMAL, spark_schema

_CTX = Context(prec=200)


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise N.NativeLibraryError("the Cobrix GPU path needs a ROCm device (torch.cuda.is_available() is False)")
    return torch


@dataclass
class ReaderParameters:
    """Subset of ReaderParameters (ReaderParameters.scala:65-103) that shapes the decode path."""
    is_ebcdic: bool = True
    ebcdic_code_page: str = "common"
    ebcdic_code_page_table: Optional[List[int]] = None   # ebcdic_code_page_class: a custom CodePage's table
    floating_point_format: str = "IBM"
    is_utf16_big_endian: bool = True
    ascii_charset: str = ""
    variable_size_occurs: bool = False
    record_length: Optional[int] = None
    is_record_sequence: bool = False
    is_text: bool = False                          # LF / CRLF separated records (TextRecordExtractor)
    is_rdw_big_endian: bool = False
    is_rdw_part_rec_length: bool = False
    rdw_adjustment: int = 0
    enable_indexes: bool = True
    input_split_records: Optional[int] = None
    input_split_size_mb: Optional[int] = None
    hdfs_default_block_size_mb: Optional[int] = None   # getSplitSizeMB fallback (VarLenNestedReader.scala:237-243)
    start_offset: int = 0
    end_offset: int = 0
    file_start_offset: int = 0
    file_end_offset: int = 0
    generate_record_id: bool = False
    schema_policy: str = "keep_original"          # or "collapse_root"
    string_trimming_policy: str = "both"
    segment_field: Optional[str] = None
    segment_id_redefine_map: Dict[str, str] = field(default_factory=dict)
    segment_id_filter: Optional[List[str]] = None
    segment_id_levels: List[str] = field(default_factory=list)   # segment_id_level0.. / segment_id_root
    segment_id_prefix: str = ""
    # segment-children: child segment redefine -> parent (MultisegmentParameters.fieldParentMap)
    segment_redefine_parents: Dict[str, str] = field(default_factory=dict)
    drop_group_fillers: bool = False
    drop_value_fillers: bool = True
    non_terminals: Sequence[str] = ()
    occurs_mappings: Dict[str, Dict[str, int]] = field(default_factory=dict)
    debug_fields_policy: str = "none"             # DebugFieldsPolicy: none / hex / raw
    window_bytes: int = 0
    # fixed-length batches of at least this many records run a copybook-specialised kernel
    # (hipRTC, compiled once per layout): 0 = library default, < 0 = never
    jit_min_records: int = 0
    # output layout of string columns: Arrow large-string (offsets, two-pass placement) or Arrow
    # string views (one pass: every value written once by the decode kernel; cobrix_hip.h)
    string_views: bool = False
    # Arrow Utf8 layout (cbx_plan_options.string_views = 2): int32 offsets relative to each slot's
    # region, a count pass + device scan, then every offset and payload byte written once at its final
    # place by the decode kernel (no placement pass); takes precedence over string_views.  The record
    # walk writes views and converts them (cbx_views_to_utf8)
    string_utf8: bool = False
    # record_length_field (VRLRecordReader.fetchRecordUsingRecordLengthField): records framed by a length
    # field inside them instead of RDW headers (not with is_record_sequence)
    record_length_field: Optional[str] = None
    # OCCURS DEPENDING ON arrays of numeric elements in the list layout (child elements packed per
    # record, absent elements unwritten; cobrix_hip.h CBX_F_LIST) instead of one slot row per element
    occurs_lists: bool = False
    # with_input_file_name_col (ReaderParameters.inputFileNameColumn): a string column holding the
    # name of the file each record came from (RecordExtractors.applyRecordPostProcessing)
    input_file_name_column: str = ""
    # debug_ignore_file_size (CobolParametersParser.PARAM_DEBUG_IGNORE_FILE_SIZE): a fixed-length file
    # whose size is not a multiple of the record size (record_length included) is read anyway, its
    # partial last record dropped, instead of being rejected (CobolScanners.scala:86-90)
    debug_ignore_file_size: bool = False


@dataclass
class SparseIndexEntry:
    """SparseIndexEntry (CP/reader/index/entry/SparseIndexEntry.scala:19)."""
    offset_from: int
    offset_to: int
    file_id: int
    record_index: int


class DecodedBatch:
    """Columnar decode of a batch of records (device tensors) + row reconstruction."""

    def __init__(self, plan: DecodePlan, n_rec: int, cols: List[Dict[str, Any]], first_record_id: int,
                 collapse_root: bool, generate_record_id: bool):
        self.plan, self.n_rec, self.cols = plan, n_rec, cols
        self.first_record_id = first_record_id
        self.collapse_root = collapse_root
        self.generate_record_id = generate_record_id
        # with_input_file_name_col: (column name, the file's name) -- a per-batch constant column
        self.input_file: Optional[Tuple[str, str]] = None

    def generated(self, column, r=None) -> List[Tuple[str, Any]]:
        """The generated leading fields of the rows: (schema name, value) pairs, value = column(ci)
        for a decoded column, the file name for the input-file-name column.  Names follow the Spark
        schema (File_Id, Record_Id, the file column, Seg_Id0..; SC/schema/CobolSchema.scala:99-110),
        values follow the Row (RecordExtractors.applyRecordPostProcessing, :409-451) -- which without
        generate_record_id puts the segment ids BEFORE the file name, so with both present the
        Row's values sit one position off the schema's names, as in the reference."""
        plan = self.plan
        gen = [("File_Id", column(plan.file_id_column)), ("Record_Id", column(plan.record_id_column))] \
            if self.generate_record_id else []
        segs = [(f"Seg_Id{lv}", column(ci)) for lv, ci in enumerate(plan.seg_id_columns)]
        if self.input_file is None:
            return gen + segs
        fname = (self.input_file[0], ("file", self.input_file[1]))
        if self.generate_record_id or not segs:
            return gen + [fname] + segs
        names = [fname[0]] + [n for n, _ in segs]
        values = [v for _, v in segs] + [fname[1]]
        return list(zip(names, values))

    # ---- host views
    def _list_dense(self, ci: int):
        """A list-layout column as dense slot rows: (values [n_slots * n_rec (, 2)], validity
        [n_slots, n_rec]) -- element j of record r at child index offsets[r] + j when j < count[r] (a valid count)."""
        info = self.plan.columns[ci]
        ar = self.plan.arrays[info.list_array]
        n, m = self.n_rec, info.n_slots
        off = self.cols[ar.offsets_column]["values"].cpu().numpy()[:n].astype(np.int64)
        cnt = self.cols[ar.count_column]["values"].cpu().numpy()[:n].astype(np.int64)
        cbits = np.unpackbits(self.cols[ar.count_column]["validity"].cpu().numpy().view(np.uint8), bitorder="little")
        cnt = np.where(cbits[:n].astype(bool), cnt, 0)   # no elements where the array's segment is inactive
        child = self.cols[ci]["values"].cpu().numpy()
        wide = info.out_type == N.O_DEC128
        if wide:
            child = child.reshape(-1, 2)
        bits = np.unpackbits(self.cols[ci]["validity"].cpu().numpy().view(np.uint8), bitorder="little").astype(bool)
        j = np.arange(m, dtype=np.int64)
        idx = off[None, :] + j[:, None]                      # [slot, record]
        present = j[:, None] < cnt[None, :]
        safe = np.where(present, idx, 0)
        valid = present & bits[safe]
        vals = child[safe.reshape(-1)]
        if wide:
            vals = np.where(present.reshape(-1)[:, None], vals, 0)
        else:
            vals = np.where(present.reshape(-1), vals, 0)
        return vals, valid

    def host_column(self, ci: int) -> Dict[str, Any]:
        c = self.cols[ci]
        info = self.plan.columns[ci]
        pitch = (self.n_rec + 63) // 64
        out: Dict[str, Any] = {"validity": None, "values": None}
        if info.list_array >= 0:
            out["values"], out["validity"] = self._list_dense(ci)
            return out
        vb = c["validity"].cpu().numpy().view(np.uint64)
        bits = np.unpackbits(vb.view(np.uint8), bitorder="little").reshape(info.n_slots, pitch * 64)
        out["validity"] = bits[:, :self.n_rec].astype(bool)
        if c.get("views") is not None:
            vw = c["views"].cpu().numpy().reshape(info.n_slots, 64 * pitch, 16)[:, : self.n_rec]
            data = c["data"].cpu().numpy().tobytes()
            out["strings"] = [decode_views(vw[s], data, c["buffer_bytes"], s * c["capacity"]) for s in range(info.n_slots)]
        elif c.get("offsets") is not None:
            # slot s: offsets[s * (pitch + 1) .. + n_rec], absolute into data (slot regions)
            out["offsets"] = c["offsets"].cpu().numpy().reshape(info.n_slots, 64 * pitch + 1)[:, : self.n_rec + 1]
            out["data"] = c["data"].cpu().numpy().tobytes()
        elif c.get("offsets32") is not None:
            # Utf8: int32 offsets relative to slot s's region -> absolute, as above
            o = c["offsets32"].cpu().numpy().reshape(info.n_slots, 64 * pitch + 1)[:, : self.n_rec + 1].astype(np.int64)
            out["offsets"] = o + (np.arange(info.n_slots, dtype=np.int64) * c["capacity"])[:, None]
            out["data"] = c["data"].cpu().numpy().tobytes()
        else:
            v = c["values"].cpu().numpy()
            if info.out_type == N.O_DEC128:
                v = v.reshape(info.n_slots, 64 * pitch, 2)[:, : self.n_rec].reshape(-1, 2)
            else:
                v = v.reshape(info.n_slots, 64 * pitch)[:, : self.n_rec].reshape(-1)
            out["values"] = v
        return out

    # ---- Arrow (the columnar bridge) ----
    def _slot_arrays(self, ci: int):
        """Per slot row of column ci: a pyarrow array of the n_rec records (values + validity bitmap,
        straight from the decode's buffers: string views / large-string offsets, unscaled decimals
        as decimal128, float bit patterns)."""
        import pyarrow as pa
        c = self.cols[ci]
        info = self.plan.columns[ci]
        n, pw = self.n_rec, (self.n_rec + 63) // 64
        pitch = 64 * pw
        ot = info.out_type
        if info.list_array >= 0:   # list layout: dense slot rows rebuilt from the child elements
            vals, valid = self._list_dense(ci)
            dense = np.zeros((info.n_slots, pw * 64), dtype=bool)
            dense[:, :n] = valid
            vbits = np.packbits(dense, axis=1, bitorder="little").view(np.uint64).reshape(info.n_slots, pw)
            vals = vals.reshape(info.n_slots, n, -1) if ot == N.O_DEC128 else vals.reshape(info.n_slots, n)
            padded = np.zeros((info.n_slots, pitch) + vals.shape[2:], dtype=vals.dtype)
            padded[:, :n] = vals
            c = {"values": _HostArray(padded.reshape(-1) if ot != N.O_DEC128 else padded.reshape(-1, 2))}
        else:
            vbits = c["validity"].cpu().numpy().view(np.uint64).reshape(info.n_slots, pw)
        out = []
        if "views" in c:
            views = c["views"].cpu().numpy().reshape(info.n_slots, pitch, 16)
            data = c["data"].cpu().numpy()
            cap, bb = c["capacity"], max(1, c["buffer_bytes"])
        elif "offsets" in c:
            offs = c["offsets"].cpu().numpy().reshape(info.n_slots, pitch + 1)
            data = c["data"].cpu().numpy()
        elif "offsets32" in c:
            offs = c["offsets32"].cpu().numpy().reshape(info.n_slots, pitch + 1)
            data = c["data"].cpu().numpy()
            cap = c["capacity"]
        else:
            vals = c["values"].cpu().numpy()
        for s in range(info.n_slots):
            valid = pa.py_buffer(vbits[s].tobytes())
            if "views" in c:
                region = data[s * cap:(s + 1) * cap]
                bufs = [pa.py_buffer(region[k:k + bb].tobytes()) for k in range(0, max(len(region), 1), bb)]
                typ = pa.string_view() if ot == N.O_STRING else pa.binary_view()
                arr = pa.Array.from_buffers(typ, n, [valid, pa.py_buffer(views[s, :n].tobytes())] + bufs)
            elif "offsets32" in c:   # Arrow Utf8 / Binary: the slot's own region, int32 offsets into it
                typ = pa.string() if ot == N.O_STRING else pa.binary()
                arr = pa.Array.from_buffers(typ, n, [valid, pa.py_buffer(offs[s, :n + 1].tobytes()),
                                                     pa.py_buffer(data[s * cap:(s + 1) * cap].tobytes())])
            elif "offsets" in c:
                typ = pa.large_string() if ot == N.O_STRING else pa.large_binary()
                arr = pa.Array.from_buffers(typ, n, [valid, pa.py_buffer(offs[s, :n + 1].tobytes()), pa.py_buffer(data.tobytes())])
            elif ot in (N.O_DEC64, N.O_DEC128):
                _, p_, s_ = info.stype
                if ot == N.O_DEC64:
                    lo = vals.reshape(info.n_slots, pitch)[s, :n].astype(np.int64)
                    w = np.stack([lo, lo >> 63], axis=1)
                else:
                    w = vals.reshape(info.n_slots, pitch, 2)[s, :n].astype(np.int64)
                arr = pa.Array.from_buffers(pa.decimal128(p_, s_), n, [valid, pa.py_buffer(np.ascontiguousarray(w).tobytes())])
            else:
                dt, typ = {N.O_I32: (np.int32, pa.int32()), N.O_I64: (np.int64, pa.int64()),
                           N.O_F32: (np.float32, pa.float32()), N.O_F64: (np.float64, pa.float64())}[ot]
                v = np.ascontiguousarray(vals.reshape(info.n_slots, pitch)[s, :n]).view(np.uint8)
                v = v.view(np.uint32 if dt in (np.int32, np.float32) else np.uint64)[:n] if v.size else v
                arr = pa.Array.from_buffers(typ, n, [valid, pa.py_buffer(np.ascontiguousarray(v).tobytes())])
            out.append(arr)
        return out

    def _arrow_builder(self, extra=None, null_segments: bool = True):
        """build(node, R, S, in_array): pyarrow array of node's values for the instances (record
        R[i], enclosing-array slot S[i]) -- groups -> structs (an inactive segment redefine -> null
        struct when null_segments), OCCURS -> lists of the records' element counts.  extra(node, R)
        may append (names, arrays) to a group's struct (hierarchical child segments)."""
        import pyarrow as pa
        plan = self.plan
        n = self.n_rec
        flat: Dict[int, Any] = {}

        def column(ci):
            if ci not in flat:
                parts = self._slot_arrays(ci)
                flat[ci] = parts[0] if len(parts) == 1 else pa.concat_arrays(parts)
            return flat[ci]

        counts: Dict[int, np.ndarray] = {}

        def count_of(ai):
            ci = plan.arrays[ai].count_column
            if ci not in counts:
                info = plan.columns[ci]
                v = self.cols[ci]["values"].cpu().numpy().reshape(info.n_slots, -1)[:, :n]
                # an invalid count cell (an array inside an inactive segment redefine the record walk
                # skips) holds no element count: no elements, as in _list_dense
                vb = np.unpackbits(self.cols[ci]["validity"].cpu().numpy().view(np.uint8), bitorder="little")
                ok = vb.reshape(info.n_slots, -1)[:, :n].astype(bool)
                counts[ci] = np.where(ok, v, 0).reshape(-1).astype(np.int64)   # slot s, record r -> s * n + r
            return counts[ci]

        seg_active = None
        if plan.segment_column >= 0 and null_segments:
            seg_active = self.cols[plan.segment_column]["values"].cpu().numpy()[:n].astype(np.int64)

        def build(node, R, S, in_array):
            if node.is_array and not in_array:
                ai = plan.array_of_node[id(node)]
                m = node.array_max_size
                cnt = count_of(ai)[(S if plan.columns[plan.arrays[ai].count_column].n_slots > 1 else 0) * n + R]
                j = np.concatenate([np.arange(k) for k in cnt]) if len(cnt) else np.zeros(0, np.int64)
                R2 = np.repeat(R, cnt)
                S2 = np.repeat(S, cnt) * m + j
                child = build(node, R2, S2, True)
                offs = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
                return pa.ListArray.from_arrays(pa.array(offs, pa.int32()), child)
            if isinstance(node, cbk.Group):
                names, kids = [], []
                for c in node.children:
                    if c.is_filler or c.is_child_segment:
                        continue
                    if isinstance(c, cbk.Group) or c.is_array or plan.field_of_node.get(id(c)) is not None:
                        names.append(c.name)
                        kids.append(build(c, R, S, False))
                if extra is not None:
                    xn, xa = extra(node, R)
                    names += xn
                    kids += xa
                mask = None
                if node.is_segment_redefine and null_segments:
                    si = plan.segment_groups.index(node)
                    mask = pa.array(seg_active[R] != si if seg_active is not None else np.ones(len(R), bool))
                return pa.StructArray.from_arrays(kids, names=names, mask=mask)
            fi = plan.field_of_node[id(node)]
            arr = column(plan.fields[fi].column)
            if len(R) == n and not S.any() and np.array_equal(R, np.arange(n)):
                return arr.slice(0, n)                       # the slot row itself, zero-copy
            if pa.types.is_string_view(arr.type) or pa.types.is_binary_view(arr.type):
                # no gather kernel for views in pyarrow: gathered OCCURS elements become large strings
                arr = arr.cast(pa.large_string() if pa.types.is_string_view(arr.type) else pa.large_binary())
            return arr.take(pa.array(S * n + R))

        build.column = column
        return build

    def to_arrow(self):
        """The batch as a pyarrow Table in the reference's Spark schema shape: groups -> structs
        (an inactive segment redefine -> null struct), OCCURS -> lists of the records' element
        counts (OCCURS DEPENDING ON), generated File_Id / Record_Id / Seg_IdN columns first."""
        import pyarrow as pa
        plan = self.plan
        n = self.n_rec
        build = self._arrow_builder()
        column = build.column
        R0 = np.arange(n, dtype=np.int64)
        S0 = np.zeros(n, dtype=np.int64)
        names, arrays = [], []
        for nm, v in self.generated(column):
            names.append(nm)
            arrays.append(_file_name_array(v[1], n) if isinstance(v, tuple) else v)
        for g in plan.copybook.ast.children:
            if not isinstance(g, cbk.Group):
                continue
            st = build(g, R0, S0, False)
            if self.collapse_root:
                for k in range(st.type.num_fields):
                    names.append(st.type.field(k).name)
                    arrays.append(st.field(k))
            else:
                names.append(g.name)
                arrays.append(st)
        return pa.Table.from_arrays(arrays, names=names)

    def _host(self, ci: int) -> Dict[str, Any]:
        cache = self.__dict__.setdefault("_host_cache", {})
        if ci not in cache:
            cache[ci] = self.host_column(ci)
        return cache[ci]

    def cell(self, ci: int, slot: int, r: int):
        """The Python value of column ci, slot, record r (None when null)."""
        c = self._host(ci)
        info = self.plan.columns[ci]
        if not c["validity"][slot, r]:
            return None
        v = slot * self.n_rec + r
        ot = info.out_type
        if ot in (N.O_STRING, N.O_BINARY) and "strings" in c:
            b = c["strings"][slot][r]
            return b.decode("utf-8") if ot == N.O_STRING else b
        if ot in (N.O_STRING, N.O_BINARY):
            off = c["offsets"][slot]
            b = c["data"][int(off[r]):int(off[r + 1])]
            return b.decode("utf-8") if ot == N.O_STRING else b
        x = c["values"][v]
        if ot == N.O_I32:
            return int(np.int32(x))
        if ot == N.O_I64:
            return int(np.int64(x))
        if ot == N.O_F32:
            return np.uint32(x).view(np.float32)
        if ot == N.O_F64:
            return np.uint64(x).view(np.float64)
        if ot == N.O_DEC64:
            u = int(np.int64(x))
        else:
            u = (int(np.int64(x[1])) << 64) | int(np.uint64(x[0]))
        return Decimal(u).scaleb(-info.stype[2], context=_CTX)

    def _row_builder(self, extra=None, null_segments: bool = True):
        """walk(group, r, idx): the dict RecordHandler.create builds for a group of record r
        (idx: enclosing OCCURS indices).  extra(group, r) may add entries (hierarchical children)."""
        plan = self.plan
        seg_col = plan.segment_column if null_segments else -1

        def walk(g: cbk.Group, r: int, idx: List[Tuple[int, int]]) -> dict:
            d = {}
            for c in g.children:
                if c.is_child_segment:
                    continue   # never in a row (hierarchical children come from `extra`)
                if c.is_array:
                    ai = plan.array_of_node[id(c)]
                    cci = plan.arrays[ai].count_column
                    cs = 0   # a count per enclosing element (record-walk plans)
                    if plan.columns[cci].n_slots > 1:
                        for i, m in idx:
                            cs = cs * m + i
                    cnt = int(np.int32(self._host(cci)["values"][cs * self.n_rec + r]))
                    vals = []
                    for i in range(cnt):
                        sub = idx + [(i, c.array_max_size)]
                        if isinstance(c, cbk.Group):
                            vals.append(walk(c, r, sub))
                        else:
                            vals.append(prim(c, r, sub))
                    val: Any = vals
                elif isinstance(c, cbk.Group):
                    if c.is_segment_redefine and seg_col >= 0:
                        si = plan.segment_groups.index(c)
                        active = int(np.int32(self._host(seg_col)["values"][r]))
                        val = walk(c, r, idx) if active == si else None
                    elif c.is_segment_redefine and null_segments:
                        val = None
                    else:
                        val = walk(c, r, idx)
                else:
                    val = prim(c, r, idx)
                if not c.is_filler and not c.is_child_segment:
                    d[c.name] = val
            if extra is not None:
                d.update(extra(g, r))
            return d

        def prim(p: cbk.Primitive, r: int, idx):
            fi = plan.field_of_node.get(id(p))
            if fi is None:
                return None
            slot = 0
            for i, m in idx:
                slot = slot * m + i
            return self.cell(plan.fields[fi].column, slot, r)

        return walk

    def to_rows(self) -> List[dict]:
        """Rebuild nested rows (RecordHandler.create + applyRecordPostProcessing)."""
        plan = self.plan
        walk = self._row_builder()
        rows = []
        for r in range(self.n_rec):
            recs = [(g.name, walk(g, r, [])) for g in plan.copybook.ast.children if isinstance(g, cbk.Group)]
            row: Dict[str, Any] = {}
            for nm, v in self.generated(lambda ci: ci):
                row[nm] = v[1] if isinstance(v, tuple) else self.cell(v, 0, r)
            if self.collapse_root:
                for _, v in recs:
                    row.update(v)
            else:
                row.update({k: v for k, v in recs})
            rows.append(row)
        return rows


def _file_name_array(name: str, n: int):
    """The input-file-name column of a batch as Arrow: one dictionary entry (the name) and n zero
    indices -- the value is constant per file, so the batch holds it once."""
    import pyarrow as pa
    return pa.DictionaryArray.from_arrays(pa.array(np.zeros(n, dtype=np.int32)), pa.array([name], pa.string()))


def _record_stream(cols: Sequence[Dict[str, Any]], stream) -> None:
    """Mark every tensor of a column table as used on `stream` (the caching allocator then keeps
    its memory until that stream's queued work is done)."""
    torch = _torch()
    for c in cols:
        for v in c.values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(stream)


def _alloc_columns(plan: DecodePlan, n_rec: int, slot_capacity: Sequence[int], device) -> Tuple[List[Dict[str, Any]], ctypes.Array]:
    """Caller-owned output buffers (cobrix_hip.h cbx_column): slot-major values, validity
    bitmaps, and for strings one Arrow large-string array per slot (regions of slot_capacity)."""
    torch = _torch()
    pitch_words = (n_rec + 63) // 64
    pitch = 64 * pitch_words          # values per slot row (cobrix_hip.h: padded to whole tiles)
    cols: List[Dict[str, Any]] = []
    cstructs = (N.CbxColumn * plan.n_columns)()
    for ci, info in enumerate(plan.columns):
        n = pitch * info.n_slots
        c: Dict[str, Any] = {"validity": torch.zeros(max(1, info.n_slots * pitch_words), dtype=torch.int64, device=device)}
        if info.out_type in (N.O_STRING, N.O_BINARY) and plan.options.string_views == 2:
            # Arrow Utf8: int32 offsets per slot (pitch + 1, relative to the slot's region) + regions
            cap = int(slot_capacity[ci])
            c["offsets32"] = torch.zeros(info.n_slots * (pitch + 1), dtype=torch.int32, device=device)
            c["data"] = torch.empty(max(1, cap * info.n_slots), dtype=torch.uint8, device=device)
            c["sizes"] = torch.zeros(info.n_slots, dtype=torch.int64, device=device)
            c["capacity"] = cap
            cstructs[ci].offsets = c["offsets32"].data_ptr()
            cstructs[ci].data = c["data"].data_ptr()
            cstructs[ci].data_capacity = cap
            cstructs[ci].data_sizes = c["sizes"].data_ptr()
        elif info.out_type in (N.O_STRING, N.O_BINARY) and plan.options.string_views:
            # string views: 16 bytes per value + per-slot regions of whole tiles (cobrix_hip.h)
            cap = int(slot_capacity[ci])
            c["views"] = torch.zeros(max(1, n * 16), dtype=torch.uint8, device=device)
            c["data"] = torch.empty(max(1, cap * info.n_slots), dtype=torch.uint8, device=device)
            c["capacity"] = cap
            c["tile_bytes"], c["buffer_bytes"] = view_geometry(cap, pitch_words)
            cstructs[ci].values = c["views"].data_ptr()
            cstructs[ci].data = c["data"].data_ptr()
            cstructs[ci].data_capacity = cap
        elif info.out_type in (N.O_STRING, N.O_BINARY):
            cap = int(slot_capacity[ci])
            c["offsets"] = torch.zeros(info.n_slots * (pitch + 1), dtype=torch.int64, device=device)
            c["data"] = torch.empty(max(1, cap * info.n_slots), dtype=torch.uint8, device=device)
            c["sizes"] = torch.zeros(info.n_slots, dtype=torch.int64, device=device)
            c["capacity"] = cap
            cstructs[ci].offsets = c["offsets"].data_ptr()
            cstructs[ci].data = c["data"].data_ptr()
            cstructs[ci].data_capacity = cap
            cstructs[ci].data_sizes = c["sizes"].data_ptr()
        elif info.list_array >= 0:
            # list layout: child elements, 64 * M per tile (M = max count rounded up to 64)
            w = N.OUT_WIDTH[info.out_type]
            dt = {4: torch.int32, 8: torch.int64, 16: torch.int64}[w]
            n_child = pitch * info.list_mpad
            c["values"] = torch.zeros(max(1, n_child * (2 if w == 16 else 1)), dtype=dt, device=device)
            c["validity"] = torch.zeros(max(1, pitch_words * info.list_mpad), dtype=torch.int64, device=device)
            cstructs[ci].values = c["values"].data_ptr()
        else:
            w = N.OUT_WIDTH[info.out_type]
            dt = {4: torch.int32, 8: torch.int64, 16: torch.int64}[w]
            c["values"] = torch.empty(max(1, n * (2 if w == 16 else 1)), dtype=dt, device=device)
            cstructs[ci].values = c["values"].data_ptr()
        cstructs[ci].validity = c["validity"].data_ptr()
        cols.append(c)
    return cols, cstructs


class _HostArray:
    """A numpy array with the tensor method _slot_arrays uses (.cpu().numpy())."""
    def __init__(self, a):
        self.a = a

    def cpu(self):
        return self

    def numpy(self):
        return self.a


def view_geometry(capacity: int, n_tiles: int) -> Tuple[int, int]:
    """String-view layout: (tile_bytes, buffer_bytes) of a slot region of `capacity` bytes for
    n_tiles tiles (cbx_string_bound's capacity; buffers of a power-of-two number of whole tiles,
    at most 1 GiB each unless one tile is larger -- cbx_string_view_geometry)."""
    if n_tiles <= 0 or capacity <= 0:
        return 0, 0
    tb = capacity // n_tiles
    cap = int(os.environ.get("CBX_VIEW_BUFFER_BYTES", "0") or 0)   # tests: multi-buffer regions (cbx_capi.hip)
    cap = cap if 16 <= cap < (1 << 30) else (1 << 30)
    tpb = max(1, cap // max(16, tb))
    return tb, (1 << (tpb.bit_length() - 1)) * tb


def decode_views(views: np.ndarray, data: bytes, buffer_bytes: int, region: int) -> List[bytes]:
    """Payload bytes of Arrow string views (16 bytes each: length, inline bytes or prefix +
    buffer index + offset) whose data buffers are cut from `data` at `region` in pieces of
    buffer_bytes."""
    v = views.reshape(-1, 16)
    ln = v[:, 0:4].copy().view(np.int32).reshape(-1)
    bi = v[:, 8:12].copy().view(np.int32).reshape(-1)
    of = v[:, 12:16].copy().view(np.int32).reshape(-1)
    out = []
    for i in range(v.shape[0]):
        n = int(ln[i])
        if n <= 12:
            out.append(bytes(v[i, 4:4 + n]))
        else:
            s = region + int(bi[i]) * buffer_bytes + int(of[i])
            out.append(data[s:s + n])
    return out


def views_to_utf8(plan: DecodePlan, cols: List[Dict[str, Any]], n_rec: int, stream) -> None:
    """String-view columns (16-byte views + per-slot regions) -> Arrow Utf8 columns (int32 offsets per
    slot, payload in the slot's own region), in place in `cols`, on the device: the record walk writes
    views (one pass with data-dependent offsets); a reader asked for string_utf8 hands out Utf8."""
    torch = _torch()
    L = N.load()
    pitch = 64 * ((n_rec + 63) // 64)
    for ci, info in enumerate(plan.columns):
        c = cols[ci]
        if "views" not in c:
            continue
        dev = c["views"].device
        cap = int(c["capacity"])
        with torch.cuda.stream(stream):
            # allocated and zero-filled on the stream the conversion runs on (ordered before its writes)
            offs = torch.zeros(info.n_slots * (pitch + 1), dtype=torch.int32, device=dev)
            sizes = torch.zeros(info.n_slots, dtype=torch.int64, device=dev)
            data = torch.empty(max(1, cap * info.n_slots), dtype=torch.uint8, device=dev)
        if stream != torch.cuda.current_stream():
            _record_stream([{"o": offs, "s": sizes, "d": data}], torch.cuda.current_stream())
        for s in range(info.n_slots):
            N.check(L.cbx_views_to_utf8(c["views"].data_ptr() + 16 * s * pitch, n_rec, c["data"].data_ptr() + s * cap,
                                        max(1, int(c["buffer_bytes"])), offs.data_ptr() + 4 * s * (pitch + 1),
                                        data.data_ptr() + s * cap, cap, sizes.data_ptr() + 8 * s,
                                        ctypes.c_void_p(stream.cuda_stream)))
        cols[ci] = {"validity": c["validity"], "offsets32": offs, "data": data, "sizes": sizes, "capacity": cap}


def string_capacity(native_plan, n_rec: int, exact: Optional[Sequence[int]] = None) -> List[int]:
    """Per-column payload bytes per slot: the exact pre-pass result or cbx_string_bound."""
    if exact is not None:
        return [int(x) for x in exact]
    out = (ctypes.c_int64 * native_plan.plan.n_columns)()
    N.check(N.load().cbx_string_bound(native_plan.handle, n_rec, out))
    return list(out)


def parse_copybook_for(copybook_contents: str, params: ReaderParameters) -> cbk.Copybook:
    """The reader's loadCopyBook (CP/reader/FixedLenNestedReader.scala:100-143,
    CP/reader/VarLenNestedReader.scala:182-226): parse options taken from ReaderParameters."""
    segment_redefines = sorted(set(params.segment_id_redefine_map.values()))
    return cbk.parse_copybook(
        copybook_contents, data_encoding=cbk.EBCDIC if params.is_ebcdic else cbk.ASCII,
        drop_group_fillers=params.drop_group_fillers, drop_value_fillers=params.drop_value_fillers,
        segment_redefines=segment_redefines, string_trimming=params.string_trimming_policy,
        code_page=params.ebcdic_code_page_table or params.ebcdic_code_page,
        floating_point_format=params.floating_point_format,
        is_utf16_big_endian=params.is_utf16_big_endian, ascii_charset=params.ascii_charset,
        non_terminals=params.non_terminals, occurs_handlers=params.occurs_mappings,
        debug_fields_policy=params.debug_fields_policy, field_parent_map=params.segment_redefine_parents)


def reader_schema(cb: cbk.Copybook, params: ReaderParameters, variable_length: bool):
    """The reader's CobolSchema -> createSparkSchema (SC/schema/CobolSchema.scala:77-113): the
    variable-length reader adds File_Id / Record_Id and one Seg_IdN column per segment level
    (CP/reader/VarLenNestedReader.scala:223-225); the fixed-length reader neither."""
    levels = len(params.segment_id_levels) if (variable_length and params.segment_field) else 0
    return spark_schema(cb, params.schema_policy == "collapse_root",
                        params.generate_record_id and variable_length, seg_id_levels=levels,
                        input_file_name_field=params.input_file_name_column if variable_length else "")


def hier_root_keys(cb: cbk.Copybook, params: ReaderParameters) -> List[str]:
    """CopybookParser.getRootSegmentIds (:751-769): the ids mapped to the segment without a parent."""
    roots = {g.name for g in cb.all_segment_redefines() if g.parent_segment is None}
    return [sid for sid, grp in params.segment_id_redefine_map.items() if cbk._transform_identifier(grp) in roots]


def hier_general_walk(params: ReaderParameters, plan: DecodePlan) -> bool:
    """Whether a segment with children is mapped from several segment ids: extractChildren stops a
    parent's children at a record with the parent's own id (or an ancestor's), so the lists then
    depend on ids, not segments, and one record can sit under several parents (cbx_hier_select's
    general walk, cbx_hier_params.flags bit 0)."""
    ids: Dict[str, List[str]] = {}
    for sid, grp in params.segment_id_redefine_map.items():
        ids.setdefault(cbk._transform_identifier(grp), []).append(sid)
    parents = {g.parent_segment.name for g in plan.segment_groups if g.parent_segment is not None}
    return any(g.name in parents and len(ids.get(g.name, [])) > 1 for g in plan.segment_groups)


def check_hierarchical(cb: cbk.Copybook, params: ReaderParameters, plan: DecodePlan) -> bool:
    """What the GPU hierarchical path assumes (cobrix_hip.h cbx_hier_select); anything else is
    reported, never decoded differently.  Returns whether a record-walk plan needs its rows' dependee
    maps seeded (cbx_plan_set_dep_seed): an OCCURS DEPENDING ON a field that another record of the
    hierarchical record registers in the shared dependFields map (RecordExtractors.scala:224-245)."""
    if not params.segment_field or not params.segment_id_redefine_map:
        raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records need segment_field and redefine-segment-id-map")
    segs = plan.segment_groups
    if len(segs) > 16:
        raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: more than 16 segment redefines")
    if plan.walk is None:
        return False

    def stmts(g):
        for c in g.children:
            yield c
            if isinstance(c, cbk.Group):
                yield from stmts(c)
    order = list(stmts(cb.ast))
    prims = [q for q in order if not isinstance(q, cbk.Group)]
    root = next((i for i, g in enumerate(segs) if g.parent_segment is None), -1)
    cross = seg_odo = False
    for st in order:
        ai = plan.array_of_node.get(id(st))
        if ai is None or st.depending_on is None:
            continue
        sa = plan.arrays[ai].segment
        q = next((q for q in prims if q.is_dependee and q.name == st.depending_on), None)
        fq = plan.field_of_node.get(id(q)) if q is not None else None
        sq = plan.fields[fq].segment if fq is not None else sa
        cross |= sa >= 0 and sq != sa and not (sa == root and sq < 0)
        seg_odo |= sa >= 0
    if not seg_odo:
        return False
    # An array of a segment reads the map another record may have filled: its dependee in another
    # segment, or its own dependee null in this row (the registration before it stays).  The seeds come
    # from the dependee fields decoded from each row's bytes at their copybook offsets
    # (cbx_hier_dependee_values): a dependee inside an OCCURS, or placed after a variable-size OCCURS
    # (variable_size_occurs: a data-dependent offset), registers what that decode cannot see -- reported
    # when the array depends on another segment, else the row's own map (a null own dependee then counts
    # the maximum instead of the earlier registration)
    first_odo = next((k for k, st in enumerate(order) if st.depending_on is not None and st.is_array), len(order))
    for k, st in enumerate(order):
        if isinstance(st, cbk.Group) or not st.is_dependee:
            continue
        fi = plan.field_of_node.get(id(st))
        if fi is None or plan.fields[fi].n_dims != 0 or (plan.walk.variable_size_occurs and k > first_odo):
            if cross:
                raise N.CbxError(N.CBX_E_UNSUPPORTED, f"hierarchical records: {st.name}, a DEPENDING ON field of "
                                                      "another segment's array, inside an OCCURS or behind a "
                                                      "variable-size one")
            return False
    return True


class HierBatch:
    """Hierarchical records decoded on the GPU (cbx_hier_select + cbx_decode_selected): `flat` holds
    one decoded row per table row -- table 0 the root records (one per hierarchical record), table
    1 + s the records of segment s placed in the tree -- and `offsets[s]` the Arrow list offsets of
    segment s's children over its parent table (cbx_hier_list_offsets)."""

    def __init__(self, flat: DecodedBatch, table_rows: List[int], offsets: Dict[int, Any],
                 collapse_root: bool, generate_record_id: bool):
        self.flat, self.plan = flat, flat.plan
        self.table_rows = table_rows
        self.table_base = [int(x) for x in np.concatenate([[0], np.cumsum(table_rows)])]
        self.d_offsets = offsets          # int32 list offsets per child segment, on the device
        self._h_offsets: Optional[Dict[int, np.ndarray]] = None
        self.collapse_root, self.generate_record_id = collapse_root, generate_record_id
        self.input_file: Optional[Tuple[str, str]] = None
        self.n_rec = table_rows[0]
        self.children = {id(g): [c for c in self.plan.segment_groups if c.parent_segment is g]
                         for g in self.plan.segment_groups}

    @property
    def offsets(self) -> Dict[int, np.ndarray]:
        """Host copies of the list offsets (made on first use by the row / pyarrow builders)."""
        if self._h_offsets is None:
            self._h_offsets = {s: (o.cpu().numpy() if hasattr(o, "cpu") else np.asarray(o)) for s, o in self.d_offsets.items()}
        return self._h_offsets

    def _seg(self, g) -> int:
        return self.plan.segment_groups.index(g)

    def _parent_base(self, child) -> int:
        """First row of the table the child's lists run over (roots for children of the root segment)."""
        p = child.parent_segment
        return 0 if p.parent_segment is None else self.table_base[1 + self._seg(p)]

    def to_rows(self) -> List[dict]:
        """getGroupValues + extractChildren + applyRecordPostProcessing (RecordExtractors.scala:298-451)."""
        plan, flat = self.plan, self.flat

        def extra(g, r):
            d = {}
            if not g.is_segment_redefine:
                return d
            for c in self.children[id(g)]:
                s = self._seg(c)
                off = self.offsets[s]
                k = r - self._parent_base(c)
                b = self.table_base[1 + s]
                d[c.name] = [walk(c, b + j, []) for j in range(int(off[k]), int(off[k + 1]))]
            return d

        walk = flat._row_builder(extra=extra, null_segments=False)
        rows = []
        for r in range(self.n_rec):
            recs = [(g.name, walk(g, r, [])) for g in plan.copybook.ast.children
                    if isinstance(g, cbk.Group) and g.parent_segment is None]
            row: Dict[str, Any] = {}
            if self.generate_record_id:
                row["File_Id"] = flat.cell(plan.file_id_column, 0, r)
                row["Record_Id"] = flat.cell(plan.record_id_column, 0, r)
            if self.input_file is not None:   # extractHierarchicalRecord: no segment ids (:384)
                row[self.input_file[0]] = self.input_file[1]
            if self.collapse_root:
                for _, v in recs:
                    row.update(v)
            else:
                row.update({k: v for k, v in recs})
            rows.append(row)
        return rows

    def to_arrow(self):
        """The hierarchical records as a pyarrow Table: each segment's children a list<struct>
        column inside its struct, built from the table rows and the GPU list offsets."""
        import pyarrow as pa
        plan, flat = self.plan, self.flat

        def extra(g, R):
            if not g.is_segment_redefine:
                return [], []
            names, arrays = [], []
            for c in self.children[id(g)]:
                s = self._seg(c)
                off = self.offsets[s]
                k = R - self._parent_base(c)
                lo, hi = off[k], off[k + 1]
                b = self.table_base[1 + s]
                rows = np.concatenate([np.arange(b + x, b + y) for x, y in zip(lo, hi)]) if len(R) else np.zeros(0, np.int64)
                child = build(c, rows.astype(np.int64), np.zeros(len(rows), np.int64), False)
                offs = np.concatenate([[0], np.cumsum(hi - lo)]).astype(np.int32)
                names.append(c.name)
                arrays.append(pa.ListArray.from_arrays(pa.array(offs, pa.int32()), child))
            return names, arrays

        build = flat._arrow_builder(extra=extra, null_segments=False)
        column = build.column
        R0 = np.arange(self.n_rec, dtype=np.int64)
        S0 = np.zeros(self.n_rec, dtype=np.int64)
        names, arrays = [], []
        if self.generate_record_id:
            names += ["File_Id", "Record_Id"]
            arrays += [column(plan.file_id_column).slice(0, self.n_rec), column(plan.record_id_column).slice(0, self.n_rec)]
        if self.input_file is not None:
            names.append(self.input_file[0])
            arrays.append(_file_name_array(self.input_file[1], self.n_rec))
        for g in plan.copybook.ast.children:
            if not isinstance(g, cbk.Group) or g.parent_segment is not None:
                continue
            st = build(g, R0, S0, False)
            if self.collapse_root:
                for k in range(st.type.num_fields):
                    names.append(st.type.field(k).name)
                    arrays.append(st.field(k))
            else:
                names.append(g.name)
                arrays.append(st)
        return pa.Table.from_arrays(arrays, names=names)


class _BaseReader:
    VARIABLE_LENGTH = False

    def __init__(self, copybook_contents: str, params: ReaderParameters):
        self.params = params
        self.copybook_contents = copybook_contents
        self.copybook = parse_copybook_for(copybook_contents, params)
        var = self.VARIABLE_LENGTH
        # the fixed-length reader only uses the redefine map (FixedLenNestedRowIterator.scala:50-70);
        # segment levels, filter and record ids belong to the variable-length iterator
        self.hierarchical = var and self.copybook.is_hierarchical
        root_keys = hier_root_keys(self.copybook, params) if self.hierarchical else ()

        def plan(walk: bool):
            # the record walk (cbx_walk.h) writes string columns as views
            return build_plan(self.copybook, segment_field=params.segment_field,
                              segment_redefine_map=params.segment_id_redefine_map or None,
                              generate_record_id=params.generate_record_id and var, window_bytes=params.window_bytes,
                              jit_min_records=params.jit_min_records,
                              segment_levels=params.segment_id_levels if var else (),
                              segment_filter=params.segment_id_filter if var else None,
                              segment_prefix=params.segment_id_prefix,
                              string_views=1 if (walk or (params.string_views and not params.string_utf8))
                              else 2 if params.string_utf8 else 0,
                              occurs_lists=params.occurs_lists, root_keys=root_keys, walk=walk,
                              variable_size_occurs=params.variable_size_occurs)

        # variable_size_occurs, DEPENDING ON inside an OCCURS, string dependees: the record walk
        walk = bool(params.variable_size_occurs)
        if not walk:
            try:
                self.plan = plan(False)
            except NeedsWalk:
                walk = True
        if walk:
            self.plan = plan(True)
        self.walk = walk
        self.walk_seeds = False
        if self.hierarchical:
            self.walk_seeds = check_hierarchical(self.copybook, params, self.plan)
        self.native = NativePlan(self.plan)

    @property
    def collapse_root(self) -> bool:
        return self.params.schema_policy == "collapse_root"

    def spark_schema(self):
        return reader_schema(self.copybook, self.params, self.VARIABLE_LENGTH)

    def _batch(self, n_rec: int, cols: List[Dict[str, Any]], first_record_id: int, gen_id: bool, stream) -> DecodedBatch:
        """The decoded columns as a batch; with string_utf8 on a record-walk plan (which writes views)
        its string columns are converted to Arrow Utf8 on the device (cbx_views_to_utf8)."""
        if self.walk and self.params.string_utf8:
            views_to_utf8(self.plan, cols, n_rec, stream)
        return DecodedBatch(self.plan, n_rec, cols, first_record_id, self.collapse_root, gen_id)

    def close(self):
        peer = getattr(self, "_peer", None)
        if peer is not None:   # (the pipelined second plan of decode_batches)
            N.check(N.load().cbx_plan_pipeline(self.native.handle, None, 0, 0))
            peer.close()
            self._peer = None
        self.native.close()


class FixedLenNestedReader(_BaseReader):
    """GPU drop-in for FixedLenNestedReader (CP/reader/FixedLenNestedReader.scala:43-144)."""

    def get_record_size(self) -> int:
        # FixedLenNestedReader.getRecordSize (:60-63)
        inner = self.params.record_length if self.params.record_length is not None else self.copybook.record_size
        return inner + self.params.start_offset + self.params.end_offset

    def check_binary_data_validity(self, n_bytes: int) -> None:
        """FixedLenNestedReader.checkBinaryDataValidity (CP/reader/FixedLenNestedReader.scala:71-90)
        and the file-size rule of the fixed-length Spark scan (SC/source/scanners/CobolScanners.scala:
        86-90), applied to a whole file / split.

        The reference runs the first check on each record Spark's binaryRecords cut at getRecordSize,
        and the second on each file before the scan: a file whose size is not a multiple of
        getRecordSize -- `record_length` included -- is rejected unless `debug_ignore_file_size` is
        set.  With it set the records are the file's whole records (the partial last one dropped)."""
        p = self.params
        if p.start_offset < 0:
            raise ValueError(f"Invalid record start offset = {p.start_offset}. A record start offset cannot be negative.")
        if p.end_offset < 0:
            raise ValueError(f"Invalid record end offset = {p.end_offset}. A record end offset cannot be negative.")
        if p.record_length is not None:
            if p.record_length < 1:
                raise ValueError(f"The specified record size {p.record_length} cannot be used. "
                                 "The record length should be greater then zero.")
            if not p.debug_ignore_file_size and n_bytes % self.get_record_size() > 0:
                raise ValueError("There are some files in the input that are NOT DIVISIBLE by the RECORD SIZE calculated "
                                 f"from the copybook ({self.get_record_size()} bytes per record). "
                                 "Check the logs for the names of the files.")
        elif not p.debug_ignore_file_size:
            exp = self.copybook.record_size + p.start_offset + p.end_offset
            if n_bytes < exp:
                raise ValueError(f"Binary record too small. Expected binary record size = {exp}, got {n_bytes} ")
            if n_bytes % exp > 0:
                raise ValueError(f"Binary record size {exp} does not divide data size {n_bytes}.")

    def decode_device(self, d_data, n_bytes: int, first_record_id: int = 0, stream=None,
                      exact_strings: bool = False) -> DecodedBatch:
        """Decode a split already resident in HBM (d_data: uint8 CUDA tensor).

        One asynchronous kernel launch; string payloads go to regions sized by the upper bound
        (or by the exact pre-pass when exact_strings=True).  cbx_plan_check synchronises and
        raises if a payload overflowed."""
        torch = _torch()
        stride = self.get_record_size()
        n_rec = n_bytes // stride
        st = stream if stream is not None else torch.cuda.current_stream()
        L = N.load()
        exact = None
        if exact_strings:
            sizes = (ctypes.c_int64 * self.plan.n_columns)()
            N.check(L.cbx_string_sizes_fixed(self.native.handle, d_data.data_ptr(), n_rec, stride,
                                             self.params.start_offset, sizes, ctypes.c_void_p(st.cuda_stream)))
            exact = list(sizes)
        cols, cs = _alloc_columns(self.plan, n_rec, string_capacity(self.native, n_rec, exact), d_data.device)
        N.check(L.cbx_decode_fixed(self.native.handle, d_data.data_ptr(), n_rec, stride, self.params.start_offset,
                                   first_record_id, cs, ctypes.c_void_p(st.cuda_stream)))
        N.check(L.cbx_plan_check(self.native.handle, ctypes.c_void_p(st.cuda_stream)))
        return self._batch(n_rec, cols, first_record_id, False, st)

    def decode_batches(self, d_data, n_bytes: int, batch_records: int, first_record_id: int = 0) -> List[DecodedBatch]:
        """A split resident in HBM decoded as consecutive batches of <= batch_records records (the
        Arrow Utf8 layout's int32 offsets cap a batch; a consumer takes one Arrow array per batch --
        a chunked array).  In the Utf8 layout the batches alternate between this plan and a second
        one on a second stream, linked by cbx_plan_pipeline: a batch's count pass runs beside the
        previous batch's decode (C3: 53.3 -> 51.3 ms per 64 GB).  Other layouts decode in turn."""
        torch = _torch()
        stride = self.get_record_size()
        n_rec = n_bytes // stride
        if n_rec == 0:
            return [self.decode_device(d_data, 0, first_record_id)]
        bs = batch_records if batch_records > 0 else n_rec
        L = N.load()
        s0 = torch.cuda.current_stream()
        targets = [(self, s0)]
        if self.params.string_utf8 and not self.walk and n_rec > bs:
            if getattr(self, "_peer", None) is None:
                self._peer = FixedLenNestedReader(self.copybook_contents, self.params)
                N.check(L.cbx_plan_pipeline(self.native.handle, self._peer.native.handle, 0, 0))
            targets.append((self._peer, torch.cuda.Stream(d_data.device)))
            targets[1][1].wait_stream(s0)   # (the data and any earlier work on the first stream)
        out, pending = [], []
        for k, r0 in enumerate(range(0, n_rec, bs)):
            rd, st = targets[k % len(targets)]
            m = min(bs, n_rec - r0)
            with torch.cuda.stream(st):
                # zero-filled on the stream that decodes the batch: a fill queued on s0 behind the
                # previous batch's decode is not ordered before the side stream's count and decode
                cols, cs = _alloc_columns(rd.plan, m, string_capacity(rd.native, m), d_data.device)
            if st is not s0:
                _record_stream(cols, s0)   # (consumed on s0 after the final wait)
            N.check(L.cbx_decode_fixed(rd.native.handle, d_data.data_ptr() + r0 * stride, m, stride, self.params.start_offset,
                                       first_record_id + r0, cs, ctypes.c_void_p(st.cuda_stream)))
            pending.append((cols, cs))   # (the column table lives until the calls are checked)
            out.append((m, cols, first_record_id + r0, st))
        for rd, st in targets:
            N.check(L.cbx_plan_check(rd.native.handle, ctypes.c_void_p(st.cuda_stream)))
        if len(targets) > 1:
            s0.wait_stream(targets[1][1])
        return [self._batch(m, cols, fid, False, st) for m, cols, fid, st in out]

    def decode(self, data: bytes, first_record_id: int = 0) -> DecodedBatch:
        torch = _torch()
        self.check_binary_data_validity(len(data))
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda") if len(data) else torch.zeros(16, dtype=torch.uint8, device="cuda")
        return self.decode_device(t, len(data), first_record_id)

    def get_row_iterator(self, data: bytes) -> Iterator[dict]:
        return iter(self.decode(data).to_rows())


class VarLenNestedReader(_BaseReader):
    """GPU drop-in for VarLenNestedReader (CP/reader/VarLenNestedReader.scala:46-310).

    Pipeline per file (what CobolScanners.buildScanForVarLenIndex runs as one Spark task per index
    entry, SC/source/scanners/CobolScanners.scala:38-55): frame (RDW walk / text lines / fixed-length
    records) -> sparse index (IndexGenerator) -> record selection (VarLenNestedIterator: Record_Id,
    Seg_IdN, segment_filter, root-reached) -> decode.  Every stage runs on the GPU."""
    VARIABLE_LENGTH = True

    def rdw_params(self) -> N.CbxRdwParams:
        p = self.params
        r = N.CbxRdwParams()
        r.big_endian = int(p.is_rdw_big_endian)
        r.adjustment = (-4 if p.is_rdw_part_rec_length else 0) + p.rdw_adjustment
        r.file_header_bytes = p.file_start_offset
        r.file_footer_bytes = p.file_end_offset
        return r

    # ---- framing
    def frame_text(self, d_data, n_bytes: int, stream=None):
        """GPU text framing (TextRecordExtractor.scala:26-108) -> (rec_off, rec_len, virtual_bytes).

        Records may reach past n_bytes up to virtual_bytes (the reference's zero-filled window):
        d_data must hold zeros there (see `read`)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        cap = n_bytes + 2
        off = torch.empty(cap, dtype=torch.int64, device=d_data.device)
        ln = torch.empty(cap, dtype=torch.int32, device=d_data.device)
        n = ctypes.c_int64(0)
        vb = ctypes.c_int64(0)
        N.check(N.load().cbx_frame_text(d_data.data_ptr(), n_bytes, self.copybook.record_size, off.data_ptr(),
                                         ln.data_ptr(), cap, ctypes.byref(n), ctypes.byref(vb),
                                         ctypes.c_void_p(st.cuda_stream)))
        return off[: n.value], ln[: n.value], vb.value

    def frame(self, d_data, n_bytes: int, seeds: Optional[Sequence[int]] = None, stream=None):
        """GPU RDW walk -> (rec_off, rec_len) device tensors of the valid records."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        seeds = list(seeds) if seeds else [0]
        cap = max(1, n_bytes // 5 + 1)
        off = torch.empty(cap, dtype=torch.int64, device=d_data.device)
        ln = torch.empty(cap, dtype=torch.int32, device=d_data.device)
        sd = (ctypes.c_int64 * len(seeds))(*seeds)
        n = ctypes.c_int64(0)
        prm = self.rdw_params()
        N.check(N.load().cbx_frame_rdw(d_data.data_ptr(), n_bytes, sd, len(seeds), ctypes.byref(prm),
                                        off.data_ptr(), ln.data_ptr(), cap, ctypes.byref(n),
                                        ctypes.c_void_p(st.cuda_stream)))
        return off[: n.value], ln[: n.value]

    def frame_fixed(self, d_data, n_bytes: int):
        """RecordHeaderParserFixedLen (CP/parser/headerparsers/RecordHeaderParserFixedLen.scala:40-50)
        through VRLRecordReader: a file header record, then records of the copybook's size while
        a whole record remains and the rest is not the footer."""
        torch = _torch()
        p = self.params
        rs = self.copybook.record_size
        first = p.file_start_offset
        n = 0
        if n_bytes - first >= rs:
            # record k valid iff n_bytes - off_k >= rs and (no footer or n_bytes - off_k > footer)
            lim = n_bytes - rs
            if p.file_end_offset > 0:
                lim = min(lim, n_bytes - p.file_end_offset - 1)
            n = max(0, (lim - first) // rs + 1) if lim >= first else 0
        off = first + rs * torch.arange(n, dtype=torch.int64, device=d_data.device)
        ln = torch.full((n,), rs, dtype=torch.int32, device=d_data.device)
        return off, ln

    def header_bytes(self) -> int:
        return 4 if self.params.is_record_sequence else 0

    def has_file_header(self) -> bool:
        p = self.params
        return p.file_start_offset > (4 if p.is_record_sequence else 0)

    # ---- sparse index
    def index_params(self, file_id: int = 0) -> N.CbxIndexParams:
        """VarLenNestedReader.generateIndex split parameters (:125-180, getSplitSizeMB :237-243)."""
        p = self.params
        prm = N.CbxIndexParams()
        split_mb = p.input_split_size_mb if p.input_split_size_mb is not None else p.hdfs_default_block_size_mb
        if p.input_split_records is not None:
            if not 1 <= p.input_split_records <= 1000000000:
                raise ValueError(f"Invalid input split size. The requested number of records is {p.input_split_records}.")
            prm.records_per_entry = p.input_split_records
        elif split_mb is not None:
            if not 1 <= split_mb <= 2000:
                raise ValueError(f"Invalid input split size of {split_mb} MB.")
            prm.bytes_per_entry, prm.subtract_size = split_mb * 1024 * 1024, 1
        else:
            prm.bytes_per_entry, prm.subtract_size = 100 * 1024 * 1024, 0   # Constants.defaultIndexEntrySizeMB
        prm.header_bytes = self.header_bytes()
        prm.has_file_header = int(self.has_file_header())
        # segmentLevelIds.nonEmpty || fieldParentMap.nonEmpty (VarLenNestedReader.scala:151-155)
        prm.hierarchical = int(bool(p.segment_field) and (bool(p.segment_id_levels) or self.hierarchical))
        prm.file_id = file_id
        return prm

    def generate_index(self, d_data, n_bytes: int, rec_off, rec_len, file_id: int = 0,
                       stream=None, start_bytes: int = 0) -> List[SparseIndexEntry]:
        """GPU sparse index over the framed file (IndexGenerator.sparseIndexGenerator).  start_bytes:
        bytesInChunk at the first record, for a piece of a file starting at one of its entries
        (cobrix_hip.h cbx_index_params; shard.index_chain)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        prm = self.index_params(file_id)
        prm.start_bytes = int(start_bytes)
        L = N.load()
        n = ctypes.c_int64(0)
        cap = 1024
        while True:
            ents = (N.CbxIndexEntry * cap)()
            rc = L.cbx_sparse_index(self.native.handle, d_data.data_ptr(), n_bytes, rec_off.data_ptr(),
                                    rec_len.data_ptr(), int(rec_off.numel()), ctypes.byref(prm), ents, cap,
                                    ctypes.byref(n), ctypes.c_void_p(st.cuda_stream))
            if rc == N.CBX_E_CAPACITY and n.value > cap:
                cap = n.value
                continue
            N.check(rc)
            break
        return [SparseIndexEntry(e.offset_from, e.offset_to, e.file_id, e.record_index) for e in ents[: n.value]]

    def split_residual_bytes(self) -> Optional[int]:
        """The split size when IndexGenerator subtracts it at every cut (isSplitBySize: an explicit
        input_split_size_mb / the HDFS block size), else None (records, or the 100 MB default that resets)."""
        p = self.params
        split_mb = p.input_split_size_mb if p.input_split_size_mb is not None else p.hdfs_default_block_size_mb
        return split_mb * 1024 * 1024 if p.input_split_records is None and split_mb is not None else None

    def index_generation_needed(self) -> bool:
        """VarLenNestedReader.isIndexGenerationNeeded (:85)."""
        p = self.params
        return (p.record_length_field is None or p.is_record_sequence) and p.enable_indexes

    def length_field(self) -> Optional[int]:
        """ReaderParametersValidator.getLengthField (CP/reader/validator/ReaderParametersValidator.scala:26-43):
        the record length field's index in the plan's field table (None: no length field), after the
        reference's checks (a primitive Integral field, not an array)."""
        name = self.params.record_length_field
        if name is None or self.params.is_record_sequence:
            return None
        node = self.copybook.get_field_by_name(name)
        if not isinstance(node, cbk.Primitive):
            raise ValueError(f"The record length field {name} must have an primitive integral type.")
        if not isinstance(node.dtype, cbk.Integral):
            raise ValueError(f"The record length field {name} must be an integral type.")
        if node.occurs is not None and node.occurs > 1:
            raise ValueError(f"The record length field '{name}' cannot be an array.")
        fi = self.plan.field_of_node.get(id(node))
        if fi is None:
            raise ValueError(f"record length field {name} is not decoded by the plan (a FILLER)")
        return fi

    def frame_length_field(self, d_data, n_bytes: int, stream=None):
        """VRLRecordReader.fetchRecordUsingRecordLengthField on the GPU (chunk-parallel framing,
        cbx_chain.h) -> (rec_off, rec_len) of the records: each starts where the previous ended, its length
        from the field inside it (+ rdw_adjustment), record_start/end_offset included."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        p = self.params
        fi = self.length_field()
        lfb = self.plan.fields[fi].offset + self.plan.fields[fi].size
        cap = max(1, n_bytes // max(1, p.start_offset + lfb) + 1)
        off = torch.empty(cap, dtype=torch.int64, device=d_data.device)
        ln = torch.empty(cap, dtype=torch.int32, device=d_data.device)
        n = ctypes.c_int64(0)
        rc = N.load().cbx_frame_length_field(self.native.handle, d_data.data_ptr(), n_bytes, fi, p.start_offset,
                                             p.end_offset, p.rdw_adjustment, off.data_ptr(), ln.data_ptr(), cap,
                                             ctypes.byref(n), ctypes.c_void_p(st.cuda_stream))
        if rc == N.CBX_E_STATE:
            # the reference's IllegalStateException names the field (VRLRecordReader.scala:131-134);
            # the C ABI knows only its byte position
            raise N.CbxError(rc, f"Record length value of the field {p.record_length_field} must be an integral type.")
        N.check(rc)
        return off[: n.value], ln[: n.value]

    # ---- selection + decode
    def select(self, d_data, n_bytes: int, rec_off, rec_len, entries: Optional[Sequence[SparseIndexEntry]] = None,
               file_id: int = 0, stream=None) -> Dict[str, Any]:
        """VarLenNestedIterator over every entry: Record_Id, Seg_IdN state, filters (GPU)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        n = int(rec_off.numel())
        dev = d_data.device
        nl = self.plan.options.segments.n_levels if self.plan.options.has_segments else 0
        sel = {"rec_off": torch.empty(max(1, n), dtype=torch.int64, device=dev),
               "rec_len": torch.empty(max(1, n), dtype=torch.int32, device=dev),
               "record_id": torch.empty(max(1, n), dtype=torch.int64, device=dev),
               "segment": torch.empty(max(1, n), dtype=torch.int32, device=dev),
               "seg_state": torch.empty(max(1, n * (1 + nl)), dtype=torch.int64, device=dev)}
        cs = N.CbxSelection()
        for k in ("rec_off", "rec_len", "record_id", "segment", "seg_state"):
            setattr(cs, k, sel[k].data_ptr())
        cs.file_id = file_id
        cs.footer_bytes = self.params.file_end_offset
        ents = None
        if entries:
            ents = (N.CbxIndexEntry * len(entries))()
            for i, e in enumerate(entries):
                ents[i].offset_from, ents[i].offset_to = e.offset_from, e.offset_to
                ents[i].record_index, ents[i].file_id = e.record_index, e.file_id
        ns = ctypes.c_int64(0)
        N.check(N.load().cbx_select_records(self.native.handle, d_data.data_ptr(), n_bytes, rec_off.data_ptr(),
                                            rec_len.data_ptr(), n, self.params.start_offset, ents,
                                            len(entries) if entries else 0, ctypes.byref(cs), ctypes.byref(ns),
                                            ctypes.c_void_p(st.cuda_stream)))
        sel["n"] = ns.value
        sel["struct"] = cs
        return sel

    def decode_selected(self, d_data, n_bytes: int, sel: Dict[str, Any], stream=None) -> DecodedBatch:
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        n_rec = sel["n"]
        cols, cs = _alloc_columns(self.plan, n_rec, string_capacity(self.native, n_rec), d_data.device)
        L = N.load()
        N.check(L.cbx_decode_selected(self.native.handle, d_data.data_ptr(), n_bytes, ctypes.byref(sel["struct"]),
                                      n_rec, self.params.start_offset, cs, ctypes.c_void_p(st.cuda_stream)))
        N.check(L.cbx_plan_check(self.native.handle, ctypes.c_void_p(st.cuda_stream)))
        return self._batch(n_rec, cols, 0, self.params.generate_record_id, st)

    def decode_device(self, d_data, n_bytes: int, rec_off, rec_len, first_record_id: int = 0,
                      stream=None, exact_strings: bool = False) -> DecodedBatch:
        """Decode framed records as one index entry starting at first_record_id, without the
        selection stage (cbx_decode_var: Record_Id = first_record_id + r).  The device-level entry
        points leave with_input_file_name_col's column to the caller (`batch.input_file`); `read`
        and `decode` set it from their input_file_name."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        n_rec = int(rec_off.numel())
        L = N.load()
        exact = None
        if exact_strings:
            sizes = (ctypes.c_int64 * self.plan.n_columns)()
            N.check(L.cbx_string_sizes_var(self.native.handle, d_data.data_ptr(), n_bytes, rec_off.data_ptr(),
                                           rec_len.data_ptr(), n_rec, self.params.start_offset, sizes,
                                           ctypes.c_void_p(st.cuda_stream)))
            exact = list(sizes)
        cols, cs = _alloc_columns(self.plan, n_rec, string_capacity(self.native, n_rec, exact), d_data.device)
        N.check(L.cbx_decode_var(self.native.handle, d_data.data_ptr(), n_bytes, rec_off.data_ptr(),
                                 rec_len.data_ptr(), n_rec, self.params.start_offset, first_record_id, cs,
                                 ctypes.c_void_p(st.cuda_stream)))
        N.check(L.cbx_plan_check(self.native.handle, ctypes.c_void_p(st.cuda_stream)))
        return self._batch(n_rec, cols, first_record_id, self.params.generate_record_id, st)

    def read_entries(self, d_data, n_bytes: int, entries: Sequence[SparseIndexEntry], entries_per_piece: int = 1,
                     file_id: int = 0, input_file_name: Optional[str] = None) -> List[DecodedBatch]:
        """An RDW file as the reference reads it -- a partition per sparse-index entry
        (CobolScanners.buildScanForVarLenIndex, SC/source/scanners/CobolScanners.scala:40-75), each with
        its own VarLenNestedIterator from the entry's offset and record index -- `entries_per_piece`
        consecutive entries to a batch: a piece's records framed from its entries' offsets (the RDW walk
        seeded at them, cbx_frame_rdw), then selected and decoded, one piece after another on the
        current stream (framing returns the piece's record count to the host, so pieces do not
        overlap).  The batches, in file order, hold the rows `read` returns.
        input_file_name: as in `read`."""
        torch = _torch()
        self._file_column(None, input_file_name, check_only=True)
        if not self.params.is_record_sequence or self.params.is_text or self.hierarchical:
            raise N.CbxError(N.CBX_E_UNSUPPORTED, "read_entries: RDW record sequences only (flat plans)")
        if entries_per_piece < 1:
            raise ValueError("entries_per_piece must be >= 1")
        ents = list(entries) or [SparseIndexEntry(0, -1, file_id, 0)]
        main = torch.cuda.current_stream()
        L = N.load()
        out: List[DecodedBatch] = []
        for k in range(0, len(ents), entries_per_piece):
            group = ents[k:k + entries_per_piece]
            a = group[0].offset_from
            known = k + entries_per_piece < len(ents)
            b = ents[k + entries_per_piece].offset_from if known else n_bytes   # (entries tile the file)
            # records of the piece: the next piece's record index minus this one's (the last: a bound)
            cap = (ents[k + entries_per_piece].record_index - group[0].record_index + 1) if known else (b - a) // 5 + 1
            off = torch.empty(max(1, cap), dtype=torch.int64, device=d_data.device)
            ln = torch.empty(max(1, cap), dtype=torch.int32, device=d_data.device)
            sd = (ctypes.c_int64 * len(group))(*[e.offset_from - a for e in group])
            # the file header record lies at the file's start, the footer before its end: a piece elsewhere
            # frames neither (the selection still drops the records within file_end_offset of each entry's
            # offset_to, as the reference's entry-bounded streams do: cbx_select.h sel_footer)
            prm = self.rdw_params()
            if a > 0:
                prm.file_header_bytes = 0
            if known:
                prm.file_footer_bytes = 0
            n = ctypes.c_int64(0)
            N.check(L.cbx_frame_rdw(d_data.data_ptr() + a, b - a, sd, len(group), ctypes.byref(prm), off.data_ptr(),
                                    ln.data_ptr(), max(1, cap), ctypes.byref(n), ctypes.c_void_p(main.cuda_stream)))
            piece = d_data[a:b]
            rebased = [SparseIndexEntry(e.offset_from - a, e.offset_to - a if e.offset_to >= 0 else -1, e.file_id,
                                        e.record_index) for e in group]
            sel = self.select(piece, b - a, off[: n.value], ln[: n.value], rebased, file_id, stream=main)
            out.append(self._file_column(self.decode_selected(piece, b - a, sel, stream=main), input_file_name))
        return out

    def _device_file(self, data: bytes):
        torch = _torch()
        # zero fill past the data: text windows and VarOccursRecordExtractor's short last record
        extra = self.copybook.record_size + 2 + 16 if (self.params.is_text or self.var_occurs_extractor()) else 0
        t = torch.zeros(max(16, len(data) + extra), dtype=torch.uint8, device="cuda")
        if len(data):
            t[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
        return t

    def frame_var_occurs(self, d_data, n_bytes: int, stream=None):
        """VarOccursRecordExtractor (GPU, chunk-parallel framing: cbx_chain.h) -> (rec_off, rec_len, virtual_bytes): the
        last record may reach past n_bytes into the reference's zero fill (d_data holds zeros there)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        cap = max(1, n_bytes)
        off = torch.empty(cap, dtype=torch.int64, device=d_data.device)
        ln = torch.empty(cap, dtype=torch.int32, device=d_data.device)
        n = ctypes.c_int64(0)
        vb = ctypes.c_int64(0)
        N.check(N.load().cbx_frame_var_occurs(self.native.handle, d_data.data_ptr(), n_bytes, 0, off.data_ptr(), ln.data_ptr(),
                                               cap, ctypes.byref(n), ctypes.byref(vb), ctypes.c_void_p(st.cuda_stream)))
        return off[: n.value], ln[: n.value], vb.value

    def var_occurs_extractor(self) -> bool:
        """VarLenNestedReader.recordExtractor (:60-78): VarOccursRecordExtractor for variable-size
        OCCURS without RDW headers or a record length field (no custom extractor / header parser here)."""
        p = self.params
        return p.variable_size_occurs and not p.is_record_sequence and not p.is_text and p.record_length_field is None

    def frame_file(self, t, n_bytes: int):
        """(rec_off, rec_len, bytes the records are decoded against) of a whole file."""
        if self.params.is_text:
            return self.frame_text(t, n_bytes)
        if self.var_occurs_extractor():
            return self.frame_var_occurs(t, n_bytes)
        if self.params.is_record_sequence:
            off, ln = self.frame(t, n_bytes)
            return off, ln, n_bytes
        if self.params.record_length_field is not None:
            off, ln = self.frame_length_field(t, n_bytes)
            return off, ln, n_bytes
        off, ln = self.frame_fixed(t, n_bytes)
        return off, ln, n_bytes

    def read_hierarchical(self, d_data, n_bytes: int, rec_off, rec_len, file_id: int = 0, first_record_id: int = 0,
                          stream=None) -> HierBatch:
        """VarLenHierarchicalIterator over framed records (GPU): cbx_hier_select -> cbx_decode_selected ->
        cbx_hier_list_offsets per child segment.  Index entries are cut at root records, so reading the
        whole stream at once gives the rows (and Record_Ids) of reading entry by entry."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream()
        sp = ctypes.c_void_p(st.cuda_stream)
        L = N.load()
        n = int(rec_off.numel())
        dev = d_data.device
        segs = self.plan.segment_groups
        prm = N.CbxHierParams()
        prm.n_segments = len(segs)
        prm.root_segment = next(i for i, g in enumerate(segs) if g.parent_segment is None)
        for i in range(N.CBX_MAX_SEG_KEYS):
            prm.parent[i] = -1
        for i, g in enumerate(segs):
            prm.parent[i] = segs.index(g.parent_segment) if g.parent_segment is not None else -1
        prm.first_record_id = first_record_id
        prm.start_offset = self.params.start_offset
        prm.flags = 1 if hier_general_walk(self.params, self.plan) else 0
        cap = max(1, n)
        while True:
            sel = {"rec_off": torch.empty(cap, dtype=torch.int64, device=dev),
                   "rec_len": torch.empty(cap, dtype=torch.int32, device=dev),
                   "record_id": torch.empty(cap, dtype=torch.int64, device=dev),
                   "segment": torch.empty(cap, dtype=torch.int32, device=dev)}
            parent_row = torch.empty(cap, dtype=torch.int64, device=dev)
            cs = N.CbxSelection()
            for k in ("rec_off", "rec_len", "record_id", "segment"):
                setattr(cs, k, sel[k].data_ptr())
            cs.file_id = file_id
            rows = (ctypes.c_int64 * (len(segs) + 1))()
            n_rows = ctypes.c_int64(0)
            prm.row_capacity = cap
            rc = L.cbx_hier_select(self.native.handle, d_data.data_ptr(), n_bytes, rec_off.data_ptr(), rec_len.data_ptr(), n,
                                   ctypes.byref(prm), ctypes.byref(cs), parent_row.data_ptr(), rows, ctypes.byref(n_rows), sp)
            if rc == N.CBX_E_CAPACITY and prm.flags and n_rows.value > cap:
                cap = n_rows.value   # the general walk: records under several parents -- more rows than records
                continue
            N.check(rc)
            break
        table_rows = [int(x) for x in rows]
        sel["n"], sel["struct"] = n_rows.value, cs
        s0 = self.params.start_offset
        if s0 and n_rows.value > table_rows[0]:
            # extractHierarchicalRecord decodes the root record from offsetBytes = record_start_offset
            # (VarLenHierarchicalIterator.scala:139-144) but each child segment at its group's own offset
            # in the child's data, without it (RecordExtractors.scala:308-310): the child rows are decoded
            # as records starting s0 bytes earlier and s0 bytes longer, so the decode's start offset
            # lands on the child's first byte and its bound on the child's own length
            kid_off = sel["rec_off"][table_rows[0]:n_rows.value]
            if int(kid_off.min().item()) < s0:
                # a child within s0 bytes of the data's start (a root shorter than the start offset): the
                # rows are decoded from a copy with s0 bytes in front, which no row reads
                d_data = torch.cat([torch.zeros(s0, dtype=torch.uint8, device=dev), d_data[:n_bytes]])
                n_bytes += s0
                sel["rec_off"][: table_rows[0]] += s0
            else:
                kid_off -= s0
            sel["rec_len"][table_rows[0]:n_rows.value] += s0
        # every child segment's list offsets over its parent table (device)
        base = np.concatenate([[0], np.cumsum(table_rows)]).astype(np.int64)
        d_offsets: Dict[int, Any] = {}
        for s, g in enumerate(segs):
            if g.parent_segment is None:
                continue
            ps = segs.index(g.parent_segment)
            pb, pn = (0, table_rows[0]) if g.parent_segment.parent_segment is None else (int(base[1 + ps]), table_rows[1 + ps])
            o = torch.empty(pn + 1, dtype=torch.int32, device=dev)
            N.check(L.cbx_hier_list_offsets(parent_row.data_ptr(), int(base[1 + s]), table_rows[1 + s], pb, pn, o.data_ptr(), sp))
            d_offsets[s] = o
        # the counts of arrays whose DEPENDING ON field another record of the hierarchical record
        # registers, resolved before the decode (one decode of the rows); on a record-walk plan each
        # row's dependee map as the hierarchical walk leaves it before the row (the walk counts itself)
        odo = seeds = None
        if self.walk_seeds:
            seeds = self._hier_walk_seeds(d_data, n_bytes, sel, table_rows, d_offsets, prm.root_segment, st)
        elif self.plan.walk is None:
            odo = self._hier_dependee_counts(d_data, n_bytes, sel, table_rows, d_offsets, prm.root_segment, st)
        if odo is not None:
            N.check(L.cbx_plan_set_odo_counts(self.native.handle, odo.data_ptr(), int(odo.shape[1])))
        if seeds is not None:
            N.check(L.cbx_plan_set_dep_seed(self.native.handle, seeds.data_ptr(), int(seeds.shape[1]), prm.root_segment))
        try:
            flat = self.decode_selected(d_data, n_bytes, sel, stream=st)
        finally:
            if odo is not None:
                N.check(L.cbx_plan_set_odo_counts(self.native.handle, None, 0))
            if seeds is not None:
                N.check(L.cbx_plan_set_dep_seed(self.native.handle, None, 0, 0))
        return HierBatch(flat, table_rows, d_offsets, self.collapse_root, self.params.generate_record_id)

    def _file_column(self, batch, input_file_name: Optional[str], check_only: bool = False):
        """with_input_file_name_col: the batch's file-name column (SimpleStream.inputFileName).  The
        schema lists the column whenever the option is set, so an entry point given no file name
        refuses rather than return a batch without it (or with empty names)."""
        if self.params.input_file_name_column:
            if not input_file_name:
                raise ValueError(f"with_input_file_name_col = '{self.params.input_file_name_column}' needs the "
                                 "input file's name (input_file_name=...)")
            if check_only:
                return batch
            batch.input_file = (self.params.input_file_name_column, input_file_name)
        return batch

    def _hier_dependee_counts(self, d_data, n_bytes: int, sel: Dict[str, Any], table_rows: List[int], child_offsets,
                              root_seg: int, stream):
        """extractHierarchicalRecord shares ONE dependFields map between the segments of a hierarchical
        record (RecordExtractors.scala:224-245): a DEPENDING ON field registers its value when a record's
        group holding it is decoded, and an array reads the value registered last -- in the walk's
        order (:324-372): the root record's groups -- the common header and every segment group, from the
        root's own bytes, with the root segment's children walked where its group ends -- then per child
        segment in copybook order each child record followed by its own subtree.  The records' own bytes
        give the same count when the dependee sits in the array's own segment and is not null there;
        otherwise (a dependee of the parent segment, of a sibling segment walked earlier, of the common
        header, of a segment group placed before the root's, or a null one) the count is the value
        registered last in the walk.  Resolved on the device BEFORE the rows are decoded: the dependee
        fields decoded from every row's bytes (cbx_hier_dependee_values), then one thread per
        hierarchical record replays the walk's events (cbx_hier_dependee_counts).  Returns the counts
        (int32 [n_arrays, rows], -1 for arrays the decode resolves from the row's own bytes), or None
        when no array depends on a numeric field of a segment."""
        torch = _torch()
        plan = self.plan
        arrays = [(ai, ar) for ai, ar in enumerate(plan.arrays) if ar.dependee >= 0 and ar.segment >= 0]
        n = int(sum(table_rows))
        if not arrays or n == 0:
            return None
        order: Dict[int, int] = {}

        def dfs(st):
            order[id(st)] = len(order)
            for c in getattr(st, "children", []) or []:
                dfs(c)
        dfs(self.copybook.ast)
        segs = plan.segment_groups
        root_pos = order[id(segs[root_seg])]
        has_kids = {sgi for sgi, g in enumerate(segs) if any(h.parent_segment is g for h in segs)}
        deps: List[int] = []               # dependee field indices, in the device table's order
        events: Dict[int, List[Tuple[int, int]]] = {}   # event row -> [(field order, event)]
        odo: List[Tuple[int, Any]] = []
        for ai, ar in arrays:
            df = plan.fields[ar.dependee]
            dcol = plan.columns[df.column]
            anode = plan.columns[ar.count_column].node
            if dcol.out_type in (N.O_STRING, N.O_BINARY):
                if df.segment != ar.segment:
                    raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: a string DEPENDING ON field "
                                                          "outside the array's segment")
                continue
            if dcol.out_type not in (N.O_I32, N.O_I64, N.O_DEC128):
                raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: a DEPENDING ON field decoded as "
                                                      "floating point")
            if ar.dependee not in deps:
                deps.append(ar.dependee)
                e = deps.index(ar.dependee)
                pos = order[id(dcol.node)]
                if df.segment < 0 or df.segment != root_seg and order[id(segs[df.segment])] < root_pos:
                    # decoded from the root's bytes ahead of the root segment's group: the common header,
                    # or a segment group placed before the root's (registered before the children walk;
                    # after the root's group, once the children are walked -- no array of theirs sees it)
                    if df.segment >= 0 and df.segment in has_kids:
                        # the root's walk also extracts that group's own children over the record's rows
                        # (getGroupValues of any segment redefine, :361-369) -- registrations not modelled
                        raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: a DEPENDING ON field in a "
                                                              "segment group with children placed before the root "
                                                              "segment's")
                    if pos < root_pos:
                        events.setdefault(N.CBX_HIER_MAX_SEG, []).append((pos, e))
                if df.segment >= 0:
                    events.setdefault(df.segment, []).append((pos, e))
            odo.append((ai, ar))
            events.setdefault(ar.segment, []).append((order[id(anode)], -len(odo)))
        if not odo:
            return None
        if len(deps) > N.CBX_HIER_MAX_DEPS or len(odo) > N.CBX_HIER_MAX_DEPS or \
                any(len(v) > N.CBX_HIER_MAX_EVENTS for v in events.values()):
            raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: more DEPENDING ON fields / arrays than "
                                                  "cbx_hier_dependee_counts takes")
        L = N.load()
        sp = ctypes.c_void_p(stream.cuda_stream)
        dev = sel["rec_off"].device
        w = self._hier_walk_struct(table_rows, child_offsets, root_seg, order, events)
        vals, valid, dt = self._hier_dependee_columns(d_data, n_bytes, sel, deps, n, stream)
        at = (N.CbxHierOdoArray * len(odo))()
        for k, (ai, ar) in enumerate(odo):
            at[k].dependee, at[k].out_row = deps.index(ar.dependee), ai
            at[k].min_count, at[k].max_count = ar.min_count, ar.max_count
            at[k].first_counts = None
        out = torch.full((len(plan.arrays), n), -1, dtype=torch.int32, device=dev)
        changed = torch.zeros(1, dtype=torch.int32, device=dev)
        N.check(L.cbx_hier_dependee_counts(ctypes.byref(w), dt, len(deps), at, len(odo), out.data_ptr(), n,
                                           changed.data_ptr(), sp))
        out._cbx_keep = (vals, valid)   # (the value columns live until the resolution has run)
        return out

    def _hier_walk_struct(self, table_rows: List[int], child_offsets, root_seg: int, order: Dict[int, int],
                          events: Dict[int, List[Tuple[int, int]]]):
        """cbx_hier_walk: tables, child segments in copybook order, their list offsets, events in field order."""
        segs = self.plan.segment_groups
        w = N.CbxHierWalk()
        w.n_segments, w.root_segment = len(segs), root_seg
        base = np.concatenate([[0], np.cumsum(table_rows)]).astype(np.int64)
        for t in range(len(table_rows)):
            w.table_base[t], w.table_rows[t] = int(base[t]), int(table_rows[t])
        for sgi in range(N.CBX_HIER_MAX_SEG):
            for k in range(N.CBX_HIER_MAX_SEG):
                w.children[sgi][k] = -1
            for k in range(N.CBX_HIER_MAX_EVENTS):
                w.events[sgi][k] = N.HIER_EVENT_END
        for k in range(N.CBX_HIER_MAX_EVENTS):
            w.events[N.CBX_HIER_MAX_SEG][k] = N.HIER_EVENT_END
        for sgi, g in enumerate(segs):
            kids = sorted((c for c, h in enumerate(segs) if h.parent_segment is g), key=lambda c: order[id(segs[c])])
            for k, c in enumerate(kids):
                w.children[sgi][k] = c
            if sgi in child_offsets:
                w.child_offsets[sgi] = child_offsets[sgi].data_ptr()
        for row, evs in events.items():
            for k, (_, e) in enumerate(sorted(evs)):
                w.events[row][k] = e
        w.seeds = None
        return w

    def _hier_dependee_columns(self, d_data, n_bytes: int, sel: Dict[str, Any], deps: List[int], n: int, stream,
                               slots: Optional[List[int]] = None):
        """Every dependee field decoded from every row's own bytes (the rows' registrations,
        cbx_hier_dependee_values): (values, validity, the cbx_hier_dependee table)."""
        torch = _torch()
        L = N.load()
        sp = ctypes.c_void_p(stream.cuda_stream)
        dev = sel["rec_off"].device
        vals = torch.empty((max(1, len(deps)), n), dtype=torch.int64, device=dev)
        valid = torch.empty((max(1, len(deps)), (n + 63) // 64), dtype=torch.int64, device=dev)
        dt = (N.CbxHierDependee * max(1, len(deps)))()
        for e, fi in enumerate(deps):
            N.check(L.cbx_hier_dependee_values(self.native.handle, d_data.data_ptr(), n_bytes, sel["rec_off"].data_ptr(),
                                               sel["rec_len"].data_ptr(), n, self.params.start_offset, fi,
                                               vals[e].data_ptr(), valid[e].data_ptr(), sp))
            is_str = self.plan.columns[self.plan.fields[fi].column].out_type in (N.O_STRING, N.O_BINARY)
            dt[e].values, dt[e].validity = vals[e].data_ptr(), valid[e].data_ptr()
            dt[e].out_type = N.O_STRING if is_str else N.O_I64
            dt[e].walk_slot = slots[e] if slots is not None else -1
        return vals, valid, dt

    def _hier_walk_seeds(self, d_data, n_bytes: int, sel: Dict[str, Any], table_rows: List[int], child_offsets,
                         root_seg: int, stream):
        """Record-walk plans: each row's dependFields map at the row's start, as extractHierarchicalRecord's
        walk leaves it (RecordExtractors.scala:224-245, walk order :324-372) -- the registrations of the
        rows before it in the walk, and for a root row those of the root's groups ahead of the root
        segment's (the common header, segment groups placed before it, from the root's bytes).  The walk
        kernel then resolves every count itself, registering the row's own dependees as it goes (a child
        row: its segment group's only).  Returns int64 [8, rows] (cbx_plan_set_dep_seed)."""
        torch = _torch()
        plan, walk = self.plan, self.plan.walk
        n = int(sum(table_rows))
        dev = sel["rec_off"].device
        seeds = torch.zeros((8, max(1, n)), dtype=torch.int64, device=dev)
        if n == 0:
            return seeds
        order: Dict[int, int] = {}

        def dfs(st):
            order[id(st)] = len(order)
            for c in getattr(st, "children", []) or []:
                dfs(c)
        dfs(self.copybook.ast)
        segs = plan.segment_groups
        root_pos = order[id(segs[root_seg])]
        has_kids = {sgi for sgi, g in enumerate(segs) if any(h.parent_segment is g for h in segs)}
        deps: List[int] = []
        slots: List[int] = []
        events: Dict[int, List[Tuple[int, int]]] = {}
        for nd in walk.nodes:
            if nd.dep_slot < 0 or nd.field < 0 or nd.field in deps:
                continue
            fi = nd.field
            df = plan.fields[fi]
            pos = order[id(plan.columns[df.column].node)]
            e = len(deps)
            deps.append(fi)
            slots.append(nd.dep_slot)
            if df.segment < 0 or df.segment != root_seg and order[id(segs[df.segment])] < root_pos:
                if df.segment >= 0 and df.segment in has_kids:
                    raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: a DEPENDING ON field in a segment "
                                                          "group with children placed before the root segment's")
                if pos < root_pos:
                    events.setdefault(N.CBX_HIER_MAX_SEG, []).append((pos, e))
            if df.segment >= 0:
                events.setdefault(df.segment, []).append((pos, e))
        if len(deps) > N.CBX_HIER_MAX_DEPS or any(len(v) > N.CBX_HIER_MAX_EVENTS for v in events.values()):
            raise N.CbxError(N.CBX_E_UNSUPPORTED, "hierarchical records: more DEPENDING ON fields than "
                                                  "cbx_hier_dependee_counts takes")
        w = self._hier_walk_struct(table_rows, child_offsets, root_seg, order, events)
        w.seeds = seeds.data_ptr()
        vals, valid, dt = self._hier_dependee_columns(d_data, n_bytes, sel, deps, n, stream, slots)
        changed = torch.zeros(1, dtype=torch.int32, device=dev)
        N.check(N.load().cbx_hier_dependee_counts(ctypes.byref(w), dt, len(deps), None, 0, None, n, changed.data_ptr(),
                                                  ctypes.c_void_p(stream.cuda_stream)))
        seeds._cbx_keep = (vals, valid)
        return seeds

    def read(self, data: bytes, file_id: int = 0, input_file_name: Optional[str] = None) -> DecodedBatch:
        """A whole file, as the reference reads it: sparse-index entries (when index generation
        applies) each read by its own VarLenNestedIterator, concatenated in file order.
        input_file_name: the file's name for the with_input_file_name_col column."""
        self._file_column(None, input_file_name, check_only=True)
        t = self._device_file(data)
        off, ln, vb = self.frame_file(t, len(data))
        if self.hierarchical:
            return self._file_column(self.read_hierarchical(t, vb, off, ln, file_id), input_file_name)
        entries = None
        if self.index_generation_needed() and not self.params.is_text:
            entries = self.generate_index(t, len(data), off, ln, file_id)
        sel = self.select(t, vb, off, ln, entries, file_id)
        return self._file_column(self.decode_selected(t, vb, sel), input_file_name)

    def decode(self, data: bytes, seeds: Optional[Sequence[int]] = None, first_record_id: int = 0,
               input_file_name: Optional[str] = None) -> DecodedBatch:
        """Frame + decode as one entry (no selection stage).  input_file_name: as in `read`."""
        self._file_column(None, input_file_name, check_only=True)
        t = self._device_file(data)
        if self.params.is_text or self.var_occurs_extractor() or (
                self.params.record_length_field is not None and not self.params.is_record_sequence):
            # framings that are not seeded by RDW headers: text lines, VarOccursRecordExtractor,
            # record_length_field (VRLRecordReader.fetchRecordUsingRecordLengthField)
            off, ln, vb = self.frame_file(t, len(data))
            return self._file_column(self.decode_device(t, vb, off, ln, first_record_id), input_file_name)
        off, ln = self.frame(t, len(data), seeds) if self.params.is_record_sequence else self.frame_fixed(t, len(data))
        return self._file_column(self.decode_device(t, len(data), off, ln, first_record_id), input_file_name)

    def get_row_iterator(self, data: bytes) -> Iterator[dict]:
        return iter(self.read(data).to_rows())
