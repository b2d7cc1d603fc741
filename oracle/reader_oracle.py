"""TEST INFRASTRUCTURE ONLY: the reference's readers around `extractRecord`, restated in Python.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.  It
restates, literally and for small inputs, the record-stream logic of the variable-length reader
that turns a file into rows (CP = cobol-parser/src/main/scala/za/co/absa/cobrix/cobol/,
SC = spark-cobol/src/main/scala/za/co/absa/cobrix/spark/cobol/):

  * FileStreamer (bounded per index entry)   SC/source/streaming/FileStreamer.scala:30-80
  * RecordHeaderParserRDW / ...FixedLen       CP/parser/headerparsers/RecordHeaderParserRDW.scala:44-85,
                                              RecordHeaderParserFixedLen.scala:40-50
  * IndexGenerator.sparseIndexGenerator       CP/reader/index/IndexGenerator.scala:33-157
  * VarLenNestedReader.generateIndex          CP/reader/VarLenNestedReader.scala:125-180
  * VRLRecordReader (record index, seg id)    CP/reader/iterator/VRLRecordReader.scala:39-198
  * VarLenNestedIterator (filter, root-reached, redefine map, Record_Id)
                                              CP/reader/iterator/VarLenNestedIterator.scala:80-147
  * SegmentIdAccumulator (Seg_IdN)            CP/reader/iterator/SegmentIdAccumulator.scala:19-86
  * VarOccursRecordExtractor                  CP/reader/extractors/raw/VarOccursRecordExtractor.scala:30-154
  * VarLenHierarchicalIterator + extractHierarchicalRecord (segment-children)
                                              CP/reader/iterator/VarLenHierarchicalIterator.scala:43-162,
                                              CP/reader/extractors/record/RecordExtractors.scala:211-385
  * applyRecordPostProcessing                 CP/reader/extractors/record/RecordExtractors.scala:409-451
  * CobolScanners.buildScanForVarLenIndex     SC/source/scanners/CobolScanners.scala:38-55

Field values themselves come from the C oracle's extractRecord restatement (oracle.py).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from decimal import Decimal as PyDecimal
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from cobrix_amd import copybook as cbk
from cobrix_amd.schema import ST_DECIMAL, spark_type
from oracle import oracle as O

MEGABYTE = 1024 * 1024
MAX_RDW = 100 * MEGABYTE      # Constants.maxRdWRecordSize (CP/parser/common/Constants.scala)
DEFAULT_ENTRY_MB = 100        # Constants.defaultIndexEntrySizeMB


class Stream:
    """FileStreamer over an in-memory file: absolute offsets, optionally bounded to
    `maximum_bytes` after `start` (checked before each read, so the last read may cross it)."""

    def __init__(self, data: bytes, start: int = 0, maximum_bytes: int = 0):
        self.data, self.start, self.maximum = data, start, maximum_bytes
        self.offset = start
        self.closed = False

    @property
    def size(self) -> int:
        return min(len(self.data), self.maximum + self.start) if self.maximum > 0 else len(self.data)

    @property
    def is_end_of_stream(self) -> bool:   # SimpleStream.isEndOfStream
        return self.offset >= self.size

    def next(self, n: int) -> bytes:
        if (self.maximum > 0 and self.offset - self.start >= self.maximum) or self.closed:
            self.closed = True
            return b""
        b = self.data[self.offset:self.offset + n]
        self.offset += len(b)
        if len(b) < n:
            self.closed = True
        return b


class RdwHeaderParser:
    """RecordHeaderParserRDW.getRecordMetadata (:44-85)."""
    header_length = 4

    def __init__(self, big_endian: bool, file_header: int, file_footer: int, adjustment: int):
        self.be, self.fh, self.ff, self.adj = big_endian, file_header, file_footer, adjustment

    def metadata(self, header: bytes, file_offset: int, file_size: int) -> Tuple[int, bool]:
        if self.fh > 4 and file_offset == 4:
            return self.fh - 4, False
        if file_size > 0 and self.ff > 0 and file_size - file_offset <= self.ff:
            return file_size - file_offset, False
        if len(header) < 4:
            return -1, False
        n = (header[1] + 256 * header[0] if self.be else header[2] + 256 * header[3]) + self.adj
        if n > 0:
            if n > MAX_RDW:
                raise RuntimeError(f"RDW headers too big (length = {n} > {MAX_RDW}) at {file_offset}.")
            return n, True
        raise RuntimeError(f"RDW headers should never be zero. Found zero size record at {file_offset}.")


class FixedLenHeaderParser:
    """RecordHeaderParserFixedLen.getRecordMetadata (:40-50): no header bytes."""
    header_length = 0

    def __init__(self, record_size: int, file_header: int, file_footer: int):
        self.rs, self.fh, self.ff = record_size, file_header, file_footer

    def metadata(self, header: bytes, file_offset: int, file_size: int) -> Tuple[int, bool]:
        if self.fh > 0 and file_offset == 0:
            return self.fh, False
        if file_size > 0 and self.ff > 0 and file_size - file_offset <= self.ff:
            return file_size - file_offset, False
        if file_size - file_offset >= self.rs:
            return self.rs, True
        return -1, False


def header_parser(cb: cbk.Copybook, p) -> Any:
    """VarLenNestedReader.getDefaultRecordHeaderParser (:267-296)."""
    adj = (-4 if p.is_rdw_part_rec_length else 0) + p.rdw_adjustment
    if p.is_record_sequence:
        return RdwHeaderParser(p.is_rdw_big_endian, p.file_start_offset, p.file_end_offset, adj)
    return FixedLenHeaderParser(cb.record_size, p.file_start_offset, p.file_end_offset)


def _java_string(v) -> str:
    """Any.toString of a decoded value (Int/Long/BigDecimal/String)."""
    if v is None:
        return ""
    if isinstance(v, PyDecimal):
        return str(v)   # BigDecimal.toString (plain for the scales Cobrix produces)
    return str(v)


class FieldReader:
    """Copybook.extractPrimitiveField(field, bytes, startOffset) (Copybook.scala:165-168)."""

    def __init__(self, cb: cbk.Copybook, field: cbk.Primitive):
        self.ast = O.OracleAst(cb)
        self.field = field
        self.node = self.ast.nodes[self.ast.node_of(field)]

    def value(self, data: bytes, start_offset: int = 0):
        f = self.field
        sl = data[f.offset + start_offset: f.offset + start_offset + f.actual_size]
        buf = np.frombuffer(sl, dtype=np.uint8) if sl else np.zeros(1, np.uint8)
        ev = np.zeros(1, dtype=O.EVENT_DTYPE)
        heap = np.zeros(4 * len(sl) + 64, dtype=np.uint8)
        hl = ctypes.c_int64(0)
        rc = O.lib().ora_decode_field(ctypes.byref(self.node), ctypes.byref(self.ast.opts), buf.ctypes.data, len(sl),
                                      ev.ctypes.data, heap.ctypes.data, len(heap), ctypes.byref(hl))
        assert rc == 0
        v = O.event_value(ev[0], heap.tobytes())
        if v is not None and int(ev[0]["stype"]) == ST_DECIMAL:
            v = PyDecimal(v).scaleb(-spark_type(f)[2])
        return v

    def segment_id(self, data: bytes, start_offset: int = 0) -> str:
        """VRLRecordReader.getSegmentId (:188-198): value.toString.trim, "" for null."""
        return _trim(_java_string(self.value(data, start_offset)))


def _trim(s: str) -> str:
    b, e = 0, len(s)
    while b < e and s[b] <= " ":
        b += 1
    while e > b and s[e - 1] <= " ":
        e -= 1
    return s[b:e]


@dataclass
class Entry:
    offset_from: int
    offset_to: int
    file_id: int
    record_index: int


def sparse_index(cb: cbk.Copybook, data: bytes, p, file_id: int = 0,
                 default_entry_bytes: Optional[int] = None, split_bytes: Optional[int] = None,
                 start_bytes: int = 0) -> List[Entry]:
    """VarLenNestedReader.generateIndex (:125-180) -> IndexGenerator.sparseIndexGenerator (:33-157).
    default_entry_bytes replaces Constants.defaultIndexEntrySizeMB (tests of the reset rule on
    small files); split_bytes replaces split_mb * MEGABYTE of an explicit (subtracted) split size (tests
    of the subtract rule on small files).  start_bytes: bytesInChunk as of the first record, taken as an
    entry already cut (a piece of a file that starts at one of its entries; 0 for a whole file -- where
    the first record is never cut either)."""
    rp = header_parser(cb, p)
    split_records = p.input_split_records
    split_mb = p.input_split_size_mb if p.input_split_size_mb is not None else p.hdfs_default_block_size_mb
    if split_records is not None and not (1 <= split_records <= 1000000000):
        raise ValueError(f"Invalid input split size. The requested number of records is {split_records}.")
    if split_records is None and split_mb is not None and not (1 <= split_mb <= 2000):
        raise ValueError(f"Invalid input split size of {split_mb} MB.")
    seg_reader = FieldReader(cb, cb.get_field_by_name(p.segment_field)) if p.segment_field else None
    parents = getattr(p, "segment_redefine_parents", {}) or {}
    is_hier = bool(p.segment_id_levels) or bool(parents)   # segmentLevelIds.nonEmpty || fieldParentMap.nonEmpty
    root_id = p.segment_id_levels[0] if p.segment_id_levels else ""
    if parents and p.segment_id_redefine_map:   # VarLenNestedReader.getRootSegmentId (:298-309)
        root_id = next(iter(root_segment_ids(cb, p)), "")
    root_ids = root_id.split(",")
    really_hier = seg_reader is not None and is_hier
    split_by_size = split_records is None and split_mb is not None
    bytes_per = split_mb * MEGABYTE if split_mb is not None else (default_entry_bytes or DEFAULT_ENTRY_MB * MEGABYTE)
    if split_bytes is not None:
        split_by_size, bytes_per = split_records is None, split_bytes

    def need_split(records: int, size: int) -> bool:
        return records >= split_records if split_records is not None else size >= bytes_per

    s = Stream(data)
    index = [Entry(0, -1, file_id, 0)]
    byte_index = records_in_chunk = record_index = 0
    bytes_in_chunk = start_bytes
    root_record_id = ""
    while True:
        hdr = s.next(rp.header_length)
        n, valid = rp.metadata(hdr, s.offset, s.size)
        record = s.next(n) if n > 0 else b""
        record_size = s.offset - byte_index
        if s.is_end_of_stream or record_size <= 0:
            break
        if valid:
            if really_hier and root_record_id == "":
                cur = _trim(seg_reader.segment_id(record))
                if (cur != "" and not root_ids) or cur in root_ids:
                    root_record_id = cur
            if record_index > 0 and need_split(records_in_chunk, bytes_in_chunk):
                if not really_hier or _trim(seg_reader.segment_id(record)) in root_ids:
                    index[-1].offset_to = byte_index
                    index.append(Entry(byte_index, -1, file_id, record_index))
                    records_in_chunk = 0
                    if split_by_size:
                        bytes_in_chunk -= bytes_per
                    else:
                        bytes_in_chunk = 0
        record_index += 1
        records_in_chunk += 1
        byte_index += record_size
        bytes_in_chunk += record_size
    return index


def root_segment_ids(cb: cbk.Copybook, p) -> List[str]:
    """CopybookParser.getRootSegmentIds (:751-769): ids mapped to a redefine without a parent."""
    parents = getattr(p, "segment_redefine_parents", {}) or {}
    roots = set(parents.values()) - set(parents)
    return [sid for sid, grp in p.segment_id_redefine_map.items() if grp in roots]


def var_occurs_records(cb: cbk.Copybook, data: bytes) -> List[bytes]:
    """VarOccursRecordExtractor.next over the whole stream (:37-154): each record is the walked
    prefix of the stream -- OCCURS DEPENDING ON counts from the dependees read so far (dependFields,
    string dependees through dependingOnHandlers), every non-redefined field advancing by its walked
    size -- zero-filled when the stream ends early; a record starts where the previous ended."""
    fields = {}

    def has_var_occurs(g) -> bool:
        for c in g.children:
            if isinstance(c, cbk.Group):
                if has_var_occurs(c):
                    return True
            elif c.is_dependee:
                return True
        return False

    max_size = cb.record_size
    out: List[bytes] = []
    pos = 0
    ast = O.OracleAst(cb)
    var = has_var_occurs(cb.ast)
    while pos < len(data):   # hasNext: offset < size
        if not var:
            out.append(data[pos:pos + max_size])
            pos += max_size
            continue
        buf = bytearray(max_size)
        got = [0]
        dep: Dict[str, Any] = {}

        def ensure(n: int):
            need = n - got[0]
            if need > 0:
                chunk = data[pos + got[0]:pos + n]
                if len(chunk) > 0:
                    buf[got[0]:got[0] + len(chunk)] = chunk
                    got[0] = n

        def extract_array(f, off: int) -> int:
            size = f.array_max_size
            if f.depending_on is not None:
                v = dep.get(f.depending_on, ("L", size))
                n = v[1] if v[0] == "L" else f.depending_on_handlers.get(v[1], size)
                size = n if f.array_min_size <= n <= f.array_max_size else f.array_max_size
            o = off
            if isinstance(f, cbk.Group):
                for _ in range(size):
                    o += extract_group(o, f)
            else:
                o += f.data_size * size
            return o - off

        def extract_value(f, off: int) -> int:
            if isinstance(f, cbk.Group):
                return extract_group(off, f)
            if f.is_dependee:
                ensure(off + f.actual_size)
                v = FieldReader(cb, f).value(bytes(buf), off - f.offset)
                if v is not None:
                    dep[f.name] = ("R", v) if isinstance(v, str) else ("L", int(v))
            return f.actual_size

        def extract_group(off: int, g) -> int:
            o = off
            for c in g.children:
                size = extract_array(c, o) if c.is_array else extract_value(c, o)
                if not c.is_redefined:
                    o += size
            return o - off

        nxt = 0
        for rec in cb.ast.children:
            nxt += extract_group(nxt, rec)
        ensure(nxt)
        out.append(bytes(buf[:nxt]))
        pos += nxt
    del fields, ast
    return out


def index_generation_needed(p) -> bool:
    """VarLenNestedReader.isIndexGenerationNeeded (:85)."""
    return (getattr(p, "record_length_field", None) is None or p.is_record_sequence) and p.enable_indexes


def _java_int(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


class LengthFieldReader:
    """VRLRecordReader.fetchRecordUsingRecordLengthField (CP/reader/iterator/VRLRecordReader.scala:114-149)
    with ReaderParametersValidator.getLengthField's checks (:26-43)."""

    def __init__(self, cb: cbk.Copybook, p):
        f = cb.get_field_by_name(p.record_length_field)
        if not isinstance(f, cbk.Primitive) or not isinstance(f.dtype, cbk.Integral):
            raise ValueError(f"The record length field {p.record_length_field} must be an integral type.")
        if f.occurs is not None and f.occurs > 1:
            raise ValueError(f"The record length field '{p.record_length_field}' cannot be an array.")
        self.reader = FieldReader(cb, f)
        self.lfb = f.offset + f.actual_size          # lengthFieldBlock
        self.start, self.end, self.adj = p.start_offset, p.end_offset, p.rdw_adjustment
        self.name = p.record_length_field

    def fetch(self, s: "Stream") -> Optional[bytes]:
        head = s.next(self.start + self.lfb)
        if len(head) < self.start + self.lfb:
            return None
        v = self.reader.value(head, self.start)
        if not isinstance(v, int) or isinstance(v, bool):   # Int / Long; null, BigDecimal: the catch-all case
            raise RuntimeError(f"Record length value of the field {self.name} must be an integral type.")
        rest = _java_int(_java_int(_java_int(v) + self.adj) - self.lfb + self.end)
        return head + s.next(rest) if rest > 0 else head


class SegmentIdAccumulator:
    """SegmentIdAccumulator.scala:19-86."""

    def __init__(self, segment_ids: Sequence[str], prefix: str, file_id: int):
        self.ids = [s.split(",") for s in segment_ids]
        self.count = len(segment_ids)
        self.acc = [0] * (self.count + 1)
        self.level = -1
        self.root = ""
        self.prefix, self.file_id = prefix, file_id

    def acquired(self, segment_id: str, record_index: int) -> None:
        if self.count == 0:
            return
        lvl = next((i for i in range(self.count) if segment_id in self.ids[i]), None)
        if lvl is not None:
            self.level = lvl
            if lvl == 0:
                self.root = f"{self.prefix}_{self.file_id}_{record_index}"
                self.acc = [0] * (self.count + 1)
            else:
                self.acc[lvl] += 1

    def level_id(self, level: int) -> Optional[str]:
        if 0 <= level <= self.level:
            return self.root if level == 0 else f"{self.root}_L{level}_{self.acc[level]}"
        return None


@dataclass
class VarRecord:
    payload: bytes
    record_id: int
    seg_ids: List[Optional[str]]
    active_segment: Optional[str]       # redefine group name (transformed identifier) or None


def var_len_records(cb: cbk.Copybook, data: bytes, p, file_id: int = 0,
                    entries: Optional[List[Entry]] = None) -> List[VarRecord]:
    """The records VarLenNestedIterator returns for every index entry, in file order."""
    rp = header_parser(cb, p)
    if entries is None:
        entries = sparse_index(cb, data, p, file_id) if index_generation_needed(p) else [Entry(0, -1, file_id, 0)]
    seg_reader = FieldReader(cb, cb.get_field_by_name(p.segment_field)) if p.segment_field else None
    levels = list(p.segment_id_levels) if p.segment_field else []
    filt = p.segment_id_filter if p.segment_field else None
    red = p.segment_id_redefine_map if p.segment_field else {}
    out: List[VarRecord] = []
    for e in entries:
        n_bytes = e.offset_to - e.offset_from if e.offset_to > 0 else 0
        s = Stream(data, e.offset_from, n_bytes)
        acc = SegmentIdAccumulator(levels, p.segment_id_prefix, e.file_id) if p.segment_field else None
        record_index = e.record_index - 1
        lf = LengthFieldReader(cb, p) if (getattr(p, "record_length_field", None) and not p.is_record_sequence) else None
        while True:
            if lf is not None:
                rec = lf.fetch(s)
                if rec is None:
                    break
            else:
                # VRLRecordReader.fetchRecordUsingRdwHeaders (:151-186)
                valid = False
                eof = False
                rec = b""
                while not valid and not eof:
                    hdr = s.next(rp.header_length)
                    n, valid = rp.metadata(hdr, s.offset, s.size)
                    if n > 0:
                        rec = s.next(n)
                    else:
                        eof = True
                if eof:
                    break
            record_index += 1
            sid = _trim(seg_reader.segment_id(rec, p.start_offset)) if seg_reader else ""
            ids: List[Optional[str]] = []
            if levels and acc is not None:
                acc.acquired(sid, record_index)
                ids = [acc.level_id(i) for i in range(len(levels))]
            root_reached = not ids or ids[0] is not None
            if not root_reached or (filt is not None and sid not in filt):
                continue
            grp = red.get(sid) if red else None
            out.append(VarRecord(rec, record_index, ids, grp))
    return out


def raw_records(cb: cbk.Copybook, data: bytes, p, e: Entry) -> List[Tuple[str, bytes]]:
    """VRLRecordReader over one entry's bounded stream: (segment id, payload) of every valid record."""
    rp = header_parser(cb, p)
    seg_reader = FieldReader(cb, cb.get_field_by_name(p.segment_field)) if p.segment_field else None
    n_bytes = e.offset_to - e.offset_from if e.offset_to > 0 else 0
    s = Stream(data, e.offset_from, n_bytes)
    out = []
    while True:
        valid, eof, rec = False, False, b""
        while not valid and not eof:
            hdr = s.next(rp.header_length)
            n, valid = rp.metadata(hdr, s.offset, s.size)
            if n > 0:
                rec = s.next(n)
            else:
                eof = True
        if eof:
            return out
        out.append((_trim(seg_reader.segment_id(rec, p.start_offset)) if seg_reader else "", rec))


def _hier_tables(cb: cbk.Copybook, ast) -> Dict[str, Any]:
    """Node-indexed tables ora_extract_hier walks by: parentChildMap (child segment group ids per
    segment redefine, in the copybook's order), each node's binary offset, child-segment and
    has-a-parent-segment flags."""
    n = len(ast.stmts)
    redefines = cb.all_segment_redefines()
    begin = np.zeros(n, np.int32)
    end = np.zeros(n, np.int32)
    kids: List[int] = []
    for i, st in enumerate(ast.stmts):
        begin[i] = len(kids)
        if isinstance(st, cbk.Group) and st.is_segment_redefine:
            kids += [ast.node_of(c) for c in redefines if c.parent_segment is st]
        end[i] = len(kids)
    return {"begin": begin, "end": end, "children": np.array(kids or [0], np.int32),
            "offset": np.array([getattr(st, "offset", 0) for st in ast.stmts], np.int32),
            "child": np.array([int(isinstance(st, cbk.Group) and st.is_child_segment) for st in ast.stmts], np.int32),
            "has_parent": np.array([int(isinstance(st, cbk.Group) and st.parent_segment is not None)
                                    for st in ast.stmts], np.int32)}


def _hier_row_values(ast, ev, heap) -> List[Tuple[Any, dict]]:
    """The event stream of one ora_extract_hier call -> [(top-level group, values)]: getGroupValues'
    shape -- no entry for a child-segment field, each segment redefine's child segments appended as
    lists (one ORA_EV_CHILDREN count, then each child's group)."""
    cb = ast.cb
    redefines = cb.all_segment_redefines()
    pos = 0

    def dec_value(st, e):
        v = O.event_value(e, heap)
        if v is not None and int(e["stype"]) == ST_DECIMAL:
            v = PyDecimal(v).scaleb(-spark_type(st)[2])
        return v

    def walk(g) -> dict:
        nonlocal pos
        d = {}
        for c in g.children:
            if isinstance(c, cbk.Group) and c.is_child_segment:
                continue   # decoded, not kept (and no events)
            if c.is_array:
                cnt = int(ev[pos]["lo"])
                pos += 1
                vals = []
                for _ in range(cnt):
                    if isinstance(c, cbk.Group):
                        vals.append(walk(c))
                    else:
                        vals.append(dec_value(c, ev[pos]))
                        pos += 1
                val: Any = vals
            elif isinstance(c, cbk.Group):
                val = walk(c)
            else:
                val = dec_value(c, ev[pos])
                pos += 1
            if not c.is_filler:
                d[c.name] = val
        if g.is_segment_redefine:
            for ch in (c for c in redefines if c.parent_segment is g):
                e = ev[pos]
                assert int(e["kind"]) == O.EV_CHILDREN and int(e["node"]) == ast.node_of(ch)
                pos += 1
                d[ch.name] = [walk(ch) for _ in range(int(e["lo"]))]
        return d

    return [(g, walk(g)) for g in cb.ast.children if isinstance(g, cbk.Group) and g.parent_segment is None]


def hier_rows(cb: cbk.Copybook, data: bytes, p, file_id: int = 0,
              entries: Optional[List[Entry]] = None) -> List[dict]:
    """VarLenHierarchicalIterator (:83-160) per index entry -- records grouped from one root segment
    record to the next -- + extractHierarchicalRecord (oracle/cobrix_oracle.c ora_extract_hier: one
    dependFields map shared by the hierarchical record's segments, the root from record_start_offset,
    children at their group's offset in their own data, the reference's DFS order) +
    applyRecordPostProcessing."""
    if entries is None:
        entries = sparse_index(cb, data, p, file_id) if index_generation_needed(p) else [Entry(0, -1, file_id, 0)]
    red = p.segment_id_redefine_map
    roots = set(root_segment_ids(cb, p))
    ast = O.OracleAst(cb)
    tb = _hier_tables(cb, ast)
    group_node = {g.name: ast.node_of(g) for g in cb.all_segment_redefines()}
    keys: Dict[str, int] = {}
    L = O.lib()
    out: List[dict] = []

    def emit(recs: List[Tuple[str, bytes]], record_id: int):
        n = len(recs)
        bufs = [np.frombuffer(r, dtype=np.uint8) if len(r) else np.zeros(1, np.uint8) for _, r in recs]
        ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
        lens = np.array([len(r) for _, r in recs], np.int32)
        seg_group = np.array([group_node.get(red.get(sid, ""), -1) for sid, _ in recs], np.int32)
        seg_key = np.array([keys.setdefault(sid, len(keys)) for sid, _ in recs], np.int32)
        ev_cap = max(1, n * ast.max_events_per_record() * 2 + 64)
        ev = np.zeros(ev_cap, dtype=O.EVENT_DTYPE)
        heap_cap = max(64, sum(len(r) for _, r in recs) * 3 * (1 + len(group_node)) + 64 * n + 64)
        heap = np.zeros(heap_cap, dtype=np.uint8)
        n_ev, hl = ctypes.c_int64(0), ctypes.c_int64(0)
        rc = L.ora_extract_hier(ctypes.addressof(ast.nodes), 0, ctypes.addressof(ast.handlers),
                                ctypes.addressof(ast.opts), n, ptrs, O._ptr(lens), O._ptr(seg_group), O._ptr(seg_key),
                                O._ptr(tb["begin"]), O._ptr(tb["end"]), O._ptr(tb["children"]), O._ptr(tb["offset"]),
                                O._ptr(tb["child"]), O._ptr(tb["has_parent"]), p.start_offset, 0, O._ptr(ev), ev_cap,
                                ctypes.byref(n_ev), O._ptr(heap), heap_cap, ctypes.byref(hl))
        if rc != 0:
            raise RuntimeError(f"oracle hierarchical decode failed: {rc}")
        recs_v = _hier_row_values(ast, ev[:n_ev.value], heap[:hl.value].tobytes())
        row: Dict[str, Any] = {}
        if p.generate_record_id:
            row["File_Id"] = e.file_id
            row["Record_Id"] = record_id
        if p.schema_policy == "collapse_root":
            for _, v in recs_v:
                row.update(v)
        else:
            row.update({g.name: v for g, v in recs_v})
        out.append(row)

    for e in entries:
        raw = raw_records(cb, data, p, e)
        record_index = e.record_index
        fetched: List[Tuple[str, bytes]] = []
        for sid, rec in raw:
            if sid in roots:
                if fetched:
                    emit(fetched, record_index)
                    fetched = []
                fetched.append((sid, rec))
            elif fetched:
                fetched.append((sid, rec))
            record_index += 1
        if fetched:
            emit(fetched, record_index)
    return out


def var_len_rows(cb: cbk.Copybook, data: bytes, p, file_id: int = 0,
                 entries: Optional[List[Entry]] = None) -> List[dict]:
    """Rows of a variable-length read (extractRecord + applyRecordPostProcessing); hierarchical
    copybooks go through VarLenHierarchicalIterator (SC/reader/VarLenNestedReader.scala:55-81)."""
    if cb.is_hierarchical:
        return hier_rows(cb, data, p, file_id, entries)
    if p.variable_size_occurs and not p.is_record_sequence and not p.is_text:
        # VarOccursRecordExtractor framing (VarLenNestedReader.recordExtractor, :60-78); one index entry
        payloads = var_occurs_records(cb, data)
        recs = [VarRecord(b, i, [], None) for i, b in enumerate(payloads)]
    else:
        recs = var_len_records(cb, data, p, file_id, entries)
    res = O.decode_records(cb, [r.payload for r in recs], start_offset=p.start_offset,
                           variable_size_occurs=p.variable_size_occurs,
                           active_segments=[r.active_segment for r in recs] if p.segment_id_redefine_map else None)
    body = O.rows(res, collapse_root=p.schema_policy == "collapse_root")
    rows = []
    for r, b in zip(recs, body):
        row: Dict[str, Any] = {}
        if p.generate_record_id:
            row["File_Id"] = file_id
            row["Record_Id"] = r.record_id
        for i, v in enumerate(r.seg_ids):
            row[f"Seg_Id{i}"] = v
        row.update(b)
        rows.append(row)
    return rows


def fixed_len_rows(cb: cbk.Copybook, data: bytes, p) -> List[dict]:
    """FixedLenNestedReader over a whole file (CobolScanners.buildScanForFixedLength + parseRecords)."""
    rs = (p.record_length if p.record_length is not None else cb.record_size)
    seg = p.segment_field if p.segment_id_redefine_map else None
    res = O.decode_fixed(cb, data, record_size=rs, start_offset=p.start_offset, end_offset=p.end_offset,
                         segment_field=seg, segment_redefine_map=p.segment_id_redefine_map or None)
    return O.rows(res, collapse_root=p.schema_policy == "collapse_root")
