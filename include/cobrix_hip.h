/*
 * cobrix_hip.h -- C ABI of the MI355X (gfx950) Cobrix record decoder (libcobrix_hip.so).
 *
 * Drop-in boundary: replaces, per BATCH of records, the per-record
 *   RecordExtractors.extractRecord(ast, data, offsetBytes, ...)            (CP/reader/extractors/record/RecordExtractors.scala:49-183)
 *   + Primitive.decodeTypeValue / DecoderSelector decoder closures        (CP/parser/ast/Primitive.scala:102-128,
 *                                                                            CP/parser/decoders/DecoderSelector.scala:54-290)
 * that sit under
 *   FixedLenReader.getRowIterator(binaryData)                              (SC/reader/FixedLenReader.scala:23-25)
 *   VarLenReader.getRowIterator(stream, startingFileOffset, fileNumber, startingRecordIndex)
 *                                                                          (SC/reader/VarLenReader.scala:44-60)
 * and, for RDW files, the sequential header walk of
 *   VRLRecordReader.fetchRecordUsingRdwHeaders / RecordHeaderParserRDW     (CP/reader/iterator/VRLRecordReader.scala:151-186,
 *                                                                            CP/parser/headerparsers/RecordHeaderParserRDW.scala:44-85)
 *   IndexGenerator.sparseIndexGenerator                                   (CP/reader/index/IndexGenerator.scala:33-127)
 * (CP = cobol-parser/src/main/scala/za/co/absa/cobrix/cobol/, SC = spark-cobol/src/main/scala/za/co/absa/cobrix/spark/cobol/)
 *
 * The JVM side flattens the parsed `Copybook` AST into the cbx_field / cbx_array tables below
 * (what the Scala/Python host does in cobrix_amd/plan.py) and calls this library through
 * JNI or Panama FFM with device (or pinned host) pointers.  Plain C types only.
 *
 * Error convention (mirrors the reference): data errors never fail a call -- a malformed value
 * decodes to null (validity bit 0), as DecoderSelector.scala:283-290 does.  Structural errors
 * return a negative status: CBX_E_ARGUMENT ~ IllegalArgumentException, CBX_E_STATE ~
 * IllegalStateException (bad RDW), with the detail in cbx_last_error().
 */
#ifndef COBRIX_HIP_H
#define COBRIX_HIP_H
#ifndef __HIPCC_RTC__
#include <stdint.h>
#else   /* compiled by hipRTC (the library's copybook-specialised kernels): its fixed-width types */
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define CBX_ABI_VERSION 20

/* status codes */
#define CBX_OK 0
#define CBX_E_ARGUMENT (-1)   /* IllegalArgumentException */
#define CBX_E_STATE (-2)      /* IllegalStateException (e.g. RDW length 0 or > 100 MiB) */
#define CBX_E_CAPACITY (-3)   /* caller buffer too small; required size reported */
#define CBX_E_HIP (-4)        /* HIP runtime failure */
#define CBX_E_UNSUPPORTED (-5)

/* field decode kinds (one per DecoderSelector branch) */
enum cbx_kind {
    CBX_K_STRING = 1,      /* EBCDIC string via code page, trimmed   StringDecoders.decodeEbcdicString */
    CBX_K_STRING_ASCII = 2,/* ASCII string                            StringDecoders.decodeAsciiString  */
    CBX_K_HEX = 3,         /* debug HEX string                        StringDecoders.decodeHex          */
    CBX_K_RAW = 4,         /* debug RAW bytes                         StringDecoders.decodeRaw          */
    CBX_K_BCD = 5,         /* COMP-3                                  BCDNumberDecoders                 */
    CBX_K_BINARY = 6,      /* COMP / COMP-4 / COMP-5 / COMP-9         BinaryNumberDecoders, BinaryUtils */
    CBX_K_ZONED = 7,       /* EBCDIC DISPLAY numeric                  StringDecoders.decodeEbcdicNumber */
    CBX_K_ASCII_NUM = 8,   /* ASCII DISPLAY numeric                   StringDecoders.decodeAsciiNumber  */
    CBX_K_FLOAT = 9,       /* COMP-1                                  FloatingPointDecoders             */
    CBX_K_DOUBLE = 10,     /* COMP-2                                  FloatingPointDecoders             */
    CBX_K_RECORD_ID = 11,  /* generated Record_Id (long)              RecordExtractors.scala:409-451    */
    CBX_K_FILE_ID = 12,    /* generated File_Id (int)                                                   */
    CBX_K_UTF16_BE = 13,   /* PIC N, is_utf16_big_endian=true         StringDecoders.decodeUtf16String  */
    CBX_K_UTF16_LE = 14    /* PIC N, is_utf16_big_endian=false                                          */
};

/* output (Spark) types -- SC/schema/CobolSchema.scala:144-173 */
enum cbx_out {
    CBX_O_I32 = 1, CBX_O_I64 = 2, CBX_O_DEC64 = 3, CBX_O_DEC128 = 4,
    CBX_O_F32 = 5, CBX_O_F64 = 6, CBX_O_STRING = 7, CBX_O_BINARY = 8
};

/* cbx_field.flags */
#define CBX_F_SIGNED 0x1        /* PIC has a sign (signPosition.isDefined) */
#define CBX_F_BIG_ENDIAN 0x2    /* binary: COMP/COMP-4/COMP-5 (COMP-9 is little-endian) */
#define CBX_F_EXPLICIT_DOT 0x4  /* DISPLAY with explicit decimal point */
#define CBX_F_INTEGRAL 0x8      /* AST type is Integral (else Decimal) */
#define CBX_F_IBM 0x10          /* COMP-1/2 in IBM hex float (else IEEE-754) */
#define CBX_F_LITTLE_ENDIAN_FP 0x20
#define CBX_F_DEPENDEE 0x40     /* an OCCURS DEPENDING ON source (isDependee) */
#define CBX_F_LIST 0x80         /* element of a list-layout OCCURS DEPENDING ON array (cbx_array.offsets_column) */

/* string trimming (StringTrimmingPolicy) */
#define CBX_TRIM_NONE 1
#define CBX_TRIM_LEFT 2
#define CBX_TRIM_RIGHT 3
#define CBX_TRIM_BOTH 4

#define CBX_MAX_DIMS 4

/* One decoded leaf (a Primitive of the AST, each OCCURS element flattened into "slots").
 * Offsets are static (variable_size_occurs = false): element (i0..ik) of the field lives at
 *   offset + sum_k i_k * dim_stride[k]  relative to the record decode base. */
typedef struct {
    int32_t kind;          /* cbx_kind */
    int32_t out_type;      /* cbx_out */
    int32_t offset;        /* binaryProperties.offset */
    int32_t size;          /* binaryProperties.dataSize (bytes per element) */
    int32_t precision, scale, scale_factor;   /* AST type */
    int32_t out_precision, out_scale;         /* Spark DecimalType(p, s) */
    int32_t flags;
    int32_t trim;          /* CBX_TRIM_* for strings */
    int32_t n_dims;        /* enclosing OCCURS levels, outermost first */
    int32_t dim_count[CBX_MAX_DIMS];   /* arrayMaxSize per level */
    int32_t dim_stride[CBX_MAX_DIMS];  /* bytes per element of that level */
    int32_t dim_array[CBX_MAX_DIMS];   /* index into the cbx_array table per level */
    int32_t segment;       /* segment-redefine group this field is under, -1 if none */
    int32_t column;        /* output column */
} cbx_field;

/* One OCCURS node. Element count per record (extractArray, RecordExtractors.scala:66-114):
 *   dependee < 0 ? max : (dependee value v valid && min <= v <= max ? v : max) */
typedef struct {
    int32_t max_count, min_count;
    int32_t dependee;      /* index into the field table, -1 for a fixed OCCURS */
    int32_t segment;       /* segment of the array node, -1 if none */
    int32_t count_column;  /* output column receiving the per-record element count (int32) */
    int32_t n_dims;        /* enclosing OCCURS levels (outer arrays of this array) */
    int32_t parent;        /* enclosing array index or -1 */
    int32_t offsets_column;/* list layout (fields flagged CBX_F_LIST): output column receiving each
                              record's int64 child offset, -1 for the slot-major layout */
} cbx_array;

/* Segment ids (the `segment_field` of a multisegment file) and everything keyed by them:
 *   - segment-redefine selection (FixedLenNestedRowIterator.getSegmentId + redefine map,
 *     CP/reader/iterator/FixedLenNestedRowIterator.scala:64-99, VarLenNestedIterator.scala:91-93),
 *   - Seg_IdN generation (segment_id_level0.., SegmentIdAccumulator.scala:19-86),
 *   - segment_filter and root-reached filtering (VarLenNestedIterator.scala:138-147),
 *   - root-segment index cuts (IndexGenerator.scala:89-113).
 * A record's segment id is extractPrimitiveField(field).toString.trim (VRLRecordReader.scala:188-198):
 * for a string field the trimmed decoded text (compared with the UTF-8 key bytes), for an integral
 * field the decimal text of its value (keys that are canonical integers are compared by value:
 * key_is_int / key_int).  Each distinct key carries everything the options say about it. */
#define CBX_MAX_SEG_KEYS 32
#define CBX_MAX_SEG_KEY_LEN 32
#define CBX_MAX_SEG_LEVELS 8
#define CBX_MAX_SEG_PREFIX 64
typedef struct {
    int32_t field_offset, field_size;   /* segment-id field (relative to decode base) */
    int32_t n_keys;
    int32_t key_len[CBX_MAX_SEG_KEYS];
    uint16_t key[CBX_MAX_SEG_KEYS][CBX_MAX_SEG_KEY_LEN];  /* UTF-16 code units */
    int32_t key_segment[CBX_MAX_SEG_KEYS];   /* redefine segment the key activates, -1 none */
    int32_t key_level[CBX_MAX_SEG_KEYS];     /* first segment_id_level listing the key (0 also for a hierarchical
                                                file's root ids: index cuts, no Seg_Id column), -1 none */
    int32_t key_in_filter[CBX_MAX_SEG_KEYS]; /* 1: listed in segment_filter */
    int32_t key_is_int[CBX_MAX_SEG_KEYS];    /* integral segment field: key is a canonical integer */
    int64_t key_int[CBX_MAX_SEG_KEYS];
    int32_t field;           /* index of the segment-id field in the field table */
    int32_t field_is_int;    /* the segment-id field is integral (compared by value) */
    int32_t n_levels;        /* segment_id_level count = Seg_IdN columns */
    int32_t has_filter;      /* segment_filter given */
    int32_t level_column[CBX_MAX_SEG_LEVELS];   /* output string column of Seg_Id<l>, -1 none */
    int32_t prefix_len;
    uint8_t prefix[CBX_MAX_SEG_PREFIX];       /* segment_id_prefix, UTF-8 */
} cbx_segment_map;

typedef struct {
    int32_t n_columns;      /* value columns + count columns */
    int32_t file_id;        /* File_Id value for CBX_K_FILE_ID */
    int32_t has_segments;   /* segment map valid */
    int32_t window_bytes;   /* LDS window per record (0 = default) */
    int32_t segment_column; /* column receiving the active segment index per record, -1 none */
    int32_t jit_min_records;/* batches of at least this many records run a kernel
                               specialised for the copybook (compiled once with hipRTC);
                               0 = default (262144), < 0 = never */
    int32_t string_views;   /* string/binary columns in the Arrow string-view layout (below) */
    int32_t reserved;
    uint32_t lut[256];      /* code page: UTF-8 bytes (0-23), length (24-25), trimmable (31) */
    cbx_segment_map segments;
} cbx_plan_options;

/* Output column buffers (caller-owned, device memory).  Every column is n_slots(c) slot rows
 * of pitch = 64 * ceil(n_rec / 64) values (one row per OCCURS element; 1 row without OCCURS):
 * value (slot s, record r) is element s * pitch + r; elements r >= n_rec are padding the
 * kernels may overwrite.  Validity is an Arrow bitmap per slot row, 64-bit words:
 *   bit r of row s = validity[s * (pitch / 64) + r / 64] >> (r % 64).
 * Strings/binary: every slot is its own Arrow large-string array.  Slot s owns the payload
 * region data[s * data_capacity, (s + 1) * data_capacity) and the offsets
 * offsets[s * (pitch + 1) + r], r = 0 .. n_rec (absolute byte positions in `data`; entries past
 * n_rec are padding).  data_capacity = cbx_string_bound(...) always suffices; a smaller
 * capacity (e.g. from cbx_string_sizes_*) is honoured: payload never overflows its region, an
 * overflow is reported by cbx_plan_check.
 *
 * List layout of an OCCURS DEPENDING ON array (cbx_array.offsets_column >= 0; its fields flagged
 * CBX_F_LIST, numeric, one OCCURS level; Arrow ListView): a field's `values` / `validity` hold
 * the CHILD elements -- tile t of 64 records owns elements [t * 64 * M, (t + 1) * 64 * M) with
 * M = max_count rounded up to 64, record r's elements start at its offsets-column value (a
 * multiple of 64) and its count column gives their number (none where the count is null: the
 * array's segment is not the record's); the run is padded to a multiple of 64 (padding values
 * unspecified, validity bits 0) and nothing past it is written.  All CBX_F_LIST fields of an
 * array share its segment.  values need ceil(n_rec / 64) * 64 * M elements, validity
 * ceil(n_rec / 64) * M words.  The elements are decoded by a second, element-parallel kernel
 * (64 consecutive elements of one record per wave step) after the record kernel.
 *
 * String-view layout (cbx_plan_options.string_views != 0; Arrow Utf8View / BinaryView): `values`
 * holds n_slots * pitch views of 16 bytes (value (s, r) at view s * pitch + r): int32 length, then
 * the UTF-8 bytes inline when length <= 12 (zero padded), else their first 4 bytes, an int32
 * data-buffer index and an int32 offset into that buffer.  `data` holds n_slots regions of
 * data_capacity bytes; a region is cut into data buffers of buffer_bytes (the last one shorter):
 * buffer k of slot s starts at data + s * data_capacity + k * buffer_bytes
 * (cbx_string_view_geometry: a power-of-two number of whole tiles, at most 1 GiB unless one tile
 * is larger).  Long payloads start at 4-byte-aligned positions of their tile.  Every tile of 64 records owns tile_bytes of its slot's region,
 * so a value is written once, where the decode kernel produces it -- no scan over the batch and
 * no placement pass.  data_capacity must be at least ceil(n_rec / 64) * tile_bytes
 * (cbx_string_bound returns that in this layout; a smaller one fails the call with
 * CBX_E_CAPACITY).  `offsets` and `data_sizes` are unused. */
typedef struct {
    void* values;          /* fixed-width values (NULL for strings) */
    uint64_t* validity;
    int64_t* offsets;      /* strings: n_slots * (pitch + 1) entries */
    uint8_t* data;         /* strings: UTF-8 payload, n_slots regions of data_capacity bytes */
    int64_t data_capacity; /* strings: bytes per slot region */
    int64_t* data_sizes;   /* strings: device array [n_slots] receiving each slot's payload bytes (may be NULL) */
} cbx_column;

typedef struct cbx_plan cbx_plan;

int32_t cbx_abi_version(void);

/* Pipelined Arrow Utf8 batches: two plans of the same layout decoding alternate batches on two
 * streams.  Each cbx_decode_fixed / cbx_decode_var call of a linked plan (Utf8 layout) makes its
 * stream wait for the peer plan's last count pass + scan before its own, and marks its own end, so
 * one plan's count pass (HBM-read bound) runs beside the other's decode (issue bound) instead of
 * after it; count_blocks_per_cu / decode_blocks_per_cu (0: the default occupancy) cap the resident
 * workgroups per CU of the two kernels so both fit on a CU at once.  B = NULL unlinks A. */
int cbx_plan_pipeline(cbx_plan* a, cbx_plan* b, int32_t count_blocks_per_cu, int32_t decode_blocks_per_cu);
const char* cbx_last_error(void);

/* Build a plan from the flattened copybook.  Copies the tables to device memory. */
int cbx_plan_create(const cbx_field* fields, int32_t n_fields, const cbx_array* arrays,
                    int32_t n_arrays, const cbx_plan_options* opts, cbx_plan** out_plan);
void cbx_plan_destroy(cbx_plan* plan);

/* Upper bound of a string column's payload per slot for n_rec records (n_rec * field size *
 * widest UTF-8 expansion of the code page; string-view layout: ceil(n_rec / 64) * tile_bytes);
 * out_bytes[n_columns] (0 for non-string columns). */
int cbx_string_bound(const cbx_plan* plan, int64_t n_rec, int64_t* out_bytes);

/* String-view layout geometry per column (0 for non-string columns): tile_bytes[n_columns] =
 * bytes of a slot region owned by one tile of 64 records, buffer_bytes[n_columns] = bytes per
 * Arrow data buffer of a slot (a whole number of tiles, at most 1 GiB). */
int cbx_string_view_geometry(const cbx_plan* plan, int64_t* tile_bytes, int64_t* buffer_bytes);

/* Exact payload sizes (optional pre-pass, synchronous): out_sizes[n_columns] receives, per
 * string column, the largest slot payload of the batch (0 for non-string columns). */
int cbx_string_sizes_fixed(cbx_plan* plan, const uint8_t* d_records, int64_t n_rec,
                           int32_t rec_stride, int32_t start_offset, int64_t* out_sizes, void* stream);

/* Fixed-length batch: record i occupies d_records[i*rec_stride, (i+1)*rec_stride) and is
 * decoded at +start_offset (CobolScanners.buildScanForFixedLength; record_start_offset).
 * Bounds rules of Primitive.decodeTypeValue apply against rec_stride.  Asynchronous on
 * `stream` (one kernel launch); calls on one plan must be issued in order on one stream. */
int cbx_decode_fixed(cbx_plan* plan, const uint8_t* d_records, int64_t n_rec, int32_t rec_stride,
                     int32_t start_offset, int64_t first_record_id, cbx_column* columns, void* stream);

/* Variable-length batch: record i is d_data[rec_off[i], rec_off[i] + rec_len[i]) (payload
 * without RDW), decoded at +start_offset; shorter records yield null numerics / truncated strings. */
int cbx_decode_var(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                   const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset,
                   int64_t first_record_id, cbx_column* columns, void* stream);
int cbx_string_sizes_var(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                         const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset,
                         int64_t* out_sizes, void* stream);

/* Multi-GPU shards of one variable-length file: d_base is a device int64 (e.g. the
 * exclusive prefix of the ranks' framed record counts, all-gathered on the device) that every later
 * decode call of the plan adds to its first_record_id when it writes Record_Id -- the shard's base
 * never visits the host.  NULL clears it.  The pointer must stay valid while calls are in flight.
 * Replaces the startingRecordIndex a Spark task passes to VarLenNestedReader.getRowIterator
 * (SC/reader/VarLenNestedReader.scala:52-81). */
int cbx_plan_set_record_base(cbx_plan* plan, const int64_t* d_base);

/* Hierarchical records (segment-children): OCCURS DEPENDING ON counts the caller resolved itself.
 * d_counts: device int32[n_arrays][pitch] -- entry (a, r) the element count of the plan's array a in
 * record r of the following decode calls (cbx_decode_selected / cbx_decode_var / cbx_decode_fixed),
 * < 0: the count the record's own dependee gives.  Replaces the dependFields map that
 * RecordExtractors.extractHierarchicalRecord shares between the segments of one hierarchical record
 * (CP/reader/extractors/record/RecordExtractors.scala:224-245): a child segment's array depending on
 * a field of its parent segment (or of a segment decoded earlier in the record) takes the value
 * registered there.  NULL clears it; the pointer must stay valid while calls are in flight.
 * CBX_E_UNSUPPORTED on a record-walk plan. */
int cbx_plan_set_odo_counts(cbx_plan* plan, const int32_t* d_counts, int64_t pitch);

/* Synchronise `stream` and report device-side errors of the plan's earlier decode calls
 * (CBX_E_CAPACITY: a string payload exceeded data_capacity). */
int cbx_plan_check(cbx_plan* plan, void* stream);

/* Optional kernel timing with HIP events on the call's stream (bench / profiling): while
 * enabled, every decode call records events around its decode kernel and around its post
 * passes (fixup of deferred values, string scan + placement), without synchronising.
 * cbx_plan_kernel_times waits for the recorded events, returns up to max_calls per-call
 * durations in ms (oldest first, *n_calls of them) and clears the record. */
int cbx_plan_set_profiling(cbx_plan* plan, int32_t enable);
int cbx_plan_kernel_times(cbx_plan* plan, float* decode_ms, float* post_ms, int32_t max_calls, int32_t* n_calls);

/* Which decode kernel the plan's last decode call ran: *kind = 0 the table-driven kernel,
 * 2 the record walk (cbx_plan_set_walk), 3 its copybook-specialised form,
 * 1 the copybook-specialised kernel.  If specialisation was attempted and failed, *kind = 0 and
 * the reason is in cbx_last_error() (the call itself succeeded on the table-driven kernel). */
int cbx_plan_kernel_kind(cbx_plan* plan, int32_t* kind);

/* Which step the plan's last cbx_frame_var_occurs call walked records with: *kind = 0 the
 * table-driven walk_length, 1 its copybook-specialised form (hipRTC, from jit_min_records records
 * estimated at the copybook's largest record; same records, tested on both). */
int cbx_plan_frame_kind(cbx_plan* plan, int32_t* kind);

/* The copybook-specialised kernel of a plan (its contiguous fixed-length variant when the layout
 * has one, else the windowed variant): writes its HIP source
 * (NUL-terminated, truncated to source_cap) and its length; with compile != 0 also compiles it
 * for gfx950 with hipRTC (no device needed) and reports a failure with the compiler log in
 * cbx_last_error().  Decode calls build and use it on their own (cbx_plan_options.jit_min_records);
 * this entry point is for inspection, ahead-of-time warm-up and tests. */
int cbx_plan_specialize(cbx_plan* plan, char* source, int64_t source_cap, int64_t* source_len, int32_t compile);

/* RDW header walk on the GPU (RecordHeaderParserRDW + VRLRecordReader), seeded by sparse-index
 * entry points: seeds[k] is a known record-header offset (offsetFrom of an index entry), the
 * chain from seeds[k] is walked up to seeds[k+1] (or n_bytes).  Writes payload offsets/lengths
 * of valid records in file order; *n_records receives the count. */
typedef struct {
    int32_t big_endian;         /* is_rdw_big_endian */
    int32_t adjustment;         /* rdw_adjustment (+ -4 if is_rdw_part_of_record_length) */
    int32_t file_header_bytes;  /* file_start_offset */
    int32_t file_footer_bytes;  /* file_end_offset */
} cbx_rdw_params;

int cbx_frame_rdw(const uint8_t* d_data, int64_t n_bytes, const int64_t* seeds, int32_t n_seeds,
                  const cbx_rdw_params* params, int64_t* d_rec_off, int32_t* d_rec_len,
                  int64_t capacity, int64_t* n_records, void* stream);

/* The same walk with no host wait: everything is enqueued on `stream` and the outcome stays on the
 * device in d_state (int64[3]): [0] the record count, [1] the first header error (-1: none; else
 * offset << 2 | kind, kind 2 = zero-length header, 3 = header above 100 MB), [2] flags (1: more
 * records than capacity).  max_rounds parallel fix rounds (0 = 3) run before a one-wave pass on the
 * device settles whatever they left (a no-op when the last round changed nothing).  A
 * multi-GPU step all-gathers d_state[0] on the device (the Record_Id bases) and decodes with the
 * count its index run predicts; cbx_frame_rdw_state reads d_state afterwards (one host wait) and
 * returns the error cbx_frame_rdw would have returned, *n_records the count.
 * (Replaces the host out-parameter of VRLRecordReader's sequential count, VarLenNestedIterator.scala:80-147,
 * for the all-gather RCCL performs) */
int cbx_frame_rdw_async(const uint8_t* d_data, int64_t n_bytes, const int64_t* seeds, int32_t n_seeds,
                        const cbx_rdw_params* params, int64_t* d_rec_off, int32_t* d_rec_len,
                        int64_t capacity, int64_t* d_state, int32_t max_rounds, void* stream);
int cbx_frame_rdw_state(const int64_t* d_state, int64_t* n_records, void* stream);

/* ---- variable-length record streams: sparse index, record selection, selected decode ----
 *
 * Sparse index (IndexGenerator.sparseIndexGenerator, CP/reader/index/IndexGenerator.scala:33-157,
 * called by VarLenNestedReader.generateIndex, CP/reader/VarLenNestedReader.scala:125-180) over a
 * file already framed on the GPU (cbx_frame_rdw over the whole file, or fixed-length records).
 * Entries are cut every records_per_entry records, or by size: bytes_per_entry with
 * subtract_size != 0 (input_split_size_mb / HDFS block size: the split size is subtracted, not
 * reset), or the 100 MB default (reset); with `hierarchical` only at records whose segment id is
 * a level-0 key of the plan's segment map.  The first entry is (0, -1, file_id, 0); the last
 * entry's offset_to is -1.  record_index counts every header read (the file header record too).
 * start_bytes: IndexGenerator's bytesInChunk as of the first framed record, which is taken as an entry
 * already cut -- 0 for a whole file; for a piece of a file that starts at one of the file's entries, that
 * entry's residual under the subtracting size split (its header offset minus the split size times the
 * cuts up to it): the piece's entries are then the file's (shard.index_chain). */
typedef struct {
    int64_t offset_from, offset_to;
    int64_t record_index;
    int32_t file_id;
    int32_t reserved;
} cbx_index_entry;

typedef struct {
    int64_t records_per_entry;  /* input_split_records; 0 = split by size */
    int64_t bytes_per_entry;    /* split size in bytes when records_per_entry == 0 */
    int32_t subtract_size;      /* isSplitBySize: an explicit MB size (subtracted) vs the default (reset) */
    int32_t header_bytes;       /* record header length: 4 (RDW) or 0 (fixed-length record parser) */
    int32_t has_file_header;    /* a file-header record precedes the first framed record */
    int32_t hierarchical;       /* cut only at level-0 segment records (segment levels given) */
    int32_t file_id;
    int32_t reserved;
    int64_t start_bytes;        /* bytesInChunk at the first framed record (0: a whole file) */
} cbx_index_params;

int cbx_sparse_index(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                     const int32_t* d_rec_len, int64_t n_rec, const cbx_index_params* params,
                     cbx_index_entry* entries, int64_t capacity, int64_t* n_entries, void* stream);

/* Record selection over framed records (VarLenNestedIterator.fetchNext + VRLRecordReader record
 * numbering, CP/reader/iterator/VarLenNestedIterator.scala:80-147, VRLRecordReader.scala:55-74):
 * records are numbered per index entry (Record_Id = entry.record_index + ordinal inside the entry;
 * entries = NULL: one entry (0, -1, file_id, 0)), Seg_IdN state is accumulated per entry,
 * records before the first root of an entry (when segment levels are given) and records outside
 * segment_filter are dropped.  Output arrays (device, capacity n_rec each) receive the selected
 * records in file order; seg_state holds (1 + n_levels) int64 per record: the root record id
 * (-1: no root seen in the entry) then per level -2 (null) or the level counter. */
typedef struct {
    int64_t* rec_off;          /* payload offsets */
    int32_t* rec_len;          /* payload lengths */
    int64_t* record_id;        /* Record_Id */
    int32_t* segment;          /* active segment redefine index, -1 none */
    int64_t* seg_state;        /* [n][1 + n_levels], may be NULL when the plan has no levels */
    int32_t file_id;           /* File_Id of the batch (written by cbx_decode_selected) */
    int32_t footer_bytes;      /* in: file_end_offset -- the reference bounds each entry's stream to
                                  offset_to and its header parser then reads records within
                                  file_end_offset of that bound as the footer: they are dropped */
} cbx_selection;

int cbx_select_records(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                       const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset,
                       const cbx_index_entry* entries, int32_t n_entries, cbx_selection* out,
                       int64_t* n_selected, void* stream);

/* Decode selected records: as cbx_decode_var, with Record_Id and the active segment taken from
 * the selection and the Seg_IdN string columns written from its seg_state
 * (SegmentIdAccumulator.getSegmentLevelId: prefix_fileId_rootRecordId[_L<level>_<counter>]). */
int cbx_decode_selected(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const cbx_selection* sel,
                        int64_t n_rec, int32_t start_offset, cbx_column* columns, void* stream);

/* ---- the record walk with data-dependent offsets ----
 *
 * Layouts the static-offset tables above cannot express run through a per-record walk of the
 * copybook (RecordExtractors.extractRecord restated per lane, cbx_walk.h): variable_size_occurs =
 * true (an OCCURS DEPENDING ON array consumes only its present elements, RecordExtractors.scala:
 * 109-113), DEPENDING ON a field inside an OCCURS, DEPENDING ON a string field through
 * occurs_mappings (dependingOnHandlers).  cbx_plan_set_walk attaches the copybook's node table to a
 * plan; every later decode call on the plan walks.  Output columns are as above, with two
 * differences: a count column of an array nested in OCCURS has one slot per enclosing element
 * (n_slots = product of the enclosing max counts), and string columns must use the string-view
 * layout.  Requires zeroed validity buffers. */
#define CBX_W_GROUP 0
#define CBX_W_PRIM 1
#define CBX_W_REDEFINED 0x1   /* isRedefined: the node does not advance the offset */
#define CBX_W_REDEFINES 0x2   /* redefines another node: a group advances by its static size */
typedef struct {
    int32_t kind;          /* CBX_W_GROUP / CBX_W_PRIM */
    int32_t next, child;   /* next sibling, first child (groups); -1 none */
    int32_t field;         /* primitive: cbx_field index, -1 when not decoded (FILLER) */
    int32_t array;         /* OCCURS node: cbx_array index, -1 */
    int32_t flags;         /* CBX_W_* */
    int32_t data_size;     /* bytes per element (binaryProperties.dataSize) */
    int32_t actual_size;   /* bytes of the whole node (binaryProperties.actualSize) */
    int32_t segment;       /* group: segment redefine index, -1 */
    int32_t dep_slot;      /* DEPENDING ON source: its dependee slot (one per name, < 8), -1 */
} cbx_walk_node;
typedef struct {
    int32_t dep_slot;      /* dependee slot of the array's DEPENDING ON name, -1: fixed OCCURS */
    int32_t h_begin, h_end;/* its occurs_mappings handlers (cbx_walk_handler range) */
    int32_t reserved;
} cbx_walk_array;
typedef struct {
    int32_t key_id;        /* distinct key strings share an id */
    int32_t key_len;       /* UTF-8 bytes */
    int32_t value;         /* element count the key stands for */
    int32_t reserved;
    uint8_t key[64];
} cbx_walk_handler;

int cbx_plan_set_walk(cbx_plan* plan, const cbx_walk_node* nodes, int32_t n_nodes, int32_t root,
                      const cbx_walk_array* arrays, const cbx_walk_handler* handlers, int32_t n_handlers,
                      int32_t variable_size_occurs);

/* VarOccursRecordExtractor (CP/reader/extractors/raw/VarOccursRecordExtractor.scala:30-154): record
 * boundaries of a file whose record size follows from its OCCURS DEPENDING ON values (no RDW, no
 * length field), from first_offset on.  A record starts where the previous one ends; the stream is
 * framed chunk-parallel (speculated chunk entries corrected until they agree with the sequential walk,
 * cbx_chain.h), with the sequential walk's results.  A short read at the end is zero-filled by
 * the reference: the last record may reach past n_bytes, up to *virtual_bytes (the buffer must hold
 * zeros there before decoding).  Needs a plan with cbx_plan_set_walk.  From jit_min_records records
 * (estimated at the copybook's largest record) the step is the copybook-specialised walk_length
 * (hipRTC; cbx_plan_frame_kind).  Device scratch, stream-ordered (hipMallocAsync, freed by the call):
 * a bitmap of one bit per byte of [first_offset, n_bytes) -- n_bytes / 8, 125 MB per GB framed --
 * plus ~60 bytes per chunk of >= 16 KiB; cbx_frame_length_field takes the same (chunks >= 1 KiB). */
int cbx_frame_var_occurs(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, int64_t first_offset,
                         int64_t* d_rec_off, int32_t* d_rec_len, int64_t capacity, int64_t* n_records,
                         int64_t* virtual_bytes, void* stream);

/* Record length field framing (record_length_field, not is_record_sequence):
 * VRLRecordReader.fetchRecordUsingRecordLengthField (CP/reader/iterator/VRLRecordReader.scala:114-149).
 * From byte 0, each record is start_offset + lfb bytes (lfb = the field's offset + size; `field` indexes
 * the plan's cbx_field table) plus max(0, value + adjustment - lfb + end_offset) more, fewer at the end
 * of the data, which ends the walk; a stream holding fewer than start_offset + lfb bytes has no further
 * record.  The field must be a primitive Integral one (ReaderParametersValidator.getLengthField); its
 * value is decoded as extractPrimitiveField does (Int / Long -> toInt) and a null or BigDecimal value
 * fails with CBX_E_STATE (the reference's IllegalStateException).  rec_off / rec_len receive
 * the record starts and lengths (decode them with cbx_decode_var at start_offset).  Framed
 * chunk-parallel like cbx_frame_var_occurs (cbx_chain.h); the error reported is the first one on the
 * record chain. */
int cbx_frame_length_field(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, int32_t field,
                           int32_t start_offset, int32_t end_offset, int32_t adjustment, int64_t* d_rec_off,
                           int32_t* d_rec_len, int64_t capacity, int64_t* n_records, void* stream);

/* ---- hierarchical records (`segment-children`) ----
 *
 * Replaces VarLenHierarchicalIterator + the structure walk of RecordExtractors.extractHierarchicalRecord
 * (CP/reader/iterator/VarLenHierarchicalIterator.scala:43-162, RecordExtractors.scala:211-385): the
 * framed records of a stream are grouped by root segment (records before the first root dropped) and
 * each record is placed under its parent instance (extractChildren's rule, :298-322: the children of
 * type C of a parent p are the C records after p up to the first record of p's segment or of one of
 * its ancestors).  With one segment id per segment that has children the reference's rule depends on
 * types only (parallel passes over the records); else flags bit 0 selects the general walk.  At most
 * 16 segments.
 *
 * Output: one cbx_selection of rows in table order -- table 0 = the root records (one row per
 * hierarchical record, Record_Id = first_record_id + the index of the next root record or n_rec,
 * VarLenHierarchicalIterator.scala:107-133), then table 1 + s = the records of segment s placed in
 * the tree, each table in record order (Record_Id = first_record_id + record index, unused by the
 * reference).  parent_row[row] = the row of the record's parent instance (-1 for roots).  Decode
 * the rows with cbx_decode_selected (segment = the record's own segment: its redefine decodes); the
 * list of segment-C children of every parent row is a contiguous run of table 1 + C
 * (cbx_hier_list_offsets).  table_rows (host, n_segments + 1 entries) receives the row count per
 * table.  Output arrays need capacity n_rec.
 * record_start_offset: extractHierarchicalRecord decodes the root at the start offset but each child
 * segment at its group's own offset, without it (RecordExtractors.scala:308-310, :376) -- the host
 * decodes the child rows as records starting start_offset bytes earlier.  The dependFields map the
 * reference shares between the segments of a hierarchical record (:224-245: a child's array DEPENDING
 * ON a field of its parent segment or of the common header, or on a null field of its own segment)
 * is resolved on the device by cbx_hier_dependee_counts and applied with cbx_plan_set_odo_counts.
 * Several segment ids mapped to one segment that has children: flags bit 0 (the general walk: one
 * thread per hierarchical record runs extractChildren's recursion with its id-based break rule).
 * The counts are resolved BEFORE the decode (one decode): cbx_hier_dependee_values decodes each
 * DEPENDING ON field from every row's bytes, cbx_hier_dependee_counts replays the walk.
 * Record-walk plans (string dependees through occurs_mappings, variable_size_occurs) take the map per
 * row instead of counts (cbx_hier_walk.seeds -> cbx_plan_set_dep_seed).
 * Not covered (reported by the host, CBX_E_UNSUPPORTED, never decoded differently): a segment group
 * placed before the root segment's that has child segments, with a cross-segment DEPENDING ON (the
 * root's record walk extracts that group's children too); on a record-walk plan, a cross-segment
 * DEPENDING ON field inside an OCCURS or behind a variable-size one. */
typedef struct {
    int32_t n_segments;               /* segment redefines (cbx_field.segment / key_segment indices) */
    int32_t root_segment;             /* the segment without a parent */
    int32_t parent[CBX_MAX_SEG_KEYS]; /* parent segment of each segment, -1 for the root */
    int64_t first_record_id;          /* startRecordId of the stream (entry.record_index) */
    int32_t start_offset;             /* record_start_offset: the segment id is read past it (VRLRecordReader) */
    int32_t flags;                    /* bit 0: the general walk -- a segment with children mapped from several
                                       * segment ids (one record can then sit under several parents: rows may
                                       * outnumber n_rec; CBX_E_CAPACITY with *n_rows / table_rows set when they
                                       * do not fit, call again with that capacity) */
    int64_t row_capacity;             /* rows the outputs hold (0: n_rec) */
} cbx_hier_params;

int cbx_hier_select(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                    const int32_t* d_rec_len, int64_t n_rec, const cbx_hier_params* params, cbx_selection* out,
                    int64_t* d_parent_row, int64_t* table_rows, int64_t* n_rows, void* stream);

/* Arrow list offsets (int32, n_parent + 1 entries) of one child table over its parent table:
 * offsets[k] = rows of the child table [child_begin, child_begin + n_child) whose parent row is
 * below parent_begin + k.  Asynchronous on `stream`. */
int cbx_hier_list_offsets(const int64_t* d_parent_row, int64_t child_begin, int64_t n_child, int64_t parent_begin,
                          int64_t n_parent, int32_t* d_offsets, void* stream);

/* A DEPENDING ON field (plan field `field`: integral COMP-3 / binary / DISPLAY) decoded from each of
 * n_rows rows' own bytes -- at rec_off + start_offset + its offset, null past rec_len or when malformed,
 * whatever the row's segment (the root record decodes every segment group from its own bytes,
 * RecordExtractors.scala:365-372) -- into d_values (int64 Number.intValue) and d_validity (one bit per
 * row, a word per 64 rows).  The dependee columns of cbx_hier_dependee_counts (out_type CBX_O_I64),
 * so the counts exist before the rows are decoded.  Asynchronous on `stream`. */
int cbx_hier_dependee_values(cbx_plan* plan, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                             const int32_t* d_rec_len, int64_t n_rows, int32_t start_offset, int32_t field,
                             int64_t* d_values, uint64_t* d_validity, void* stream);

/* The dependFields map extractHierarchicalRecord shares between the segments of one hierarchical
 * record (RecordExtractors.scala:224-245, walk order :324-370), on the device: one thread per
 * hierarchical record walks its rows as the reference does -- the root, then per child segment in
 * copybook order (getParentToChildrenMap, CopybookParser.scala:702-727) each child row followed by
 * its own subtree -- replaying at every row its segment's events in field order: a numeric DEPENDING
 * ON field registers its value (Number.intValue) when the row decodes it non-null; an array takes the
 * value registered last (its maximum when none is, or the value is outside [min, max]).
 * counts (device, [n_arrays_out][pitch] int32) receives the count of every array event's rows, root
 * rows included, and *d_changed (device int32) is set to 1 when some count differs from first_counts
 * (when given); apply with cbx_plan_set_odo_counts to the decode.  Rows as cbx_hier_select emits them.
 * Root-record registrations that precede the root segment's group (the common header, a segment group
 * placed before it, decoded from the root's bytes) are events[CBX_HIER_MAX_SEG]. */
#define CBX_HIER_MAX_SEG 16       /* segments of a hierarchical layout (cbx_hier_select's limit) */
#define CBX_HIER_MAX_EVENTS 32    /* events per segment */
#define CBX_HIER_MAX_DEPS 16      /* dependees and arrays of one cbx_hier_dependee_counts call */
typedef struct {
    const void* values;               /* device: the dependee column's values, slot 0 (row-indexed) */
    const uint64_t* validity;         /* device: its validity words, slot 0 */
    int32_t out_type;                 /* CBX_O_I32 / CBX_O_I64 / CBX_O_DEC128; CBX_O_STRING: int64 values are the
                                       * occurs_mappings key id + 1 of a string dependee (cbx_hier_dependee_values) */
    int32_t walk_slot;                /* its dependee slot in the plan's record walk (seeds), -1 none */
} cbx_hier_dependee;

typedef struct {
    int32_t dependee;                 /* index into the dependee table */
    int32_t out_row;                  /* row of `counts` receiving this array's counts (the plan array index) */
    int32_t min_count, max_count;
    const int32_t* first_counts;      /* device: the first decode's counts of the array (row-indexed), may be NULL */
} cbx_hier_odo_array;

typedef struct {
    int32_t n_segments;
    int32_t root_segment;
    int64_t table_base[CBX_HIER_MAX_SEG + 1];        /* first row of table t (0: roots, 1 + s: segment s) */
    int64_t table_rows[CBX_HIER_MAX_SEG + 1];
    const int32_t* child_offsets[CBX_HIER_MAX_SEG];  /* device: segment s's list offsets over its parent table */
    int8_t children[CBX_HIER_MAX_SEG][CBX_HIER_MAX_SEG]; /* child segments of s in copybook order, -1 ends */
    /* events of a row of segment s in field order (s = CBX_HIER_MAX_SEG: the root record's common-header
     * registrations before the root segment's group): e >= 0 registers dependee e, e < 0 resolves
     * array -e - 1; -32768 ends */
    int16_t events[CBX_HIER_MAX_SEG + 1][CBX_HIER_MAX_EVENTS];
    /* device, or NULL: [8][pitch] int64, each row's record-walk dependee slots as the walk leaves the map
     * before the row (after the root's registrations that precede the root segment's group, for a root
     * row): kind << 32 | value, kind 0 unseen, 1 Left(int), 2 Right(key id + 1) -- cbx_plan_set_dep_seed */
    int64_t* seeds;
} cbx_hier_walk;

/* Record-walk plans (cbx_plan_set_walk: variable_size_occurs, string dependees through occurs_mappings,
 * DEPENDING ON inside an OCCURS): the walk resolves a row's counts itself from its dependFields map; for
 * hierarchical rows that map starts as the walk of the hierarchical record left it (cbx_hier_walk.seeds),
 * and a child row registers no common-header dependee (it decodes its own segment group only,
 * RecordExtractors.scala:300-322).  d_seed = NULL clears it.  Asynchronous use by later decode calls. */
int cbx_plan_set_dep_seed(cbx_plan* plan, const int64_t* d_seed, int64_t pitch, int32_t root_segment);

int cbx_hier_dependee_counts(const cbx_hier_walk* walk, const cbx_hier_dependee* deps, int32_t n_deps,
                             const cbx_hier_odo_array* arrays, int32_t n_arrays, int32_t* d_counts, int64_t pitch,
                             int32_t* d_changed, void* stream);

/* One string slot in the string-view layout (Utf8View: 16-byte views, long payloads in data buffers of
 * buffer_bytes each starting at region, cbx_string_view_geometry) -> Arrow Utf8 (int32 offsets
 * [n + 1] + the payload written contiguously into data, data_capacity bytes).  The record walk
 * (cbx_plan_set_walk: data-dependent offsets, one pass) writes views; this converts its columns for a
 * consumer of the Utf8 layout the reference's StringType maps to (SC/schema/CobolSchema.scala:
 * StringType).  Validity is unchanged (null values are empty).  *d_size (device int64) receives the
 * payload bytes; CBX_E_CAPACITY when they exceed data_capacity or an int32 offset (Arrow's limit). */
int cbx_views_to_utf8(const uint8_t* d_views, int64_t n, const uint8_t* d_region, int64_t buffer_bytes,
                      int32_t* d_offsets, uint8_t* d_data, int64_t data_capacity, int64_t* d_size, void* stream);

/* Text record framing (is_text = true) on the GPU: replaces TextRecordExtractor
 * (cobol-parser/.../reader/extractors/raw/TextRecordExtractor.scala:26-108, chosen by
 * VarLenNestedReader.scala:69-70).  Records end at LF or CR LF (payload without the line
 * ending) inside a window of record_size + 2 bytes (record_size = copybook.getRecordSize); a
 * window without one gives a forced record.  Writes payload offsets/lengths in file order.
 * *virtual_bytes receives the stream length the reference decodes against: its read helper
 * treats a short last read as a full window of zero bytes, so records may reach past n_bytes
 * (by at most record_size + 2); the buffer must hold zeros there before records are decoded
 * (pass *virtual_bytes as n_bytes to cbx_decode_var). */
int cbx_frame_text(const uint8_t* d_data, int64_t n_bytes, int32_t record_size, int64_t* d_rec_off,
                   int32_t* d_rec_len, int64_t capacity, int64_t* n_records, int64_t* virtual_bytes,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif
