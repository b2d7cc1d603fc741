/*
 * cobrix_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the Cobrix record-extraction hot path, used as the parity checker for the
 * HIP path (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).  Never linked into or
 * called by the product library (libcobrix_hip.so).
 *
 * Parity pinning: the restatement is checked against the reference's own golden outputs
 * (the data/testN_expected goldens, copied under tests/golden/data) and its unit-test literals
 * (tests/golden/unit_vectors.json); see tests/test_oracle_golden.py.
 */
#ifndef COBRIX_ORACLE_H
#define COBRIX_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORA_GROUP = 0, ORA_PRIMITIVE = 1 };
enum { ORA_ALPHA = 1, ORA_INTEGRAL = 2, ORA_DECIMAL = 3 };
enum { ORA_EBCDIC = 0, ORA_ASCII = 1, ORA_UTF16 = 2, ORA_HEX = 3, ORA_RAW = 4 };
enum { ORA_DISPLAY = 0, ORA_COMP1 = 1, ORA_COMP2 = 2, ORA_COMP3 = 3, ORA_COMP4 = 4, ORA_COMP5 = 5, ORA_COMP9 = 9 };
enum { ORA_TRIM_NONE = 1, ORA_TRIM_LEFT = 2, ORA_TRIM_RIGHT = 3, ORA_TRIM_BOTH = 4 };
enum { ORA_FP_IBM = 0, ORA_FP_IBM_LE = 1, ORA_FP_IEEE = 2, ORA_FP_IEEE_LE = 3 };

/* Spark result types (SC/schema/CobolSchema.scala:144-173) */
enum { ORA_ST_INT = 1, ORA_ST_LONG = 2, ORA_ST_DECIMAL = 3, ORA_ST_FLOAT = 4, ORA_ST_DOUBLE = 5,
       ORA_ST_STRING = 6, ORA_ST_BINARY = 7 };

/* events, emitted in extractRecord walk order */
enum { ORA_EV_VALUE = 1, ORA_EV_ARRAY = 2, ORA_EV_SEGNULL = 3, ORA_EV_CHILDREN = 4 };

typedef struct {
    int32_t kind;             /* ORA_GROUP / ORA_PRIMITIVE */
    int32_t first_child;      /* -1 if none */
    int32_t next_sibling;     /* -1 if none */
    int32_t name_id;          /* interned exact name */
    int32_t name_upper_id;    /* interned upper-case name */
    int32_t depending_on_id;  /* interned exact DEPENDING ON name, -1 if none */
    int32_t is_array, occurs_min, occurs_max;
    int32_t is_redefined, has_redefines, is_filler;
    int32_t is_segment_redefine, is_dependee;
    int32_t data_size, actual_size;
    int32_t tclass, enc, compact;
    int32_t precision, scale, scale_factor;
    int32_t explicit_decimal, is_signed, sign_separate;
    int32_t handlers_begin, handlers_end; /* range into the handler table (occurs_mappings) */
} ora_node;

typedef struct {
    uint16_t key[64];
    int32_t key_len;
    int32_t value;
} ora_handler;

typedef struct {
    int32_t trimming;
    int32_t float_format;
    int32_t variable_size_occurs;
    int32_t utf16_big_endian;   /* is_utf16_big_endian (DecoderSelector.scala:86) */
    const uint16_t* lut;      /* 256-entry EBCDIC -> UTF-16 table */
    const uint16_t* ascii_lut;/* ascii_charset other than US-ASCII: byte -> UTF-16 of that charset
                                 (AsciiStringDecoderWrapper), else NULL */
} ora_options;

typedef struct {
    uint32_t rec;
    int32_t node;
    int32_t kind;
    int32_t isnull;
    int32_t slot;             /* flattened element index over the enclosing arrays */
    int32_t stype;            /* ORA_ST_* */
    int64_t lo, hi;           /* int/decimal unscaled (128-bit two's complement), float bits,
                                 string/binary: lo = heap offset, hi = length; array: lo = count */
} ora_event;

/* Decode one record (RecordExtractors.extractRecord). Returns 0 on success, <0 on error
 * (-1 event buffer full, -2 heap full, -3 non-integral dependee). */
/* active_segment_upper_id = ORA_ALL_SEGMENTS: every segment redefine is decoded (no nulls) -- the
 * hierarchical walk decodes each segment group from its own record (RecordExtractors.scala:298-322) */
#define ORA_ALL_SEGMENTS (-3)
int ora_extract_record(const ora_node* nodes, int32_t root, const ora_handler* handlers,
                       const ora_options* opt, const uint8_t* data, int32_t data_len,
                       int32_t offset_bytes, int32_t active_segment_upper_id, uint32_t rec,
                       ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                       uint8_t* heap, int64_t heap_cap, int64_t* heap_len);

/* One hierarchical record (RecordExtractors.extractHierarchicalRecord, :211-385): records[0] is the root
 * segment record, the others the records accumulated after it (VarLenHierarchicalIterator).  One
 * dependFields map is shared by every segment of the record.  The root's top-level groups without a
 * parent segment are walked from offset_bytes; at the end of a segment-redefine group the group's child
 * segments (child_begin/child_end/children: parentChildMap, node ids) are extracted from the records after
 * the current one (extractChildren) -- each child group at its own offset (node_offset) in its record's
 * data -- preceded by one ORA_EV_CHILDREN event (node = the child group, lo = the count).  Fields that are
 * child segments (is_child_seg) are decoded where they sit -- their dependees register -- but emit no
 * events, as getGroupValues keeps no value for them.  seg_group: per record the node id of the
 * segment-redefine group its segment id maps to (-1: none); seg_key: per record its segment id as an int
 * key (equal ids, equal keys).  Events carry rec = rec_base + the record's index. */
int ora_extract_hier(const ora_node* nodes, int32_t root, const ora_handler* handlers, const ora_options* opt,
                     int32_t n_records, const uint8_t* const* datas, const int32_t* lens,
                     const int32_t* seg_group, const int32_t* seg_key, const int32_t* child_begin,
                     const int32_t* child_end, const int32_t* children, const int32_t* node_offset,
                     const int32_t* is_child_seg, const int32_t* has_parent_seg, int32_t offset_bytes,
                     uint32_t rec_base, ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                     uint8_t* heap, int64_t heap_cap, int64_t* heap_len);

/* Batch of variable-length records: record i = data[rec_off[i], + rec_len[i]), active segment act[i]. */
int ora_extract_var(const ora_node* nodes, int32_t root, const ora_handler* handlers,
                    const ora_options* opt, const uint8_t* data, const int64_t* rec_off,
                    const int32_t* rec_len, const int32_t* act, int64_t n, int32_t offset_bytes,
                    ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                    uint8_t* heap, int64_t heap_cap, int64_t* heap_len);

/* Fixed-length batch: record i is data[i*stride, (i+1)*stride), decoded at +start_offset
 * (CobolScanners.buildScanForFixedLength + FixedLenNestedRowIterator).  Segment redefine per
 * record: if seg_field >= 0 the field's trimmed string value is looked up in seg_keys. */
int ora_decode_fixed(const ora_node* nodes, int32_t root, const ora_handler* handlers,
                     const ora_options* opt, const uint8_t* data, int64_t n_rec, int32_t stride,
                     int32_t start_offset, int32_t seg_field, int32_t seg_field_offset,
                     const ora_handler* seg_keys, int32_t n_seg_keys,
                     ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                     uint8_t* heap, int64_t heap_cap, int64_t* heap_len);

/* RDW framing (RecordHeaderParserRDW.getRecordMetadata + VRLRecordReader.fetchRecordUsingRdwHeaders).
 * Emits payload (offset, length) per valid record. Returns number of records, <0 on error:
 * -1 capacity, -2 zero-length RDW, -3 RDW too big. err_offset receives the failing header offset. */
int64_t ora_frame_text(const uint8_t* data, int64_t n_bytes, int32_t record_size, int64_t* off, int32_t* len,
                       int64_t cap, int64_t* virtual_bytes);
int64_t ora_frame_rdw(const uint8_t* data, int64_t n_bytes, int32_t big_endian, int32_t adjustment,
                      int32_t file_header_bytes, int32_t file_footer_bytes,
                      int64_t* rec_off, int32_t* rec_len, int64_t cap, int64_t* err_offset);

/* Sparse index (IndexGenerator.sparseIndexGenerator) over an RDW stream, non-hierarchical or
 * root-segment-aware. out entries: (offset_from, offset_to, record_index). Returns count. */
int64_t ora_sparse_index(const uint8_t* data, int64_t n_bytes, int32_t big_endian, int32_t adjustment,
                         int32_t file_header_bytes, int32_t file_footer_bytes,
                         int64_t records_per_entry, int64_t size_per_entry_mb,
                         const int32_t* is_root, /* per-record root flag or NULL */
                         int64_t* out_from, int64_t* out_to, int64_t* out_rec, int64_t cap);

/* Single-field decoders (unit-test surface). value out: same encoding as ora_event. */
int ora_decode_field(const ora_node* node, const ora_options* opt, const uint8_t* bytes,
                     int32_t n, ora_event* out, uint8_t* heap, int64_t heap_cap, int64_t* heap_len);

int32_t ora_spark_type(const ora_node* node, int32_t* precision, int32_t* scale);

#ifdef __cplusplus
}
#endif
#endif
