// cbx_internal.h -- device-side plan layout shared by the kernels and the C ABI.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif   /* hipRTC (cbx_jit.h) provides the runtime and the fixed-width types */

#include "cbx_decode.h"
#include "cobrix_hip.h"

// Plan tables are read-only for the whole launch: address space 4 ("constant") lets the
// compiler fetch uniform descriptors with scalar loads (s_load) through the scalar cache
// instead of vector memory round trips.
#define CBX_CONST __attribute__((address_space(4)))

namespace cbx {

constexpr int kWave = 64;              // one wave = one tile of 64 consecutive records (lane = record)
constexpr int kWavesPerBlock = 2;      // waves per workgroup (each works on its own tile)
constexpr int kGuard = 16;             // LDS guard bytes in front of / behind a record image
// LDS in front of the waves' regions: the code page LUT (256 x 4 bytes) + the 16 pattern selectors
// of the 2-byte-page string compose (group_sel, 16 x 8 bytes).  (Every byte counts: SYN200's two
// 12.8 KB record images per workgroup sit at 6 workgroups per CU by a margin of ~200 bytes.)
constexpr int kLutLds = 1024 + 128;
constexpr int kMaxWindowBytes = 1024;  // fields wider than this are read from HBM directly
constexpr int kStrStageBytes = 4096;   // per-wave LDS staging of one string item's tile payload
constexpr int kMaxStrItems = 256;      // string (field, slot) items per window (plan splits windows)

// One string element (field, slot), pre-resolved by the plan (cf. NumOp in cbx_decode.h).
struct StrOp {
    int32_t eo;                       // element offset in the record (before start_off)
    int32_t size;
    uint8_t kind, trim, n_odo, pad;   // pad: widest UTF-8 expansion of a byte (1..3)
    int32_t column;
    int32_t slot;
    int32_t seq;                      // look-back sequence
    int32_t segment;
    int16_t odo_arr[CBX_MAX_DIMS];
    int16_t odo_idx[CBX_MAX_DIMS];
    int32_t reserved;
};

// A run of numeric ops of one window sharing decoder variant and output width: the kernel
// runs each batch with a loop specialised for that pair.
struct Batch {
    int32_t variant, width;           // Variant, output bytes per value (4, 8, 16)
    int32_t begin, end;               // NumOp range
    int32_t odo;                      // ops carry OCCURS DEPENDING ON conditions
    int32_t runs;                     // some op of the batch stands for a run of OCCURS elements
};

// Per-call output addresses of one numeric op (host-resolved column + slot bases).
struct NumCall {
    uint8_t* values;          // values of (column, slot): element r at values + r * width
    uint64_t* validity;       // validity words of (column, slot): word t = tile t
    uint64_t* defer;          // deferral words of the op's sequence (null if never deferred)
    uint64_t reserved;
};

// Per-call addresses of one string op (tile-local pass).
struct StrCall {
    uint64_t* validity;       // validity words of (column, slot)
    uint32_t* local;          // tile-local start of every value of the slot (pitch entries)
                              // (Utf8 layout: the slot's int32 Arrow offsets, pitch + 1 entries)
    uint8_t* scratch;         // tile regions of the slot: tile t at scratch + t * tile_cap
                              // (string-view and Utf8 layouts: the slot's region of the caller's data buffer)
    int64_t tile_cap;         // bytes per tile region (64 * size * widest UTF-8 expansion, 16-aligned)
                              // (Utf8 layout: the region's capacity)
    uint8_t* views;           // string-view layout: the slot's 16-byte views (pitch entries)
    int64_t tiles_per_buf;    // string-view layout: tiles per Arrow data buffer
    const int64_t* excl;      // Utf8 layout: exclusive scan of the (sequence, tile) payload totals, this
                              // sequence's row (entry 0 = the sequence's start)
    int64_t* size;            // Utf8 layout: the slot's payload bytes (data_sizes, may be null)
};

// One field of a list-layout OCCURS DEPENDING ON array (CBX_F_LIST): the list kernel decodes its
// elements k = 0 .. len-1 at op.eo + k * stride.
struct ListOp {
    NumOp op;                 // element 0 (fast-path constants of the field)
    int32_t field;            // field index (byte-loop decoder for wide / deferred forms)
    int32_t array;            // its array (ListOps of one array are adjacent)
    int32_t stride;           // bytes between elements
    int32_t elem_lo;          // offset of the array's first element (lowest eo of its ListOps)
};

// Generated column (File_Id / Record_Id).
struct GenOp {
    int32_t kind, column, out_type, reserved;
};

// Byte range [lo, hi) of each record (relative to the decode base) staged into LDS together,
// with the numeric / string ops whose bytes lie inside it.  The window with global != 0 is
// never staged: its ops read HBM (oversized fields) or are generated.
struct Window {
    int32_t lo, hi;
    int32_t nop_begin, nop_end;
    int32_t batch_begin, batch_end;
    int32_t sop_begin, sop_end;
    int32_t gen_begin, gen_end;
    int32_t pitch;         // LDS row pitch in bytes (odd number of dwords)
    int32_t global;
};

// Per output column device pointers.
struct DevColumn {
    void* values;
    uint64_t* validity;
    int64_t* offsets;
    uint8_t* data;
    int64_t capacity;      // strings: bytes per slot region
    int64_t* sizes;        // strings: per-slot payload bytes (device, may be null)
};

struct KernelArgs {
    // input
    const uint8_t* data;
    int64_t data_len;          // bytes addressable from data (bounds for staging loads)
    int64_t base_shift;        // data is 16-byte aligned down; record bases are shifted by this
    const int64_t* rec_off;    // var-len: payload offsets (nullptr for fixed)
    const int32_t* rec_len;    // var-len: payload lengths
    int64_t n_rec;
    int64_t n_tiles;
    int64_t pitch;             // values per slot row of every output column (64 * n_tiles)
    int32_t stride;            // fixed: record stride (avail length)
    int32_t start_off;         // record_start_offset
    int64_t first_record_id;
    const int64_t* rec_id;     // per-record Record_Id (selected records), nullptr: first_record_id + r
    const int64_t* rec_id_base;// device int64 added to first_record_id (cbx_plan_set_record_base), nullptr: 0
    const int32_t* rec_seg;    // per-record active segment (selected records), nullptr: from segmap
    const int32_t* odo_count;  // [n_arrays][odo_pitch] OCCURS DEPENDING ON counts given by the caller
                               // (cbx_plan_set_odo_counts; < 0: from the record), nullptr: none
    int64_t odo_pitch;
    int32_t file_id;
    int32_t mode;              // 0 decode, 1 string sizes only
    int32_t str_view;          // string columns: 0 Arrow large-string (scratch + placement), 1 string views,
                               // 2 Arrow Utf8 (int32 offsets; payload written at its final place)
    // fixed-length contiguous staging: the tile's byte span is loaded with 16-byte loads and
    // scattered dword-wise into rows of `cpitch` bytes (odd dword count: conflict-free lanes)
    int32_t contig;
    // variable-length span staging (span_loop): bytes a record's fields reach past its decode base
    // plus start_off, and the row pitch of the record-by-record fallback
    int32_t span_ext;
    int32_t span_pitch;
    int32_t cpitch;
    int32_t stride_dw;         // stride / 4
    float inv_stride_dw;       // 1 / stride_dw
    // plan
    const CBX_CONST Field* fields;
    const CBX_CONST Window* windows;
    int32_t n_windows;
    const CBX_CONST NumOp* nops;
    const CBX_CONST NumCall* ncall;
    const CBX_CONST Batch* batches;
    const CBX_CONST StrOp* sops;
    const CBX_CONST StrCall* scall;
    const CBX_CONST GenOp* gops;
    const CBX_CONST cbx_array* arrays;
    int32_t n_arrays;
    int32_t seg_col;           // column receiving the active segment index, -1 none
    const CBX_CONST cbx_segment_map* segmap;  // nullptr if none
    const uint32_t* lut;       // 256 entries
    const CBX_CONST DevColumn* cols;
    // strings
    int32_t n_seq;             // string sequences = sum over string fields of n_slots
    uint32_t* str_tot;         // [n_seq][n_tiles] payload bytes of every (sequence, tile)
    int32_t* status;           // [0]: capacity overflow flag
    int32_t* list_len;         // list-layout arrays: [n_arrays][pitch] present elements per record
    int32_t* list_flag;        // per tile: the list kernel left elements to its byte-loop pass
    uint64_t* defer_bits;      // [n_defer][n_tiles] values left to the fixup kernel
    // LDS layout (bytes, per wave)
    int32_t lds_rows;          // record image incl. guards
    int32_t lds_counts;        // OCCURS element counts
    int32_t str_stage;         // string payload staging bytes
    int32_t lds_wave;          // total per wave
    int32_t dump_stride;       // bytes between the lanes' string dump slots (4, or 0 = one shared slot)
    uint64_t* stamps;          // diagnostic build (CBX_STAMPS) only: per-segment wave-cycle sums
};

}  // namespace cbx
