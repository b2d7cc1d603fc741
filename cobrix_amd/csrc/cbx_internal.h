// cbx_internal.h -- device-side plan layout shared by the kernels and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cbx_decode.h"
#include "cobrix_hip.h"

namespace cbx {

constexpr int kWave = 64;            // one wave = one 64-record tile
constexpr int kMaxWindowBytes = 1024;  // fields wider than this are read from HBM directly

// A run of consecutive slots of one field staged in the same LDS window.
struct Run {
    int32_t field;
    int32_t slot_begin, slot_end;
    int32_t reserved;
};

// Byte range [lo, hi) of each record (relative to the decode base) staged into LDS together.
struct Window {
    int32_t lo, hi;
    int32_t run_begin, run_end;
    int32_t has_strings;   // any string run (needed by the sizing pass)
    int32_t pitch;         // LDS row pitch in bytes (4 * odd)
    int32_t reserved[2];
};

// Per output column device pointers.
struct DevColumn {
    void* values;
    uint64_t* validity;
    int64_t* offsets;
    uint8_t* data;
};

struct KernelArgs {
    // input
    const uint8_t* data;
    int64_t data_len;          // bytes addressable from data (bounds for staging loads)
    int64_t base_shift;        // data is 16-byte aligned down; record bases are shifted by this
    const int64_t* rec_off;    // var-len: payload offsets (nullptr for fixed)
    const int32_t* rec_len;    // var-len: payload lengths
    int64_t n_rec;
    int32_t stride;            // fixed: record stride (avail length)
    int32_t start_off;         // record_start_offset
    int64_t first_record_id;
    int32_t file_id;
    int32_t mode;              // 0 decode, 1 string sizes
    // plan
    const Field* fields;
    const Window* windows;
    int32_t n_windows;
    const Run* runs;
    const cbx_array* arrays;
    int32_t n_arrays;
    int32_t seg_col;           // column receiving the active segment index, -1 none
    const cbx_segment_map* segmap;  // nullptr if none
    const uint32_t* lut;       // 256 entries
    DevColumn* cols;
    // string offsets: per string column base of its (slot, tile) sequence in tile_sums/scan
    const int64_t* str_seq_base;     // [n_columns] index of the column's first (slot,tile) entry, -1 non-string
    int64_t* tile_sums;              // sizes pass: written; decode pass: exclusive scan (read)
    int64_t n_tiles;
    int32_t max_pitch;         // LDS bytes per row of the widest window
    int32_t contig;            // fixed-length: stage each tile's contiguous byte span (all windows at once)
};

}  // namespace cbx
