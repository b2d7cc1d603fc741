// cbx_kernels.hip -- gfx950 kernels of the copybook decode hot path.
//
// Work decomposition (DESIGN.md "Kernels"): one wave = one tile of 64 consecutive records,
// lane r = record r of the tile; a workgroup holds kWavesPerBlock independent waves.  The field
// loop walks the plan's descriptor tables (scalar loads: the tables live in address space 4),
// so decode dispatch is wave-uniform -- every lane decodes the same field of a different record
// -- and every output store is a coalesced 64-value row of a slot-major column.
//
// Record bytes reach LDS in one of two ways:
//   * contiguous (fixed-length records, 64 * stride <= 16 KiB): the tile's whole byte span is
//     fetched with 16-byte loads (consecutive lanes on consecutive chunks, 1 KiB per
//     wave-instruction, all chunks in flight at once) and written to LDS rows padded to an odd
//     number of dwords, so the per-lane dword reads of a field hit 32 distinct banks;
//   * windowed (variable-length records, wide records): per window of <= 1 KiB of each record,
//     (record, 16-byte chunk) pairs are spread over the lanes.
// Validity bits come from one 64-lane ballot per (field, slot).
//
// String columns: the decode kernel computes every value's trimmed span and UTF-8 length, a
// DPP wave scan gives tile-local positions, and the tile's payload (staged in LDS, copied with
// dword stores) goes to a per-tile scratch region; a device-wide scan of the per-tile totals
// and the placement kernel then write the final payload and absolute offsets.  (A single-pass
// decoupled look-back was measured slower on this chip: device-scope atomics and look-back
// probes are memory-side round trips, and ~2,500 tiles are in flight at once -- DESIGN.md.)
#include <hip/hip_runtime.h>

#include "cbx_internal.h"

namespace cbx {

// Exclusive scan of a 32-bit value over the wave with DPP row shifts (Hillis-Steele inside
// each 16-lane row) plus the preceding rows' totals read with v_readlane.  All lanes active.
__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t x, int lane, uint32_t& total) {
    uint32_t v = x;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    const int row = lane >> 4;
    v += (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
    total = r0 + r1 + r2 + r3;
    return v - x;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Copy a plan-table entry out of the constant address space (scalar loads when uniform).
template <typename T>
__device__ __forceinline__ T ldc(const CBX_CONST T* p) {
    static_assert(sizeof(T) % 4 == 0, "plan tables are dword structs");
    int32_t w[sizeof(T) / 4];
    const CBX_CONST int32_t* q = (const CBX_CONST int32_t*)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) w[i] = q[i];
    T r;
    __builtin_memcpy(&r, w, sizeof(T));
    return r;
}

// 16 bytes at data + ga (ga 16-byte aligned); bytes outside [0, len) read as 0.
__device__ __forceinline__ uint4 load16_guarded(const uint8_t* data, int64_t ga, int64_t len) {
    if (ga >= 0 && ga + 16 <= len) return *(const uint4*)(data + ga);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int64_t g = ga + j;
        const uint32_t b = (g >= 0 && g < len) ? data[g] : 0u;
        w[j >> 2] |= b << (8 * (j & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// FixedLenNestedRowIterator.getSegmentId / VRLRecordReader.getSegmentId:
// extractPrimitiveField(field).toString.trim, looked up in the segment-redefine map.
__device__ int segment_of(const KernelArgs& a, const uint32_t* lut, const uint8_t* rec, int avail) {
    const CBX_CONST cbx_segment_map* m = a.segmap;
    int o = a.start_off + m->field_offset;
    int n = m->field_size;
    if (o > avail) o = avail;
    if (o + n > avail) n = avail - o;
    if (n < 0) n = 0;
    const uint8_t* p = rec + o;
    int b = 0, e = n;
    while (b < e && (lut[p[b]] >> 31)) b++;
    while (e > b && (lut[p[e - 1]] >> 31)) e--;
    // keys are stored as UTF-8 (key[k][] holds bytes, key_len[k] their count)
    for (int k = 0; k < m->n_keys; k++) {
        const CBX_CONST uint16_t* key = m->key[k];
        int kl = m->key_len[k];
        int pos = 0;
        bool eq = true;
        for (int i = b; i < e && eq; i++) {
            uint32_t en = lut[p[i]];
            int l = (en >> 24) & 3;
            for (int j = 0; j < l; j++) {
                if (pos >= kl || key[pos] != ((en >> (8 * j)) & 0xFF)) { eq = false; break; }
                pos++;
            }
        }
        if (eq && pos == kl) return m->key_segment[k];
    }
    return -1;
}

__device__ __forceinline__ void store_value(const DevColumn& c, int out_type, int64_t v, const Val& x) {
    switch (out_type) {
    case CBX_O_I32: ((int32_t*)c.values)[v] = (int32_t)x.lo; break;
    case CBX_O_F32: ((uint32_t*)c.values)[v] = (uint32_t)x.lo; break;
    case CBX_O_DEC128: ((uint64_t*)c.values)[2 * v] = x.lo; ((uint64_t*)c.values)[2 * v + 1] = x.hi; break;
    default: ((uint64_t*)c.values)[v] = x.lo; break;
    }
}

// Per-lane state of the tile being decoded.
struct TileCtx {
    int64_t tile;
    int64_t rec;        // record index of this lane
    bool active;        // rec < n_rec
    int64_t base;       // byte offset of the record (relative to a.data) -- decode base minus start_off
    int avail;          // bytes available in the record (rec_len / stride)
    int seg;            // active segment-redefine index, -1 none
};

// OCCURS DEPENDING ON presence of an element: every ODO level's element index is below the
// record's count (read through the table pointer: a dynamic index into a register copy of
// the op would force it to scratch).
template <typename OP>
__device__ __forceinline__ bool odo_present(const CBX_CONST OP* opp, int n_odo, const int32_t* s_cnt, int lane) {
    bool el = true;
    for (int j = 0; j < n_odo; j++) el &= opp->odo_idx[j] < s_cnt[opp->odo_arr[j] * kWave + lane];
    return el;
}

__device__ __forceinline__ uint32_t str_lut(int kind, const uint32_t* s_lut, uint32_t b) {
    return kind == CBX_K_STRING_ASCII ? ascii_lut(b) : s_lut[b];
}

// String element of the current tile: trimmed span + UTF-8 length (StringDecoders / StringTools).
// Elements of at most kStrFastBytes EBCDIC/ASCII bytes keep their bytes in `w` (register path).
__device__ __forceinline__ StrSpan sop_span(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp,
                                            const TileCtx& t, const int32_t* s_cnt, int lane, const uint8_t* src,
                                            uint32_t rec_addr, const uint32_t* s_lut, bool& ok, bool fast, uint32_t w[8]) {
    bool el = t.active && (op.segment < 0 || op.segment == t.seg);
    if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
    const int o = a.start_off + op.eo;
    ok = el && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    auto lutf = [&](uint32_t b) { return str_lut(op.kind, s_lut, b); };
    if (fast) {
        img_bytes32(src, rec_addr + (ok ? (uint32_t)op.eo : 0u), op.size, w);
        return string_span32(op.trim, w, n, op.size, lutf);
    }
    StrSpan sp{0, 0, 0};
    if (ok) sp = string_span(op.kind, op.trim, src + rec_addr + (uint32_t)op.eo, n, lutf);
    return sp;
}

__device__ __forceinline__ bool sop_fast(const StrOp& op, bool global) {
    return !global && op.size <= kStrFastBytes && (op.kind == CBX_K_STRING || op.kind == CBX_K_STRING_ASCII);
}

template <int W>
__device__ __forceinline__ void store_w(void* values, int64_t v, const Val& x, int out_type) {
    // v: element index within the slot row
    const int w = W ? W : (out_type == CBX_O_I32 || out_type == CBX_O_F32 ? 4 : out_type == CBX_O_DEC128 ? 16 : 8);
    if (w == 4) ((uint32_t*)values)[v] = (uint32_t)x.lo;
    else if (w == 8) ((uint64_t*)values)[v] = x.lo;
    else { ((uint64_t*)values)[2 * v] = x.lo; ((uint64_t*)values)[2 * v + 1] = x.hi; }
}

// One batch of numeric ops (same decoder variant V, output width W).  Decoding is branch-free
// per lane: every lane reads its (clamped) element and computes, the bounds / segment / OCCURS
// conditions only select validity.  The validity (and deferral) word of each op is a wave
// ballot stored by every lane to the same address.
template <int V, int W, bool kOdo, bool kGlobal>
__device__ __forceinline__ void num_one(const KernelArgs& a, const NumOp& op, int i, const TileCtx& t,
                                        bool ok, uint64_t r1, uint64_t r0, const int32_t* s_cnt, int lane) {
    if (op.segment >= 0) ok &= op.segment == t.seg;
    if (kOdo) ok &= odo_present(a.nops + i, op.n_odo, s_cnt, lane);
    Val x = null_val();
    bool defer = false;
    if (kGlobal || V == V_GENERIC) {
        defer = ok;
    } else {
        if (V == V_BCD8) x = bcd8_raw(op, r1);
        else if (V == V_BCD16) x = bcd16_raw(op, r1, r0);
        else if (V == V_BIN8) x = bin8_raw(op, r1);
        else if (V == V_ZONED16) { x = zoned16_raw(op, r1, r0, defer); defer &= ok; }
        else if (V == V_FP) x = fp_raw(op, r1);
        x.valid &= ok;
    }
    const NumCall c = ldc(a.ncall + i);
    // every lane stores (slot rows are padded to 64 * n_tiles values): no exec-mask branches
    store_w<W>(c.values, t.rec, x, op.out_type);
    const uint64_t m = __ballot(x.valid);
    c.validity[t.tile] = m;
    if (V == V_ZONED16 || V == V_GENERIC || kGlobal) {
        const uint64_t dm = __ballot(defer);
        if (c.defer) c.defer[t.tile] = dm;
    }
}

// One batch of numeric ops (same decoder variant V, output width W), four ops per step: the
// LDS reads of the four elements are issued before any of them is decoded.  Decoding is
// branch-free per lane: every lane reads its (clamped) element and computes, the bounds /
// segment / OCCURS conditions only select validity.  The validity (and deferral) word of each
// op is a wave ballot stored by every lane to the same address.
template <int V, int W, bool kOdo, bool kGlobal>
__device__ __forceinline__ void num_batch(const KernelArgs& a, const Batch& b, const TileCtx& t, const uint8_t* src,
                                          uint32_t rec_addr, const int32_t* s_cnt, int lane) {
    constexpr bool kWide = V == V_BCD16 || V == V_ZONED16;   // two 8-byte reads per element
    constexpr bool kRead = !(kGlobal || V == V_GENERIC);
    const int lim = t.active ? t.avail - a.start_off : -1;   // element must end within the record
    constexpr int U = 4;
    int i = b.begin;
    for (; i + U <= b.end; i += U) {
        NumOp op[U];
        bool ok[U];
        uint64_t r1[U], r0[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            op[u] = ldc(a.nops + i + u);
            ok[u] = op[u].eo + op[u].size <= lim;
            r1[u] = r0[u] = 0;
            if (kRead) {
                const uint32_t end = rec_addr + (ok[u] ? (uint32_t)op[u].eo : 0u) + op[u].size;
                r1[u] = img_le64_ending(src, end);
                if (kWide) r0[u] = img_le64_ending(src, end - 8);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) num_one<V, W, kOdo, kGlobal>(a, op[u], i + u, t, ok[u], r1[u], r0[u], s_cnt, lane);
    }
    for (; i < b.end; i++) {
        const NumOp op = ldc(a.nops + i);
        const bool ok = op.eo + op.size <= lim;
        uint64_t r1 = 0, r0 = 0;
        if (kRead) {
            const uint32_t end = rec_addr + (ok ? (uint32_t)op.eo : 0u) + op.size;
            r1 = img_le64_ending(src, end);
            if (kWide) r0 = img_le64_ending(src, end - 8);
        }
        num_one<V, W, kOdo, kGlobal>(a, op, i, t, ok, r1, r0, s_cnt, lane);
    }
}

// One string element of the tile (StringDecoders.decodeEbcdicString / decodeAsciiString):
// span + tile-local scan; the tile's payload is staged contiguously in LDS and copied with
// dword stores to the tile's scratch region; the tile-local start of every value and the
// tile's byte total are recorded for the compaction kernel, which places tiles after a
// device-wide scan of the totals (two-pass string offsets, no cross-tile waiting).
__device__ __forceinline__ void str_element(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp,
                                            const StrCall& c, const TileCtx& t, const int32_t* s_cnt,
                                            const uint8_t* src, uint32_t rec_addr, bool global,
                                            const uint32_t* s_lut, uint8_t* s_str, int lane) {
    const bool fast = sop_fast(op, global);
    bool ok;
    uint32_t wb[8];
    const StrSpan sp = sop_span(a, op, opp, t, s_cnt, lane, src, rec_addr, s_lut, ok, fast, wb);
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32((uint32_t)sp.utf8_len, lane, tot);
    if (a.mode == 1) {
        if (lane == 0) a.str_tot[(int64_t)op.seq * a.n_tiles + t.tile] = tot;
        return;
    }
    c.validity[t.tile] = __ballot(ok);
    c.local[t.rec] = ex;
    if (lane == 0) a.str_tot[(int64_t)op.seq * a.n_tiles + t.tile] = tot;
    auto lutf = [&](uint32_t b) { return str_lut(op.kind, s_lut, b); };
    const uint8_t* sp_src = src + rec_addr + (uint32_t)op.eo;
    uint32_t* dst32 = (uint32_t*)(c.scratch + t.tile * (int64_t)c.tile_cap);   // 16-byte aligned region
    if ((int)tot <= a.str_stage) {
        if (fast) string_write32(wb, sp, s_str + ex, s_str + a.str_stage, op.size, op.pad > 1, lutf);
        else if (ok) string_write(op.kind, sp_src, sp, s_str + ex, lutf);
        wave_sync_lds();
        const uint32_t* s32 = (const uint32_t*)s_str;
        for (int q = lane; 4 * q < (int)tot; q += kWave) dst32[q] = s32[q];
        wave_sync_lds();
    } else if (ok) {
        uint8_t* dst = (uint8_t*)dst32 + ex;
        if (fast) {
            uint8_t dump[4];
            string_write32(wb, sp, dst, dump, op.size, op.pad > 1, lutf);
        } else {
            string_write(op.kind, sp_src, sp, dst, lutf);
        }
    }
}

// Decode one window of the current tile.  src + rec_addr is the record's decode base (LDS
// image, or HBM for the global window).
template <bool kGlobal>
__device__ __forceinline__ void decode_window(const KernelArgs& a, const Window& w, const TileCtx& t, const uint8_t* src,
                                              uint32_t rec_addr, const int32_t* s_cnt, const uint32_t* s_lut,
                                              uint8_t* s_str, int lane) {
    const bool sizes = a.mode == 1;
    // ---- strings (tile-local; placed by the compaction kernel)
    for (int i = w.sop_begin; i < w.sop_end; i++) {
        const StrOp op = ldc(a.sops + i);
        const StrCall c = sizes ? StrCall{} : ldc(a.scall + i);
        str_element(a, op, a.sops + i, c, t, s_cnt, src, rec_addr, kGlobal, s_lut, s_str, lane);
    }
    if (sizes) return;
    // ---- generated columns (File_Id / Record_Id)
    for (int i = w.gen_begin; i < w.gen_end; i++) {
        const GenOp g = ldc(a.gops + i);
        const DevColumn col = ldc(a.cols + g.column);
        Val x{g.kind == CBX_K_RECORD_ID ? (uint64_t)(a.first_record_id + t.rec) : (uint64_t)(int64_t)a.file_id, 0, true};
        if (t.active) store_value(col, g.out_type, t.rec, x);
        const uint64_t m = __ballot(t.active);
        if (lane == 0) col.validity[t.tile] = m;
    }
    // ---- numerics (look-back words of earlier tiles land meanwhile), one specialised loop per batch
    for (int bi = w.batch_begin; bi < w.batch_end; bi++) {
        const Batch b = ldc(a.batches + bi);
        if (kGlobal) {
            if (b.odo) num_batch<V_GENERIC, 8, true, true>(a, b, t, src, rec_addr, s_cnt, lane);
            else num_batch<V_GENERIC, 8, false, true>(a, b, t, src, rec_addr, s_cnt, lane);
            continue;
        }
        if (b.odo) {   // elements under OCCURS DEPENDING ON: one generic-width loop per variant
            switch (b.variant) {
            case V_BCD8: num_batch<V_BCD8, 0, true, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
            case V_BCD16: num_batch<V_BCD16, 0, true, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
            case V_BIN8: num_batch<V_BIN8, 0, true, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
            case V_ZONED16: num_batch<V_ZONED16, 0, true, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
            case V_FP: num_batch<V_FP, 0, true, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
            default: num_batch<V_GENERIC, 0, true, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
            }
            continue;
        }
#define CBX_BATCH(V)                                                                                  \
    case V:                                                                                           \
        if (b.width == 4) num_batch<V, 4, false, false>(a, b, t, src, rec_addr, s_cnt, lane);        \
        else if (b.width == 8) num_batch<V, 8, false, false>(a, b, t, src, rec_addr, s_cnt, lane);   \
        else num_batch<V, 16, false, false>(a, b, t, src, rec_addr, s_cnt, lane);                    \
        break;
        switch (b.variant) {
            CBX_BATCH(V_BCD8)
            CBX_BATCH(V_BCD16)
            CBX_BATCH(V_BIN8)
            CBX_BATCH(V_ZONED16)
            CBX_BATCH(V_FP)
            default: num_batch<V_GENERIC, 0, false, false>(a, b, t, src, rec_addr, s_cnt, lane); break;
        }
#undef CBX_BATCH
    }
    if (w.sop_begin == w.sop_end) return;
}

// Contiguous staging of a fixed-length tile: the tile's byte span [t0b, t0b + n * stride) is
// fetched in rounds of 8 KiB per wave (16-byte loads, consecutive lanes on consecutive chunks)
// and written to LDS rows of cpitch bytes (odd dword count).  Returns the lane's record base.
__device__ __forceinline__ uint32_t stage_contig(const KernelArgs& a, int64_t tile, uint8_t* s_img, int lane) {
    const int64_t t0b = a.base_shift + tile * kWave * (int64_t)a.stride;
    const int64_t left = a.n_rec - tile * kWave;
    const int nrec_tile = left < kWave ? (int)left : kWave;
    const int64_t a0 = t0b & ~(int64_t)15;
    const int mis_dw = (int)((t0b - a0) >> 2);
    const int span_dw = nrec_tile * a.stride_dw;
    const int nch = (mis_dw + span_dw + 3) >> 2;
    const bool pad = a.cpitch != 4 * a.stride_dw;
    constexpr int kRound = 8;   // 16-byte chunks per lane in flight (8 KiB per wave)
    uint32_t* img32 = (uint32_t*)s_img;
    for (int c0 = 0; c0 < nch; c0 += kRound * kWave) {
        uint4 buf[kRound];
#pragma unroll
        for (int u = 0; u < kRound; u++) {
            const int c = c0 + u * kWave + lane;
            buf[u] = c < nch ? load16_guarded(a.data, a0 + 16 * (int64_t)c, a.data_len) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kRound; u++) {
            const int c = c0 + u * kWave + lane;
            if (c < nch) {
                if (!pad) {
                    *(uint4*)(s_img + 16 * c) = buf[u];
                } else {
                    const uint32_t wv[4] = {buf[u].x, buf[u].y, buf[u].z, buf[u].w};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int d = 4 * c + k - mis_dw;
                        if (d >= 0 && d < span_dw) {
                            const int r = (int)(((float)d + 0.5f) * a.inv_stride_dw);
                            img32[d + mis_dw + r] = wv[k];
                        }
                    }
                }
            }
        }
    }
    return (uint32_t)(lane * a.cpitch + 4 * mis_dw + a.start_off);
}

// Windowed staging: bytes [w.lo, w.hi) of every record of the tile, (record, 16-byte chunk)
// pairs spread over the lanes, rows of w.pitch bytes.  Returns the lane's record base.
__device__ __forceinline__ uint32_t stage_window(const KernelArgs& a, const Window& w, const TileCtx& t,
                                                 uint8_t* s_img, int lane) {
    const int W = w.hi - w.lo;
    const int pitch = w.pitch;
    const int nch = (W + 15 + 15) >> 4;
    const float inv_nch = 1.0f / (float)nch;
    const int64_t my_g = t.base + a.start_off + w.lo;
    const int my_mis = (int)(my_g & 15);
    const int total = kWave * nch;
    for (int t0 = 0; t0 < total; t0 += 8 * kWave) {
        uint4 buf[8];
        int rr[8], kk[8];
        bool ld[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int q = t0 + u * kWave + lane;
            int r = (int)(((float)q + 0.5f) * inv_nch);
            r = r < kWave ? r : kWave - 1;
            const int k = q - r * nch;
            rr[u] = r; kk[u] = k;
            const int64_t gb = __shfl(my_g, r, kWave);
            const bool ract = __shfl((int)t.active, r, kWave) != 0;
            ld[u] = q < total && ract;
            const int64_t ga = (gb & ~(int64_t)15) + 16 * (int64_t)k;
            buf[u] = ld[u] ? load16_guarded(a.data, ga, a.data_len) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (ld[u]) {
                uint32_t* dst = (uint32_t*)(s_img + rr[u] * pitch + 16 * kk[u]);
                dst[0] = buf[u].x; dst[1] = buf[u].y; dst[2] = buf[u].z; dst[3] = buf[u].w;
            }
        }
    }
    return (uint32_t)(lane * pitch + my_mis - w.lo);
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void decode_kernel(KernelArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* s_lut = (uint32_t*)smem;
    const int wid = threadIdx.x / kWave;
    const int lane = threadIdx.x % kWave;
    uint8_t* wbase = smem + 1024 + wid * a.lds_wave;
    uint8_t* s_img = wbase + kGuard;
    int32_t* s_cnt = (int32_t*)(wbase + a.lds_rows);
    uint8_t* s_str = wbase + a.lds_rows + a.lds_counts;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lut[i] = a.lut[i];
    __syncthreads();

    // static grid-stride tile order (tiles are independent)
    int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    const int64_t tstep = (int64_t)gridDim.x * kWavesPerBlock;

    while (tile < a.n_tiles) {
        TileCtx t;
        t.tile = tile;
        t.rec = tile * kWave + lane;
        t.active = t.rec < a.n_rec;
        t.base = a.base_shift;
        t.avail = 0;
        if (a.rec_off) {
            if (t.active) { t.base += a.rec_off[t.rec]; t.avail = a.rec_len[t.rec]; }
        } else if (t.active) {
            t.base += t.rec * (int64_t)a.stride;
            t.avail = a.stride;
        }
        const uint8_t* rp = a.data + t.base;

        // ---- segment redefine selection
        t.seg = -1;
        if (a.segmap && t.active) t.seg = segment_of(a, s_lut, rp, t.avail);
        if (a.mode == 0 && a.seg_col >= 0) {
            const DevColumn c = ldc(a.cols + a.seg_col);
            if (t.active) ((int32_t*)c.values)[t.rec] = t.seg;
            const uint64_t m = __ballot(t.active);
            if (lane == 0) c.validity[tile] = m;
        }

        // ---- OCCURS DEPENDING ON element counts (extractArray, RecordExtractors.scala:66-114)
        for (int ai = 0; ai < a.n_arrays; ai++) {
            const cbx_array ar = ldc(a.arrays + ai);
            int cnt = ar.max_count;
            if (ar.dependee >= 0 && t.active) {
                const Field df = ldc(a.fields + ar.dependee);
                const int o = a.start_off + df.offset;
                const bool seg_ok = df.segment < 0 || df.segment == t.seg;
                if (seg_ok && o + df.size <= t.avail) {
                    Val dv = decode_count_int(df, rp + o);
                    if (dv.valid) {
                        const int32_t v = (int32_t)dv.lo;   // Number.intValue
                        if (v >= ar.min_count && v <= ar.max_count) cnt = v;
                    }
                }
            }
            s_cnt[ai * kWave + lane] = cnt;
            if (a.mode == 0 && ar.count_column >= 0) {
                const DevColumn c = ldc(a.cols + ar.count_column);
                const bool ok = t.active && (ar.segment < 0 || ar.segment == t.seg);
                if (t.active) ((int32_t*)c.values)[t.rec] = cnt;
                const uint64_t m = __ballot(ok);
                if (lane == 0) c.validity[tile] = m;
            }
        }

        for (int wi = 0; wi < a.n_windows; wi++) {
            const Window w = ldc(a.windows + wi);
            if (a.mode == 1 && w.sop_begin == w.sop_end) continue;
            if (w.global) {
                decode_window<true>(a, w, t, rp, 0u, s_cnt, s_lut, s_str, lane);
                continue;
            }
            const uint32_t rec_addr = a.contig ? stage_contig(a, tile, s_img, lane) : stage_window(a, w, t, s_img, lane);
            wave_sync_lds();
            decode_window<false>(a, w, t, (const uint8_t*)s_img, rec_addr, s_cnt, s_lut, s_str, lane);
            wave_sync_lds();
        }
        tile += tstep;
    }
}

// ------------------------------------------------------------------------------------------
// String placement.  Exclusive scan of the per-(sequence, tile) payload totals (one int64 array
// over all sequences; a sequence's base is subtracted by the compaction kernel), then one wave
// per (sequence, tile) copies the tile's payload from its scratch region to its final place and
// writes the absolute Arrow offsets.
// ------------------------------------------------------------------------------------------
constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ int64_t block_excl_scan64(int64_t x, int64_t* s_w, int64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t v = x;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int64_t y = __shfl_up(v, d, kWave);
        if (lane >= d) v += y;
    }
    if (lane == kWave - 1) s_w[wid] = v;
    __syncthreads();
    int64_t pre = 0, all = 0;
    for (int i = 0; i < kScanBlock / kWave; i++) {
        if (i < wid) pre += s_w[i];
        all += s_w[i];
    }
    __syncthreads();
    *total = all;
    return pre + v - x;
}

// pass 1: per-block sums of uint32 totals
__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(const uint32_t* in, int64_t n, int64_t* block_sums) {
    __shared__ int64_t s_w[kScanBlock / kWave];
    const int64_t b0 = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int64_t sum = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) sum += b0 + i < n ? in[b0 + i] : 0u;
    int64_t total;
    block_excl_scan64(sum, s_w, &total);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

// pass 2: exclusive scan of the block sums (one block, loops)
__global__ __launch_bounds__(kScanBlock) void scan_block_sums_kernel(int64_t* block_sums, int64_t nb) {
    __shared__ int64_t s_w[kScanBlock / kWave];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += kScanBlock) {
        const int64_t i = b0 + threadIdx.x;
        const int64_t x = i < nb ? block_sums[i] : 0;
        int64_t total;
        const int64_t ex = block_excl_scan64(x, s_w, &total);
        if (i < nb) block_sums[i] = carry + ex;
        carry += total;
    }
}

// pass 3: exclusive prefix of every element
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const uint32_t* in, int64_t n, const int64_t* block_sums,
                                                                int64_t* out) {
    __shared__ int64_t s_w[kScanBlock / kWave];
    const int64_t b0 = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    int64_t sum = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        v[i] = b0 + i < n ? in[b0 + i] : 0u;
        sum += v[i];
    }
    int64_t total;
    int64_t ex = block_excl_scan64(sum, s_w, &total) + block_sums[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        if (b0 + i < n) out[b0 + i] = ex;
        ex += v[i];
    }
}

struct SeqCall {
    int64_t* offsets;       // slot offsets (pitch + 1 entries)
    uint8_t* data;          // slot payload region
    const uint32_t* local;  // tile-local starts of the slot's values
    const uint8_t* scratch; // tile regions of the slot
    int64_t* size;          // slot payload bytes (may be null)
    int64_t region;         // region position in the column's data
    int64_t capacity;
    int32_t tile_cap;
    int32_t reserved;
};

__global__ __launch_bounds__(kWave) void str_place_kernel(const CBX_CONST SeqCall* seqs, const uint32_t* tot,
                                                          const int64_t* excl, int64_t n_tiles, int64_t n_rec,
                                                          int32_t* status) {
    const int seq = blockIdx.y;
    const int lane = threadIdx.x;
    const SeqCall q = ldc(seqs + seq);
    const int64_t seq0 = excl[(int64_t)seq * n_tiles];
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = excl[(int64_t)seq * n_tiles + tile] - seq0;
        const uint32_t n = tot[(int64_t)seq * n_tiles + tile];
        const int64_t rec = tile * kWave + lane;
        q.offsets[rec] = q.region + base + q.local[rec];   // lanes past n_rec write padding entries
        if (tile == n_tiles - 1 && lane == 0) {
            q.offsets[n_rec] = q.region + base + n;
            if (q.size) *q.size = base + n;
        }
        if (base + (int64_t)n > q.capacity) {
            if (lane == 0) atomicOr(status, 1);
            continue;
        }
        // payload: scratch (aligned) -> data + base (any alignment); dword stores in the middle,
        // byte stores for the unaligned head and tail
        const uint32_t* src = (const uint32_t*)(q.scratch + tile * (int64_t)q.tile_cap);
        uint8_t* dst = q.data + base;
        const uint64_t g0 = (uint64_t)dst;
        const uint64_t A = (g0 + 3) & ~3ull, B = (g0 + n) & ~3ull;
        const uint8_t* s8 = (const uint8_t*)src;
        if (A > B) {
            if (lane < (int)n) dst[lane] = s8[lane];
            continue;
        }
        const int head = (int)(A - g0), tail = (int)(g0 + n - B);
        if (lane < head) dst[lane] = s8[lane];
        if (lane < tail) dst[(int)(B - g0) + lane] = s8[(int)(B - g0) + lane];
        const int ndw = (int)((B - A) >> 2);
        uint32_t* d32 = (uint32_t*)A;
        for (int i = lane; i < ndw; i += kWave) {
            const uint32_t byte = (uint32_t)head + 4u * (uint32_t)i;
            const uint32_t lo = src[byte >> 2], hi = src[(byte >> 2) + 1];
            d32[i] = align_bytes(hi, lo, byte & 3u);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Fixup: values the fast paths deferred (zoned forms other than F-zone digits + overpunch,
// wide / P-scaled numerics) are decoded here with the byte-loop decoders, straight from HBM.
// One thread per (deferral sequence, tile) word of the deferral bitmap; almost all are zero.
// ------------------------------------------------------------------------------------------
struct DeferSeq {
    int32_t field, slot;
};

__global__ __launch_bounds__(256) void fixup_kernel(KernelArgs a, const CBX_CONST DeferSeq* dseq, int32_t n_defer) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_defer * a.n_tiles) return;
    uint64_t bits = a.defer_bits[i];
    if (!bits) return;
    const int d = (int)(i / a.n_tiles);
    const int64_t tile = i - (int64_t)d * a.n_tiles;
    const DeferSeq ds = ldc(dseq + d);
    const CBX_CONST Field* fp = a.fields + ds.field;
    const Field f = ldc(fp);
    int eo = f.offset, rem = ds.slot;
    for (int k = f.n_dims - 1; k >= 0; k--) {
        const int dc = fp->dim_count[k];
        eo += (rem % dc) * fp->dim_stride[k];
        rem /= dc;
    }
    const DevColumn col = ldc(a.cols + f.column);
    uint64_t vbits = 0;
    while (bits) {
        const int b = __builtin_ctzll(bits);
        bits &= bits - 1;
        const int64_t rec = tile * kWave + b;
        const int64_t base = a.base_shift + (a.rec_off ? a.rec_off[rec] : rec * (int64_t)a.stride);
        const Val x = decode_numeric(f, a.data + base + a.start_off + eo);
        store_value(col, f.out_type, (int64_t)ds.slot * a.pitch + rec, x);
        if (x.valid) vbits |= 1ull << b;
    }
    if (vbits) col.validity[(int64_t)ds.slot * a.n_tiles + tile] |= vbits;
}

// ------------------------------------------------------------------------------------------
// RDW framing (RecordHeaderParserRDW.getRecordMetadata + VRLRecordReader.fetchRecordUsingRdwHeaders)
// One lane per seed segment [seeds[k], seeds[k+1]); pass 0 counts, pass 1 writes.
// ------------------------------------------------------------------------------------------
struct RdwArgs {
    const uint8_t* data;
    int64_t n_bytes;
    const int64_t* seeds;
    int32_t n_seeds;
    cbx_rdw_params p;
    int64_t* counts;       // per seed: pass 0 out, pass 1 in (exclusive scan)
    int64_t* rec_off;
    int32_t* rec_len;
    int64_t capacity;
    int64_t* error;        // [0] = code (0 ok, -2 zero, -3 too big), [1] = offset
};

__global__ void rdw_walk_kernel(RdwArgs a, int pass) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n_seeds) return;
    int64_t pos = a.seeds[k];
    const int64_t end = k + 1 < a.n_seeds ? a.seeds[k + 1] : a.n_bytes;
    int64_t out = pass ? a.counts[k] : 0;
    int64_t cnt = 0;
    while (pos < end) {
        int64_t avail = a.n_bytes - pos;
        int64_t hl = avail < 4 ? avail : 4;
        const uint8_t* h = a.data + pos;
        pos += hl;
        const int64_t file_offset = pos;
        int64_t rlen;
        bool valid;
        if (a.p.file_header_bytes > 4 && file_offset == 4) {
            rlen = a.p.file_header_bytes - 4; valid = false;
        } else if (a.n_bytes > 0 && a.p.file_footer_bytes > 0 && a.n_bytes - file_offset <= a.p.file_footer_bytes) {
            rlen = a.n_bytes - file_offset; valid = false;
        } else if (hl < 4) {
            rlen = -1; valid = false;
        } else {
            rlen = a.p.big_endian ? (int64_t)h[1] + 256 * (int64_t)h[0] + a.p.adjustment
                                  : (int64_t)h[2] + 256 * (int64_t)h[3] + a.p.adjustment;
            if (rlen <= 0) { atomicCAS((unsigned long long*)a.error, 0ull, (unsigned long long)-2ll); a.error[1] = file_offset; return; }
            if (rlen > 100ll * 1024 * 1024) { atomicCAS((unsigned long long*)a.error, 0ull, (unsigned long long)-3ll); a.error[1] = file_offset; return; }
            valid = true;
        }
        if (rlen <= 0) break;
        int64_t rem = a.n_bytes - pos;
        int64_t got = rlen < rem ? rlen : rem;
        if (valid) {
            if (pass && out < a.capacity) { a.rec_off[out] = pos; a.rec_len[out] = (int32_t)got; }
            out++;
            cnt++;
        }
        pos += got;
    }
    if (!pass) a.counts[k] = cnt;
}

}  // namespace cbx
