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
// String columns are produced in ONE pass with a decoupled look-back across tiles: a tile
// publishes its per-sequence UTF-8 byte total (aggregate) before decoding its numeric fields,
// then resolves its exclusive base from its predecessors' words, publishes its inclusive prefix
// and writes its payload (staged in LDS, copied out with dword stores).  Tiles are handed out
// by an atomic ticket so every tile a wave waits on is already owned by a running wave.
#include <hip/hip_runtime.h>

#include "cbx_internal.h"

namespace cbx {

__device__ __forceinline__ int64_t wave_excl_scan(int64_t x, int lane, int64_t* total) {
    int64_t v = x;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        int64_t y = __shfl_up(v, d, kWave);
        if (lane >= d) v += y;
    }
    *total = __shfl(v, kWave - 1, kWave);
    return v - x;
}

__device__ __forceinline__ int32_t wave_sum32(int32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, kWave);
    return x;
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

__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
__device__ __forceinline__ StrSpan sop_span(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp,
                                            const TileCtx& t, const int32_t* s_cnt, int lane, const uint8_t* src,
                                            uint32_t rec_addr, const uint32_t* s_lut, bool& ok) {
    bool el = t.active && (op.segment < 0 || op.segment == t.seg);
    if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
    const int o = a.start_off + op.eo;
    ok = el && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    StrSpan sp{0, 0, 0};
    if (ok) sp = string_span(op.kind, op.trim, src + rec_addr + (uint32_t)op.eo, n,
                             [&](uint32_t b) { return str_lut(op.kind, s_lut, b); });
    return sp;
}

// W = output bytes per value; W = 0: width from the op's output type (generic batches)
template <int W>
__device__ __forceinline__ void store_w(void* values, int64_t v, const Val& x, int out_type) {
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
__device__ __forceinline__ void num_batch(const KernelArgs& a, const Batch& b, const TileCtx& t, const uint8_t* src,
                                          uint32_t rec_addr, const int32_t* s_cnt, int lane) {
    const int lim = t.active ? t.avail - a.start_off : -1;   // element must end within the record
    for (int i = b.begin; i < b.end; i++) {
        const NumOp op = ldc(a.nops + i);
        bool ok = op.eo + op.size <= lim;
        if (op.segment >= 0) ok &= op.segment == t.seg;
        if (kOdo) ok &= odo_present(a.nops + i, op.n_odo, s_cnt, lane);
        Val x = null_val();
        bool defer = false;
        if (kGlobal || V == V_GENERIC) {
            defer = ok;
        } else {
            const uint32_t addr = rec_addr + (ok ? (uint32_t)op.eo : 0u);
            if (V == V_BCD8) x = decode_bcd8(op, src, addr);
            else if (V == V_BCD16) x = decode_bcd16(op, src, addr);
            else if (V == V_BIN8) x = decode_bin8(op, src, addr);
            else if (V == V_ZONED16) { x = decode_zoned16(op, src, addr, defer); defer &= ok; }
            else if (V == V_FP) x = decode_fp(op, src, addr);
            x.valid &= ok;
        }
        const DevColumn col = ldc(a.cols + op.column);
        if (t.active) store_w<W>(col.values, (int64_t)op.slot * a.n_rec + t.rec, x, op.out_type);
        const uint64_t m = __ballot(x.valid);
        col.validity[(int64_t)op.slot * a.n_tiles + t.tile] = m;
        if (V == V_ZONED16 || V == V_GENERIC || kGlobal) {
            const uint64_t dm = __ballot(defer);
            if (op.defer >= 0) a.defer_bits[(int64_t)op.defer * a.n_tiles + t.tile] = dm;
        }
    }
}

// Decode one window of the current tile.  src + rec_addr is the record's decode base (LDS
// image, or HBM for the global window).
template <bool kGlobal>
__device__ __forceinline__ void decode_window(const KernelArgs& a, const Window& w, const TileCtx& t, const uint8_t* src,
                                              uint32_t rec_addr, const int32_t* s_cnt, const uint32_t* s_lut,
                                              uint8_t* s_str, uint64_t* s_scr, uint32_t* s_agg, int lane) {
    const bool sizes = a.mode == 1;
    // ---- strings, phase A: per-element tile aggregates (kept in LDS for phase C)
    for (int i = w.sop_begin; i < w.sop_end; i++) {
        const StrOp op = ldc(a.sops + i);
        bool ok;
        const StrSpan sp = sop_span(a, op, a.sops + i, t, s_cnt, lane, src, rec_addr, s_lut, ok);
        const int32_t agg = wave_sum32(sp.utf8_len);
        if (lane == 0) {
            s_agg[i - w.sop_begin] = (uint32_t)agg;
            if (sizes) atomicAdd((unsigned long long*)&a.seq_totals[op.seq], (unsigned long long)agg);
            else lb_store(&a.lookback[t.tile * a.n_seq + op.seq], (t.tile == 0 ? kLbPrefix : kLbAgg) | (uint64_t)agg);
        }
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
    wave_sync_lds();
    // ---- strings, phase C: resolve bases (look-back), write offsets + payload
    for (int i0 = w.sop_begin; i0 < w.sop_end; i0 += kWave) {
        const int ni = min(kWave, w.sop_end - i0);
        // lane k resolves element i0 + k
        if (lane < ni) {
            const int seq = a.sops[i0 + lane].seq;
            uint64_t* me = &a.lookback[t.tile * a.n_seq + seq];
            uint64_t excl = 0;
            if (t.tile > 0) {
                int64_t j = t.tile - 1;
                while (true) {
                    const uint64_t wv = lb_load(&a.lookback[j * a.n_seq + seq]);
                    const uint64_t st = wv >> 62;
                    if (st == 0) { __builtin_amdgcn_s_sleep(1); continue; }
                    excl += wv & kLbValue;
                    if (st == 2) break;
                    j--;
                }
                lb_store(me, kLbPrefix | (excl + s_agg[i0 - w.sop_begin + lane]));
            }
            s_scr[lane] = excl;
        }
        wave_sync_lds();
        for (int k = 0; k < ni; k++) {
            const StrOp op = ldc(a.sops + i0 + k);
            const DevColumn col = ldc(a.cols + op.column);
            bool ok;
            const StrSpan sp = sop_span(a, op, a.sops + i0 + k, t, s_cnt, lane, src, rec_addr, s_lut, ok);
            int64_t tot;
            const int64_t ex = wave_excl_scan(sp.utf8_len, lane, &tot);
            const int64_t tbase = (int64_t)s_scr[k];
            const int64_t region = (int64_t)op.slot * col.capacity;
            const bool fits = tbase + tot <= col.capacity;
            const int64_t ob = (int64_t)op.slot * (a.n_rec + 1);
            if (t.active) {
                col.offsets[ob + t.rec] = region + tbase + ex;
                if (t.rec == a.n_rec - 1) {
                    col.offsets[ob + a.n_rec] = region + tbase + ex + sp.utf8_len;
                    if (col.sizes) col.sizes[op.slot] = tbase + ex + sp.utf8_len;
                }
            }
            const uint64_t m = __ballot(ok);
            if (lane == 0) col.validity[(int64_t)op.slot * a.n_tiles + t.tile] = m;
            if (!fits) {
                if (lane == 0) atomicOr(a.status, 1);
                continue;
            }
            auto lutf = [&](uint32_t b) { return str_lut(op.kind, s_lut, b); };
            const uint8_t* sp_src = src + rec_addr + (uint32_t)op.eo;
            uint8_t* gdst = col.data + region + tbase;
            if (tot <= a.str_stage) {
                // stage the tile's payload contiguously in LDS, copy out with dword stores
                if (ok) string_write(op.kind, sp_src, sp, s_str + ex, lutf);
                wave_sync_lds();
                const uint64_t g0 = (uint64_t)gdst;
                const uint64_t A = (g0 + 3) & ~3ull, B = (g0 + tot) & ~3ull;
                if (A > B) {   // payload inside one dword: byte stores
                    if (lane < tot) gdst[lane] = s_str[lane];
                } else {
                    const int head = (int)(A - g0), tail = (int)(g0 + tot - B);
                    if (lane < head) gdst[lane] = s_str[lane];
                    if (lane < tail) gdst[(int)(B - g0) + lane] = s_str[(int)(B - g0) + lane];
                    const int ndw = (int)((B - A) >> 2);
                    const uint32_t* s32 = (const uint32_t*)s_str;
                    uint32_t* d32 = (uint32_t*)A;
                    for (int q = lane; q < ndw; q += kWave) {
                        const uint32_t byte = (uint32_t)head + 4u * (uint32_t)q;
                        const uint32_t lo = s32[byte >> 2], hi = s32[(byte >> 2) + 1];
                        d32[q] = align_bytes(hi, lo, byte & 3u);
                    }
                }
                wave_sync_lds();
            } else if (ok) {
                string_write(op.kind, sp_src, sp, gdst + ex, lutf);
            }
        }
    }
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
    uint64_t* s_scr = (uint64_t*)(wbase + a.lds_rows + a.lds_counts);
    uint32_t* s_agg = (uint32_t*)(wbase + a.lds_rows + a.lds_counts + kWave * 8);
    uint8_t* s_str = wbase + a.lds_rows + a.lds_counts + kWave * 8 + a.lds_agg;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lut[i] = a.lut[i];
    __syncthreads();

    const bool dynamic = a.n_seq > 0 && a.mode == 0;
    int64_t tile;
    if (dynamic) {
        uint32_t tk = 0;
        if (lane == 0) tk = atomicAdd(a.ticket, 1u);
        tile = __shfl((int)tk, 0, kWave);
    } else {
        tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    }
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

        // ---- next tile (ticket taken early: its owner is this wave, so waiters progress)
        int64_t next;
        if (dynamic) {
            uint32_t tk = 0;
            if (lane == 0) tk = atomicAdd(a.ticket, 1u);
            next = __shfl((int)tk, 0, kWave);
        } else {
            next = tile + tstep;
        }

        for (int wi = 0; wi < a.n_windows; wi++) {
            const Window w = ldc(a.windows + wi);
            if (a.mode == 1 && w.sop_begin == w.sop_end) continue;
            if (w.global) {
                decode_window<true>(a, w, t, rp, 0u, s_cnt, s_lut, s_str, s_scr, s_agg, lane);
                continue;
            }
            const uint32_t rec_addr = a.contig ? stage_contig(a, tile, s_img, lane) : stage_window(a, w, t, s_img, lane);
            wave_sync_lds();
            decode_window<false>(a, w, t, (const uint8_t*)s_img, rec_addr, s_cnt, s_lut, s_str, s_scr, s_agg, lane);
            wave_sync_lds();
        }
        tile = next;
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
        store_value(col, f.out_type, (int64_t)ds.slot * a.n_rec + rec, x);
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
