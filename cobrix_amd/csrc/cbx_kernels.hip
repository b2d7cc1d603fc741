// cbx_kernels.hip -- gfx950 kernels of the copybook decode hot path.
//
// Work decomposition (DESIGN.md "Kernels"): one wave = one tile of 64 consecutive records,
// lane r = record r of the tile.  The field loop runs over the plan's descriptor table, so the
// decode dispatch is wave-uniform (every lane decodes the same field of a different record) and
// every output store is a coalesced 64-value row of a slot-major column.  Record bytes are
// staged window by window into a per-wave LDS region with 16-byte global loads (consecutive
// lanes take consecutive 16-byte chunks of the same record, which handles odd record lengths
// and arbitrary var-len offsets); rows use an odd-dword pitch so the per-lane byte reads of a
// field hit distinct banks.  Validity bits come from one 64-lane ballot per (field, slot).
// String offsets use a two-pass scheme: a sizing pass writes per-(column, slot, tile) UTF-8
// totals, a device scan turns them into bases, and the decode pass adds a wave-level scan.
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

// FixedLenNestedRowIterator.getSegmentId / VRLRecordReader.getSegmentId:
// extractPrimitiveField(field).toString.trim, looked up in the segment-redefine map.
__device__ int segment_of(const KernelArgs& a, const uint32_t* lut, const uint8_t* rec, int avail) {
    const cbx_segment_map* m = a.segmap;
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
        const uint16_t* key = m->key[k];
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

__global__ __launch_bounds__(64) void decode_kernel(KernelArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* s_lut = (uint32_t*)smem;
    int32_t* s_cnt = (int32_t*)(smem + 1024);
    uint8_t* s_rows = smem + 1024 + ((a.n_arrays * kWave * 4 + 15) & ~15);
    const int lane = threadIdx.x;
    for (int i = lane; i < 256; i += kWave) s_lut[i] = a.lut[i];
    __syncthreads();
    const bool sizes = a.mode == 1;

    for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const int64_t rec = tile * kWave + lane;
        const bool active = rec < a.n_rec;
        int64_t base = a.base_shift;
        int avail = 0;
        if (a.rec_off) {
            if (active) { base += a.rec_off[rec]; avail = a.rec_len[rec]; }
        } else if (active) {
            base += rec * (int64_t)a.stride;
            avail = a.stride;
        }
        const uint8_t* rp = a.data + base;

        // ---- segment redefine selection
        int seg = -1;
        if (a.segmap && active) seg = segment_of(a, s_lut, rp, avail);
        if (!sizes && a.seg_col >= 0) {
            const DevColumn& c = a.cols[a.seg_col];
            if (active) ((int32_t*)c.values)[rec] = seg;
            uint64_t m = __ballot(active);
            if (lane == 0) c.validity[tile] = m;
        }

        // ---- OCCURS DEPENDING ON element counts (extractArray, RecordExtractors.scala:66-114)
        for (int ai = 0; ai < a.n_arrays; ai++) {
            const cbx_array& ar = a.arrays[ai];
            int cnt = ar.max_count;
            if (ar.dependee >= 0 && active) {
                const Field& df = a.fields[ar.dependee];
                int o = a.start_off + df.offset;
                bool seg_ok = df.segment < 0 || df.segment == seg;
                if (seg_ok && o + df.size <= avail) {
                    Val dv = decode_numeric(df, rp + o);
                    if (dv.valid) {
                        int32_t v = (int32_t)dv.lo;   // Number.intValue
                        if (v >= ar.min_count && v <= ar.max_count) cnt = v;
                    }
                }
            }
            s_cnt[ai * kWave + lane] = cnt;
            if (!sizes && ar.count_column >= 0) {
                const DevColumn& c = a.cols[ar.count_column];
                bool ok = active && (ar.segment < 0 || ar.segment == seg);
                if (active) ((int32_t*)c.values)[rec] = cnt;
                uint64_t m = __ballot(ok);
                if (lane == 0) c.validity[tile] = m;
            }
        }

        // ---- stage record bytes into the wave's LDS image
        uint32_t contig_addr = 0;
        if (a.contig) {
            // fixed-length tile: one contiguous span [t0b, t0b + nrec * stride), 16-byte chunks,
            // consecutive lanes on consecutive chunks (1 KiB per wave-instruction)
            const int64_t t0b = a.base_shift + tile * kWave * (int64_t)a.stride;
            const int64_t left = a.n_rec - tile * kWave;
            const int nrec_tile = left < kWave ? (int)left : kWave;
            const int64_t a0 = t0b & ~(int64_t)15;
            const int mis = (int)(t0b - a0);
            const int nch = (int)((t0b + (int64_t)nrec_tile * a.stride - a0 + 15) >> 4);
            for (int c0 = 0; c0 < nch; c0 += 8 * kWave) {
                uint4 buf[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int c = c0 + u * kWave + lane;
                    const int64_t ga = a0 + 16 * (int64_t)c;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (c < nch) {
                        if (ga + 16 <= a.data_len) {
                            buf[u] = *(const uint4*)(a.data + ga);
                        } else {
                            uint32_t wv[4] = {0, 0, 0, 0};
                            for (int j = 0; j < 16; j++)
                                if (ga + j < a.data_len) wv[j >> 2] |= (uint32_t)a.data[ga + j] << (8 * (j & 3));
                            buf[u] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int c = c0 + u * kWave + lane;
                    if (c < nch) *(uint4*)(s_rows + 16 * c) = buf[u];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            contig_addr = (uint32_t)(mis + lane * a.stride + a.start_off);
        }
        for (int wi = 0; wi < a.n_windows; wi++) {
            const Window& w = a.windows[wi];
            if (sizes && !w.has_strings) continue;
            const int W = w.hi - w.lo;
            const int pitch = w.pitch;
            const int nch = (W + 15 + 15) >> 4;
            uint8_t* my_row = s_rows + lane * pitch;
            const int64_t my_g = base + a.start_off + w.lo;
            const int my_mis = (int)(my_g & 15);
            // stage: flattened (record, chunk) -> lane, 4 chunks in flight per lane
            const int total = a.contig ? 0 : kWave * nch;
            for (int t0 = 0; t0 < total; t0 += 4 * kWave) {
                uint4 buf[4];
                int rr[4], kk[4];
                bool ld[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    int t = t0 + u * kWave + lane;
                    int r = t / nch;
                    int k = t - r * nch;
                    rr[u] = r; kk[u] = k;
                    int64_t gb = __shfl(my_g, r < kWave ? r : 0, kWave);
                    bool ract = __shfl((int)active, r < kWave ? r : 0, kWave) != 0;
                    ld[u] = t < total && ract;
                    int64_t ga = (gb & ~(int64_t)15) + 16 * (int64_t)k;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (ld[u]) {
                        if (ga >= 0 && ga + 16 <= a.data_len) {
                            buf[u] = *(const uint4*)(a.data + ga);
                        } else {
                            uint32_t wv[4] = {0, 0, 0, 0};
                            for (int j = 0; j < 16; j++) {
                                int64_t q = ga + j;
                                if (q >= 0 && q < a.data_len) wv[j >> 2] |= (uint32_t)a.data[q] << (8 * (j & 3));
                            }
                            buf[u] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (ld[u]) {
                        uint32_t* dst = (uint32_t*)(s_rows + rr[u] * pitch + 16 * kk[u]);
                        dst[0] = buf[u].x; dst[1] = buf[u].y; dst[2] = buf[u].z; dst[3] = buf[u].w;
                    }
                }
            }
            if (!a.contig) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            // LDS byte address of the record's decode base (element offset eo is added per field)
            const uint32_t rec_addr = a.contig ? contig_addr : (uint32_t)(lane * pitch + my_mis - w.lo);
            (void)my_row;
            for (int ri = w.run_begin; ri < w.run_end; ri++) {
                const Run run = a.runs[ri];
                const Field& f = a.fields[run.field];
                const bool is_str = f.out_type == CBX_O_STRING || f.out_type == CBX_O_BINARY;
                if (sizes && !is_str) continue;
                const DevColumn col = a.cols[f.column];
                for (int s = run.slot_begin; s < run.slot_end; s++) {
                    int eo = f.offset;
                    int rem = s;
                    bool el = active && (f.segment < 0 || f.segment == seg);
                    for (int k = f.n_dims - 1; k >= 0; k--) {
                        int dc = f.dim_count[k];
                        int idx = rem % dc;
                        rem /= dc;
                        eo += idx * f.dim_stride[k];
                        el &= idx < s_cnt[f.dim_array[k] * kWave + lane];
                    }
                    const int o = a.start_off + eo;
                    const int64_t v = (int64_t)s * a.n_rec + rec;
                    const uint32_t addr = rec_addr + (uint32_t)eo;
                    const uint8_t* p = s_rows + addr;
                    if (!is_str) {
                        bool ok = el && o + f.size <= avail;
                        Val x = null_val();
                        if (ok) x = decode_numeric_at(f, s_rows, addr);
                        if (active) store_value(col, f.out_type, v, x);
                        uint64_t m = __ballot(x.valid);
                        if (lane == 0) col.validity[(int64_t)s * a.n_tiles + tile] = m;
                    } else {
                        bool ok = el && o <= avail;
                        int n = ok ? (f.size < avail - o ? f.size : avail - o) : 0;
                        StrSpan sp{0, 0, 0};
                        auto lutf = [&](uint32_t b) -> uint32_t {
                            return f.kind == CBX_K_STRING_ASCII ? ascii_lut(b) : s_lut[b];
                        };
                        if (ok) sp = string_span(f, p, n, lutf);
                        int64_t tot;
                        int64_t ex = wave_excl_scan(sp.utf8_len, lane, &tot);
                        const int64_t seq = a.str_seq_base[f.column] + (int64_t)s * a.n_tiles + tile;
                        if (sizes) {
                            if (lane == 0) a.tile_sums[seq] = tot;
                        } else {
                            int64_t off = a.tile_sums[seq] - a.tile_sums[a.str_seq_base[f.column]] + ex;
                            if (active) {
                                col.offsets[v] = off;
                                if (ok) string_write(f, p, sp, col.data + off, lutf);
                                if (v == (int64_t)f.n_slots * a.n_rec - 1) col.offsets[v + 1] = off + sp.utf8_len;
                            }
                            uint64_t m = __ballot(ok);
                            if (lane == 0) col.validity[(int64_t)s * a.n_tiles + tile] = m;
                        }
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// Fields outside any window: generated Record_Id / File_Id and oversized fields, read from HBM.
__global__ __launch_bounds__(64) void decode_global_kernel(KernelArgs a, const int32_t* gfields, int32_t n_g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* s_lut = (uint32_t*)smem;
    const int lane = threadIdx.x;
    for (int i = lane; i < 256; i += kWave) s_lut[i] = a.lut[i];
    __syncthreads();
    const bool sizes = a.mode == 1;
    for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const int64_t rec = tile * kWave + lane;
        const bool active = rec < a.n_rec;
        int64_t base = a.base_shift;
        int avail = 0;
        if (a.rec_off) {
            if (active) { base += a.rec_off[rec]; avail = a.rec_len[rec]; }
        } else if (active) {
            base += rec * (int64_t)a.stride;
            avail = a.stride;
        }
        const uint8_t* rp = a.data + base;
        int seg = -1;
        if (a.segmap && active) seg = segment_of(a, s_lut, rp, avail);
        for (int gi = 0; gi < n_g; gi++) {
            const Field& f = a.fields[gfields[gi]];
            const DevColumn col = a.cols[f.column];
            if (f.kind == CBX_K_RECORD_ID || f.kind == CBX_K_FILE_ID) {
                if (sizes) continue;
                Val x{f.kind == CBX_K_RECORD_ID ? (uint64_t)(a.first_record_id + rec) : (uint64_t)(int64_t)a.file_id, 0, true};
                if (active) store_value(col, f.out_type, rec, x);
                uint64_t m = __ballot(active);
                if (lane == 0) col.validity[tile] = m;
                continue;
            }
            const bool is_str = f.out_type == CBX_O_STRING || f.out_type == CBX_O_BINARY;
            if (sizes && !is_str) continue;
            for (int s = 0; s < f.n_slots; s++) {
                int eo = f.offset;
                int rem = s;
                bool el = active && (f.segment < 0 || f.segment == seg);
                for (int k = f.n_dims - 1; k >= 0; k--) {
                    int dc = f.dim_count[k];
                    int idx = rem % dc;
                    rem /= dc;
                    eo += idx * f.dim_stride[k];
                    // element counts: recomputed per record (rare path)
                    const cbx_array& ar = a.arrays[f.dim_array[k]];
                    int cnt = ar.max_count;
                    if (ar.dependee >= 0 && active) {
                        const Field& df = a.fields[ar.dependee];
                        int od = a.start_off + df.offset;
                        if ((df.segment < 0 || df.segment == seg) && od + df.size <= avail) {
                            Val dv = decode_numeric(df, rp + od);
                            int32_t dvi = (int32_t)dv.lo;
                            if (dv.valid && dvi >= ar.min_count && dvi <= ar.max_count) cnt = dvi;
                        }
                    }
                    el &= idx < cnt;
                }
                const int o = a.start_off + eo;
                const int64_t v = (int64_t)s * a.n_rec + rec;
                const uint8_t* p = rp + o;
                if (!is_str) {
                    bool ok = el && o + f.size <= avail;
                    Val x = null_val();
                    if (ok) x = decode_numeric(f, p);
                    if (active) store_value(col, f.out_type, v, x);
                    uint64_t m = __ballot(x.valid);
                    if (lane == 0) col.validity[(int64_t)s * a.n_tiles + tile] = m;
                } else {
                    bool ok = el && o <= avail;
                    int n = ok ? (f.size < avail - o ? f.size : avail - o) : 0;
                    StrSpan sp{0, 0, 0};
                    auto lutf = [&](uint32_t b) -> uint32_t {
                        return f.kind == CBX_K_STRING_ASCII ? ascii_lut(b) : s_lut[b];
                    };
                    if (ok) sp = string_span(f, p, n, lutf);
                    int64_t tot;
                    int64_t ex = wave_excl_scan(sp.utf8_len, lane, &tot);
                    const int64_t seq = a.str_seq_base[f.column] + (int64_t)s * a.n_tiles + tile;
                    if (sizes) {
                        if (lane == 0) a.tile_sums[seq] = tot;
                    } else {
                        int64_t off = a.tile_sums[seq] - a.tile_sums[a.str_seq_base[f.column]] + ex;
                        if (active) {
                            col.offsets[v] = off;
                            if (ok) string_write(f, p, sp, col.data + off, lutf);
                            if (v == (int64_t)f.n_slots * a.n_rec - 1) col.offsets[v + 1] = off + sp.utf8_len;
                        }
                        uint64_t m = __ballot(ok);
                        if (lane == 0) col.validity[(int64_t)s * a.n_tiles + tile] = m;
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Exclusive scan of int64 (string tile sums -> tile bases): block reduce / scan of block sums /
// block scan + add.  1024 elements per 256-thread block.
// ------------------------------------------------------------------------------------------
constexpr int kScanBlock = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ int64_t block_excl_scan(int64_t x, int64_t* s_warp, int64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t t;
    int64_t ex = wave_excl_scan(x, lane, &t);
    if (lane == 0) s_warp[wid] = t;
    __syncthreads();
    int64_t pre = 0, all = 0;
    for (int i = 0; i < kScanBlock / 64; i++) {
        if (i < wid) pre += s_warp[i];
        all += s_warp[i];
    }
    __syncthreads();
    *total = all;
    return pre + ex;
}

__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(const int64_t* in, int64_t n, int64_t* block_sums) {
    __shared__ int64_t s_warp[kScanBlock / 64];
    int64_t b0 = (int64_t)blockIdx.x * kScanTile;
    int64_t sum = 0;
    for (int i = 0; i < kScanItems; i++) {
        int64_t idx = b0 + (int64_t)threadIdx.x * kScanItems + i;
        if (idx < n) sum += in[idx];
    }
    int64_t total;
    block_excl_scan(sum, s_warp, &total);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanBlock) void scan_block_sums_kernel(int64_t* block_sums, int64_t nb) {
    __shared__ int64_t s_warp[kScanBlock / 64];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += kScanBlock) {
        int64_t idx = b0 + threadIdx.x;
        int64_t x = idx < nb ? block_sums[idx] : 0;
        int64_t total;
        int64_t ex = block_excl_scan(x, s_warp, &total);
        if (idx < nb) block_sums[idx] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(int64_t* data, int64_t n, const int64_t* block_sums) {
    __shared__ int64_t s_warp[kScanBlock / 64];
    int64_t b0 = (int64_t)blockIdx.x * kScanTile;
    int64_t v[kScanItems];
    int64_t sum = 0;
    for (int i = 0; i < kScanItems; i++) {
        int64_t idx = b0 + (int64_t)threadIdx.x * kScanItems + i;
        v[i] = idx < n ? data[idx] : 0;
        sum += v[i];
    }
    int64_t total;
    int64_t ex = block_excl_scan(sum, s_warp, &total) + block_sums[blockIdx.x];
    for (int i = 0; i < kScanItems; i++) {
        int64_t idx = b0 + (int64_t)threadIdx.x * kScanItems + i;
        if (idx < n) data[idx] = ex;
        ex += v[i];
    }
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
