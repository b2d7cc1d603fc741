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

#include "cbx_device.h"

namespace cbx {

// Interpreter body of the contiguous loop: the plan's windows, read from the tables at run time.
struct InterpBody {
    static constexpr int kWords = 0;   // validity words stored per tile (DirectSink)
    __device__ __forceinline__ void begin(int64_t) {}
    __device__ __forceinline__ void flush(const KernelArgs&, int64_t, int) {}
    __device__ __forceinline__ void post(const KernelArgs&, const TileCtx&, const uint8_t*, uint32_t, const WaveLds&, int,
                                         Stamps&) const {}
    __device__ __forceinline__ void pre(const KernelArgs& a, const TileCtx& t, const uint8_t* img,
                                        uint32_t rec_addr, const WaveLds& l, int lane, Stamps& st) const {
        for (int wi = 0; wi < a.n_windows; wi++) {
            const Window w = ldc(a.windows + wi);
            if (a.mode == 1 && w.sop_begin == w.sop_end) continue;
            if (w.global) {
                decode_generated<false>(a, w, t, lane);   // contig plans: generated columns only
                continue;
            }
#ifdef CBX_STAMPS
            Window ws = w, wn = w;
            ws.batch_begin = ws.batch_end; ws.gen_begin = ws.gen_end;
            wn.sop_begin = wn.sop_end;
            decode_window<false>(a, ws, t, img, rec_addr, l.cnt, l.lut, l.str, lane);
            st.mark(3);   // strings
            decode_window<false>(a, wn, t, img, rec_addr, l.cnt, l.lut, l.str, lane);
            st.mark(4);   // numerics + generated
#else
            decode_window<false>(a, w, t, img, rec_addr, l.cnt, l.lut, l.str, lane);
#endif
        }
    }
};

__global__ __launch_bounds__(kWave * kWavesPerBlock) void decode_kernel(KernelArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // wave-uniform to the compiler
    const int lane = threadIdx.x % kWave;
    const WaveLds l = wave_lds(a, smem, wid);
    for (int i = threadIdx.x; i < 256; i += blockDim.x) l.lut[i] = a.lut[i];
    __syncthreads();

    // static grid-stride tile order (tiles are independent)
    int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    const int64_t tstep = (int64_t)gridDim.x * kWavesPerBlock;

    if (a.contig) {
        contig_loop<kPre, 3, false>(a, l, tile, tstep, lane, InterpBody{});
        return;
    }

    while (tile < a.n_tiles) {
        TileCtx t = tile_ctx(a, tile, lane);
        const uint8_t* rp = a.data + t.base;
        tile_prologue(a, t, rp, lane, l.lut, l.cnt);
        for (int wi = 0; wi < a.n_windows; wi++) {
            const Window w = ldc(a.windows + wi);
            if (a.mode == 1 && w.sop_begin == w.sop_end) continue;
            if (w.global) {
                decode_window<true>(a, w, t, rp, 0u, l.cnt, l.lut, l.str, lane);
                continue;
            }
            const uint32_t rec_addr = stage_window(a, w, t, l.img, lane);
            wave_sync_lds();
            decode_window<false>(a, w, t, (const uint8_t*)l.img, rec_addr, l.cnt, l.lut, l.str, lane);
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

// One wave per (sequence, kPlaceTiles consecutive tiles), 4 waves per workgroup.  The pass is
// bound by load latency per resident wave (each tile is ~1 KiB), so every wave first issues the
// loads of all its tiles -- scanned bases, totals, tile-local starts and the first 20 scratch
// bytes of every lane -- and only then stores: two dependent memory round trips per wave
// instead of two per tile.  The payload moves in 16-byte pieces: each lane reads 5 dwords of
// the (aligned) scratch region and writes 4 realigned dwords at the destination (any
// alignment; byte stores at the unaligned ends).
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
constexpr int kPlaceWaves = 4;
constexpr int kPlaceTiles = 4;

__global__ __launch_bounds__(kWave * kPlaceWaves) void str_place_kernel(const CBX_CONST SeqCall* seqs, const uint32_t* tot,
                                                                         const int64_t* excl, int64_t n_tiles, int64_t n_rec,
                                                                         int32_t n_seq, int32_t* status) {
    const int lane = threadIdx.x % kWave;
    const int64_t tile0 = ((int64_t)blockIdx.x * kPlaceWaves + threadIdx.x / kWave) * kPlaceTiles;
    if (tile0 >= n_tiles) return;
    for (int seq = blockIdx.y; seq < n_seq; seq += gridDim.y) {
        const SeqCall q = ldc(seqs + seq);
        const int64_t* ex = excl + (int64_t)seq * n_tiles;
        const uint32_t* tt = tot + (int64_t)seq * n_tiles;
        const int64_t seq0 = ex[0];
        const bool pre = 16 * lane + 20 <= q.tile_cap;   // this lane's first piece lies in the region
        int64_t base[kPlaceTiles];
        uint32_t n[kPlaceTiles], loc[kPlaceTiles], e0[kPlaceTiles];
        u32x4a v0[kPlaceTiles];
#pragma unroll
        for (int u = 0; u < kPlaceTiles; u++) {
            const int64_t tile = tile0 + u < n_tiles ? tile0 + u : n_tiles - 1;
            base[u] = ex[tile] - seq0;
            n[u] = tt[tile];
            loc[u] = gp(q.local)[tile * kWave + lane];
            const CBX_GLOBAL uint32_t* src = gp((const uint32_t*)(q.scratch + tile * (int64_t)q.tile_cap));
            v0[u] = pre ? *(const CBX_GLOBAL u32x4a*)(src + 4 * lane) : u32x4a{0, 0, 0, 0};
            e0[u] = pre ? src[4 * lane + 4] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kPlaceTiles; u++) {
            const int64_t tile = tile0 + u;
            if (tile >= n_tiles) break;
            const int64_t rec = tile * kWave + lane;
            gp(q.offsets)[rec] = q.region + base[u] + loc[u];   // lanes past n_rec write padding entries
            if (tile == n_tiles - 1 && lane == 0) {
                gp(q.offsets)[n_rec] = q.region + base[u] + n[u];
                if (q.size) *gp(q.size) = base[u] + n[u];
            }
            if (base[u] + (int64_t)n[u] > q.capacity) {
                if (lane == 0) atomicOr(status, 1);
                continue;
            }
            const CBX_GLOBAL uint32_t* src = gp((const uint32_t*)(q.scratch + tile * (int64_t)q.tile_cap));
            const CBX_GLOBAL uint8_t* s8 = (const CBX_GLOBAL uint8_t*)src;
            CBX_GLOBAL uint8_t* dst = gp(q.data + base[u]);
            const uint32_t g0 = (uint32_t)((uint64_t)(q.data + base[u]) & 3);
            const uint32_t head = (4 - g0) & 3;                 // bytes before the first aligned dword
            if (n[u] <= head) {
                if (lane < (int)n[u]) dst[lane] = s8[lane];
                continue;
            }
            const uint32_t ndw = (n[u] - head) >> 2;            // whole destination dwords
            const uint32_t tail = (n[u] - head) & 3;
            if (lane < (int)head) dst[lane] = s8[lane];
            if (lane < (int)tail) dst[head + 4 * ndw + lane] = s8[head + 4 * ndw + lane];
            CBX_GLOBAL uint32_t* d32 = (CBX_GLOBAL uint32_t*)(dst + head);
            const uint32_t sh = head & 3;                       // source byte shift (scratch is 16-aligned)
            for (uint32_t d = 4u * lane; d < ndw; d += 4u * kWave) {
                u32x4a v = v0[u];
                uint32_t e = e0[u];
                if (d != 4u * lane || !pre) {
                    v = *(const CBX_GLOBAL u32x4a*)(src + d);
                    e = src[d + 4];
                }
                const uint32_t w0 = align_bytes(v.y, v.x, sh), w1 = align_bytes(v.z, v.y, sh);
                const uint32_t w2 = align_bytes(v.w, v.z, sh), w3 = align_bytes(e, v.w, sh);
                if (d + 4 <= ndw) {
                    *(CBX_GLOBAL u32x4a*)(d32 + d) = u32x4a{w0, w1, w2, w3};
                } else {
                    d32[d] = w0;
                    if (d + 1 < ndw) d32[d + 1] = w1;
                    if (d + 2 < ndw) d32[d + 2] = w2;
                }
            }
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

// One wave per 64 tiles of a deferral sequence: the wave's deferred values (set bits of its 64
// words, ~0.5 % of the zoned values of SYN200) are enumerated with a wave scan and spread over
// the lanes one value each, so a word with many deferrals does not serialise its wave.
__global__ __launch_bounds__(256) void fixup_kernel(KernelArgs a, const CBX_CONST DeferSeq* dseq, int32_t n_defer) {
    const int lane = threadIdx.x % kWave;
    const int64_t tile = ((int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave) * kWave + lane;
    for (int d = blockIdx.y; d < n_defer; d += gridDim.y) {
        const uint64_t bits = tile < a.n_tiles ? a.defer_bits[(int64_t)d * a.n_tiles + tile] : 0ull;
        uint32_t total;
        const uint32_t ex = wave_excl_scan32((uint32_t)__popcll(bits), lane, total);
        if (total == 0) continue;
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
        for (uint32_t j = lane; j < total + (kWave - 1) - ((total + kWave - 1) % kWave); j += kWave) {
            // owner lane: the last lane whose exclusive prefix is <= j (binary search over the wave)
            int lo = 0;
#pragma unroll
            for (int step = kWave / 2; step >= 1; step >>= 1) {
                const uint32_t e = (uint32_t)__shfl((int)ex, lo + step, kWave);
                if (e <= j) lo += step;
            }
            // every lane takes part in the shuffles (a shuffle from an inactive lane reads 0)
            const uint64_t wb = __shfl(bits, lo, kWave);
            const int64_t wt = __shfl(tile, lo, kWave);
            const uint32_t we = (uint32_t)__shfl((int)ex, lo, kWave);
            if (j >= total) continue;
            uint64_t m = wb;
            for (uint32_t r = j - we; r > 0; r--) m &= m - 1;   // r-th set bit of the owner's word
            const int b = __builtin_ctzll(m);
            const int64_t rec = wt * kWave + b;
            const int64_t base = a.base_shift + (a.rec_off ? a.rec_off[rec] : rec * (int64_t)a.stride);
            const Val x = decode_numeric(f, a.data + base + a.start_off + eo);
            store_value(col, f.out_type, (int64_t)ds.slot * a.pitch + rec, x);
            if (x.valid) atomicOr((unsigned long long*)(col.validity + (int64_t)ds.slot * a.n_tiles + wt), 1ull << b);
        }
    }
}

// ------------------------------------------------------------------------------------------
// List layout (CBX_F_LIST): the child elements of OCCURS DEPENDING ON arrays, element-parallel.
// The decode kernel's prologue left every record's present element count (list_len) and its
// child start (offsets column, a multiple of 64).  One wave per tile of 64 records takes the
// tile's records with elements one at a time and their elements 64 per step, lane = element:
// the value stores are one contiguous run and a step's validity exactly one bitmap word.
// Element bytes: arrays whose 64 elements fit the staging area are staged a group of steps at a
// time with 16-byte loads (1 KiB per wave instruction) and read from LDS; wider elements are read
// per lane with dword loads.  The record's bytes are read through a buffer descriptor bounded by
// the record, so bytes past it read as zeros (elements past the record's end are null, as
// extractArray's bounds check makes them).  Reference: the OCCURS loop of
// RecordExtractors.extractRecord (RecordExtractors.scala:66-114) with the element decoders.
// ------------------------------------------------------------------------------------------
constexpr int kListWaves = 4;      // waves per workgroup
constexpr int kListStage = 4096;   // LDS staging bytes per wave (staged: elements of up to 63 bytes)
constexpr int kListKP = kListStage / (16 * kWave);   // 16-byte loads per lane per group

// Dword at byte offset o of the record's descriptor; offsets before the record read as zero.
__device__ __forceinline__ uint32_t list_dword(__amdgpu_buffer_rsrc_t rs, int o) {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, o < 0 ? 0x7ffffff0 : o, 0, 0);
}

// bytes [end - 8, end) of the descriptor as a little-endian u64 (cf. img_le64_ending)
__device__ __forceinline__ uint64_t list_le64_ending(__amdgpu_buffer_rsrc_t rs, int end) {
    const int s = end - 8;
    const int a0 = s & ~3;
    const uint32_t sh = (uint32_t)s & 3u;
    const uint32_t d0 = list_dword(rs, a0), d1 = list_dword(rs, a0 + 4), d2 = list_dword(rs, a0 + 8);
    return ((uint64_t)align_bytes(d2, d1, sh) << 32) | align_bytes(d1, d0, sh);
}

// Decode + store element k of a record (its step starts at element c0) for one field.
// r1 / r0: the 8 (and 8 more) bytes ending at the element's end.
// kFix = false: the fast decoders; lanes that need the byte loops (wide fields, zoned forms the
// fast path defers, an element ending in the input's last partial dword) only raise `deferred`.
// kFix = true (the second pass, over tiles that raised it): exactly those items again, byte loops
// for the deferred lanes (the byte-loop decoders use scratch: they stay out of the first pass).
// V >= 0: the fast decoder of variant V; V < 0: the variant read from the op (the byte-loop pass).
// clean (wave-uniform): every present element of the step ends inside the record and before rsafe.
// Every lane stores: lanes past the record's count write the padding of its 64-aligned run.
template <int V, bool kFix>
__device__ __forceinline__ void list_item(const KernelArgs& a, const ListOp& L, const DevColumn& col, int k, int c0,
                                          int rlen, int ravail, int rsafe, bool clean, int64_t rbase, int64_t rstart,
                                          uint64_t r1, uint64_t r0, bool& deferred) {
    const NumOp& op = L.op;
    const int v = V >= 0 ? V : op.variant;
    const int eo = a.start_off + op.eo + k * L.stride;
    const bool present = k < rlen;
    const bool ok = present && (clean || eo + op.size <= ravail);
    Val x = null_val();
    bool slow = v == V_GENERIC;
    if (v == V_BCD8) x = bcd8_raw<0>(op, r1);
    else if (v == V_BCD16) x = bcd16_raw<0>(op, r1, r0);
    else if (v == V_BIN8) x = bin8_raw<0>(op, r1);
    else if (v == V_ZONED16) x = zoned16_raw<0>(op, r1, r0, slow);
    else if (v == V_FP) x = fp_raw(op, r1);
    if (kFix || !clean || v == V_ZONED16 || v == V_GENERIC) {
        slow = (slow || eo + op.size > rsafe) && ok;   // (or ends in the input's last, partial dword)
        const uint64_t sm = __ballot(slow);
        if (!kFix) {
            deferred |= sm != 0;
            x.valid &= !slow;
        } else {
            if (sm == 0) return;
            if (slow) x = decode_numeric(ldc(a.fields + L.field), a.data + rbase + eo);
        }
    }
    x.valid &= ok;
    store_value(col, op.out_type, rstart + k, x);
    const uint64_t vm = __ballot(x.valid);
    gp(col.validity)[(rstart + c0) >> 6] = vm;
}

constexpr int kListSteps = 4;   // element steps per round: reads first

// One field over a group of element steps g0 .. g0+gn-1 of a record.  kStaged: the group's bytes are
// in img (rel: the field's end in element 0 of the group, from img - kGuard); else read per lane
// from the record's descriptor (rel: from the descriptor base).
template <int V, bool kStaged, bool kFix = false>
__device__ __forceinline__ void list_field(const KernelArgs& a, const ListOp& L, const DevColumn& col, const uint8_t* img,
                                           __amdgpu_buffer_rsrc_t rs, int rel, int g0, int gn, int rlen, int ravail,
                                           int rsafe, int64_t rbase, int64_t rstart, int lane, bool& deferred) {
    const bool kWide = V >= 0 ? (V == V_BCD16 || V == V_ZONED16) : (L.op.variant == V_BCD16 || L.op.variant == V_ZONED16);
    const int step_bytes = kWave * L.stride;
    const int mine = rel + lane * L.stride;
    // the group's last present element of this field ends inside the record, before rsafe
    const int kmax = ((g0 + gn) * kWave < rlen ? (g0 + gn) * kWave : rlen) - 1;
    const bool clean = a.start_off + L.op.eo + L.op.size + kmax * L.stride <= (ravail < rsafe ? ravail : rsafe);
    if (kFix) {   // byte-loop pass: one step at a time (its decoders are large)
        for (int st = 0; st < gn; st++) {
            const int end = mine + st * step_bytes;
            uint64_t r1, r0 = 0;
            if (kStaged) {
                r1 = img_le64_ending(img - kGuard, (uint32_t)end);
                if (kWide) r0 = img_le64_ending(img - kGuard, (uint32_t)end - 8);
            } else {
                r1 = list_le64_ending(rs, end);
                if (kWide) r0 = list_le64_ending(rs, end - 8);
            }
            const int c0 = (g0 + st) * kWave;
            list_item<-1, true>(a, L, col, c0 + lane, c0, rlen, ravail, rsafe, clean, rbase, rstart, r1, r0, deferred);
        }
        return;
    }
    for (int st0 = 0; st0 < gn; st0 += kListSteps) {
        uint64_t r1[kListSteps], r0[kListSteps];
#pragma unroll
        for (int u = 0; u < kListSteps; u++) {
            const int st = st0 + u < gn ? st0 + u : gn - 1;   // (a repeat is not decoded)
            const int end = mine + st * step_bytes;
            r0[u] = 0;
            if (V == V_GENERIC) { r1[u] = 0; continue; }
            if (kStaged) {
                r1[u] = img_le64_ending(img - kGuard, (uint32_t)end);
                if (kWide) r0[u] = img_le64_ending(img - kGuard, (uint32_t)end - 8);
            } else {
                r1[u] = list_le64_ending(rs, end);
                if (kWide) r0[u] = list_le64_ending(rs, end - 8);
            }
        }
#pragma unroll
        for (int u = 0; u < kListSteps; u++) {
            if (st0 + u >= gn) break;
            const int c0 = (g0 + st0 + u) * kWave;
            list_item<V, false>(a, L, col, c0 + lane, c0, rlen, ravail, rsafe, clean, rbase, rstart, r1[u], r0[u], deferred);
        }
    }
}

template <bool kStaged, bool kFix>
__device__ __forceinline__ void list_field_v(const KernelArgs& a, const ListOp& L, const DevColumn& col, const uint8_t* img,
                                             __amdgpu_buffer_rsrc_t rs, int rel, int g0, int gn, int rlen, int ravail,
                                             int rsafe, int64_t rbase, int64_t rstart, int lane, bool& deferred) {
#define CBX_LIST_V(VV) list_field<VV, kStaged>(a, L, col, img, rs, rel, g0, gn, rlen, ravail, rsafe, rbase, rstart, lane, deferred)
    if (kFix) {
        list_field<-1, kStaged, true>(a, L, col, img, rs, rel, g0, gn, rlen, ravail, rsafe, rbase, rstart, lane, deferred);
        return;
    }
    switch (L.op.variant) {
    case V_BCD8: CBX_LIST_V(V_BCD8); break;
    case V_BCD16: CBX_LIST_V(V_BCD16); break;
    case V_BIN8: CBX_LIST_V(V_BIN8); break;
    case V_ZONED16: CBX_LIST_V(V_ZONED16); break;
    case V_FP: CBX_LIST_V(V_FP); break;
    default: CBX_LIST_V(V_GENERIC); break;
    }
#undef CBX_LIST_V
}

// A record with list elements (wave-uniform): its count, child start, byte offset and length, and
// a buffer descriptor over its bytes from a 16-byte aligned base, rounded up to whole dwords (the
// range check drops a dword that crosses it) within the input: elements ending past rsafe (only
// in a last, partial dword of the input) take the byte-loop pass.
struct ListRec {
    int rlen, ravail, rsafe, bias;
    int64_t rstart, rbase;
    __amdgpu_buffer_rsrc_t rs;
};

__device__ __forceinline__ ListRec list_rec(const KernelArgs& a, int b, int len, int64_t start, int64_t base, int avail) {
    ListRec r;
    r.rlen = __builtin_amdgcn_readlane(len, b);
    r.rstart = ((int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(start >> 32), b) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)start, b);
    r.rbase = ((int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(base >> 32), b) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)base, b);
    r.ravail = __builtin_amdgcn_readlane(avail, b);
    const uint64_t addr = (uint64_t)(a.data + r.rbase);
    r.bias = (int)(addr & 15);
    const int64_t in_left = (a.data_len - r.rbase + r.bias) & ~(int64_t)3;
    const int64_t want = ((int64_t)r.ravail + r.bias + 3) & ~(int64_t)3;
    const int range = (int)(want < in_left ? want : in_left);
    r.rsafe = range - r.bias;
    r.rs = __builtin_amdgcn_make_buffer_rsrc((void*)(addr - r.bias), (short)0, range, 0x00020000);
    return r;
}

// 16-byte chunks of group g0 of record r (its elements' bytes from the array's first field byte)
__device__ __forceinline__ int list_n16(const ListRec& r, int s0, int s16, int g0, int gsteps, int stride) {
    const int left = r.rlen - g0 * kWave;
    const int ne = left < gsteps * kWave ? left : gsteps * kWave;
    return (s0 - s16 + ne * stride + 15) >> 4;
}

// Issue the staging loads of group g0 of record r (chunks past the group: no access).
__device__ __forceinline__ void list_issue(const KernelArgs& a, const ListRec& r, int elo, int stride, int g0, int gsteps,
                                           int lane, uint4 (&v)[kListKP]) {
    const int s0 = r.bias + a.start_off + elo + g0 * kWave * stride;
    const int s16 = s0 & ~15;
    const int n16 = list_n16(r, s0, s16, g0, gsteps, stride);
#pragma unroll
    for (int u = 0; u < kListKP; u++) {
        const int c = u * kWave + lane;
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(r.rs, c < n16 ? s16 + 16 * c : 0x7ffffff0, 0, 0);
        v[u] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

template <bool kFix>
__global__ __launch_bounds__(kWave * kListWaves) void list_kernel(KernelArgs a, const CBX_CONST ListOp* lops, int32_t n_lops) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x % kWave;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint8_t* img = smem + wid * (kGuard + kListStage + kGuard) + kGuard;
    const int64_t nw = (int64_t)gridDim.x * kListWaves;
    for (int64_t tile = (int64_t)blockIdx.x * kListWaves + wid; tile < a.n_tiles; tile += nw) {
        if (kFix && a.list_flag[tile] == 0) continue;
        bool deferred = false;
        const int64_t rec = tile * kWave + lane;
        const bool active = rec < a.n_rec;
        int64_t base = a.base_shift;
        int avail = 0;
        if (active) {
            if (a.rec_off) { base += a.rec_off[rec]; avail = a.rec_len[rec]; }
            else { base += rec * (int64_t)a.stride; avail = a.stride; }
        }
        for (int i0 = 0; i0 < n_lops;) {
            const int ai = lops[i0].array;
            int i1 = i0 + 1;
            while (i1 < n_lops && lops[i1].array == ai) i1++;
            const int nops = i1 - i0;
            const int stride = lops[i0].stride;
            const int elo = lops[i0].elem_lo;             // the array's first byte in an element
            // a staged group of element steps plus up to 15 bytes of alignment fits kListStage
            const bool staged = kWave * stride <= kListStage - 16;
            const int gsteps = staged ? (kListStage - 16) / (kWave * stride) : 1;
            const DevColumn oc = ldc(a.cols + a.arrays[ai].offsets_column);
            const int len = active ? a.list_len[(int64_t)ai * a.pitch + rec] : 0;
            const int64_t start = active ? ((const int64_t*)oc.values)[rec] : 0;
            uint64_t m = __ballot(len > 0);
            if (m == 0) { i0 = i1; continue; }
            // the tile's records with elements, a staged group at a time; the loads of the next
            // group (of this record or the next one) are issued before the current group is decoded
            ListRec cur = list_rec(a, __builtin_ctzll(m), len, start, base, avail);
            m &= m - 1;
            int g0 = 0;
            uint4 v[kListKP];
            if (staged) list_issue(a, cur, elo, stride, g0, gsteps, lane, v);
            for (;;) {
                const int nsteps = (cur.rlen + kWave - 1) / kWave;
                const int gn = nsteps - g0 < gsteps ? nsteps - g0 : gsteps;
                const int s0 = cur.bias + a.start_off + elo + g0 * kWave * stride;
                const int s16 = s0 & ~15;
                ListRec nxt = cur;
                int ng0 = g0 + gsteps;
                bool more = true;
                if (ng0 >= nsteps) {
                    if (m) { nxt = list_rec(a, __builtin_ctzll(m), len, start, base, avail); m &= m - 1; ng0 = 0; }
                    else more = false;
                }
                if (staged) {
                    const int n16 = list_n16(cur, s0, s16, g0, gsteps, stride);
#pragma unroll
                    for (int u = 0; u < kListKP; u++)
                        if (u * kWave + lane < n16) *(uint4*)(img + 16 * (u * kWave + lane)) = v[u];
                    wave_sync_lds();
                    if (more) list_issue(a, nxt, elo, stride, ng0, gsteps, lane, v);
                }
                // field by field (its descriptor loaded once per group), the group's steps
                for (int i = i0; i < i1; i++) {
                    const ListOp L = ldc(lops + i);
                    const DevColumn col = ldc(a.cols + L.op.column);
                    const int rel = L.op.eo - elo + L.op.size;
                    if (staged)
                        list_field_v<true, kFix>(a, L, col, img, cur.rs, kGuard + s0 - s16 + rel, g0, gn, cur.rlen, cur.ravail,
                                                 cur.rsafe, cur.rbase, cur.rstart, lane, deferred);
                    else
                        list_field_v<false, kFix>(a, L, col, img, cur.rs, s0 + rel, g0, gn, cur.rlen, cur.ravail, cur.rsafe,
                                                  cur.rbase, cur.rstart, lane, deferred);
                }
                if (staged) wave_sync_lds();
                if (!more) break;
                cur = nxt;
                g0 = ng0;
            }
            i0 = i1;
        }
        if (!kFix) gp(a.list_flag)[tile] = deferred ? 1 : 0;
    }
}

// ------------------------------------------------------------------------------------------
// RDW framing (RecordHeaderParserRDW.getRecordMetadata + VRLRecordReader.fetchRecordUsingRdwHeaders)
// One lane per chunk of a seed range walks its header chain; the walk stages the records it finds
// in a per-chunk region, and one placement pass moves them to their final positions.
// ------------------------------------------------------------------------------------------
struct RdwArgs {
    const uint8_t* data;
    int64_t n_bytes;
    cbx_rdw_params p;
};

// Header walk step (RecordHeaderParserRDW.getRecordMetadata + VRLRecordReader.fetchRecordUsingRdwHeaders):
// the header at pos gives the next header position, the payload (off, len) and whether the
// record is valid (file header / footer records are not).  err: -2 length <= 0, -3 > 100 MiB.
struct RdwStep {
    int64_t next, off;
    int32_t len;
    bool valid, stop;
    int32_t err;
};

__device__ __forceinline__ uint32_t rdw_header(const RdwArgs& a, int64_t pos) {
    // 4 bytes at any alignment (caller guarantees pos + 4 <= n_bytes): the two dwords around them
    // (two loads per header instead of four byte loads -- the walks' lanes hit 64 different lines
    // per instruction), byte loads only where the second dword would pass the end of the input
    // (dwords aligned in memory: the one holding data[pos] starts at most 3 bytes before it, in the
    // same page as the input's first byte when pos < 4)
    const uintptr_t u = (uintptr_t)(a.data + pos);
    const uint32_t* q = (const uint32_t*)(u & ~(uintptr_t)3);
    if ((const uint8_t*)q + 8 <= a.data + a.n_bytes) return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(u & 3));
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) w |= (uint32_t)a.data[pos + j] << (8 * j);
    return w;
}

__device__ __forceinline__ int64_t rdw_len(const RdwArgs& a, uint32_t h) {
    const uint32_t b0 = h & 0xFF, b1 = (h >> 8) & 0xFF, b2 = (h >> 16) & 0xFF, b3 = h >> 24;
    return (a.p.big_endian ? (int64_t)b1 + 256 * (int64_t)b0 : (int64_t)b2 + 256 * (int64_t)b3) + a.p.adjustment;
}

__device__ __forceinline__ RdwStep rdw_step(const RdwArgs& a, int64_t pos) {
    RdwStep s{0, 0, 0, false, false, 0};
    const int64_t avail = a.n_bytes - pos;
    const int64_t hl = avail < 4 ? avail : 4;
    const int64_t fo = pos + hl;   // file offset after the header
    int64_t rlen;
    if (a.p.file_header_bytes > 4 && fo == 4) {
        rlen = a.p.file_header_bytes - 4;
    } else if (a.n_bytes > 0 && a.p.file_footer_bytes > 0 && a.n_bytes - fo <= a.p.file_footer_bytes) {
        rlen = a.n_bytes - fo;
    } else if (hl < 4) {
        s.stop = true;
        s.next = a.n_bytes;
        return s;
    } else {
        rlen = rdw_len(a, rdw_header(a, pos));
        if (rlen <= 0) { s.err = -2; return s; }
        if (rlen > 100ll * 1024 * 1024) { s.err = -3; return s; }
        s.valid = true;
    }
    if (rlen <= 0) { s.stop = true; s.next = a.n_bytes; return s; }
    const int64_t rem = a.n_bytes - fo;
    const int64_t got = rlen < rem ? rlen : rem;
    s.off = fo;
    s.len = (int32_t)got;
    s.next = fo + got;
    return s;
}

// Chunk-parallel RDW offset discovery.  The byte range of every sparse-
// index seed is cut into chunks; a chunk holds the records whose header starts in
// [start, end).  Every chunk walks from a speculated entry (a plausible header chain near its
// start; the seed itself for a range's first chunk) to its exit (first header position >= end);
// then rounds of the fix kernel replace each entry with the predecessor's exit and re-walk the
// chunks that change, until no chunk changes: by induction from the seeds the entries are then
// exactly the sequential walk's header positions.  Every walk stages (offset, length) of the
// valid records it finds in its chunk's region of a staging area (up to `stage_cap` records, in
// 64-byte pieces: a lane buffers 8 records in registers, so its stores are whole segments instead
// of 8-byte scatters); after a device scan of the counts, the placement kernel copies each
// chunk's records to its base with coalesced wave loads / stores (a chunk with more records than
// its region holds is walked again and written directly).  The data is walked once per
// speculation round; in the common case (every speculated entry right) exactly once.
struct RdwRange {
    int64_t r0, r1;          // seed range [r0, r1)
    int64_t first;           // index of its first chunk
};

struct RdwChunkArgs {
    const RdwRange* ranges;  // chunk k of range i: [r0 + (k - first) * chunk, min(.. + chunk, r1))
    int32_t n_ranges;
    int64_t chunk;
    int64_t* entry;
    int64_t* exit_in;
    int64_t* exit_out;
    uint32_t* count;         // valid records from the current entry
    int64_t* err;            // per chunk: (error position << 2 | code) or -1
    int32_t* changed;
    int64_t n;
    int64_t* stage_off;      // chunk k's records: [k * stage_cap, k * stage_cap + min(count, stage_cap))
    int32_t* stage_len;
    int64_t stage_cap;       // a multiple of 8
};

struct RdwWalk {
    int64_t exit;            // first header position >= end; -2 after an error (dead chain)
    uint32_t count;
    int64_t err;
};

// kMode 0: count; 1: stage the records at rec_off/rec_len[0, cap) (cap a multiple of 8; records
// past cap are counted, not kept); 2: write them at rec_off/rec_len[out ..) below cap.
template <int kMode>
__device__ RdwWalk rdw_walk(const RdwArgs& a, int64_t pos, int64_t end, int64_t* rec_off, int32_t* rec_len,
                            int64_t out, int64_t cap) {
    RdwWalk w{pos, 0, -1};
    if (pos < 0) { w.exit = pos; return w; }
    int64_t bo[8];
    int32_t bl[8];
    while (pos < end) {
        const RdwStep s = rdw_step(a, pos);
        if (s.err) {
            w.err = ((pos + 4) << 2) | (s.err == -2 ? 2 : 3);   // reported at the payload offset
            w.exit = -2;
            return w;
        }
        if (s.stop) { pos = s.next; break; }
        if (s.valid) {
            if (kMode == 2 && out < cap) { rec_off[out] = s.off; rec_len[out] = s.len; }
            if (kMode == 1) {
                const uint32_t slot = w.count & 7u;
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if ((uint32_t)j == slot) { bo[j] = s.off; bl[j] = s.len; }
                if (slot == 7u && (int64_t)w.count < cap) {   // 8 records: 64 + 32 contiguous bytes
                    int64_t* d = rec_off + (w.count - 7);
                    int32_t* e = rec_len + (w.count - 7);
#pragma unroll
                    for (int j = 0; j < 8; j += 2) *(int4*)(d + j) = make_int4((int)bo[j], (int)(bo[j] >> 32), (int)bo[j + 1], (int)(bo[j + 1] >> 32));
                    *(int4*)e = make_int4(bl[0], bl[1], bl[2], bl[3]);
                    *(int4*)(e + 4) = make_int4(bl[4], bl[5], bl[6], bl[7]);
                }
            }
            out++;
            w.count++;
        }
        pos = s.next;
    }
    if (kMode == 1) {   // the last partial group
        const uint32_t done = w.count & ~7u;
#pragma unroll
        for (int j = 0; j < 7; j++)
            if ((uint32_t)j < (w.count & 7u) && (int64_t)(done + j) < cap) { rec_off[done + j] = bo[j]; rec_len[done + j] = bl[j]; }
    }
    w.exit = pos;
    return w;
}

// A plausible header chain starting at q: kHops headers with lengths in (0, 100 MiB] inside the
// range (strict: the two bytes that do not carry the length are zero, as RDWs write them).
__device__ __forceinline__ bool rdw_plausible(const RdwArgs& a, int64_t q, int64_t range_end, bool strict) {
    constexpr int kHops = 4;
    int64_t pos = q;
    for (int k = 0; k < kHops; k++) {
        if (pos >= range_end || pos + 4 > a.n_bytes) return k > 0;
        const uint32_t h = rdw_header(a, pos);
        const int64_t len = rdw_len(a, h);
        if (len <= 0 || len > 100ll * 1024 * 1024) return false;
        if (strict && (a.p.big_endian ? (h >> 16) : (h & 0xFFFF)) != 0) return false;
        pos += 4 + len;
    }
    return true;
}

struct RdwChunk {
    int64_t start, end, range_end;
    bool known;              // the entry is a seed (a range's first chunk)
};

__device__ __forceinline__ RdwChunk rdw_chunk(const RdwChunkArgs& c, int64_t k) {
    int lo = 0, hi = c.n_ranges - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (c.ranges[mid].first <= k) lo = mid; else hi = mid - 1;
    }
    const RdwRange r = c.ranges[lo];
    RdwChunk ch;
    ch.start = r.r0 + (k - r.first) * c.chunk;
    ch.end = ch.start + c.chunk < r.r1 ? ch.start + c.chunk : r.r1;
    ch.range_end = r.r1;
    ch.known = k == r.first;
    return ch;
}

// First q in [s, e) that starts a strictly plausible chain.  A strict header has two zero bytes
// (LE: bytes 0-1, BE: bytes 2-3), so only zero-byte pairs are candidates: the chunk is scanned
// a dword at a time with an exact zero-byte mask, and the chain test runs on candidates only.
__device__ __forceinline__ uint32_t zero_bytes4(uint32_t x) {   // bit j: byte j of x is zero
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// ---- the walk as one wave per chunk, headers read from an LDS ring (rdw_wave_kernel) ----
// The lane-per-chunk walk above makes every header a dependent HBM load in a line no other lane
// touches; with ~2,300 waves for 150 k chunks (C4) it is latency-bound (SQ_WAIT_ANY 83 % of its
// wave cycles, profiles/r03_a).  Here a wave owns a chunk: the chunk's bytes stream through a
// 4-window LDS ring (1 KiB windows, one 16-byte buffer load per lane, two windows in flight), the
// header chain is walked wave-uniformly from LDS, and the wave's 64 lanes hold the last 64 records
// found so the staging stores are whole 512 + 256-byte rows.  A walk whose next header lies past the
// windows in flight (records longer than a window, C5) restarts the stream at that header.  The
// speculated entry of a chunk (no seed) is the first strict candidate that starts a plausible chain:
// the lanes test the zero-byte pairs of a window in parallel and the lowest plausible one wins.
// Fix rounds walk in place: a chunk whose entry differs from its predecessor's exit re-walks; a
// round that changed nothing ends the loop (device flag per round, checked by the next round's
// kernel, so rounds are launched without waiting for the host).
constexpr int kRdwWin = 1024;                  // window bytes: one 16-byte load per lane
constexpr int kRdwRingWins = 4;                // windows resident in the wave's ring
constexpr int kRdwRing = kRdwWin * kRdwRingWins;
constexpr int kRdwWaveLds = kRdwRing + 16;     // + a copy of the ring's first 16 bytes (reads across its end)
constexpr int kRdwWaves = 4;                   // waves per workgroup

struct RdwStream {
    const uint8_t* base;   // 16-byte aligned address at or before data
    int64_t shift;         // data - base
    int64_t limit;         // input bytes from base (shift + n_bytes)
    uint8_t* ring;         // the wave's LDS ring
    int64_t hi;            // next window (index from base) to enter the ring
    uint4 nx0, nx1;        // windows hi, hi + 1 in flight
};

__device__ __forceinline__ uint4 rdw_win_load(const RdwStream& s, int64_t win, int lane) {
    const int64_t a0 = win * kRdwWin;
    int64_t left = s.limit - a0;
    left = left < 0 ? 0 : (left > kRdwWin ? kRdwWin : left);
    const uint64_t b = (uint64_t)(s.base + (a0 < s.limit ? a0 : 0));
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane((int)left);
    void* bp = (void*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(bp, (short)0, nbytes, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 0, 0);   // past the input: zeros
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void rdw_win_put(RdwStream& s, int64_t win, uint4 v, int lane) {
    const int slot = (int)(win & (kRdwRingWins - 1));
    *(uint4*)(s.ring + slot * kRdwWin + 16 * lane) = v;
    if (slot == 0 && lane == 0) *(uint4*)(s.ring + kRdwRing) = v;
}

__device__ __forceinline__ void rdw_stream_start(RdwStream& s, int64_t win, int lane) {
    s.hi = win;
    s.nx0 = rdw_win_load(s, win, lane);
    s.nx1 = rdw_win_load(s, win + 1, lane);
}

// Bring the windows holding [pos, pos + 4) into the ring (pos: wave-uniform, relative to data).
__device__ __forceinline__ void rdw_stream_need(RdwStream& s, int64_t pos, int lane) {
    const int64_t w0 = (s.shift + pos) >> 10, w1 = (s.shift + pos + 3) >> 10;
    if (w1 < s.hi) return;
    if (w0 > s.hi + 1) rdw_stream_start(s, w0, lane);   // a jump past the windows in flight
    while (w1 >= s.hi) {
        rdw_win_put(s, s.hi, s.nx0, lane);
        s.nx0 = s.nx1;
        s.hi++;
        s.nx1 = rdw_win_load(s, s.hi + 1, lane);
    }
    wave_sync_lds();
}

// The 4 header bytes at pos (in the ring).
__device__ __forceinline__ uint32_t rdw_ring_header(const RdwStream& s, int64_t pos) {
    const uint32_t o = (uint32_t)((s.shift + pos) & (kRdwRing - 1));
    const uint32_t* q = (const uint32_t*)(s.ring + (o & ~3u));
    return __builtin_amdgcn_alignbyte(q[1], q[0], o & 3u);
}

// rdw_step with the header read from the ring (RecordHeaderParserRDW.getRecordMetadata + the
// reader's next-record arithmetic)
__device__ __forceinline__ RdwStep rdw_step_ring(const RdwArgs& a, RdwStream& s, int64_t pos, int lane) {
    RdwStep r{0, 0, 0, false, false, 0};
    const int64_t avail = a.n_bytes - pos;
    const int64_t hl = avail < 4 ? avail : 4;
    const int64_t fo = pos + hl;
    int64_t rlen;
    if (a.p.file_header_bytes > 4 && fo == 4) {
        rlen = a.p.file_header_bytes - 4;
    } else if (a.n_bytes > 0 && a.p.file_footer_bytes > 0 && a.n_bytes - fo <= a.p.file_footer_bytes) {
        rlen = a.n_bytes - fo;
    } else if (hl < 4) {
        r.stop = true;
        r.next = a.n_bytes;
        return r;
    } else {
        rdw_stream_need(s, pos, lane);
        rlen = rdw_len(a, rdw_ring_header(s, pos));
        if (rlen <= 0) { r.err = -2; return r; }
        if (rlen > 100ll * 1024 * 1024) { r.err = -3; return r; }
        r.valid = true;
    }
    if (rlen <= 0) { r.stop = true; r.next = a.n_bytes; return r; }
    const int64_t rem = a.n_bytes - fo;
    const int64_t got = rlen < rem ? rlen : rem;
    r.off = fo;
    r.len = (int32_t)got;
    r.next = fo + got;
    return r;
}

// The chain from pos to the first header at or past end, staging (offset, length) of the valid
// records at so / sl [0, cap) in rows of 64 (records past cap are counted, not kept).
__device__ RdwWalk rdw_walk_wave(const RdwArgs& a, RdwStream& s, int64_t pos, int64_t end, int64_t* so, int32_t* sl,
                                 int64_t cap, int lane) {
    RdwWalk w{pos, 0, -1};
    if (pos < 0) { w.exit = pos; return w; }
    if (pos < end) rdw_stream_start(s, (s.shift + pos) >> 10, lane);
    int64_t my_off = 0;
    int32_t my_len = 0;
    uint32_t count = 0;
    while (pos < end) {
        const RdwStep st = rdw_step_ring(a, s, pos, lane);
        if (st.err) {
            w.err = ((pos + 4) << 2) | (st.err == -2 ? 2 : 3);   // reported at the payload offset
            w.exit = -2;
            w.count = count;
            return w;
        }
        if (st.stop) { pos = st.next; break; }
        if (st.valid) {
            if ((uint32_t)lane == (count & 63u)) { my_off = st.off; my_len = st.len; }
            count++;
            if ((count & 63u) == 0 && (int64_t)count <= cap) {
                so[count - 64 + lane] = my_off;
                sl[count - 64 + lane] = my_len;
            }
        }
        pos = st.next;
    }
    const uint32_t done = count & ~63u;
    if ((uint32_t)lane < (count & 63u) && (int64_t)(done + lane) < cap) {
        so[done + lane] = my_off;
        sl[done + lane] = my_len;
    }
    w.exit = pos;
    w.count = count;
    return w;
}

// Speculated entry of a chunk [s0, e) of a range ending at re: the first strict candidate (the two
// non-length header bytes zero) starting a plausible chain, else the first position starting a
// plausible chain at all (the chunk's start when none: the fix rounds correct it).
__device__ int64_t rdw_entry_wave(const RdwArgs& a, RdwStream& s, int64_t s0, int64_t e, int64_t re, int lane) {
    const int64_t off = a.p.big_endian ? 2 : 0;   // position of the zero pair inside a header
    for (int64_t w = (s.shift + s0 + off) >> 10; ; w++) {
        const int64_t wa = w * kRdwWin - s.shift;   // window start relative to data
        if (wa >= e + off || wa >= a.n_bytes) break;
        // the lane's 16 bytes + the next one (from the following lane's slice, or the next window)
        const uint4 v = rdw_win_load(s, w, lane);
        const uint32_t nb_in = __shfl_down(v.x, 1, kWave) & 0xFFu;
        uint32_t next_byte = nb_in;
        if (lane == kWave - 1) {
            const int64_t q = wa + kRdwWin;
            next_byte = q < a.n_bytes ? a.data[q] : 1u;
        }
        const uint32_t zb = zero_bytes4(v.x) | zero_bytes4(v.y) << 4 | zero_bytes4(v.z) << 8 | zero_bytes4(v.w) << 12 |
                            (next_byte == 0 ? 1u << 16 : 0u);
        uint32_t pairs = zb & (zb >> 1) & 0xFFFFu;   // bit i: bytes i, i + 1 of the slice are zero
        int64_t found = -1;
        while (pairs) {
            const int i = __builtin_ctz(pairs);
            pairs &= pairs - 1;
            const int64_t p = wa + 16 * lane + i;   // pair position (relative to data)
            const int64_t q = p - off;              // header position
            if (p < s0 + off || q >= e || p < 0) continue;
            if (rdw_plausible(a, q, re, true)) { found = q; break; }
        }
        const uint64_t m = __ballot(found >= 0);
        if (m) return __shfl(found, __builtin_ctzll(m), kWave);
    }
    // no strict candidate: any plausible chain (lanes over consecutive positions)
    for (int64_t p0 = s0; p0 < e; p0 += kWave) {
        const int64_t p = p0 + lane;
        const bool ok = p < e && rdw_plausible(a, p, re, false);
        const uint64_t m = __ballot(ok);
        if (m) return p0 + __builtin_ctzll(m);
    }
    return s0;
}

__device__ __forceinline__ RdwStream rdw_stream(const RdwArgs& a, uint8_t* ring) {
    RdwStream s;
    const uintptr_t d = (uintptr_t)a.data;
    s.base = (const uint8_t*)(d & ~(uintptr_t)15);
    s.shift = (int64_t)(d & 15);
    s.limit = s.shift + a.n_bytes;
    s.ring = ring;
    s.hi = 0;
    s.nx0 = s.nx1 = make_uint4(0, 0, 0, 0);
    return s;
}

// kFix false: speculate every chunk's entry and walk it; true: one fix round (changed[round - 1] == 0
// ends the loop: every thread returns).
template <bool kFix>
__global__ __launch_bounds__(kWave * kRdwWaves) void rdw_wave_kernel(RdwArgs a, RdwChunkArgs c, int32_t round) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kRdwWaves * kRdwWaveLds];
    const int lane = threadIdx.x % kWave;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if (kFix && round > 0 && c.changed[round - 1] == 0) return;
    RdwStream s = rdw_stream(a, smem + wid * kRdwWaveLds);
    for (int64_t k = (int64_t)blockIdx.x * kRdwWaves + wid; k < c.n; k += (int64_t)gridDim.x * kRdwWaves) {
        const RdwChunk ch = rdw_chunk(c, k);
        int64_t entry;
        if (kFix) {
            if (ch.known) continue;
            entry = c.exit_out[k - 1];   // in place: the predecessor's exit of this round or the last
            if (entry == c.entry[k]) continue;
            if (lane == 0) { c.entry[k] = entry; c.changed[round] = 1; }
        } else {
            entry = ch.known ? ch.start : rdw_entry_wave(a, s, ch.start, ch.end, ch.range_end, lane);
            if (lane == 0) c.entry[k] = entry;
        }
        const RdwWalk w = rdw_walk_wave(a, s, entry, ch.end, c.stage_off + k * c.stage_cap, c.stage_len + k * c.stage_cap,
                                        c.stage_cap, lane);
        if (lane == 0) {
            c.exit_out[k] = w.exit;
            c.count[k] = w.count;
            c.err[k] = w.err;
        }
    }
}

// One wave per chunk: its staged records -> rec_off / rec_len[base, base + count) (coalesced);
// a chunk whose count passed the staging capacity is walked again by one lane, writing directly.
constexpr int kRdwPlaceWaves = 4;

__global__ __launch_bounds__(kWave * kRdwPlaceWaves) void rdw_place_kernel(RdwArgs a, RdwChunkArgs c, const int64_t* base,
                                                                          int64_t* rec_off, int32_t* rec_len, int64_t cap,
                                                                          unsigned long long* first_err) {
    const int lane = threadIdx.x % kWave;
    const int64_t k = (int64_t)blockIdx.x * kRdwPlaceWaves + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if (k >= c.n) return;
    const int64_t b = base[k];
    const int64_t n = c.count[k];
    if (lane == 0) {
        if (c.err[k] >= 0) atomicMin(first_err, (unsigned long long)c.err[k]);
        if (k == c.n - 1) first_err[1] = (unsigned long long)(b + n);   // record total
    }
    if (c.err[k] >= 0) return;
    if (n > c.stage_cap) {
        if (lane == 0) rdw_walk<2>(a, c.entry[k], rdw_chunk(c, k).end, rec_off, rec_len, b, cap);
        return;
    }
    const int64_t* so = c.stage_off + k * c.stage_cap;
    const int32_t* sl = c.stage_len + k * c.stage_cap;
    for (int64_t j = lane; j < n && b + j < cap; j += kWave) {
        rec_off[b + j] = so[j];
        rec_len[b + j] = sl[j];
    }
}

}  // namespace cbx
