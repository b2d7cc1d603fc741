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
#include "cbx_list.h"

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
    if (!lds_base_ok(smem)) { if (threadIdx.x == 0) atomicOr(a.status, 4); return; }   // (lds_ld)
    const WaveLds l = wave_lds(a, smem, wid);
    lut_lds_fill(a, l.lut);
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
template <bool kFix>
__global__ __launch_bounds__(kWave * kListWaves) void list_kernel(KernelArgs a, const CBX_CONST ListOp* lops, int32_t n_lops) {
    ListFieldLoop body;
    list_run<kFix>(a, lops, n_lops, body);
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
    uint32_t* stage_off;     // chunk k's records: [k * stage_cap, k * stage_cap + min(count, stage_cap)), payload
                             // offsets relative to the chunk's entry
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
constexpr int kRdwRingWins = 8;                // windows in the wave's ring (resident + loading ahead)
constexpr int kRdwRing = kRdwWin * kRdwRingWins;
constexpr int kRdwWaveLds = kRdwRing;
constexpr int kRdwWaves = 4;                   // waves per workgroup
#ifndef CBX_RDW_SPEC_GROUP
#define CBX_RDW_SPEC_GROUP 4
#endif
constexpr int kRdwSpecGroup = CBX_RDW_SPEC_GROUP;   // speculation windows loaded together

// The ring is filled by LDS-DMA (buffer_load_dwordx4 ... lds: one instruction per window, 16 bytes
// per lane straight into the window's slot, no registers).  The loads are issued as inline asm so
// the compiler does not drain them (it waits vmcnt(0) before any LDS read after an LDS-DMA it
// knows of); the walk waits for exactly the window it needs with a counted s_waitcnt vmcnt(N),
// N = the windows issued after it: vector memory operations complete in issue order, and other
// loads / stores issued after it only make the wait stricter.  (Register-held windows moved between
// registers at each refill waited vmcnt(0) per window: C4 framing 10 ms.)
struct RdwStream {
    const uint8_t* base;   // 16-byte aligned address at or before data
    int64_t shift;         // data - base
    int64_t limit;         // input bytes from base (shift + n_bytes)
    uint8_t* ring;         // the wave's LDS ring
    uint32_t ring_lds;     // its LDS address (M0 of the DMA)
    int64_t hi;            // next window (index from base) to issue
    int64_t ready;         // windows <= ready are in the ring
};

__device__ __forceinline__ void rdw_vmwait(int n) { lds_dma_wait(n); }

// Issue the DMA of window win into its slot (bytes past the input: zeros, range-checked).
__device__ __forceinline__ void rdw_win_dma(const RdwStream& s, int64_t win, int lane) {
    const int64_t a0 = win * kRdwWin;
    int64_t left = s.limit - a0;
    left = left < 0 ? 0 : (left > kRdwWin ? kRdwWin : left);
    const uint64_t b = (uint64_t)(s.base + (a0 < s.limit ? a0 : 0));
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane((int)left);
    void* bp = (void*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(bp, (short)0, nbytes, 0x00020000);
    const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)(s.ring_lds + (uint32_t)(win & (kRdwRingWins - 1)) * kRdwWin));
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %3\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(16 * lane), "s"(rs), "s"(dst) : "memory");
}

// Window win into registers (the speculation's scan): 16 bytes per lane, past the input zeros.
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
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// (re)start the stream at window win: 4 windows (a jump over a long record then costs 4 KiB, not
// the ring); later calls top the ring up to 8 windows ahead of the position
__device__ __forceinline__ void rdw_stream_start(RdwStream& s, int64_t win, int lane) {
    for (int j = 0; j < 4; j++) rdw_win_dma(s, win + j, lane);
    s.hi = win + 4;
    s.ready = win - 1;
}

// Bring the windows holding [pos, pos_hi) into the ring (wave-uniform positions relative to data,
// pos_hi - pos <= 4 KiB), keeping the ring's other slots loading ahead.
__device__ __forceinline__ void rdw_stream_range(RdwStream& s, int64_t pos, int64_t pos_hi, int lane) {
    const int64_t w0 = (s.shift + pos) >> 10, w1 = (s.shift + pos_hi - 1) >> 10;
    if (w1 <= s.ready && w0 >= s.hi - kRdwRingWins) return;
    if (w0 >= s.hi || w0 < s.hi - kRdwRingWins) {   // a jump past the windows issued
        rdw_stream_start(s, w0, lane);
    } else {
        while (s.hi <= w0 + kRdwRingWins - 1) rdw_win_dma(s, s.hi++, lane);   // slots of windows < w0 are free
    }
    const int64_t n_after = s.hi - 1 - w1;   // the windows issued after w1 may stay in flight
    rdw_vmwait((int)(n_after < 0 ? 0 : n_after));
    s.ready = w1;
}

__device__ __forceinline__ void rdw_stream_need(RdwStream& s, int64_t pos, int lane) { rdw_stream_range(s, pos, pos + 4, lane); }

// The 4 header bytes at pos (in the ring; the second dword wraps at the ring's end).
__device__ __forceinline__ uint32_t rdw_ring_header(const RdwStream& s, int64_t pos) {
    const uint32_t o = (uint32_t)((s.shift + pos) & (kRdwRing - 1));
    const uint32_t d0 = o & ~3u, d1 = (d0 + 4u) & (kRdwRing - 1);
    return __builtin_amdgcn_alignbyte(*(const uint32_t*)(s.ring + d1), *(const uint32_t*)(s.ring + d0), o & 3u);
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

// wave-uniform 64-bit value (SGPR pair): the walk's positions and lengths stay scalar
__device__ __forceinline__ int64_t uni64(int64_t v) {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)v));
}

// Staging of a walk: the lane that keeps record `count` of the current row of 64 (payload offset
// relative to the walk's entry, 32 bits; length), stored as a row when it fills.
struct RdwStage {
    uint32_t* so;
    int32_t* sl;
    uint32_t cap;            // (uniform: row bases scalar, the row stores take the saddr form)
    uint32_t count, my_off;
    int32_t my_len;
    __device__ __forceinline__ void push(uint32_t off, int32_t len, int lane) {
        if ((uint32_t)lane == (count & 63u)) { my_off = off; my_len = len; }
        count++;
        if ((count & 63u) == 0 && count <= cap) {
            (gp(so) + (count - 64))[lane] = my_off;
            (gp(sl) + (count - 64))[lane] = my_len;
        }
    }
    __device__ __forceinline__ void finish(int lane) {
        const uint32_t done = count & ~63u;
        if ((uint32_t)lane < (count & 63u) && done + (uint32_t)lane < cap) {
            (gp(so) + done)[lane] = my_off;
            (gp(sl) + done)[lane] = my_len;
        }
    }
};

// Ordinary headers from rp (relative to base) while rp < lim: the header from the ring made
// wave-uniform (readfirstlane), so position and length arithmetic is 32-bit scalar and a record costs
// a few vector instructions (the LDS read, the lane that keeps it).  With the generic step per header
// (vector compares and branches on vector values) C4's 150 M headers took 11.4 G VALU instructions,
// 24 ms (profiles/r03_a).  Returns false at a length the reference rejects (rp left at its header).
template <bool kBE>
__device__ __forceinline__ bool rdw_fast_run(const RdwArgs& a, RdwStream& s, int64_t base, int32_t& rp, int32_t lim,
                                             int32_t in_left, uint32_t rel0, RdwStage& sg, int lane) {
    const int32_t adj = a.p.adjustment;
    while (rp < lim) {
        rdw_stream_need(s, base + rp, lane);
        const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)rdw_ring_header(s, base + rp));
        const int32_t rlen = (kBE ? (int32_t)(((h & 0xFFu) << 8) | ((h >> 8) & 0xFFu)) : (int32_t)(h >> 16)) + adj;
        if (rlen <= 0 || rlen > 100 * 1024 * 1024) return false;
        const int32_t fo = rp + 4;
        const int32_t rem = in_left - fo;
        const int32_t got = rlen < rem ? rlen : rem;
        sg.push(rel0 + (uint32_t)fo, got, lane);
        rp = fo + got;
    }
    return true;
}

// The chain from pos to the first header at or past end, staging (offset relative to pos, length)
// of the valid records at so / sl [0, cap) in rows of 64 (records past cap are counted, not kept).
// Ordinary headers (not the file header record, not in the footer, 4 header bytes in the input)
// take rdw_fast_run; the others the generic step.
__device__ RdwWalk rdw_walk_wave(const RdwArgs& a, RdwStream& s, int64_t pos, int64_t end, uint32_t* so, int32_t* sl,
                                 int64_t cap, int lane) {
    RdwWalk w{pos, 0, -1};
    pos = uni64(pos);
    end = uni64(end);
    if (pos < 0) { w.exit = pos; return w; }
    const int64_t entry = pos;
    if (pos < end) rdw_stream_start(s, (s.shift + pos) >> 10, lane);
    RdwStage sg{so, sl, (uint32_t)(cap < 0x7fffffffll ? cap : 0x7fffffffll), 0u, 0u, 0};
    // ordinary headers: pos >= fast_lo (past a file header record at 0) and pos < fast_hi (4 header
    // bytes in the input, the payload start before the footer: n - (pos + 4) > footer)
    const int64_t fast_lo = a.p.file_header_bytes > 4 ? 1 : 0;
    const int64_t fast_hi = a.n_bytes - 4 - (a.p.file_footer_bytes > 0 ? (int64_t)a.p.file_footer_bytes : 0);
    while (pos < end) {
        if (pos >= fast_lo && pos < fast_hi) {
            // 32-bit positions relative to the run's start: scalar compares (no 64-bit SALU compare)
            const int64_t base = pos;
            const int64_t lim64 = (end < fast_hi ? end : fast_hi) - base;
            const int32_t lim = (int32_t)(lim64 < 0x40000000ll ? lim64 : 0x40000000ll);
            const int64_t in64 = a.n_bytes - base;
            const int32_t in_left = (int32_t)(in64 < 0x7fff0000ll ? in64 : 0x7fff0000ll);
            int32_t rp = 0;
            const uint32_t rel0 = (uint32_t)(base - entry);
            const bool ok = a.p.big_endian ? rdw_fast_run<true>(a, s, base, rp, lim, in_left, rel0, sg, lane)
                                           : rdw_fast_run<false>(a, s, base, rp, lim, in_left, rel0, sg, lane);
            pos = base + rp;
            if (ok) continue;
        }
        const RdwStep st = rdw_step_ring(a, s, pos, lane);
        if (st.err) {
            w.err = ((pos + 4) << 2) | (st.err == -2 ? 2 : 3);   // reported at the payload offset
            w.exit = -2;
            w.count = sg.count;
            return w;
        }
        if (st.stop) { pos = st.next; break; }
        if (st.valid) sg.push((uint32_t)(st.off - entry), st.len, lane);
        pos = uni64(st.next);
    }
    sg.finish(lane);
    w.exit = pos;
    w.count = sg.count;
    return w;
}

// ---- the walk over lane windows (dense records) ----
// A wave walks its chunk in windows of 2 KiB from the chain position P (a header): lane i owns
// [P + 32 i, P + 32 i + 32).  Every lane speculates the first header of its span (lane 0: P) -- the
// first strict candidate (the two non-length RDW bytes zero) whose next two hops are plausible --
// and walks from it to its span's end (headers read from the LDS ring): exit y_i and count c_i.  A
// lane without a candidate assumes the chain jumps over its span.  Resolution: the true position
// entering lane i is the exit of the last lane before it that holds a header (a ballot and a
// shuffle); lanes whose assumption fails re-walk (or become jumps), until none fails.  Then the
// counts are scanned over the wave and every lane walks its span once more, staging its records at
// their indices.  Per 2 KiB about two hundred wave instructions instead of a serial wave-uniform
// step per header (whose scalar instructions bound C4's framing: ~22 SALU per header, one SALU per
// cycle per CU).
constexpr int kLaneSpan = 32;
constexpr int kLaneWin = kWave * kLaneSpan;   // 2 KiB

// header at relative position rp (data position base + rp), from the ring
__device__ __forceinline__ int32_t rdw_lane_len(const RdwArgs& a, const RdwStream& s, int64_t base, int32_t rp,
                                                uint32_t& h) {
    h = rdw_ring_header(s, base + rp);
    return (a.p.big_endian ? (int32_t)(((h & 0xFFu) << 8) | ((h >> 8) & 0xFFu)) : (int32_t)(h >> 16)) + a.p.adjustment;
}

__device__ __forceinline__ bool rdw_lane_strict(const RdwArgs& a, uint32_t h, int32_t rl) {
    return rl > 0 && rl <= 100 * 1024 * 1024 && (a.p.big_endian ? (h >> 16) : (h & 0xFFFFu)) == 0;
}

// Walk a lane's span from rp while rp < r1: records counted, exit position, first error (relative
// position of the header, or -1).  kStore: stage record k at so / sl[idx + k] (idx < cap).
template <bool kStore>
__device__ __forceinline__ int32_t rdw_lane_walk(const RdwArgs& a, const RdwStream& s, int64_t base, int32_t rp, int32_t r1,
                                                 int32_t in_left, uint32_t& cnt, int32_t& err, uint32_t rel0,
                                                 uint32_t* so, int32_t* sl, uint32_t idx, uint32_t cap) {
    cnt = 0;
    err = -1;
    while (rp < r1) {
        uint32_t h;
        const int32_t rl = rdw_lane_len(a, s, base, rp, h);
        if (rl <= 0 || rl > 100 * 1024 * 1024) { err = rp; break; }
        const int32_t fo = rp + 4;
        const int32_t rem = in_left - fo;
        const int32_t got = rl < rem ? rl : rem;
        if (kStore && idx + cnt < cap) {
            gp(so)[idx + cnt] = rel0 + (uint32_t)fo;
            gp(sl)[idx + cnt] = got;
        }
        cnt++;
        rp = fo + got;
    }
    return rp;
}

// The lanes' parallel walk of one window from P = base (relative positions, every header in
// [base, base + kLaneWin) an ordinary one; lim = min(kLaneWin, end - base)).  Returns the exit
// (relative), adds the records to `count` (staged from index count), err: the relative position of
// a rejected header (-1 none) -- records before it are counted and staged.
// Strict candidates (the zero pair of a header: bytes 0-1 little-endian, 2-3 big-endian) of the
// lane's span [r0, r1) of the window at base: bit j <-> a header at relative position r0 + j.
__device__ __forceinline__ uint32_t rdw_lane_pairs(const RdwArgs& a, const RdwStream& s, int64_t base, int32_t r0, int32_t r1) {
    const int32_t off = a.p.big_endian ? 2 : 0;   // zero pair inside a header
    const uint32_t o0 = (uint32_t)((s.shift + base + r0 + off) & (kRdwRing - 1));
    const uint32_t a16 = o0 & ~15u, m = o0 & 15u;
    // zero bytes as 0x80 per byte (exact: no carry leaves a byte), a pair as a byte and the next
    // one (a funnel shift brings the next dword's byte 0 in), each dword's 4 pair bits gathered
    // into a nibble by one dot product of the 0/1 bytes with (1, 2, 4, 8)
    uint32_t z[13];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const u32x4 v = *(const u32x4*)(s.ring + ((a16 + 16u * j) & (kRdwRing - 1)));
        const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) z[4 * j + k] = ~(((x[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x[k]) & 0x80808080u;
    }
    z[12] = 0u;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const uint32_t pz = z[k] & __builtin_amdgcn_alignbit(z[k + 1], z[k], 8);
        const uint32_t nib = __builtin_amdgcn_udot4(pz >> 7, 0x08040201u, 0u, false);
        if (k < 8) lo |= nib << (4 * k);
        else hi |= nib << (4 * (k - 8));
    }
    const uint64_t zp = (uint64_t)lo | (uint64_t)hi << 32;
    return (uint32_t)((zp >> m) & ((1ull << (r1 - r0)) - 1));
}

// The chained-candidate form of a window (dense text-like records, C4): when the window's strict
// candidates are exactly a chain from P -- P is the first one, every candidate's next header is
// the following candidate, the last one's lies at or past the window's end -- they are exactly the
// headers the sequential walk visits (by induction from P: no header lies between a header and its
// next), so the window needs no speculation, hops, resolution rounds or walks: one candidate scan,
// one header read per candidate, a wave scan of the counts and the stores.  Any other window (a
// zero pair inside a payload, a non-strict or rejected header) returns false and takes the general
// form.  Returns the exit; adds the records to count (staged from index count).
__device__ __forceinline__ bool rdw_chain_window(const RdwArgs& a, const RdwStream& s, int64_t base, int32_t lim, int32_t in_left,
                                                 uint32_t rel0, uint32_t* so, int32_t* sl, uint32_t cap, uint32_t& count,
                                                 int32_t& exit, int lane, uint32_t pairs, int32_t r0) {
    int32_t first = 0x7fffffff, next = -1;
    uint32_t nc = 0;
    bool bad = false;
    for (uint32_t pm = pairs; pm; pm &= pm - 1) {
        const int32_t q = r0 + (int32_t)__builtin_ctz(pm);
        uint32_t h;
        const int32_t rl = rdw_lane_len(a, s, base, q, h);
        if (rl <= 0 || rl > 100 * 1024 * 1024 || (next >= 0 && next != q)) { bad = true; break; }
        if (nc == 0) first = q;
        const int32_t fo = q + 4;
        const int32_t rem = in_left - fo;
        next = fo + (rl < rem ? rl : rem);
        nc++;
    }
    const uint64_t hold = __ballot(nc > 0);
    // the first candidate of the next lane holding one (or none): the chain must enter it there
    const uint64_t above = lane < kWave - 1 ? hold & ~((2ull << lane) - 1) : 0ull;
    const int src = above ? __builtin_ctzll(above) : lane;
    const int32_t nf = __shfl(first, src, kWave);
    if (nc > 0) bad |= above ? next != nf : next < lim;
    if (lane == 0) bad |= first != 0;
    if (__ballot(bad)) return false;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(nc, lane, tot);
    uint32_t idx = count + ex;
    for (uint32_t pm = pairs; pm; pm &= pm - 1, idx++) {
        const int32_t q = r0 + (int32_t)__builtin_ctz(pm);
        uint32_t h;
        const int32_t rl = rdw_lane_len(a, s, base, q, h);
        const int32_t fo = q + 4;
        const int32_t rem = in_left - fo;
        if (idx < cap) {
            gp(so)[idx] = rel0 + (uint32_t)fo;
            gp(sl)[idx] = rl < rem ? rl : rem;
        }
    }
    count += tot;
    exit = __shfl(next, hold ? 63 - __builtin_clzll(hold) : 0, kWave);
    return true;
}

__device__ int32_t rdw_lane_window(const RdwArgs& a, const RdwStream& s, int64_t base, int32_t lim, int32_t in_left,
                                   int32_t resident, uint32_t rel0, uint32_t* so, int32_t* sl, uint32_t cap,
                                   uint32_t& count, int32_t& err, int lane) {
    err = -1;
    {
        // a record spanning the window (C5's 16 KB roots): the chain goes from P straight past the
        // window end, so P is the window's only header whatever the payload holds -- no candidate
        // scan (binary payloads are full of zero pairs) and no lane walks
        uint32_t h;
        const int32_t rl = rdw_lane_len(a, s, base, 0, h);   // (the same LDS dwords for every lane)
        const int32_t rem = in_left - 4;
        const int32_t nx = 4 + (rl < rem ? rl : rem);
        if (rl > 0 && rl <= 100 * 1024 * 1024 && nx >= lim) {
            if (lane == 0 && count < cap) {
                gp(so)[count] = rel0 + 4u;
                gp(sl)[count] = nx - 4;
            }
            count += 1;
            return nx;
        }
    }
    const int32_t r0 = lane * kLaneSpan;
    const int32_t r1 = r0 + kLaneSpan < lim ? r0 + kLaneSpan : lim;
    const bool live = r0 < lim;
    const uint32_t all_pairs = live ? rdw_lane_pairs(a, s, base, r0, r1) : 0u;
    int32_t cx;
    if (rdw_chain_window(a, s, base, lim, in_left, rel0, so, sl, cap, count, cx, lane, all_pairs, r0)) return cx;
    // speculation: the first strict candidate of the span with two plausible hops
    int32_t e = -1;
    if (lane == 0) {
        e = 0;
    } else if (live) {
        uint32_t pairs = all_pairs;
        while (pairs) {
            const int32_t q = r0 + (int32_t)__builtin_ctz(pairs);
            pairs &= pairs - 1;
            uint32_t h;
            int32_t rl = rdw_lane_len(a, s, base, q, h);
            if (!rdw_lane_strict(a, h, rl)) continue;
            bool ok = true;
            int32_t p = q + 4 + rl;
            for (int hop = 0; hop < 2 && ok; hop++) {   // hops past the resident bytes: not contradicted
                if (p + 4 > resident || p + 4 > in_left) break;
                rl = rdw_lane_len(a, s, base, p, h);
                ok = rdw_lane_strict(a, h, rl);
                p += 4 + rl;
            }
            if (ok) { e = q; break; }
        }
    }
    // speculative walks
    uint32_t c = 0;
    int32_t er = -1;
    int32_t y = e >= 0 ? rdw_lane_walk<false>(a, s, base, e, r1, in_left, c, er, 0u, nullptr, nullptr, 0u, 0u) : 0;
    // resolution: the position entering lane i is the exit of the last holding lane before it
    for (int round = 0; round <= kWave; round++) {
        const uint64_t hold = __ballot(e >= 0 && live);
        const uint64_t below = lane ? (hold & ((1ull << lane) - 1)) : 0ull;
        const int src = below ? 63 - __builtin_clzll(below) : 0;
        const int32_t x = __shfl(er >= 0 ? 0x7fffffff : y, src, kWave);   // (an error ends the chain)
        bool bad = false;
        if (lane > 0 && live) {
            if (e >= 0 && x != e) {            // a false candidate (or a chain entering elsewhere)
                bad = true;
                e = x < r1 ? x : -1;
            } else if (e < 0 && x < r1) {      // a header the speculation missed
                bad = true;
                e = x;
            }
            if (bad && e >= 0) y = rdw_lane_walk<false>(a, s, base, e, r1, in_left, c, er, 0u, nullptr, nullptr, 0u, 0u);
            if (bad && e < 0) { c = 0; er = -1; }
        }
        if (!__ballot(bad)) break;
    }
    // the first error of the chain (holding lanes only) ends the window: lanes after it keep nothing
    const uint64_t errs = __ballot(e >= 0 && live && er >= 0);
    const int first_err = errs ? __builtin_ctzll(errs) : kWave;
    const bool keep = e >= 0 && live && lane <= first_err;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(keep ? c : 0u, lane, tot);
    if (keep) {
        uint32_t c2;
        int32_t er2;
        rdw_lane_walk<true>(a, s, base, e, r1, in_left, c2, er2, rel0, so, sl, count + ex, cap);
    }
    count += tot;
    const uint64_t hold = __ballot(keep);
    const int last = 63 - __builtin_clzll(hold | 1ull);
    err = first_err < kWave ? __shfl(er, first_err, kWave) : -1;
    return __shfl(y, last, kWave);
}

// The chain from pos to the first header at or past end: windows of ordinary headers through the
// lanes (rdw_lane_window), the file header record and footer records through the generic step.
// Stages (offset relative to pos, length) of the valid records at so / sl [0, cap).
__device__ RdwWalk rdw_walk_lanes(const RdwArgs& a, RdwStream& s, int64_t pos, int64_t end, uint32_t* so, int32_t* sl,
                                  int64_t cap64, int lane) {
    RdwWalk w{pos, 0, -1};
    pos = uni64(pos);
    end = uni64(end);
    if (pos < 0) { w.exit = pos; return w; }
    const int64_t entry = pos;
    const uint32_t cap = (uint32_t)(cap64 < 0x7fffffffll ? cap64 : 0x7fffffffll);
    const int64_t fast_lo = a.p.file_header_bytes > 4 ? 1 : 0;
    const int64_t fast_hi = a.n_bytes - 4 - (a.p.file_footer_bytes > 0 ? (int64_t)a.p.file_footer_bytes : 0);
    uint32_t count = 0;
    while (pos < end) {
        if (pos >= fast_lo && pos < fast_hi) {
            // every header of [pos, pos + lim) is an ordinary one (lim clipped at fast_hi and the chunk end)
            const int64_t lim64 = (end < fast_hi ? end : fast_hi) - pos;
            const int32_t lim = (int32_t)(lim64 < kLaneWin ? lim64 : kLaneWin);
            const int64_t in64 = a.n_bytes - pos;
            const int32_t in_left = (int32_t)(in64 < 0x7fff0000ll ? in64 : 0x7fff0000ll);
            const int64_t res64 = pos + 3 * 1024 < a.n_bytes ? pos + 3 * 1024 : a.n_bytes;
            rdw_stream_range(s, pos, res64 > pos + 4 ? res64 : pos + 4, lane);
            const int32_t resident = (int32_t)(res64 - pos);
            int32_t err;
            const int32_t x = rdw_lane_window(a, s, pos, lim, in_left, resident, (uint32_t)(pos - entry), so, sl, cap,
                                              count, err, lane);
            if (err >= 0) {
                w.err = ((pos + err + 4) << 2) | 2;   // (the header's length: <= 0 or > 100 MiB; the code below)
                const int64_t ep = uni64(pos + err);
                const RdwStep st = rdw_step_ring(a, s, ep, lane);
                w.err = ((ep + 4) << 2) | (st.err == -3 ? 3 : 2);
                w.exit = -2;
                w.count = count;
                return w;
            }
            pos = uni64(pos + (int64_t)x);
            continue;
        }
        const RdwStep st = rdw_step_ring(a, s, pos, lane);
        if (st.err) {
            w.err = ((pos + 4) << 2) | (st.err == -2 ? 2 : 3);   // reported at the payload offset
            w.exit = -2;
            w.count = count;
            return w;
        }
        if (st.stop) { pos = st.next; break; }
        if (st.valid) {
            if (lane == 0 && count < cap) {
                gp(so)[count] = (uint32_t)(st.off - entry);
                gp(sl)[count] = st.len;
            }
            count++;
        }
        pos = uni64(st.next);
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
    // windows in groups of kRdwSpecGroup, all of a group's loads issued before the first is scanned: the
    // first header of a chunk of 16 KB records lies ~8 windows in (C5), one load latency per group
    // instead of one per window (C5 framing -7 %, C4 unchanged; 8 windows: C4 +1.5 %)
    for (int64_t w0 = (s.shift + s0 + off) >> 10; ; w0 += kRdwSpecGroup) {
        if (w0 * kRdwWin - s.shift >= e + off || w0 * kRdwWin - s.shift >= a.n_bytes) break;
        uint4 vg[kRdwSpecGroup];
#pragma unroll
        for (int g = 0; g < kRdwSpecGroup; g++) {
            const int64_t wa = (w0 + g) * kRdwWin - s.shift;
            vg[g] = (wa < e + off && wa < a.n_bytes) ? rdw_win_load(s, w0 + g, lane) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int g = 0; g < kRdwSpecGroup; g++) {
            const int64_t wa = (w0 + g) * kRdwWin - s.shift;   // window start relative to data
            if (wa >= e + off || wa >= a.n_bytes) break;
            // the lane's 16 bytes + the next one (from the following lane's slice, or the next window)
            const uint4 v = vg[g];
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
    s.ring_lds = (uint32_t)(uintptr_t)ring;   // a generic LDS address: the LDS offset in its low 32 bits
    s.hi = 0;
    s.ready = -1;
    return s;
}

// A chunk the lane walk (rdw_lane_walk_kernel) hands back to the wave walk: its count word.
constexpr uint32_t kRdwToWave = 0xFFFFFFFFu;

// kFix false: `round` is the phase -- 0 speculate every chunk's entry and walk it; 1 speculate only
// (the entries for rdw_lane_walk_kernel); 2 walk, from its entry, every chunk the lane walk handed
// back (count == kRdwToWave).  kFix true: one fix round (changed[round - 1] == 0 ends the loop: every
// thread returns).
template <bool kFix>
__global__ __launch_bounds__(kWave * kRdwWaves) void rdw_wave_kernel(RdwArgs a, RdwChunkArgs c, int32_t round) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kRdwWaves * kRdwWaveLds];
    const int lane = threadIdx.x % kWave;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if (kFix && round > 0 && c.changed[round - 1] == 0) return;
    if (kFix && round == 0 && c.changed[c.n + 1] == 0) return;   // rdw_check_kernel found every entry right
    RdwStream s = rdw_stream(a, smem + wid * kRdwWaveLds);
    for (int64_t k = (int64_t)blockIdx.x * kRdwWaves + wid; k < c.n; k += (int64_t)gridDim.x * kRdwWaves) {
        const RdwChunk ch = rdw_chunk(c, k);
        int64_t entry;
        if (kFix) {
            if (ch.known) continue;
            entry = c.exit_out[k - 1];   // in place: the predecessor's exit of this round or the last
            if (entry == c.entry[k]) continue;
            if (lane == 0) { c.entry[k] = entry; c.changed[round] = 1; }
        } else if (round == 2) {
            if (__builtin_amdgcn_readfirstlane((int)c.count[k]) != (int)kRdwToWave) continue;
            entry = uni64(c.entry[k]);
        } else {
            entry = ch.known ? ch.start : rdw_entry_wave(a, s, ch.start, ch.end, ch.range_end, lane);
            if (lane == 0) c.entry[k] = entry;
            if (round == 1) continue;
        }
        const RdwWalk w = rdw_walk_lanes(a, s, entry, ch.end, c.stage_off + k * c.stage_cap, c.stage_len + k * c.stage_cap,
                                         c.stage_cap, lane);
        if (lane == 0) {
            c.exit_out[k] = w.exit;
            c.count[k] = w.count;
            c.err[k] = w.err;
        }
    }
}

// Phase 1 as a kernel of its own: the speculation reads its windows into registers, so without the
// walk's LDS ring (8 KiB a wave) more waves are resident per CU.
__global__ __launch_bounds__(kWave * kRdwWaves) __attribute__((amdgpu_waves_per_eu(8))) void rdw_spec_kernel(RdwArgs a,
                                                                                                         RdwChunkArgs c) {
    const int lane = threadIdx.x % kWave;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    RdwStream s = rdw_stream(a, nullptr);
    for (int64_t k = (int64_t)blockIdx.x * kRdwWaves + wid; k < c.n; k += (int64_t)gridDim.x * kRdwWaves) {
        const RdwChunk ch = rdw_chunk(c, k);
        const int64_t entry = ch.known ? ch.start : rdw_entry_wave(a, s, ch.start, ch.end, ch.range_end, lane);
        if (lane == 0) c.entry[k] = entry;
    }
}

// The walk of chunks of long records, one lane per chunk (phase 1's entries): headers read straight
// from HBM, so a wave has 64 chains in flight where the wave walk has one -- a chunk of 16 KB records
// is ~16 dependent header loads, which the wave walk pays as 16 DMA round trips of one wave (C5).  A
// chunk that turns out dense -- its first kRdwLaneProbe records span less than kRdwLaneProbe x 1 KiB, or
// it holds more than kRdwLaneMax records -- is handed to the wave walk (phase 2) untouched.  Results as
// rdw_walk_lanes': exit (or -2 after an error), valid-record count, first error, records staged as
// (payload offset relative to the entry, length).
constexpr int kRdwLaneProbe = 8;
constexpr uint32_t kRdwLaneMax = 256;

__global__ __launch_bounds__(256) void rdw_lane_walk_kernel(RdwArgs a, RdwChunkArgs c) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n) return;
    const RdwChunk ch = rdw_chunk(c, k);
    const int64_t entry = c.entry[k];
    uint32_t* so = c.stage_off + k * c.stage_cap;
    int32_t* sl = c.stage_len + k * c.stage_cap;
    int64_t pos = entry;
    uint32_t count = 0, steps = 0;
    int64_t err = -1;
    while (pos < ch.end) {
        const RdwStep st = rdw_step(a, pos);
        if (st.err) {
            err = ((pos + 4) << 2) | (st.err == -2 ? 2 : 3);   // reported at the payload offset
            pos = -2;
            break;
        }
        if (st.stop) { pos = st.next; break; }
        if (st.valid) {
            if ((int64_t)count < c.stage_cap) { so[count] = (uint32_t)(st.off - entry); sl[count] = st.len; }
            count++;
        }
        pos = st.next;
        steps++;
        if ((steps == kRdwLaneProbe && pos - entry < (int64_t)kRdwLaneProbe * 1024) || count > kRdwLaneMax) {
            c.count[k] = kRdwToWave;   // dense: the wave walk's
            return;
        }
    }
    c.exit_out[k] = pos;
    c.count[k] = count;
    c.err[k] = err;
}

// Before the fix rounds: does any chunk's entry differ from its predecessor's exit?  (changed[n + 1]; a
// lane per chunk -- the first fix round's wave per chunk spent ~40-80 us finding that out on C5.)
__global__ __launch_bounds__(256) void rdw_check_kernel(RdwChunkArgs c) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n || k == 0) return;
    if (!rdw_chunk(c, k).known && c.exit_out[k - 1] != c.entry[k]) c.changed[c.n + 1] = 1;
}

// Settles the walk on the device after the parallel fix rounds (cbx_frame_rdw_async, no host check
// between rounds): returns at once when the last round changed nothing; otherwise one wave goes over
// the chunks in file order -- 64 (predecessor exit, entry) pairs per ballot -- and walks again every
// chunk whose entry differs from its predecessor's exit, so a chain of failed speculations of any
// length resolves in one pass (sequential along that chain only; rare).
__global__ __launch_bounds__(kWave) void rdw_settle_kernel(RdwArgs a, RdwChunkArgs c, int32_t last_round) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kRdwWaveLds];
    const int lane = threadIdx.x;
    if (c.changed[last_round] == 0) return;
    RdwStream s = rdw_stream(a, smem);
    for (int64_t k0 = 1; k0 < c.n;) {
        const int64_t k = k0 + lane;
        bool bad = false;
        if (k < c.n) bad = !rdw_chunk(c, k).known && c.exit_out[k - 1] != c.entry[k];
        const uint64_t m = __ballot(bad);
        if (m == 0) {
            k0 += kWave;
            continue;
        }
        const int64_t kb = k0 + __builtin_ctzll(m);
        const int64_t entry = uni64(c.exit_out[kb - 1]);
        const RdwChunk ch = rdw_chunk(c, kb);
        const RdwWalk w = rdw_walk_lanes(a, s, entry, ch.end, c.stage_off + kb * c.stage_cap,
                                         c.stage_len + kb * c.stage_cap, c.stage_cap, lane);
        if (lane == 0) {
            c.entry[kb] = entry;
            c.exit_out[kb] = w.exit;
            c.count[kb] = w.count;
            c.err[kb] = w.err;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        k0 = kb + 1;   // the next pair reads exit_out[kb]: lane 0 wrote it, lane 0 reads it
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
    const uint32_t* so = c.stage_off + k * c.stage_cap;
    const int32_t* sl = c.stage_len + k * c.stage_cap;
    const int64_t e0 = c.entry[k];   // staged offsets are relative to the walk's entry
    for (int64_t j = lane; j < n && b + j < cap; j += kWave) {
        rec_off[b + j] = e0 + so[j];
        rec_len[b + j] = sl[j];
    }
}

}  // namespace cbx
