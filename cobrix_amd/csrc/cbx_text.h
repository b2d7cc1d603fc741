// Text record framing (is_text = true): the records of an ASCII file separated by LF / CRLF,
// restating TextRecordExtractor (CP/reader/extractors/raw/TextRecordExtractor.scala:26-108) as
// data-parallel passes.
//
// The reference reads the stream through a window of M = record_size + 2 bytes and takes the
// first LF (or CR LF) inside it as the end of the record (payload without the line ending); a
// window without one yields a forced record of M - (previous line ending's length) bytes, and
// at the end of the stream the rest of the window.  Its read helper (ensureBytesRead, :98-107)
// marks the whole window as filled even when the last read came back short, so the stream
// behaves as if M - (bytes read) zero bytes followed the data: the "virtual" length.
//
// Parallel form: every LF of the data ends one segment; a segment shorter than M is one record,
// a longer one starts with forced records whose lengths follow from the previous line ending
// (closed form below).  A CR counts as part of the line ending only when it lies inside the
// record that ends at the LF, so the line-ending length depends on where the previous segment's
// last record started: a scan of per-segment maps over {1, 2} resolves it.  Passes: LF count per
// 16 KiB chunk (one wave each) -> scan -> LF positions -> line-ending map scan -> per-segment
// record counts -> scan -> records; the final record after the last LF (its length depends on
// the virtual length) is settled by the host.
#pragma once

namespace cbx {

constexpr int kForcedInline = 64;   // forced records a segment's own thread writes; more -> text_forced_kernel
constexpr int kBigSegCap = 1024;    // segments listed for text_forced_kernel (beyond: written inline)
constexpr int kTextChunk = 16384;   // bytes per wave in the LF passes (64 lanes x 16 B x 16 steps)

__device__ __forceinline__ uint32_t lf_mask16(const uint8_t* p, int64_t i, int64_t n, bool vec) {
    // bit b set when byte i + b is an LF (bytes at or past n never are)
    uint32_t m = 0;
    if (vec && i + 16 <= n) {
        const uint4 v = *(const uint4*)(p + i);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int b = 0; b < 4; b++) m |= (((w[k] >> (8 * b)) & 0xFFu) == 0x0Au ? 1u : 0u) << (4 * k + b);
    } else {
        for (int b = 0; b < 16 && i + b < n; b++) m |= (p[i + b] == 0x0A ? 1u : 0u) << b;
    }
    return m;
}

// One wave per kTextChunk-byte chunk, lanes on consecutive 16-byte groups (coalesced).
// mode 0: LF count of the chunk into count[chunk]; mode 1: LF positions in file order at
// lf[base[chunk]...] (wave prefix sums of the lanes' counts per step).
__global__ __launch_bounds__(256) void text_lf_kernel(const uint8_t* __restrict__ data, int64_t n, int64_t n_chunks,
                                                      int mode, uint32_t* __restrict__ count,
                                                      const int64_t* __restrict__ base, int64_t* __restrict__ lf) {
    const int lane = threadIdx.x & 63;
    const int64_t chunk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (chunk >= n_chunks) return;
    const bool vec = ((uintptr_t)data & 15u) == 0;
    const int64_t c0 = chunk * kTextChunk;
    uint32_t c = 0;
    int64_t out = mode ? base[chunk] : 0;
    for (int step = 0; step < kTextChunk / (64 * 16); step++) {
        const int64_t i = c0 + (int64_t)step * 1024 + lane * 16;
        if (c0 + (int64_t)step * 1024 >= n) break;   // wave-uniform
        uint32_t m = i < n ? lf_mask16(data, i, n, vec) : 0u;
        const uint32_t k = (uint32_t)__popc(m);
        if (mode == 0) { c += k; continue; }
        uint32_t pre = k;   // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(pre, d, 64);
            if (lane >= d) pre += y;
        }
        const uint32_t tot = __shfl(pre, 63, 64);
        int64_t o = out + (pre - k);
        while (m) {
            const int b = __ffs(m) - 1;
            lf[o++] = i + b;
            m &= m - 1;
        }
        out += tot;
    }
    if (mode == 0) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
        if (lane == 0) count[chunk] = c;
    }
}

__device__ __forceinline__ int64_t text_ceil_div(int64_t a, int64_t b) { return a <= 0 ? 0 : (a + b - 1) / b; }

// Start of the record that ends at the LF p of a segment starting at s0 (forced records first
// while the LF lies outside the window), and the number of forced records.
__device__ __forceinline__ int64_t text_final_start(int64_t s0, int64_t p, int64_t M, int f, int64_t* forced) {
    if (p - s0 < M) { *forced = 0; return s0; }
    const int64_t s1 = s0 + M - f;
    const int64_t c = 1 + text_ceil_div(p - M + 1 - s1, M);
    *forced = c;
    return s1 + (c - 1) * M;
}

__device__ __forceinline__ int text_eol_len(const uint8_t* data, int64_t p, int64_t start) {
    return (p - 1 >= start && data[p - 1] == 0x0D) ? 2 : 1;
}

// Line-ending length of the EOL that ends segment i, given the line-ending length f before it.
__device__ __forceinline__ int text_seg_out(const uint8_t* data, const int64_t* lf, int64_t i, int64_t M, int f) {
    const int64_t s0 = i > 0 ? lf[i - 1] + 1 : 0;
    if (lf[i] - s0 < M) return text_eol_len(data, lf[i], s0);
    int64_t c;
    return text_eol_len(data, lf[i], text_final_start(s0, lf[i], M, f, &c));
}

// Line-ending length of the EOL before every segment (1 before the first record, :31).  Segment i
// maps the length before it, f in {1, 2}, to the length of its own line ending: a 2-bit map
// (bit 0: f = 1 -> 2, bit 1: f = 2 -> 2).  The lengths are an exclusive scan of those maps under
// composition, applied to f = 1 -- three passes (block compositions, their scan, apply), linear
// in the segment count whatever the data (long lines ending right after a CR chain every
// segment's result to its predecessor's).
constexpr int kEolThreads = 256;
constexpr int kEolItems = 8;
constexpr int kEolTile = kEolThreads * kEolItems;

__device__ __forceinline__ uint32_t eol_map(const uint8_t* data, const int64_t* lf, int64_t i, int64_t M) {
    return (text_seg_out(data, lf, i, M, 1) == 2 ? 1u : 0u) | (text_seg_out(data, lf, i, M, 2) == 2 ? 2u : 0u);
}
__device__ __forceinline__ uint32_t eol_apply(uint32_t m, uint32_t f) { return ((m >> (f - 1)) & 1u) ? 2u : 1u; }
// a then b
__device__ __forceinline__ uint32_t eol_compose(uint32_t a, uint32_t b) {
    return (eol_apply(b, eol_apply(a, 1)) == 2 ? 1u : 0u) | (eol_apply(b, eol_apply(a, 2)) == 2 ? 2u : 0u);
}
constexpr uint32_t kEolIdentity = 2u;   // 1 -> 1, 2 -> 2

// pass 0: composition of each tile's maps -> tot[tile]; pass 2: f before every segment j <= n_lf,
// starting from the tile's incoming map pre[tile]
__global__ __launch_bounds__(kEolThreads) void text_eol_kernel(const uint8_t* __restrict__ data, const int64_t* __restrict__ lf,
                                                               int64_t n_lf, int64_t M, int pass, uint8_t* __restrict__ tot,
                                                               const uint8_t* __restrict__ pre, uint8_t* __restrict__ f_before) {
    __shared__ uint8_t s_m[kEolThreads];
    const int64_t i0 = (int64_t)blockIdx.x * kEolTile + (int64_t)threadIdx.x * kEolItems;
    uint32_t maps[kEolItems];
    uint32_t acc = kEolIdentity;
#pragma unroll
    for (int k = 0; k < kEolItems; k++) {
        maps[k] = i0 + k < n_lf ? eol_map(data, lf, i0 + k, M) : kEolIdentity;
        acc = eol_compose(acc, maps[k]);
    }
    s_m[threadIdx.x] = (uint8_t)acc;
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive scan of the threads' compositions (in place)
        uint32_t run = kEolIdentity;
        for (int t = 0; t < kEolThreads; t++) {
            const uint32_t x = s_m[t];
            s_m[t] = (uint8_t)run;
            run = eol_compose(run, x);
        }
        if (pass == 0) tot[blockIdx.x] = (uint8_t)run;
    }
    __syncthreads();
    if (pass == 0) return;
    uint32_t f = eol_apply(eol_compose(pre[blockIdx.x], s_m[threadIdx.x]), 1);
#pragma unroll
    for (int k = 0; k < kEolItems; k++) {
        if (i0 + k <= n_lf) f_before[i0 + k] = (uint8_t)f;
        f = eol_apply(maps[k], f);
    }
}

// pass 1: exclusive scan of the tile compositions (one thread: a tile covers 2048 segments)
__global__ void text_eol_scan_kernel(uint8_t* tot, int64_t n_tiles) {
    uint32_t run = kEolIdentity;
    for (int64_t t = 0; t < n_tiles; t++) {
        const uint32_t x = tot[t];
        tot[t] = (uint8_t)run;
        run = eol_compose(run, x);
    }
}

// One thread per segment j in [0, n_lf]: segment n_lf is the tail after the last LF (forced
// records while the window ends inside the data; its final record is left to the host).
// mode 0: record counts into cnt[j] (+ the tail's final start into *tail_start); mode 1: records.
__global__ __launch_bounds__(256) void text_seg_kernel(const uint8_t* __restrict__ data, int64_t n,
                                                       const int64_t* __restrict__ lf, int64_t n_lf, int64_t M,
                                                       int mode, uint32_t* __restrict__ cnt,
                                                       const int64_t* __restrict__ base, int64_t* __restrict__ rec_off,
                                                       int32_t* __restrict__ rec_len, int64_t* __restrict__ tail_start,
                                                       unsigned long long* __restrict__ big, int32_t big_ok,
                                                       const uint8_t* __restrict__ f_before) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n_lf) return;
    const int64_t s0 = j > 0 ? lf[j - 1] + 1 : 0;
    const bool tail = j == n_lf;
    const int f = f_before[j];
    int64_t c, fs;
    if (!tail) {
        fs = text_final_start(s0, lf[j], M, f, &c);
    } else if (s0 + M >= n) {
        c = 0; fs = s0;
    } else {
        const int64_t s1 = s0 + M - f;
        c = 1 + text_ceil_div(n - M - s1, M);
        fs = s1 + (c - 1) * M;
    }
    if (mode == 0) {
        cnt[j] = (uint32_t)(c + (tail ? 0 : 1));
        if (tail) *tail_start = fs;
        if (c > kForcedInline) {   // big[0]: count, big[1..]: segment indices
            const unsigned long long k = atomicAdd(big, 1ull);
            if (k < (unsigned long long)kBigSegCap) big[1 + k] = (unsigned long long)j;
        }
        return;
    }
    int64_t o = base[j];
    if (c > 0) {
        rec_off[o] = s0;
        rec_len[o] = (int32_t)(M - f);
        o++;
        const int64_t s1 = s0 + M - f;
        if (c > kForcedInline && big_ok) {
            o += c - 1;   // text_forced_kernel
        } else {
            for (int64_t i = 1; i < c; i++, o++) {
                rec_off[o] = s1 + (i - 1) * M;
                rec_len[o] = (int32_t)M;
            }
        }
    }
    if (!tail) {
        const int64_t p = lf[j];
        rec_off[o] = fs;
        rec_len[o] = (int32_t)(p - fs - (text_eol_len(data, p, fs) - 1));
    }
}

// The forced records 1..c-1 of the listed long segments, spread over gridDim.y blocks each.
__global__ __launch_bounds__(256) void text_forced_kernel(const uint8_t* __restrict__ data, int64_t n,
                                                          const int64_t* __restrict__ lf, int64_t n_lf, int64_t M,
                                                          const unsigned long long* __restrict__ big,
                                                          const int64_t* __restrict__ base, int64_t* __restrict__ rec_off,
                                                          int32_t* __restrict__ rec_len, const uint8_t* __restrict__ f_before) {
    const int64_t j = (int64_t)big[1 + blockIdx.x];
    const int64_t s0 = j > 0 ? lf[j - 1] + 1 : 0;
    const int f = f_before[j];
    int64_t c;
    if (j < n_lf) {
        text_final_start(s0, lf[j], M, f, &c);
    } else {
        const int64_t s1 = s0 + M - f;
        c = s0 + M >= n ? 0 : 1 + text_ceil_div(n - M - s1, M);
    }
    const int64_t s1 = s0 + M - f;
    const int64_t o = base[j];
    for (int64_t i = 1 + (int64_t)blockIdx.y * blockDim.x + threadIdx.x; i < c; i += (int64_t)gridDim.y * blockDim.x) {
        rec_off[o + i] = s1 + (i - 1) * M;
        rec_len[o + i] = (int32_t)M;
    }
}

}  // namespace cbx
