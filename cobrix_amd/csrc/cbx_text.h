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
// last record started: a segment walks back only while that dependence is real (rare).  Passes: LF count per 16 KiB chunk (one wave each) -> scan -> LF positions -> per-segment
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

// Line-ending length of the EOL before segment j (1 before the first record, :31).  Walks back
// only while a segment's result depends on its input (a long segment whose last record starts
// right at a CR): short segments and almost all long ones map both inputs to the same length.
__device__ int text_footer_before(const uint8_t* data, const int64_t* lf, int64_t j, int64_t M) {
    int64_t k = j - 1;
    int f = 1;
    for (; k >= 0; k--) {
        const int a = text_seg_out(data, lf, k, M, 1), b = text_seg_out(data, lf, k, M, 2);
        if (a == b) { f = a; break; }
    }
    for (int64_t i = k + 1; i < j; i++) f = text_seg_out(data, lf, i, M, f);
    return f;
}

// One thread per segment j in [0, n_lf]: segment n_lf is the tail after the last LF (forced
// records while the window ends inside the data; its final record is left to the host).
// mode 0: record counts into cnt[j] (+ the tail's final start into *tail_start); mode 1: records.
__global__ __launch_bounds__(256) void text_seg_kernel(const uint8_t* __restrict__ data, int64_t n,
                                                       const int64_t* __restrict__ lf, int64_t n_lf, int64_t M,
                                                       int mode, uint32_t* __restrict__ cnt,
                                                       const int64_t* __restrict__ base, int64_t* __restrict__ rec_off,
                                                       int32_t* __restrict__ rec_len, int64_t* __restrict__ tail_start,
                                                       unsigned long long* __restrict__ big, int32_t big_ok) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n_lf) return;
    const int64_t s0 = j > 0 ? lf[j - 1] + 1 : 0;
    const bool tail = j == n_lf;
    const int f = text_footer_before(data, lf, j, M);
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
                                                          int32_t* __restrict__ rec_len) {
    const int64_t j = (int64_t)big[1 + blockIdx.x];
    const int64_t s0 = j > 0 ? lf[j - 1] + 1 : 0;
    const int f = text_footer_before(data, lf, j, M);
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
