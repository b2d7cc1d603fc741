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
// last record started: a segment walks back over the run of long segments before it (none in
// ordinary text).  Passes: LF count per 256-byte chunk -> scan -> LF positions -> per-segment
// record counts -> scan -> records; the final record after the last LF (its length depends on
// the virtual length) is settled by the host.
#pragma once

namespace cbx {

constexpr int kTextChunk = 256;   // bytes per thread in the LF passes

__device__ __forceinline__ int lf_in_word(uint32_t w) {
    const uint32_t x = w ^ 0x0A0A0A0Au;   // LF bytes -> 0
    int c = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) c += ((x >> (8 * b)) & 0xFFu) == 0u;
    return c;
}

// mode 0: LF count of the thread's chunk into count[t]; mode 1: LF positions at lf[base[t]...]
__global__ __launch_bounds__(256) void text_lf_kernel(const uint8_t* __restrict__ data, int64_t n, int64_t n_chunks,
                                                      int mode, uint32_t* __restrict__ count,
                                                      const int64_t* __restrict__ base, int64_t* __restrict__ lf) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_chunks) return;
    const int64_t b0 = t * kTextChunk, b1 = b0 + kTextChunk < n ? b0 + kTextChunk : n;
    const bool words = ((uintptr_t)data & 3u) == 0;
    uint32_t c = 0;
    int64_t out = mode ? base[t] : 0;
    int64_t i = b0;
    if (words) {
        for (; i + 4 <= b1; i += 4) {
            const uint32_t w = *(const uint32_t*)(data + i);
            if (mode == 0) {
                c += (uint32_t)lf_in_word(w);
            } else if (lf_in_word(w)) {
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if (((w >> (8 * b)) & 0xFFu) == 0x0Au) lf[out++] = i + b;
            }
        }
    }
    for (; i < b1; i++) {
        if (data[i] == 0x0A) {
            if (mode == 0) c++;
            else lf[out++] = i;
        }
    }
    if (mode == 0) count[t] = c;
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

// Line-ending length of the EOL before segment j (1 before the first record, :31).
__device__ int text_footer_before(const uint8_t* data, const int64_t* lf, int64_t j, int64_t M) {
    int64_t k = j - 1;
    while (k >= 0 && lf[k] - (k > 0 ? lf[k - 1] + 1 : 0) >= M) k--;
    int f = k < 0 ? 1 : text_eol_len(data, lf[k], k > 0 ? lf[k - 1] + 1 : 0);
    for (int64_t i = k + 1; i < j; i++) {
        int64_t c;
        const int64_t fs = text_final_start(i > 0 ? lf[i - 1] + 1 : 0, lf[i], M, f, &c);
        f = text_eol_len(data, lf[i], fs);
    }
    return f;
}

// One thread per segment j in [0, n_lf]: segment n_lf is the tail after the last LF (forced
// records while the window ends inside the data; its final record is left to the host).
// mode 0: record counts into cnt[j] (+ the tail's final start into *tail_start); mode 1: records.
__global__ __launch_bounds__(256) void text_seg_kernel(const uint8_t* __restrict__ data, int64_t n,
                                                       const int64_t* __restrict__ lf, int64_t n_lf, int64_t M,
                                                       int mode, uint32_t* __restrict__ cnt,
                                                       const int64_t* __restrict__ base, int64_t* __restrict__ rec_off,
                                                       int32_t* __restrict__ rec_len, int64_t* __restrict__ tail_start) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n_lf) return;
    const int64_t s0 = j > 0 ? lf[j - 1] + 1 : 0;
    const bool tail = j == n_lf;
    // fast path: a short segment after a short segment needs no walk back
    int f;
    if (j == 0) f = 1;
    else {
        const int64_t sp = j > 1 ? lf[j - 2] + 1 : 0;
        f = lf[j - 1] - sp < M ? text_eol_len(data, lf[j - 1], sp) : text_footer_before(data, lf, j, M);
    }
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
        return;
    }
    int64_t o = base[j];
    if (c > 0) {
        rec_off[o] = s0;
        rec_len[o] = (int32_t)(M - f);
        o++;
        const int64_t s1 = s0 + M - f;
        for (int64_t i = 1; i < c; i++, o++) {
            rec_off[o] = s1 + (i - 1) * M;
            rec_len[o] = (int32_t)M;
        }
    }
    if (!tail) {
        const int64_t p = lf[j];
        rec_off[o] = fs;
        rec_len[o] = (int32_t)(p - fs - (text_eol_len(data, p, fs) - 1));
    }
}

}  // namespace cbx
