// cbx_chain.h -- chunk-parallel framing of record chains: streams where a record starts where the
// previous one ends and its length is read from its own bytes.
//
// * record_length_field (VRLRecordReader.fetchRecordUsingRecordLengthField,
//   CP/reader/iterator/VRLRecordReader.scala:114-149): the length field decoded at the record start.
// * variable_size_occurs framing (VarOccursRecordExtractor.extractVarOccursRecordBytes,
//   CP/reader/extractors/raw/VarOccursRecordExtractor.scala:51-136): the record's length walked over
//   its dependees (walk_length).
//
// Sequential as the reference reads it, but not sequential in structure: from any byte position p the
// next record start next(p) is a function of the bytes at p.  So the stream is cut into chunks of C
// bytes and every chunk is framed from an assumed entry (its first record start), then corrected:
//
// 1. chain_sample: one thread walks the first records (the true chain) for the length range [lo, hi].
// 2. chain_spec (one lane per chunk): the speculated entry -- the first position of the chunk that
//    starts 4 records whose lengths lie in [lo, hi] (chunk 0: the stream start, exact) -- and the walk
//    from it to the chunk end: every visited position marked in a bitmap, the count and the exit (the
//    first chain position at or past the chunk end).
// 3. chain_fix rounds (one lane per chunk): a chunk whose entry differs from its predecessor's exit
//    walks again from that exit until it reaches a position the speculated walk visited -- from there
//    on the two chains are one (next() is deterministic), so the count is the walked prefix plus the
//    speculated walk's records from that position (a popcount of the bitmap) and the exit is the
//    speculated one.  A chunk whose exit changes sends its successor into the next round.  By
//    induction from chunk 0 every entry is then the sequential walk's; speculation only moves work.
//    Rounds run until none changes (chains from wrong entries mostly meet the true one within a few
//    records: an implausible length breaks a candidate at once, a plausible one lands on a record
//    start); after kChainRounds a one-lane settle pass resolves the rest in chunk order.
// 4. a device scan of the counts, then chain_write (one lane per chunk) walks its chunk from its entry
//    writing the record offsets / lengths at the chunk's base, and the chunk holding the chain's end
//    records it (the error of a record-length field, the end of the last record).
#pragma once
#include "cbx_walk.h"

namespace cbx {

constexpr int64_t kChainStop = 0x7fffffffffffffffll;   // the chain has ended
constexpr int kChainHops = 4;                             // plausible records a speculated entry starts
constexpr int kChainRounds = 8;                           // fix rounds before the settle pass
constexpr int kChainSearch = 512;                         // candidate entries tried per chunk

// One record at pos: len 0 = no record starts there (the chain ends at pos); next = kChainStop after
// the stream's last record; err != 0 = the reference fails at pos.
struct ChainStep {
    int64_t next;
    int32_t len;
    int32_t err;
};

// ---- VRLRecordReader.fetchRecordUsingRecordLengthField (CP/reader/iterator/VRLRecordReader.scala:114-149) ----
// A record's first start_offset + lfb bytes (lfb = the length field's offset + size) carry the length
// field, decoded as extractPrimitiveField does; the record is those bytes + max(0, length + adjustment -
// lfb + end_offset) more (fewer at the end of the stream, which then ends).  Error (the reference throws
// IllegalStateException): 1 a null or non-Int/Long value.
struct LenFieldArgs {
    const uint8_t* data;
    int64_t n_bytes;
    const CBX_CONST Field* field;     // the length field (decode offset relative to the record start + start_off)
    int32_t start_off, end_off, adjustment, lfb;
};

struct LenFieldStep {
    LenFieldArgs a;
    __device__ __forceinline__ ChainStep at(int64_t pos) const {
        ChainStep s{kChainStop, 0, 0};
        const int64_t head = (int64_t)a.start_off + a.lfb;
        if (pos + head > a.n_bytes) return s;   // dataStream.next(startOffset + lengthFieldBlock) short: the end
        const Field f = ldc(a.field);
        // an Integral field (ReaderParametersValidator.getLengthField): Int / Long -> toInt; a null or
        // a BigDecimal (precision > 18) value: "must be an integral type"
        const Val x = decode_numeric(f, a.data + pos + a.start_off + f.offset);
        if (!x.valid || (f.out_type != CBX_O_I32 && f.out_type != CBX_O_I64)) { s.err = 1; return s; }
        const int32_t len = (int32_t)(uint32_t)x.lo;
        // Java int arithmetic: recordLength = value + adjustment; rest = recordLength - lfb + endOffset
        const int32_t rest = (int32_t)((uint32_t)len + (uint32_t)a.adjustment - (uint32_t)a.lfb + (uint32_t)a.end_off);
        const int64_t left = a.n_bytes - (pos + head);
        const int64_t take = rest > 0 ? (rest < left ? rest : left) : 0;
        s.len = (int32_t)(head + take);
        s.next = (rest > 0 && take < rest) ? kChainStop : pos + head + take;   // a short read closes the stream
        return s;
    }
};

// ---- VarOccursRecordExtractor: a record's length walked over its dependees ----
// hasNext while offset < size; a record may reach past n_bytes (zero-filled, the virtual length).
// walk_length: > 0 the record's length, 0 nothing to walk, -1 the copybook nests deeper than the walk.
#ifndef CBX_JIT_WALK
struct VarOccursStep {
    WalkArgs a;
    int64_t n_bytes;
    __device__ __forceinline__ ChainStep at(int64_t pos) const {
        ChainStep s{kChainStop, 0, 0};
        if (pos >= n_bytes) return s;
        const int64_t left = n_bytes - pos;
        const int len = walk_length(a, a.data + pos, left < 0x7fffffff ? (int)left : 0x7fffffff);
        if (len <= 0) { s.err = len < 0 ? 2 : 0; return s; }
        s.len = len;
        s.next = pos + len;
        return s;
    }
};
#endif

// Chunk state (device, one entry per chunk).  out: [0] records (the write pass), [1] the chain's end
// position, [2] error kind, [3] error position, [4] the fix rounds' changed flag, [5] lo, [6] hi.
struct ChainArgs {
    int64_t first, chunk, n_chunks;
    int64_t n_bits;                   // positions the bitmap covers (records start before first + n_bits)
    uint32_t* bits;                   // bit (pos - first): a position the speculated walk visited
    int64_t* ent;                     // the entry each chunk's result was computed from
    int64_t* spec_exit;               // exit of the speculated walk
    int64_t* spec_cnt;                // records of the speculated walk
    uint32_t* cnt;                    // records starting in the chunk (given ent)
    int64_t* out;
};

__device__ __forceinline__ int64_t chunk_begin(const ChainArgs& c, int64_t k) { return c.first + k * c.chunk; }
__device__ __forceinline__ int64_t chunk_end(const ChainArgs& c, int64_t k) {
    return k + 1 >= c.n_chunks ? kChainStop : c.first + (k + 1) * c.chunk;   // the last chunk holds the rest
}

__device__ __forceinline__ bool chain_bit(const ChainArgs& c, int64_t pos) {
    const int64_t i = pos - c.first;
    return i < c.n_bits && ((c.bits[i >> 5] >> (i & 31)) & 1u);
}

// Visited positions of chunk k's speculated walk in [chunk start, pos).
__device__ __forceinline__ int64_t chain_rank(const ChainArgs& c, int64_t k, int64_t pos) {
    const int64_t i0 = k * c.chunk, i1 = pos - c.first;   // chunk starts are 32-bit aligned (chunk % 32 == 0)
    int64_t n = 0;
    for (int64_t w = i0 >> 5; w < (i1 >> 5); w++) n += __popc(c.bits[w]);
    if (i1 & 31) n += __popc(c.bits[i1 >> 5] & ((1u << (i1 & 31)) - 1u));
    return n;
}

// The true chain's first records: the plausible length range [lo, hi] for the speculation.
template <typename Step>
__device__ __forceinline__ void chain_sample_run(const Step& s, const ChainArgs& c, int n_max) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int64_t pos = c.first;
    int64_t lo = 0x7fffffff, hi = 0;
    for (int k = 0; k < n_max && pos != kChainStop; k++) {
        const ChainStep r = s.at(pos);
        if (r.len <= 0) break;
        lo = r.len < lo ? r.len : lo;
        hi = r.len > hi ? r.len : hi;
        pos = r.next;
    }
    c.out[5] = lo > hi ? 1 : lo;
    c.out[6] = hi;
}

// Whether pos starts kChainHops records of plausible lengths (or records running into the chain's end).
template <typename Step>
__device__ __forceinline__ bool chain_plausible(const Step& s, int64_t pos, int64_t lo, int64_t hi) {
    for (int h = 0; h < kChainHops; h++) {
        const ChainStep r = s.at(pos);
        if (r.len <= 0) return h > 0 && r.err == 0;
        if (r.len < lo || r.len > hi) return false;
        if (r.next == kChainStop) return true;
        pos = r.next;
    }
    return true;
}

template <typename Step>
__device__ __forceinline__ void chain_spec_run(const Step& s, const ChainArgs& c) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n_chunks) return;
    const int64_t b = chunk_begin(c, k), e = chunk_end(c, k);
    int64_t entry = b;
    if (k > 0) {
        const int64_t lo = c.out[5], hi = c.out[6];
        for (int i = 0; i < kChainSearch && b + i < e; i++)
            if (chain_plausible(s, b + i, lo, hi)) { entry = b + i; break; }
    }
    // the walk: visited positions into the chunk's bitmap words (this lane's alone), one store per word
    int64_t pos = entry, n = 0, wi = -1;
    uint32_t wv = 0;
    while (pos < e) {
        const ChainStep r = s.at(pos);
        if (r.len <= 0) { pos = kChainStop; break; }
        const int64_t i = pos - c.first;
        if ((i >> 5) != wi) {
            if (wi >= 0) c.bits[wi] = wv;
            wi = i >> 5;
            wv = 0;
        }
        wv |= 1u << (i & 31);
        n++;
        pos = r.next;
    }
    if (wi >= 0) c.bits[wi] = wv;
    c.ent[k] = entry;
    c.spec_exit[k] = pos;
    c.spec_cnt[k] = n;
    c.cnt[k] = (uint32_t)n;
}

// Chunk k framed from `in` (its predecessor's exit): walked until the speculated walk's positions are
// reached.  Returns the exit; *n the chunk's records.
template <typename Step>
__device__ __forceinline__ int64_t chain_refit(const Step& s, const ChainArgs& c, int64_t k, int64_t in, int64_t* n) {
    const int64_t e = chunk_end(c, k);
    int64_t pos = in, f = 0;
    while (pos < e) {
        if (chain_bit(c, pos)) { *n = f + c.spec_cnt[k] - chain_rank(c, k, pos); return c.spec_exit[k]; }
        const ChainStep r = s.at(pos);
        if (r.len <= 0) { *n = f; return kChainStop; }
        f++;
        pos = r.next;
    }
    *n = f;
    return pos;
}

// One fix round: exits read from ex_in (the previous round's), written to ex_out.
template <typename Step>
__device__ __forceinline__ void chain_fix_run(const Step& s, const ChainArgs& c, const int64_t* ex_in, int64_t* ex_out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n_chunks) return;
    const int64_t old = ex_in[k];
    if (k == 0) { ex_out[0] = old; return; }
    const int64_t in = ex_in[k - 1];
    if (in == c.ent[k]) { ex_out[k] = old; return; }
    int64_t n = 0;
    const int64_t x = chain_refit(s, c, k, in, &n);
    c.ent[k] = in;
    c.cnt[k] = (uint32_t)n;
    ex_out[k] = x;
    if (x != old) __hip_atomic_store(c.out + 4, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The settle pass: chunks in order, one lane (what the fix rounds left: a ripple longer than them).
template <typename Step>
__device__ __forceinline__ void chain_settle_run(const Step& s, const ChainArgs& c, int64_t* ex) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int64_t k = 1; k < c.n_chunks; k++) {
        const int64_t in = ex[k - 1];
        if (in == c.ent[k]) continue;
        int64_t n = 0;
        ex[k] = chain_refit(s, c, k, in, &n);
        c.ent[k] = in;
        c.cnt[k] = (uint32_t)n;
    }
}

// Records of chunk k at base[k] (exclusive scan of cnt), at most capacity of them; the chunk where the
// chain ends records its end position and error.
template <typename Step>
__device__ __forceinline__ void chain_write_run(const Step& s, const ChainArgs& c, const int64_t* base, int64_t capacity,
                                                int64_t* rec_off, int32_t* rec_len) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n_chunks) return;
    const int64_t e = chunk_end(c, k);
    int64_t pos = c.ent[k], j = base[k];
    while (pos < e) {
        const ChainStep r = s.at(pos);
        if (r.len <= 0) {   // the chain's end (one chunk holds it)
            c.out[1] = pos;
            if (r.err) { c.out[2] = r.err; c.out[3] = pos; }
            break;
        }
        if (j < capacity) { rec_off[j] = pos; rec_len[j] = r.len; }
        j++;
        if (r.next == kChainStop) { c.out[1] = pos + r.len; break; }
        pos = r.next;
    }
    if (k == c.n_chunks - 1) c.out[0] = base[k] + c.cnt[k];
}

// The passes as kernels of the library (the specialised var-occurs framing wraps the same bodies in
// its own extern "C" kernels, cbx_capi.hip: jit_chain_source).
template <typename Step>
__global__ void chain_sample(Step s, ChainArgs c, int n_max) { chain_sample_run(s, c, n_max); }
template <typename Step>
__global__ void chain_spec(Step s, ChainArgs c) { chain_spec_run(s, c); }
template <typename Step>
__global__ void chain_fix(Step s, ChainArgs c, const int64_t* ex_in, int64_t* ex_out) { chain_fix_run(s, c, ex_in, ex_out); }
template <typename Step>
__global__ void chain_settle(Step s, ChainArgs c, int64_t* ex) { chain_settle_run(s, c, ex); }
template <typename Step>
__global__ void chain_write(Step s, ChainArgs c, const int64_t* base, int64_t capacity, int64_t* rec_off, int32_t* rec_len) {
    chain_write_run(s, c, base, capacity, rec_off, rec_len);
}

}  // namespace cbx
