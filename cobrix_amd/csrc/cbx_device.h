// cbx_device.h -- device-side building blocks of the decode hot path, shared by the
// interpreter kernel (cbx_kernels.hip: plan tables read at run time) and the per-copybook
// specialised kernels compiled at run time with hipRTC (cbx_jit.cpp: the same functions with the
// op records as compile-time constants).  See cbx_kernels.hip for the work decomposition.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "cbx_internal.h"

// Diagnostic builds only (tools/build_variant.py . NAME -DCBX_DIAG=N): bit 0 drops the numeric
// validity / deferral stores, bit 1 the numeric value stores, bit 2 has one lane store a word (not
// all 64) -- to price the stores.  The product build is 0.
#ifndef CBX_DIAG
#define CBX_DIAG 0
#endif

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

// Plan-table and column pointers are plain (generic) pointers; stores through them would be
// `flat_*` instructions, which also count in lgkmcnt -- every later LDS / scalar-load wait
// would then wait for those stores to reach memory.  gp() re-qualifies them as global.
#define CBX_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ CBX_GLOBAL T* gp(T* p) { return (CBX_GLOBAL T*)p; }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Whole-line output stores (numeric values, string views, Utf8 offsets: 4-16 bytes per lane of 64
// consecutive lanes, written once, never read back by the decode) are nontemporal: SYN200 (C2) 4.63
// -> 4.38 ms, measured same-box (env A/B: CBX_JIT_DEFINES=CBX_NO_NT_STORES).  String payloads keep
// plain stores (st_pay): their pieces cover parts of lines that the L2 merges with the neighbouring
// values' pieces -- nontemporal there made SYNSTR200's views decode 10 % slower (5.32 -> 5.85 ms).
template <typename T>
__device__ __forceinline__ void st_out(CBX_GLOBAL T* p, T v) {
#ifdef CBX_NO_NT_STORES
    *p = v;
#else
    __builtin_nontemporal_store(v, p);
#endif
}
template <typename T>
__device__ __forceinline__ void st_pay(CBX_GLOBAL T* p, T v) {
#ifdef CBX_NT_PAYLOAD   // (A/B)
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
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

// FixedLenNestedRowIterator.getSegmentId / VRLRecordReader.getSegmentId (VRLRecordReader.scala:188-198):
// extractPrimitiveField(field, record, start_off).toString.trim, looked up in the segment map's
// keys.  Returns the key index, -1 when no key matches.  A string field is compared as trimmed
// UTF-8 text; an integral field by value (its decimal text equals a key exactly when the key is
// that integer written canonically); a null value is the empty id "".
// Every read of the map is indexed by wave-uniform values (scalar loads): a per-lane index would
// make it a vector load, and its wait inside the decode loop would also cover the prefetched tile.
__device__ int segment_key(const CBX_CONST cbx_segment_map* m, const uint32_t* lut, const CBX_CONST Field* fields,
                           const uint8_t* rec, int avail, int start_off) {
    int o = start_off + m->field_offset;
    int found = -1;
    if (m->field_is_int) {
        const Field f = ldc(fields + m->field);
        Val v = null_val();
        if (o + f.size <= avail) v = decode_count_int(f, rec + o);
        for (int k = m->n_keys - 1; k >= 0; k--) {   // the first matching key wins
            if (v.valid ? (m->key_is_int[k] && m->key_int[k] == (int64_t)v.lo) : m->key_len[k] == 0) found = k;
        }
        return found;
    }
    int n = m->field_size;
    if (o > avail) o = avail;
    if (o + n > avail) n = avail - o;
    if (n < 0) n = 0;
    const uint8_t* p = rec + o;
    int b = 0, e = n;
    while (b < e && (lut[p[b]] >> 31)) b++;
    while (e > b && (lut[p[e - 1]] >> 31)) e--;
    // keys are stored as UTF-8 (key[k][] holds bytes, key_len[k] their count); each lane walks its
    // trimmed field's UTF-8 bytes in step with the key position
    for (int k = 0; k < m->n_keys; k++) {
        const int kl = m->key_len[k];
        int i = b, j = 0;
        bool eq = found < 0;
        for (int pos = 0; pos < kl; pos++) {
            // dword reads (there is no 16-bit scalar load): key rows are dword aligned
            const uint32_t kw = ((const CBX_CONST uint32_t*)m->key[k])[pos >> 1];
            const uint32_t kb = (pos & 1) ? kw >> 16 : kw & 0xFFFF;
            uint32_t en = 0;
            while (eq && i < e && ((en = lut[p[i]]) >> 24 & 3) == 0) i++;   // characters with no output bytes
            if (eq) {
                if (i >= e || ((en >> (8 * j)) & 0xFF) != kb) eq = false;
                else if (++j >= (int)((en >> 24) & 3)) { j = 0; i++; }
            }
        }
        while (eq && i < e && ((lut[p[i]] >> 24) & 3) == 0) i++;
        if (eq && i == e) found = k;
    }
    return found;
}

__device__ __forceinline__ int segment_of(const KernelArgs& a, const uint32_t* lut, const uint8_t* rec, int avail) {
    const int k = segment_key(a.segmap, lut, a.fields, rec, avail, a.start_off);
    int seg = -1;
    for (int j = 0; j < a.segmap->n_keys; j++) {
        int ks = a.segmap->key_segment[j];
        asm volatile("" : "+s"(ks));   // a scalar load: keeps the compiler from folding the select into a lane-indexed load
        seg = k == j ? ks : seg;
    }
    return seg;
}

__device__ __forceinline__ void store_value(const DevColumn& c, int out_type, int64_t v, const Val& x) {
    switch (out_type) {
    case CBX_O_I32: gp((int32_t*)c.values)[v] = (int32_t)x.lo; break;
    case CBX_O_F32: gp((uint32_t*)c.values)[v] = (uint32_t)x.lo; break;
    case CBX_O_DEC128: gp((uint64_t*)c.values)[2 * v] = x.lo; gp((uint64_t*)c.values)[2 * v + 1] = x.hi; break;
    default: gp((uint64_t*)c.values)[v] = x.lo; break;
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
                                            uint32_t rec_addr, const uint32_t* s_lut, bool& ok, bool fast,
                                            uint32_t ev[kStrFastBytes]) {
    bool el = t.active && (op.segment < 0 || op.segment == t.seg);
    if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
    const int o = a.start_off + op.eo;
    ok = el && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    auto lutf = [&](uint32_t b) { return str_lut(op.kind, s_lut, b); };
    if (fast) {
        uint32_t w[8];
        img_bytes32(src, rec_addr + (ok ? (uint32_t)op.eo : 0u), op.size, w);
        lut_entries32(w, op.size, lutf, ev);
        return string_span32e(op.trim, ev, n, op.size);
    }
    StrSpan sp{0, 0, 0};
    if (ok) sp = string_span(op.kind, op.trim, src + rec_addr + (uint32_t)op.eo, n, lutf);
    return sp;
}

__device__ __forceinline__ bool sop_fast(const StrOp& op, bool global) {
    return !global && op.size <= kStrFastBytes && (op.kind == CBX_K_STRING || op.kind == CBX_K_STRING_ASCII);
}

// Value of record (tile * 64 + lane) of a slot row: the tile's row base is wave-uniform (scalar
// registers) and the lane offset a 32-bit vector offset, so the store takes the saddr form.
template <int W>
__device__ __forceinline__ void store_w(void* values, int64_t tile, int lane, const Val& x, int out_type) {
    const int w = W ? W : (out_type == CBX_O_I32 || out_type == CBX_O_F32 ? 4 : out_type == CBX_O_DEC128 ? 16 : 8);
    if (w == 4) st_out(gp((uint32_t*)values) + tile * kWave + lane, (uint32_t)x.lo);
    else if (w == 8) st_out(gp((uint64_t*)values) + tile * kWave + lane, x.lo);
    else st_out(gp((u32x4*)values) + tile * kWave + lane, u32x4{(uint32_t)x.lo, (uint32_t)(x.lo >> 32), (uint32_t)x.hi, (uint32_t)(x.hi >> 32)});
}

// Where a numeric op's validity / deferral word of a tile goes.  DirectSink: a wave ballot stored
// by every lane to its address (8 bytes per (op, tile)).  VWords: gathered in lanes over a run of
// kVRun consecutive tiles and stored 64 bytes at a time (VWords::flush) -- one 8-byte store per
// (word, tile) cost the SYN200 kernel a fifth of its time (4.78 -> 3.85 ms without them, measured).
struct DirectSink {
    __device__ __forceinline__ void valid(const NumCall& c, int, int64_t tile, uint64_t m) const {
        if (!(CBX_DIAG & 4) || __builtin_amdgcn_mbcnt_lo(~0u, 0u) == 0) gp(c.validity)[tile] = m;   // (diag 4: one lane stores)
    }
    __device__ __forceinline__ void defer(const NumCall& c, int, int64_t tile, uint64_t m) const {
        if (c.defer && (!(CBX_DIAG & 4) || __builtin_amdgcn_mbcnt_lo(~0u, 0u) == 0)) gp(c.defer)[tile] = m;
    }
    __device__ __forceinline__ void svalid(const StrCall& c, int, int64_t tile, uint64_t m) const { gp(c.validity)[tile] = m; }
};

constexpr int kVRun = 8;   // consecutive tiles per run of a wave (the words of 8 tiles = 64 bytes)

// NV VGPR pairs: word w of the run's tile j sits in lane 8 (w % 8) + j of pair w / 8.  Validity
// words are numbered by op (NNUM ops), deferral words follow (NNUM + deferral sequence, NDEF of
// them), then the string elements' validity words (NNUM + NDEF + string op).  Every
// index is a compile-time constant after inlining (specialised kernels), so the pairs stay in
// registers.
template <int NV, int NNUM, int NDEF = 0>
struct VWords {
    uint32_t lo[NV], hi[NV];
    int j;   // the current tile's place in its run
    __device__ __forceinline__ void put(int w, uint64_t m) {
        // v_writelane: the wave-uniform word from SGPRs into one lane (a lane compare + select per
        // word costs ~20 VGPRs more: 174 -> 191, below 3 waves per SIMD).  The lane select goes
        // through M0: with both operands in SGPRs gfx950 rejects the instruction (constant bus).
        const int reg = w >> 3;
        const int ln = __builtin_amdgcn_readfirstlane(((w & 7) << 3) | j);   // provably uniform: an SGPR
        const uint32_t mlo = __builtin_amdgcn_readfirstlane((uint32_t)m), mhi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
        asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(lo[reg]) : "s"(mlo), "s"(ln) : "m0");
        asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(hi[reg]) : "s"(mhi), "s"(ln) : "m0");
    }
    __device__ __forceinline__ void valid(const NumCall&, int i, int64_t, uint64_t m) { put(i, m); }
    __device__ __forceinline__ void defer(const NumCall&, int d, int64_t, uint64_t m) { if (d >= 0) put(NNUM + d, m); }
    __device__ __forceinline__ void svalid(const StrCall&, int i, int64_t, uint64_t m) { put(NNUM + NDEF + i, m); }
    // the run starting at tile t0: lanes 8k..8k+7 of pair r store word 8r + k of its tiles (64 B)
    // own: the words this wave gathered (a cooperative tile's waves each flush their own ops' words)
    // The 8 word pointers of a pair come from scalar loads (the word index is a compile-time constant
    // per k) and are selected per lane: a per-lane load of the pointer table was a vector load whose
    // wait (vmcnt(0), in issue order) also waited for every value store of the tile before it.
    __device__ __forceinline__ static uint64_t* word_ptr(const KernelArgs& a, int w) {
        return w < NNUM ? ldc(a.ncall + w).validity
             : w < NNUM + NDEF ? a.defer_bits + (int64_t)(w - NNUM) * a.n_tiles
                               : ldc(a.scall + (w - NNUM - NDEF)).validity;
    }
    __device__ __forceinline__ void flush(const KernelArgs& a, int n_words, int64_t t0, int lane, uint64_t own = ~0ull) {
        const int jj = lane & 7;
        const int kk = lane >> 3;
#pragma unroll
        for (int r = 0; r < NV; r++) {
            uint64_t* p = nullptr;
            bool mine = false;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int w = 8 * r + k;
                if (w < n_words && ((own >> (w & 63)) & 1)) {
                    uint64_t* q = word_ptr(a, w);
                    p = kk == k ? q : p;
                    mine |= kk == k;
                }
            }
            if (mine && t0 + jj < a.n_tiles) gp(p)[t0 + jj] = ((uint64_t)hi[r] << 32) | lo[r];
        }
    }
};

// One batch of numeric ops (same decoder variant V, output width W).  Decoding is branch-free
// per lane: every lane reads its (clamped) element and computes, the bounds / segment / OCCURS
// conditions only select validity.  The validity (and deferral) word of each op goes to the sink.
template <int V, int W, bool kOdo, bool kGlobal, typename Sink>
__device__ __forceinline__ void num_one(const KernelArgs& a, const NumOp& op, int i, const TileCtx& t,
                                        bool ok, uint64_t r1, uint64_t r0, const int32_t* s_cnt, int lane, Sink& sk) {
    if (op.segment >= 0) ok &= op.segment == t.seg;
    if (kOdo) ok &= odo_present(a.nops + i, op.n_odo, s_cnt, lane);
    Val x = null_val();
    bool defer = false;
    if (kGlobal || V == V_GENERIC) {
        defer = ok;
    } else {
        if (V == V_BCD8) x = bcd8_raw<W>(op, r1);
        else if (V == V_BCD16) x = bcd16_raw<W>(op, r1, r0);
        else if (V == V_BIN8) x = bin8_raw<W>(op, r1);
        else if (V == V_ZONED16) { x = zoned16_raw<W>(op, r1, r0, defer); defer &= ok; }
        else if (V == V_FP) x = fp_raw(op, r1);
        x.valid &= ok;
    }
    const NumCall c = ldc(a.ncall + i);
    // every lane stores (slot rows are padded to 64 * n_tiles values): no exec-mask branches
    if (!(CBX_DIAG & 2)) store_w<W>(c.values, t.tile, lane, x, op.out_type);
    const uint64_t m = __ballot(x.valid);
    if (!(CBX_DIAG & 1)) sk.valid(c, i, t.tile, m);
    if ((V == V_ZONED16 || V == V_GENERIC || kGlobal) && !(CBX_DIAG & 1)) sk.defer(c, op.defer, t.tile, __ballot(defer));
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
    DirectSink ds;
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
        for (int u = 0; u < U; u++) num_one<V, W, kOdo, kGlobal>(a, op[u], i + u, t, ok[u], r1[u], r0[u], s_cnt, lane, ds);
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
        num_one<V, W, kOdo, kGlobal>(a, op, i, t, ok, r1, r0, s_cnt, lane, ds);
    }
}

// Element r of an OCCURS run op (NumOp.run): offset, slot row, deferral row and innermost ODO
// index advance with r; otherwise num_one.
template <int V, int W, bool kOdo>
__device__ __forceinline__ void run_elem(const KernelArgs& a, const NumOp& op, const CBX_CONST NumOp* opp, const NumCall& c,
                                         int r, const TileCtx& t, bool ok, uint64_t r1, uint64_t r0, const int32_t* s_cnt,
                                         int lane) {
    if (op.segment >= 0) ok &= op.segment == t.seg;
    if (kOdo) {
        // ODO levels read through the op pointer (indexing the local copy would force it to scratch)
        for (int j = 0; j < op.n_odo; j++) {
            const int idx = opp->odo_idx[j] + (j == op.n_odo - 1 && op.run_odo ? r : 0);
            ok &= idx < s_cnt[opp->odo_arr[j] * kWave + lane];
        }
    }
    Val x = null_val();
    bool defer = false;
    if (V == V_GENERIC) {
        defer = ok;
    } else {
        if (V == V_BCD8) x = bcd8_raw<W>(op, r1);
        else if (V == V_BCD16) x = bcd16_raw<W>(op, r1, r0);
        else if (V == V_BIN8) x = bin8_raw<W>(op, r1);
        else if (V == V_ZONED16) { x = zoned16_raw<W>(op, r1, r0, defer); defer &= ok; }
        else if (V == V_FP) x = fp_raw(op, r1);
        x.valid &= ok;
    }
    const int w = W ? W : (op.out_type == CBX_O_I32 || op.out_type == CBX_O_F32 ? 4 : op.out_type == CBX_O_DEC128 ? 16 : 8);
    store_w<W>(c.values + (int64_t)r * a.pitch * w, t.tile, lane, x, op.out_type);
    const uint64_t m = __ballot(x.valid);
    gp(c.validity + (int64_t)r * a.n_tiles)[t.tile] = m;
    if (V == V_ZONED16 || V == V_GENERIC) {
        const uint64_t dm = __ballot(defer);
        if (c.defer) gp(c.defer + (int64_t)r * a.n_tiles)[t.tile] = dm;
    }
}

constexpr int kRunU = 4;   // run elements decoded per step (reads first)

// A batch holding OCCURS runs: per op, its elements kRunU at a time (reads first).
template <int V, int W, bool kOdo>
__device__ __forceinline__ void run_batch(const KernelArgs& a, const Batch& b, const TileCtx& t, const uint8_t* src,
                                          uint32_t rec_addr, const int32_t* s_cnt, int lane) {
    constexpr bool kWide = V == V_BCD16 || V == V_ZONED16;
    constexpr bool kRead = V != V_GENERIC;
    const int lim = t.active ? t.avail - a.start_off : -1;
    for (int i = b.begin; i < b.end; i++) {
        const NumOp op = ldc(a.nops + i);
        const NumCall c = ldc(a.ncall + i);
        const int run = op.run > 1 ? op.run : 1;
        for (int r0 = 0; r0 < run; r0 += kRunU) {
            bool ok[kRunU];
            uint64_t q1[kRunU], q0[kRunU];
#pragma unroll
            for (int u = 0; u < kRunU; u++) {
                const int eo = op.eo + (r0 + u) * op.run_stride;
                ok[u] = r0 + u < run && eo + op.size <= lim;
                q1[u] = q0[u] = 0;
                if (kRead) {
                    const uint32_t end = rec_addr + (ok[u] ? (uint32_t)eo : 0u) + op.size;
                    q1[u] = img_le64_ending(src, end);
                    if (kWide) q0[u] = img_le64_ending(src, end - 8);
                }
            }
#pragma unroll
            for (int u = 0; u < kRunU; u++)
                if (r0 + u < run) run_elem<V, W, kOdo>(a, op, a.nops + i, c, r0 + u, t, ok[u], q1[u], q0[u], s_cnt, lane);
        }
    }
}

// A group of N <= 4 numeric ops with the op records known at compile time (the specialised
// kernels of cbx_jit.h): the interpreter's batch step with every descriptor field folded.
template <int V, int W, bool kOdo, int N, typename Sink>
__device__ __forceinline__ void num_group(const KernelArgs& a, const NumOp (&op)[N], int i0, const TileCtx& t,
                                          const uint8_t* src, uint32_t rec_addr, const int32_t* s_cnt, int lane, Sink& sk) {
    constexpr bool kWide = V == V_BCD16 || V == V_ZONED16;
    constexpr bool kRead = V != V_GENERIC;
    const int lim = t.active ? t.avail - a.start_off : -1;
    bool ok[N];
    uint64_t r1[N], r0[N];
#pragma unroll
    for (int u = 0; u < N; u++) {
        ok[u] = op[u].eo + op[u].size <= lim;
        r1[u] = r0[u] = 0;
        if (kRead) {
            const uint32_t end = rec_addr + (ok[u] ? (uint32_t)op[u].eo : 0u) + op[u].size;
            r1[u] = img_le64_ending(src, end);
            if (kWide) r0[u] = img_le64_ending(src, end - 8);
        }
    }
#pragma unroll
    for (int u = 0; u < N; u++) num_one<V, W, kOdo, false>(a, op[u], i0 + u, t, ok[u], r1[u], r0[u], s_cnt, lane, sk);
}

// String-view layout (cbx_plan_options.string_views): the element's Arrow view -- length, then the
// UTF-8 bytes inline (<= 12, zero padded) or their first 4 bytes + data buffer index + offset.
// Payloads longer than 12 bytes are packed (wave scan) into the tile's region of the slot's data
// buffer: staged in LDS and copied out in 16-byte pieces when the tile's long payload fits the
// staging area, else written straight from the lanes.  Short payloads go to 16-byte LDS slots in
// front of the long ones (one scan places both: every lane takes 16 bytes or its length, so the
// area a plan sizes for 64 values of the field -- at least 1 KiB -- holds the tile) and into the
// view.  One pass, no scan across tiles, no placement kernel.
// Data buffer of a tile and a position in it (tiles_per_buf is a power of two: a shift, not a
// 64-bit division per element).
__device__ __forceinline__ uint32_t view_buf(int64_t tile, const StrCall& c) {
    return (uint32_t)(tile >> __builtin_ctzll((unsigned long long)c.tiles_per_buf));
}
__device__ __forceinline__ uint32_t view_pos(int64_t tile, const StrCall& c, uint32_t ex) {
    return (uint32_t)((tile & (c.tiles_per_buf - 1)) * c.tile_cap + ex);
}

template <typename Sink>
__device__ __forceinline__ void str_view_element(const KernelArgs& a, const StrOp& op, int i, const StrCall& c, const TileCtx& t,
                                                 const StrSpan& sp, bool ok, bool fast, const uint32_t (&ev)[kStrFastBytes],
                                                 const uint8_t* sp_src, const uint32_t* s_lut, uint8_t* s_str, int lane,
                                                 Sink& sk) {
    const int len = ok ? sp.utf8_len : 0;
    const bool lng = len > 12;
    // one scan: short slots counted above bit 20, long payload bytes below (<= 64 * 96 bytes)
    uint32_t both;
    const uint32_t exb = wave_excl_scan32(lng ? (uint32_t)len : (1u << 20), lane, both);
    const uint32_t ex = exb & 0xFFFFFu, tot = both & 0xFFFFFu, n_short = both >> 20;
    sk.svalid(c, i, t.tile, __ballot(ok));
    auto lutf = [&](uint32_t b) { return str_lut(op.kind, s_lut, b); };
    uint8_t* s_short = s_str + 16 * (exb >> 20);   // this lane's inline bytes
    uint8_t* s_long = s_str + 16 * n_short;        // the tile's long payloads, packed (16-aligned)
    // wave-uniform; always true for the register path (the plan sizes the staging area for it in
    // this layout), so its unrolled byte writes never target global memory
    const bool staged = fast || (int)(16 * n_short + tot) <= a.str_stage;
    uint8_t* region = c.scratch + t.tile * c.tile_cap;           // 16-byte aligned
    uint8_t* dump = s_str + a.str_stage + a.dump_stride * lane;
    if (!lng) *(u32x4*)s_short = u32x4{0u, 0u, 0u, 0u};   // inline bytes are zero padded
    if (lng && !staged) {
        if (fast) string_write32e(ev, sp, region + ex, dump, op.size, op.pad);
        else string_write(op.kind, sp_src, sp, region + ex, lutf);
    } else {
        uint8_t* dst = lng ? s_long + ex : s_short;
        if (fast) string_write32e(ev, sp, dst, dump, op.size, op.pad);
        else if (ok) string_write(op.kind, sp_src, sp, dst, lutf);
    }
    wave_sync_lds();
    if (staged) {
        const u32x4* s128 = (const u32x4*)s_long;
        for (int q = lane; 16 * q < (int)tot; q += kWave) gp((u32x4*)region)[q] = s128[q];
    }
    u32x4 v;
    if (!lng) {
        const u32x4 w = *(const u32x4*)s_short;
        v = u32x4{(uint32_t)len, w.x, w.y, w.z};
    } else {
        uint32_t pre;
        if (staged) {
            const uint32_t* q = (const uint32_t*)(s_long + (ex & ~3u));
            pre = align_bytes(q[1], q[0], ex & 3u);
        } else {
            // the lane's own bytes, written above through the vector memory path
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const CBX_GLOBAL uint8_t* g = gp(region + ex);
            pre = (uint32_t)g[0] | (uint32_t)g[1] << 8 | (uint32_t)g[2] << 16 | (uint32_t)g[3] << 24;
        }
        v = u32x4{(uint32_t)len, pre, view_buf(t.tile, c), view_pos(t.tile, c, ex)};
    }
    st_out(gp((u32x4*)c.views) + t.tile * kWave + lane, v);
    wave_sync_lds();   // the staging area is reused by the next element
}

// LDS reads at an LDS byte address (a 32-bit integer): typed address-space-3 loads, so the
// compiler emits no generic-to-LDS pointer conversion per read (torch's bundled compiler, the one the
// specialised kernels are built with, null-checks each such conversion: v_cmp + v_cndmask per read).
// lds_addr: the LDS address of a generic pointer into the workgroup's LDS (one conversion, hoisted).
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
template <typename T>
__device__ __forceinline__ T lds_ld(uint32_t addr) {
    return *(const __attribute__((address_space(3))) T*)(lds_cu8*)addr;
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(size_t)(lds_cu8*)p;
}

// Diagnostic (CBX_DIAG & 32, timing only, wrong values): a LUT read's address replaced by the lane's
// own bank (conflict-free), still issued after the address it replaces (one extra VALU) -- prices the
// LUT's bank conflicts.
__device__ __forceinline__ uint32_t diag_bank(uint32_t x) {
    asm volatile("v_and_b32 %0, 0, %0" : "+v"(x));
    return x | ((__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 31u) << 2);
}

// bits (byte k of w) & mask, one SDWA op (mask in a VGPR: SDWA takes no literal)
__device__ __forceinline__ uint32_t byte_and(uint32_t w, int k, uint32_t mask) {
    uint32_t r;
    switch (k) {
    case 0: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(mask), "v"(w)); break;
    case 1: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(mask), "v"(w)); break;
    case 2: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(mask), "v"(w)); break;
    default: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(mask), "v"(w)); break;
    }
    return r;
}

// (byte k of w) * 4: the byte offset of its 4-byte LUT entry, one SDWA shift
__device__ __forceinline__ uint32_t byte_x4(uint32_t w, int k) {
    uint32_t r;
    switch (k) {
    case 0: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w)); break;
    case 1: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w)); break;
    case 2: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w)); break;
    default: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w)); break;
    }
    return r;
}

// Lane-private LDS slot of a register-path element in the view layout: its UTF-8 bytes (<= size *
// width) + the bytes written past them (<= 3), rounded to 8 bytes with an odd count of 8-byte
// words -- lanes at the same position fall on different banks (2-way at most for the byte stores;
// the 8-byte read-backs conflict-free), where a 16-byte multiple put lanes 8 apart on one bank.
__host__ __device__ constexpr int str_lane_slot(int size, int width) {
    // an odd dword count: the lanes' byte stores at similar positions land on distinct banks
    // (ds_write_b8: bank (a / 4) mod 32), and the dword read-backs are conflict-free.  (Odd counts of
    // 8-byte words, read back as 8-byte words, left every byte store 2-way conflicted: 14 dwords
    // per lane.)  2-byte pages (str_lane_group2): the phase (<= 3 bytes), <= 8 bytes per group of 4
    // characters and the carried dword written past them.
    return width == 2 ? ((((3 + 8 * ((size + 3) / 4)) >> 2) + 1) | 1) << 2 : (((size * width + 3 + 3) >> 2) | 1) << 2;
}

// Pattern selectors of a group of 4 characters of a 2-byte code page (str_lane_group2): entry h (bit k
// = character k takes 2 UTF-8 bytes) lists, for v_perm over (U23, U01) -- character k's first UTF-8
// byte at source 2k, its second at 2k + 1 -- the first bytes in order with each wide character's
// second byte after its first, then zero bytes (0x0C).  Two dwords per entry, 16 entries.
__host__ __device__ constexpr uint32_t group_sel(int i) {
    const int h = i >> 1;
    uint64_t v = 0x0C0C0C0C0C0C0C0Cull;   // the 8 selector bytes (no array: a run-time i indexed one in scratch)
    int n = 0;
    for (int k = 0; k < 4; k++) {
        v = (v & ~(0xFFull << (8 * n))) | ((uint64_t)(2 * k) << (8 * n));
        n++;
        if ((h >> k) & 1) {
            v = (v & ~(0xFFull << (8 * n))) | ((uint64_t)(2 * k + 1) << (8 * n));
            n++;
        }
    }
    return (uint32_t)(v >> (32 * (i & 1)));
}

// The code page LUT and the group selectors into the workgroup's LDS (kLutLds bytes at lut).
__device__ __forceinline__ void lut_lds_fill(const KernelArgs& a, uint32_t* lut) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = a.lut[i];
    if (threadIdx.x < 32) lut[256 + threadIdx.x] = group_sel((int)threadIdx.x);
}

// The view layout's register-path string element (fields of <= kStrFastBytes EBCDIC / ASCII bytes,
// StringDecoders.decodeEbcdicString / decodeAsciiString + StringTools.trim*): every byte's LUT
// entry once, the trim range from the entries' trim bits, then the UTF-8 bytes written at running
// positions into the lane's own LDS slot -- a byte outside the range adds no length, so its writes
// land where the next kept byte's go, or past the end.  No cross-lane staging and no wave barrier:
// the lane builds its view from its slot, and a long payload (> 12 bytes) goes from registers to the
// tile's region at a 4-byte-aligned packed position (exact dword counts, so lanes never overlap).
constexpr int kStrNC = (kStrFastBytes * 3 + 15) / 16;   // 16-byte words of a lane slot's read-back

// The lane's field of a register-path view element: bytes [eo, eo + n) of its record (n <= size
// <= smax; smax bounds the unrolled loops), composed in the lane's slot and read back into q.
// Returns the UTF-8 length.
__device__ __forceinline__ int str_lane_compose(int kind, int trim, int width, int smax, int eo, int n, bool ok,
                                                const uint8_t* src, uint32_t rec_addr, const uint32_t* s_lut,
                                                uint8_t* s_str, int lane, u32x4 (&q)[kStrNC], bool zero_tail = true);

// Single-byte code pages: the kept bytes [b, e) are the mapped bytes shifted down by b -- packed
// into dwords, a 3-stage dword shift by b / 4 and one byte align, in registers (no LDS).
__device__ __forceinline__ int str_lane_shift(int smax, const uint32_t (&ev)[kStrFastBytes], int b, int e,
                                              u32x4 (&q)[kStrNC]) {
    uint32_t s[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint32_t v = 0;
        if (k < 8) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (4 * k + u < smax) v |= (ev[4 * k + u] & 0xFFu) << (8 * u);
        }
        s[k] = v;
    }
    // the stages as bit blends on sbfe masks (0 / ~0): written as selects, the compiler turned the
    // network into a lane-indexed array in scratch
    const int qd = b >> 2;
    const uint32_t m4 = (uint32_t)__builtin_amdgcn_sbfe(qd, 2, 1), m2 = (uint32_t)__builtin_amdgcn_sbfe(qd, 1, 1),
                   m1 = (uint32_t)__builtin_amdgcn_sbfe(qd, 0, 1);
#pragma unroll
    for (int k = 0; k < 12; k++) s[k] = (s[k + 4] & m4) | (s[k] & ~m4);
#pragma unroll
    for (int k = 0; k < 10; k++) s[k] = (s[k + 2] & m2) | (s[k] & ~m2);
#pragma unroll
    for (int k = 0; k < 9; k++) s[k] = (s[k + 1] & m1) | (s[k] & ~m1);
    const int len = e - b;
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t x = __builtin_amdgcn_alignbyte(s[k + 1], s[k], (uint32_t)(b & 3));
        const int r = len - 4 * k;   // bytes of this dword inside the value
        o[k] = r >= 4 ? x : r <= 0 ? 0u : x & ((1u << (8 * r)) - 1u);
    }
    q[0] = u32x4{o[0], o[1], o[2], o[3]};   // <= 32 bytes: the other words are never read (cap)
    q[1] = u32x4{o[4], o[5], o[6], o[7]};
    return len;
}

// 2-byte code pages (every character 1 or 2 UTF-8 bytes: cp037, cp500, cp875, ...): the field's
// UTF-8 bytes composed 4 characters at a time in registers and placed in the lane's LDS slot with
// dword stores only.  A group's characters give two dwords of byte pairs (U01, U23: first byte, then
// the second one or 0); one pattern selector (group_sel: which of the 4 are wide) and two v_perm
// compact them to the group's 4..8 bytes; the group lands at its running byte position through a
// 64-bit shift, OR-ed into the partial dword carried from the previous group, as one 2-dword store
// at a dword boundary.  The untrimmed field is composed (a trimmed leading character is <= U+0020,
// one UTF-8 byte), starting at phase (-b) & 3, so the kept bytes [b, e) begin on a dword and are
// read back packed from byte 0.  Per group, from the 4 entries' byte 3 gathered into one dword (two
// v_perm: trim flag bit 7, UTF-8 length bits 0-1 per byte): the selector's byte offset and the
// group's byte count as one v_dot4 each.  Every group's selector is read before the first slot
// store (the reads do not wait behind the stores).  zero_tail: the bytes of q[0] past the value
// zeroed (a short string view inlines them; the Utf8 store writes exactly len bytes and skips it).
// Read-backs past the lane's slot (dwords beyond the value) land in the next lane's slot or read 0
// past the workgroup's LDS -- never part of a value.
constexpr int kStrNG = (kStrFastBytes + 3) / 4;   // groups of 4 characters of a register-path field

// The placement half of the 2-byte compose: groups g < ceil(smax / 4) (byte pairs u01 / u23, byte
// count nb, selector sel) into the lane's slot from phase (-b) & 3, the kept bytes read back into q.
// The groups alone, from slot byte s0 on.
__device__ __forceinline__ void group2_put(int smax, const uint32_t (&u01)[kStrNG], const uint32_t (&u23)[kStrNG],
                                           const uint32_t (&nb)[kStrNG], const uint2 (&sel)[kStrNG], uint32_t s0,
                                           uint8_t* slot) {
    uint32_t carry = 0, pos = s0;
#pragma unroll
    for (int g = 0; g < kStrNG; g++) {
        if (4 * g >= smax) break;
        const uint32_t lo = __builtin_amdgcn_perm(u23[g], u01[g], sel[g].x), hi = __builtin_amdgcn_perm(u23[g], u01[g], sel[g].y);
        const uint32_t k8 = 8u * (pos & 3u);
        const uint64_t v = (((uint64_t)hi << 32) | lo) << k8;
        const uint32_t w0 = (uint32_t)v | carry, w1 = (uint32_t)(v >> 32);
        const uint32_t w2 = (uint32_t)(((uint64_t)hi << k8) >> 32);   // the group's bytes past w1 (k8 > 0)
        uint32_t* d = (uint32_t*)(slot + (pos & ~3u));
        d[0] = w0;
        d[1] = w1;
        const uint32_t np = pos + nb[g];
        const uint32_t dd = (np >> 2) - (pos >> 2);   // 1 or 2 for 4 characters (>= 4 bytes); 0 too for a last partial group
        carry = dd == 2u ? w2 : (4 * g + 4 <= smax || dd == 1u) ? w1 : w0;
        pos = np;
    }
    *(uint32_t*)(slot + (pos & ~3u)) = carry;
}

__device__ __forceinline__ void group2_place(int smax, const uint32_t (&u01)[kStrNG], const uint32_t (&u23)[kStrNG],
                                             const uint32_t (&nb)[kStrNG], const uint2 (&sel)[kStrNG], int b, int len,
                                             uint8_t* slot, u32x4 (&q)[kStrNC], bool zero_tail) {
    const uint32_t s0 = (uint32_t)(-b) & 3u;
    group2_put(smax, u01, u23, nb, sel, s0, slot);
    // the kept bytes, packed from byte 0
    const uint32_t* sd = (const uint32_t*)slot + ((s0 + (uint32_t)b) >> 2);
#pragma unroll
    for (int k = 0; k < kStrNC; k++) {
        if (16 * k < 2 * smax) {
            uint32_t d4[4];
#pragma unroll
            for (int m = 0; m < 4; m++) d4[m] = 16 * k + 4 * m < 2 * smax ? sd[4 * k + m] : 0u;
            if (k == 0 && zero_tail) {
                // a short string view inlines these dwords: zero the bytes past the value (the
                // slot holds the untrimmed field there)
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    const int r = len - 4 * m;
                    d4[m] = r >= 4 ? d4[m] : r <= 0 ? 0u : d4[m] & ((1u << (8 * r)) - 1u);
                }
            }
            q[k] = u32x4{d4[0], d4[1], d4[2], d4[3]};
        }
    }
}

__device__ __forceinline__ uint2 group2_sel(uint32_t so) {
    const uint64_t sv = lds_ld<uint64_t>(1024u + so);   // the selectors after the LUT (lut_lds_fill; the LUT at LDS 0)
    return make_uint2((uint32_t)sv, (uint32_t)(sv >> 32));
}

__device__ __forceinline__ int str_lane_group2(int smax, const uint32_t (&ev)[kStrFastBytes], int b, int e,
                                               uint8_t* slot, u32x4 (&q)[kStrNC], bool zero_tail = true) {
    uint32_t u01[kStrNG], u23[kStrNG], nb[kStrNG];
    uint2 sel[kStrNG];
    uint32_t wide = 0;   // bit j: character j is 2 UTF-8 bytes
#pragma unroll
    for (int g = 0; g < kStrNG; g++) {
        if (4 * g >= smax) break;
        const uint32_t e0 = ev[4 * g], e1 = 4 * g + 1 < smax ? ev[4 * g + 1] : 0u;
        const uint32_t e2 = 4 * g + 2 < smax ? ev[4 * g + 2] : 0u, e3 = 4 * g + 3 < smax ? ev[4 * g + 3] : 0u;
        u01[g] = __builtin_amdgcn_perm(e1, e0, 0x05040100u);   // c0.b0 c0.b1 c1.b0 c1.b1
        u23[g] = __builtin_amdgcn_perm(e3, e2, 0x05040100u);
        const uint32_t lb = __builtin_amdgcn_perm(e1, e0, 0x0C0C0703u) | __builtin_amdgcn_perm(e3, e2, 0x07030C0Cu);
        const uint32_t so = __builtin_amdgcn_udot4(lb & 0x02020202u, 0x20100804u, 0u, false);   // 8 * (wide bits h)
        nb[g] = __builtin_amdgcn_udot4(lb & 0x03030303u, 0x01010101u, 0u, false);            // 4 + popc(h)
        wide |= g == 0 ? so >> 3 : so << (4 * g - 3);
        sel[g] = group2_sel(so);
    }
    const int len = (e - b) + (int)popc32(wide & bits_below(e) & ~bits_below(b));
    group2_place(smax, u01, u23, nb, sel, b, len, slot, q, zero_tail);
    return len;
}


__device__ __forceinline__ int str_lane_compose(int kind, int trim, int width, int smax, int eo, int n, bool ok,
                                                const uint8_t* src, uint32_t rec_addr, const uint32_t* s_lut,
                                                uint8_t* s_str, int lane, u32x4 (&q)[kStrNC], bool zero_tail) {
    uint32_t w[8], ev[kStrFastBytes];
    img_bytes32(src, rec_addr + (ok ? (uint32_t)eo : 0u), smax, w);
    // the LUT's LDS address: 0 in every kernel (wave_lds / coop_lds put it at smem, lds_base_ok);
    // the constant lets each read's address be the SDWA shift's result itself
    const uint32_t lut_a = 0;
    (void)s_lut;
#ifndef CBX_STR_NO_SDWA
    if (kind == CBX_K_STRING) {   // code page: LDS entries, byte offsets straight from the image dwords
#pragma unroll
        for (int j = 0; j < kStrFastBytes; j++)
            ev[j] = j < smax ? lds_ld<uint32_t>(lut_a + ((CBX_DIAG & 32) ? diag_bank(byte_x4(w[j >> 2], j & 3)) : byte_x4(w[j >> 2], j & 3))) : 0u;
    } else {
        lut_entries32(w, smax, [&](uint32_t b) { return ascii_lut(b); }, ev);
    }
#else
    lut_entries32(w, smax, [&](uint32_t b) { return str_lut(kind, s_lut, b); }, ev);
#endif
    // bit j: byte j trimmable (entry bit 31) -- collected reversed with one funnel shift per byte
    // ((tr << 1) | bit 31), then bit-reversed: 1 VALU per byte instead of shift, mask and OR
    uint32_t tr = 0;
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++)
        if (j < smax) tr = __builtin_amdgcn_alignbit(tr, ev[j], 31);
    const uint32_t tm = __builtin_bitreverse32(tr) >> (32 - smax);
    const uint32_t keep = ~tm & bits_below(n);
    int b = 0, e = n;
    if (trim == CBX_TRIM_LEFT || trim == CBX_TRIM_BOTH) b = keep ? (int)ctz32(keep) : n;
    if (trim == CBX_TRIM_RIGHT || trim == CBX_TRIM_BOTH) e = keep ? 32 - (int)clz32(keep) : b;
#ifndef CBX_STR_NO_SHIFT
    if (width == 1) return str_lane_shift(smax, ev, b, e, q);
#endif
#ifndef CBX_STR_W2_BYTES   // (A/B: the byte-store compose below for 2-byte pages too)
    if (width == 2) return str_lane_group2(smax, ev, b, e, s_str + lane * str_lane_slot(smax, 2), q, zero_tail);
#endif
    const uint32_t range = bits_below(e) & ~bits_below(b);
    uint8_t* slot = s_str + lane * str_lane_slot(smax, width);
    uint8_t* p = slot;
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++) {
        if (j < smax) {
            const uint32_t ej = ev[j];
            // byte stores: one unaligned 2-byte LDS store instead made SYNSTR200 2.8x slower (6.54 ->
            // 18.3 ms, measured)
            p[0] = (uint8_t)ej;
            if (width > 1) p[1] = (uint8_t)(ej >> 8);
            if (width > 2) p[2] = (uint8_t)(ej >> 16);
            p += ((ej >> 24) & 3u) & (uint32_t)__builtin_amdgcn_sbfe((int)range, j, 1);
        }
    }
    const int len = (int)(p - slot);
    slot[len] = 0; slot[len + 1] = 0; slot[len + 2] = 0;   // the partial dword's tail
#pragma unroll
    for (int k = 0; k < kStrNC; k++) {
        if (16 * k < smax * width) {   // dword reads (the slot is 4-byte aligned)
            const uint32_t* sd = (const uint32_t*)slot + 4 * k;
            uint32_t d[4];
#pragma unroll
            for (int m = 0; m < 4; m++) d[m] = 16 * k + 4 * m < smax * width ? sd[m] : 0u;
            q[k] = u32x4{d[0], d[1], d[2], d[3]};
        }
    }
    return len;
}

// A long payload (len > 12) from registers to dst (4-byte aligned): exact dword count.
__device__ __forceinline__ void str_store_long(CBX_GLOBAL uint8_t* dst, int len, int cap, const u32x4 (&q)[kStrNC]) {
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
    const int n4 = (len + 3) >> 2;
#pragma unroll
    for (int k = 0; k < kStrNC; k++) {
        if (16 * k < cap) {
            const int r = n4 - 4 * k;
            CBX_GLOBAL uint8_t* d = dst + 16 * k;
            if (r >= 4) {
                st_pay((CBX_GLOBAL u32x4a*)(d), u32x4a{q[k].x, q[k].y, q[k].z, q[k].w});
            } else if (r >= 2) {
                st_pay((CBX_GLOBAL u32x2a*)(d), u32x2a{q[k].x, q[k].y});
                if (r == 3) ((CBX_GLOBAL uint32_t*)d)[2] = q[k].z;
            } else if (r == 1) {
                st_pay((CBX_GLOBAL uint32_t*)(d), q[k].x);
            }
        }
    }
}

__device__ __forceinline__ u32x4 str_short_view(int len, const u32x4 (&q)[kStrNC]) {
    return u32x4{(uint32_t)len, len > 0 ? q[0].x : 0u, len > 4 ? q[0].y : 0u, len > 8 ? q[0].z : 0u};
}

template <typename Sink>
__device__ __forceinline__ void str_view_fast(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp, int i,
                                              const StrCall& c, const TileCtx& t, const int32_t* s_cnt,
                                              const uint8_t* src, uint32_t rec_addr, const uint32_t* s_lut,
                                              uint8_t* s_str, int lane, Sink& sk) {
    bool el = t.active && (op.segment < 0 || op.segment == t.seg);
    if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
    const int o = a.start_off + op.eo;
    const bool ok = el && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    u32x4 q[kStrNC];
    const int len = str_lane_compose(op.kind, op.trim, op.pad, op.size, op.eo, n, ok, src, rec_addr, s_lut, s_str, lane, q);
    sk.svalid(c, i, t.tile, __ballot(ok));
    const bool lng = len > 12;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(lng ? (uint32_t)(len + 3) & ~3u : 0u, lane, tot);
    u32x4 v;
    if (!lng) {
        v = str_short_view(len, q);
    } else {
        str_store_long(gp(c.scratch + t.tile * c.tile_cap + ex), len, op.size * op.pad, q);
        v = u32x4{(uint32_t)len, q[0].x, view_buf(t.tile, c), view_pos(t.tile, c, ex)};
    }
    st_out(gp((u32x4*)c.views) + t.tile * kWave + lane, v);
}

// Two register-path view elements of mutually exclusive segment redefines (the same record bytes
// read as fields of different segments, e.g. exp2's STATIC-DETAILS / CONTACTS) in one pass: each
// lane composes the field of its record's segment, so the tile pays the byte loop once for the
// pair (the longer field's).  The specialised kernel pairs them (cbx_jit.h: same kind, trim and
// code page, no OCCURS); each column gets its validity word, the lane's view where its record holds
// the field and a null view elsewhere; one wave scan places both columns' long payloads (16-bit
// halves: a tile's payload per column is < 64 KiB).
template <typename Sink>
__device__ __forceinline__ void str_view_pair(const KernelArgs& a, const StrOp& A, int ia, const StrCall& ca,
                                              const StrOp& B, int ib, const StrCall& cb, const TileCtx& t,
                                              const uint8_t* src, uint32_t rec_addr, const uint32_t* s_lut,
                                              uint8_t* s_str, int lane, Sink& sk) {
    const bool sa = t.seg == A.segment;
    const int eo = sa ? A.eo : B.eo, size = sa ? A.size : B.size;
    const int smax = A.size > B.size ? A.size : B.size;
    const int o = a.start_off + eo;
    const bool ok = t.active && (sa || t.seg == B.segment) && o <= t.avail;
    const int n = ok ? (size < t.avail - o ? size : t.avail - o) : 0;
    u32x4 q[kStrNC];
    const int len = str_lane_compose(A.kind, A.trim, A.pad, smax, eo, n, ok, src, rec_addr, s_lut, s_str, lane, q);
    sk.svalid(ca, ia, t.tile, __ballot(ok && sa));
    sk.svalid(cb, ib, t.tile, __ballot(ok && !sa));
    const bool lng = len > 12;
    uint32_t tot;
    const uint32_t r4 = lng ? (uint32_t)(len + 3) & ~3u : 0u;
    const uint32_t exb = wave_excl_scan32(sa ? r4 : r4 << 16, lane, tot);
    const uint32_t ex = sa ? exb & 0xFFFFu : exb >> 16;
    u32x4 v;
    if (!lng) {
        v = str_short_view(len, q);
    } else {
        CBX_GLOBAL uint8_t* dst = sa ? gp(ca.scratch + t.tile * ca.tile_cap + ex) : gp(cb.scratch + t.tile * cb.tile_cap + ex);
        str_store_long(dst, len, smax * A.pad, q);
        v = sa ? u32x4{(uint32_t)len, q[0].x, view_buf(t.tile, ca), view_pos(t.tile, ca, ex)}
               : u32x4{(uint32_t)len, q[0].x, view_buf(t.tile, cb), view_pos(t.tile, cb, ex)};
    }
    const u32x4 z = u32x4{0u, 0u, 0u, 0u};
    // whole 1 KiB rows per column, written once: nontemporal like every other view row (st_out)
    st_out(gp((u32x4*)ca.views) + t.tile * kWave + lane, sa ? v : z);
    st_out(gp((u32x4*)cb.views) + t.tile * kWave + lane, sa ? z : v);
}

// n bytes from the 16-byte aligned LDS staging s to global d at any alignment: the bytes up to d's
// next 16-byte boundary and the tail past the last whole chunk as byte stores (neighbouring tiles
// own the bytes on either side, so no store may cover them), 16-byte stores in between, each
// composed from five LDS dwords and a byte align.
__device__ __forceinline__ void lds_to_global_any(const uint8_t* s, CBX_GLOBAL uint8_t* d, uint32_t n, int lane) {
    const uint32_t mis = (uint32_t)((uint64_t)(size_t)d & 15u);
    uint32_t head = (16u - mis) & 15u;
    if (head > n) head = n;
    const uint32_t body = (n - head) >> 4;
    const uint32_t tail0 = head + 16u * body;
    if ((uint32_t)lane < head) d[lane] = s[lane];
    if (tail0 + (uint32_t)lane < n) d[tail0 + lane] = s[tail0 + lane];
    const uint32_t sh = head & 3u;
    for (uint32_t q = lane; q < body; q += kWave) {
        const uint32_t o = head + 16u * q;
        const uint32_t* w = (const uint32_t*)(s + (o & ~3u));
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        *(CBX_GLOBAL u32x4*)(d + o) = u32x4{align_bytes(w1, w0, sh), align_bytes(w2, w1, sh), align_bytes(w3, w2, sh),
                                           align_bytes(w4, w3, sh)};
    }
}

// The launch's mode (KernelArgs.mode: 0 decode, 1 the string sizes / Utf8 count pass): a
// compile-time constant in the specialised kernels (CBX_MODE), so a count kernel carries no decode
// code (and its register allocation) and a decode kernel no count branches.
__device__ __forceinline__ int kmode(const KernelArgs& a) {
#ifdef CBX_MODE
    (void)a;
    return CBX_MODE;
#else
    return a.mode;
#endif
}

// The plan's string layout (KernelArgs.str_view): a compile-time constant in the specialised
// kernels (cbx_jit.h defines CBX_STR_LAYOUT), so a kernel inlines only its own layout's string path
// per element -- with all three, layouts of hundreds of string elements took minutes in hipRTC.
__device__ __forceinline__ int str_layout(const KernelArgs& a) {
#ifdef CBX_STR_LAYOUT
    (void)a;
    return CBX_STR_LAYOUT;
#else
    return a.str_view;
#endif
}

// ---- LDS-DMA (buffer_load_dwordx4 ... lds) ----
// 16 bytes per lane from the buffer resource at voffset (out of range: no access) into LDS at
// lds_base + 16 * lane (lds_base wave-uniform: the instruction's M0).  Issued as inline asm so the
// compiler does not drain it at the next LDS read (it waits vmcnt(0) after any LDS-DMA it knows of):
// the caller waits with a counted s_waitcnt vmcnt (lds_dma_wait) before it reads the bytes.
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voffset, const void* lds_base) {
    const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(size_t)lds_base);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %3\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voffset), "s"(rs), "s"(dst) : "memory");
}

// wait until at most n vector memory operations are outstanding (n: the ones issued after the
// DMA the caller needs; memory operations complete in issue order).  The s_waitcnt builtin (not
// asm): the compiler's own wait insertion sees it, so it does not wait again for older loads or
// stores it tracks (a later wait of its own would also drain DMAs issued after this one).
// Encoding (gfx9): vmcnt bits 3:0, expcnt 6:4 and lgkmcnt 11:8 left at their maxima.
__device__ __forceinline__ void lds_dma_wait(int n) {
    switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(0x0F70); break;
    case 1: __builtin_amdgcn_s_waitcnt(0x0F71); break;
    case 2: __builtin_amdgcn_s_waitcnt(0x0F72); break;
    case 3: __builtin_amdgcn_s_waitcnt(0x0F73); break;
    case 4: __builtin_amdgcn_s_waitcnt(0x0F74); break;
    case 5: __builtin_amdgcn_s_waitcnt(0x0F75); break;
    case 6: __builtin_amdgcn_s_waitcnt(0x0F76); break;
    default: __builtin_amdgcn_s_waitcnt(0x0F77); break;
    }
    asm volatile("" ::: "memory");   // no LDS read hoisted above the wait
}

// ---- Utf8 decode of a register-path element (str_view 2, decode mode) ----
// The value is composed in the lane's registers exactly as in the view layout (str_lane_compose:
// single-byte pages in registers, multi-byte ones through the lane's conflict-free LDS slot), the
// tile's lengths are scanned, and every lane stores its own bytes at their final byte offset
// straight from registers: the bytes up to the next 4-byte boundary and the bytes past the last
// whole dword as byte stores (the neighbouring values own the rest of those dwords), the whole
// dwords in between as 16 / 8 / 4-byte stores.  No LDS staging, no wave barrier.  (The earlier form
// OR-ed the lanes' shifted dwords into a zeroed LDS staging and copied whole 16-byte chunks out:
// ~130 VALU, 13 LDS instructions and three waits per element -- SYNSTR200 decode 10.75 ms,
// profiles/r03_b.)  str_utf8_two runs two elements with one scan of 16-bit halves.

// The lane's value of element op (composed; length, 0 when the record lacks it).
__device__ __forceinline__ int utf8_compose(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp, const TileCtx& t,
                                            const int32_t* s_cnt, const uint8_t* src, uint32_t rec_addr,
                                            const uint32_t* s_lut, uint8_t* s_str, int lane, bool& ok, u32x4 (&q)[kStrNC]) {
    bool el = t.active && (op.segment < 0 || op.segment == t.seg);
    if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
    const int o = a.start_off + op.eo;
    ok = el && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    const int len = str_lane_compose(op.kind, op.trim, op.pad, op.size, op.eo, n, ok, src, rec_addr, s_lut, s_str, lane, q, false);
    return ok ? len : 0;
}

// The tile's place in the element's slot region (the count pass's exclusive scan).  The
// specialised kernel loads it for all of a tile's elements before the first is decoded (one wait
// for the tile instead of a dependent scalar load in front of every element's stores).
// (scalar loads through the constant address space: with the generic pointer they were flat loads,
// which count in vmcnt AND lgkmcnt out of order -- every element then waited vmcnt(0), draining the
// wave's value stores and the next tile's prefetched loads, 5 times per SYNSTR200 tile and wave)
__device__ __forceinline__ int64_t utf8_tile_base(const StrCall& c, const TileCtx& t) {
    const CBX_CONST int64_t* x = (const CBX_CONST int64_t*)c.excl;
    return x[t.tile] - x[0];
}

// The element's int32 offsets (from the tile's place, base) and the slot's size; returns the tile's
// destination, or null when the region (or an int32 offset) overflows.
__device__ __forceinline__ CBX_GLOBAL uint8_t* utf8_offsets(const KernelArgs& a, const StrCall& c, const TileCtx& t, int64_t base,
                                                            uint32_t ex, int len, uint32_t tot, int lane) {
    CBX_GLOBAL int32_t* offs = gp((int32_t*)c.local);
    st_out(offs + t.tile * kWave + lane, (int32_t)(base + ex));
    if (t.rec == a.n_rec - 1) {   // the closing offset and the slot's size
        offs[a.n_rec] = (int32_t)(base + ex + len);
        if (c.size) *gp(c.size) = base + ex + len;
    }
    if (base + tot > c.tile_cap || base + tot > 0x7fffffffll) {
        if (lane == 0) atomicOr(a.status, 1);
        return nullptr;
    }
    return gp(c.scratch + base);
}

// The lane's len bytes (q, packed from byte 0; nbytes: the compile-time bound of len) to d at any
// byte alignment, in few store instructions (a wave issues every variant any lane needs, so the
// variants are kept to: head byte + head short, whole 16-byte chunks, a remainder of 8 + 4 bytes
// at a per-lane address, tail short + tail byte -- at most 9 stores with the offsets, 14 before).
__device__ __forceinline__ void utf8_store_direct(CBX_GLOBAL uint8_t* d, int len, int nbytes, const u32x4 (&q)[kStrNC]) {
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
    constexpr int kNW = 4 * kStrNC;
    uint32_t w[kNW + 1];
#pragma unroll
    for (int k = 0; k < kStrNC; k++) {
        w[4 * k] = q[k].x;
        w[4 * k + 1] = q[k].y;
        w[4 * k + 2] = q[k].z;
        w[4 * k + 3] = q[k].w;
    }
    w[kNW] = 0u;
    const uint32_t mis = (uint32_t)((uint64_t)(size_t)d & 3u);
    int head = (int)((4u - mis) & 3u);
    head = head < len ? head : len;
    // head: a byte at an odd address, then 2 bytes at the (2-aligned) next one or a last byte (a
    // value shorter than its first dword's remainder)
    const int b1 = (head > 0 && (mis & 1u)) ? 1 : 0;
    const int h2 = head - b1;
    if (b1) d[0] = (uint8_t)w[0];
    if (h2 >= 2) st_pay((CBX_GLOBAL uint16_t*)(d + b1), (uint16_t)(w[0] >> (8 * b1)));
    else if (h2 == 1) d[b1] = (uint8_t)(w[0] >> (8 * b1));
    const int nb = (len - head) >> 2;   // whole dwords from d + head (4-byte aligned)
    const int nbmax = nbytes / 4 + 1;   // (compile-time bound of nb + 1: the tail's dword)
    uint32_t s[kNW];
#pragma unroll
    for (int k = 0; k < kNW; k++)
        if (k < nbmax) s[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)head);
    CBX_GLOBAL uint8_t* body = d + head;
#pragma unroll
    for (int k = 0; 4 * k < kNW; k++)
        if (16 * k + 16 <= nbytes && 4 * k + 4 <= nb)
            st_pay((CBX_GLOBAL u32x4a*)(body + 16 * k), u32x4a{s[4 * k], s[4 * k + 1], s[4 * k + 2], s[4 * k + 3]});
    // the remainder (nb & 3 dwords of chunk nb / 4) and the tail dword (s[nb]), selected by chunk
    const int kr = nb >> 2, r = nb & 3;
    uint32_t r0 = 0, r1 = 0, r2 = 0, tl = 0;
#pragma unroll
    for (int k = 0; 4 * k < kNW; k++) {
        if (4 * k < nbmax) {
            if (kr == k) {
                r0 = s[4 * k];
                if (4 * k + 1 < nbmax) r1 = s[4 * k + 1];
                if (4 * k + 2 < nbmax) r2 = s[4 * k + 2];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kNW; k++)
        if (k < nbmax && k == nb) tl = s[k];
    CBX_GLOBAL uint8_t* rp = body + 16 * kr;
    if (r & 2) st_pay((CBX_GLOBAL u32x2a*)(rp), u32x2a{r0, r1});
    if (r & 1) st_pay((CBX_GLOBAL uint32_t*)(rp + 4 * (r & 2)), (uint32_t)((r & 2) ? r2 : r0));
    // tail: 2 bytes at the 4-aligned tail, then 1 byte
    const int rem = len - head - 4 * nb;   // 0..3 tail bytes
    CBX_GLOBAL uint8_t* tp = body + 4 * nb;
    if (rem >= 2) st_pay((CBX_GLOBAL uint16_t*)(tp), (uint16_t)tl);
    if (rem & 1) tp[rem & 2] = (uint8_t)(tl >> (8 * (rem & 2)));
}

// The Utf8 store of a 2-byte-page element from the lane's slot, its bytes placed at the phase of
// the destination: the value's byte i at slot byte 4 * d0 + ph + i, where ph = dst & 3, so slot dword
// d0 + k is destination dword k of A = dst - ph.  Every dword then goes out as it lies in the slot --
// the bytes of the first dword from ph (byte / short), the whole dwords in 16-byte pieces plus a
// remainder of 8 + 4 bytes, the bytes of the last one (short / byte) -- each piece read from LDS at
// its own place: no alignbyte per dword and no register select of the remainder or the tail dword
// (utf8_store_direct's ~100 instructions per element, half of the Utf8 decode's per-element store work).
__device__ __forceinline__ void utf8_store_slot(CBX_GLOBAL uint8_t* dst, int len, int nbytes, const uint32_t* sd) {
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
    if (len <= 0) return;
    const int ph = (int)((uint64_t)(size_t)dst & 3u);
    CBX_GLOBAL uint8_t* A = dst - ph;
    const int T = ph + len;   // bytes from A
    // head: bytes [ph, min(4, T)) of dword 0
    if (ph) {
        const uint32_t d0 = sd[0];
        const int he = T < 4 ? T : 4;
        if (ph & 1) A[ph] = (uint8_t)(d0 >> (8 * ph));
        const int p2 = ph + (ph & 1);   // 2 or 4
        if (p2 == 2 && he == 4) st_pay((CBX_GLOBAL uint16_t*)(A + 2), (uint16_t)(d0 >> 16));
        else if (p2 == 2 && he == 3) A[2] = (uint8_t)(d0 >> 16);
    }
    // whole dwords [k0, k1)
    const int k0 = ph ? 1 : 0, k1 = T >> 2;
    const int n = k1 - k0;   // whole dwords: <= (nbytes + 3) / 4, nbytes the compile-time bound of len
    const uint32_t* m = sd + k0;
    CBX_GLOBAL uint8_t* mp = A + 4 * k0;
#pragma unroll
    for (int c = 0; 16 * c + 16 <= nbytes + 3; c++)
        if (n >= 4 * c + 4) st_pay((CBX_GLOBAL u32x4a*)(mp + 16 * c), u32x4a{m[4 * c], m[4 * c + 1], m[4 * c + 2], m[4 * c + 3]});
    const int j0 = n > 0 ? (n & ~3) : 0, r = n > 0 ? (n & 3) : 0;
    if (r) {
        const uint32_t* rm = m + j0;
        const uint32_t r0 = rm[0], r1 = rm[1], r2 = rm[2];
        CBX_GLOBAL uint8_t* rp = mp + 4 * j0;
        if (r & 2) st_pay((CBX_GLOBAL u32x2a*)(rp), u32x2a{r0, r1});
        if (r & 1) st_pay((CBX_GLOBAL uint32_t*)(rp + 4 * (r & 2)), (uint32_t)((r & 2) ? r2 : r0));
    }
    // tail: bytes [0, T & 3) of dword T >> 2 (unless that is dword 0, done above)
    const int tb = T & 3;
    if (tb && (k1 > 0 || !ph)) {
        const uint32_t td = sd[k1];
        CBX_GLOBAL uint8_t* tp = A + 4 * k1;
        if (tb >= 2) st_pay((CBX_GLOBAL uint16_t*)(tp), (uint16_t)td);
        if (tb & 1) tp[tb & 2] = (uint8_t)(td >> (8 * (tb & 2)));
    }
}

// Utf8 decode of a register-path element of a 2-byte code page: the LUT entries, trim range and
// length first (str_lane_compose's first half and str_lane_group2's group build: g2_prep), then the
// tile scan, then the groups placed in the lane's slot at the destination's phase (g2_store:
// group2_put + utf8_store_slot).
struct G2 {   // a lane's composed value: byte pairs, byte counts and selectors per group of 4 characters
    uint32_t u01[kStrNG], u23[kStrNG], nb[kStrNG];
    uint2 sel[kStrNG];
    int b, e, len;   // kept characters [b, e), UTF-8 length (0 when !ok)
};

// smax: the compile-time bound of the field's bytes; bytes [eo, eo + n) of the lane's record at rec_addr.
__device__ __forceinline__ void g2_prep(int trim, int smax, int eo, int n, bool ok, const uint8_t* src, uint32_t rec_addr, G2& g) {
    uint32_t w[8], ev[kStrFastBytes];
    img_bytes32(src, rec_addr + (ok ? (uint32_t)eo : 0u), smax, w);
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++)
        ev[j] = j < smax ? lds_ld<uint32_t>(byte_x4(w[j >> 2], j & 3)) : 0u;   // (the LUT at LDS 0)
    uint32_t tr = 0;
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++)
        if (j < smax) tr = __builtin_amdgcn_alignbit(tr, ev[j], 31);
    const uint32_t keep = ~(__builtin_bitreverse32(tr) >> (32 - smax)) & bits_below(n);
    int b = 0, e = n;
    if (trim == CBX_TRIM_LEFT || trim == CBX_TRIM_BOTH) b = keep ? (int)ctz32(keep) : n;
    if (trim == CBX_TRIM_RIGHT || trim == CBX_TRIM_BOTH) e = keep ? 32 - (int)clz32(keep) : b;
    uint32_t wide = 0;
#pragma unroll
    for (int q = 0; q < kStrNG; q++) {
        if (4 * q >= smax) break;
        const uint32_t e0 = ev[4 * q], e1 = 4 * q + 1 < smax ? ev[4 * q + 1] : 0u;
        const uint32_t e2 = 4 * q + 2 < smax ? ev[4 * q + 2] : 0u, e3 = 4 * q + 3 < smax ? ev[4 * q + 3] : 0u;
        g.u01[q] = __builtin_amdgcn_perm(e1, e0, 0x05040100u);
        g.u23[q] = __builtin_amdgcn_perm(e3, e2, 0x05040100u);
        const uint32_t lb = __builtin_amdgcn_perm(e1, e0, 0x0C0C0703u) | __builtin_amdgcn_perm(e3, e2, 0x07030C0Cu);
        const uint32_t so = __builtin_amdgcn_udot4(lb & 0x02020202u, 0x20100804u, 0u, false);
        g.nb[q] = __builtin_amdgcn_udot4(lb & 0x03030303u, 0x01010101u, 0u, false);
        wide |= q == 0 ? so >> 3 : so << (4 * q - 3);
        g.sel[q] = group2_sel(so);
    }
    g.b = b;
    g.e = e;
    g.len = ok ? (e - b) + (int)popc32(wide & bits_below(e) & ~bits_below(b)) : 0;
}

// The lane's value to d (its final place) through the lane's slot, placed at d's byte phase.
__device__ __forceinline__ void g2_store(CBX_GLOBAL uint8_t* d, int smax, const G2& g, uint8_t* s_str, int lane) {
    const uint32_t ph = (uint32_t)((uint64_t)(size_t)d & 3u);
    const uint32_t s0 = (ph - (uint32_t)g.b) & 3u;   // character b lands at slot byte s0 + b = ph (mod 4)
    uint8_t* slot = s_str + lane * str_lane_slot(smax, 2);
    group2_put(smax, g.u01, g.u23, g.nb, g.sel, s0, slot);
    utf8_store_slot(d, g.len, 2 * smax, (const uint32_t*)slot + ((s0 + (uint32_t)g.b) >> 2));
}

// The tile's payload of one element through a tile-contiguous LDS staging (the wave's string area),
// copied out with aligned 16-byte stores: staging byte k is global byte A + k (A = D rounded down to
// 16, D the tile's destination), so the body moves as whole 16-byte chunks -- ~2 coalesced store
// instructions per element where each lane's own head / dword / tail stores were ~8 scattered ones
// (SYNSTR200 Utf8 chain 8.08 -> 8.03 and 8.26 -> 8.03 ms, same-box A/B; CBX_U8_DIRECT: the old form).
// Every lane ORs its composed groups into the zeroed staging at its tile-local place, the characters
// outside its kept range [b, e) zeroed first (their bytes then land as zeros in the neighbours' bytes:
// OR-ing zeros changes nothing), 32 guard bytes in front for lane 0's leading characters.  The two
// partial chunks at the ends go out as byte stores (the neighbouring tiles own the bytes around).
constexpr uint32_t kU8StageGuard = 32;

__device__ __forceinline__ void lds_or32(uint32_t addr, uint32_t v) {
    __hip_atomic_fetch_or((__attribute__((address_space(3))) uint32_t*)(size_t)addr, v, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void g2_stage_store(CBX_GLOBAL uint8_t* D, uint32_t ex, uint32_t tot, int smax, const G2& gin, bool on,
                                               uint8_t* s_str, int lane) {
    G2 g = gin;   // (on: the lane's value belongs to this column -- a segment-redefine pair stages one column at a time)
    const uint32_t ph = (uint32_t)((uint64_t)(size_t)D & 15u);
    CBX_GLOBAL uint8_t* A = D - ph;
    const uint32_t sb = lds_addr(s_str) + kU8StageGuard;   // staging byte 0 (16-aligned)
    const uint32_t end = ph + tot;
    for (uint32_t q = (uint32_t)lane; 16u * q < end + 2u * (uint32_t)smax + 8u; q += kWave)
        *(__attribute__((address_space(3))) u32x4*)(size_t)(sb + 16u * q) = u32x4{0u, 0u, 0u, 0u};
    // the kept characters' bytes only (a leading / trailing trimmed character is one byte: zeroed)
    const uint32_t bb = (uint32_t)g.b * 0x01010101u, eb = (uint32_t)(on ? g.e : 0) * 0x01010101u + 0x7F7F7F7Fu;
#pragma unroll
    for (int q = 0; q < kStrNG; q++) {
        if (4 * q >= smax) break;
        const uint32_t pos4 = 0x03020100u + 0x04040404u * (uint32_t)q;
        const uint32_t km = ((((pos4 | 0x80808080u) - bb) & (eb - pos4)) >> 7) & 0x01010101u;   // 1 per kept character
        g.u01[q] &= __builtin_amdgcn_perm(km, km, 0x01010000u) * 0xFFu;
        g.u23[q] &= __builtin_amdgcn_perm(km, km, 0x03030202u) * 0xFFu;
    }
    // character b lands at staging byte ph + ex (the stream's leading b one-byte characters before it)
    uint32_t pos = sb + ph + ex - (uint32_t)g.b, carry = 0;
#pragma unroll
    for (int q = 0; q < kStrNG; q++) {
        if (4 * q >= smax) break;
        const uint32_t lo = __builtin_amdgcn_perm(g.u23[q], g.u01[q], g.sel[q].x), hi = __builtin_amdgcn_perm(g.u23[q], g.u01[q], g.sel[q].y);
        const uint32_t k8 = 8u * (pos & 3u);
        const uint64_t v = (((uint64_t)hi << 32) | lo) << k8;
        const uint32_t w0 = (uint32_t)v | carry, w1 = (uint32_t)(v >> 32);
        const uint32_t w2 = (uint32_t)(((uint64_t)hi << k8) >> 32);
        lds_or32(pos & ~3u, w0);
        lds_or32((pos & ~3u) + 4u, w1);
        const uint32_t np = pos + g.nb[q];
        const uint32_t dd = (np >> 2) - (pos >> 2);
        carry = dd == 0u ? w0 : dd == 1u ? w1 : w2;
        pos = np;
    }
    lds_or32(pos & ~3u, carry);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the wave's ORs landed before its reads
    // copy out: whole chunks [q_lo, q_hi), the head bytes [ph, 16) of chunk 0 and the tail of chunk q_hi
    const uint32_t q_lo = ph ? 1u : 0u, q_hi = end >> 4;
    for (uint32_t q = q_lo + (uint32_t)lane; q < q_hi; q += kWave)
        st_pay((CBX_GLOBAL u32x4*)(A + 16u * q), lds_ld<u32x4>(sb + 16u * q));
    const uint32_t he = end < 16u ? end : 16u;
    if (ph && (uint32_t)lane >= ph && (uint32_t)lane < he) A[lane] = lds_ld<uint8_t>(sb + (uint32_t)lane);
    const uint32_t t0 = 16u * q_hi;
    if (t0 >= 16u * q_lo && t0 + (uint32_t)lane < end && (t0 > 0 || !ph)) A[t0 + lane] = lds_ld<uint8_t>(sb + t0 + (uint32_t)lane);
}

__device__ __forceinline__ void str_utf8_fast2(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp,
                                               const StrCall& c, const TileCtx& t, const int32_t* s_cnt,
                                               const uint8_t* src, uint32_t rec_addr, uint8_t* s_str, int lane) {
    bool el = t.active && (op.segment < 0 || op.segment == t.seg);
    if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
    const int o = a.start_off + op.eo;
    const bool ok = el && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    G2 g;
    g2_prep(op.trim, op.size, op.eo, n, ok, src, rec_addr, g);
    gp(c.validity)[t.tile] = __ballot(ok);
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32((uint32_t)g.len, lane, tot);
    CBX_GLOBAL uint8_t* dst = utf8_offsets(a, c, t, utf8_tile_base(c, t), ex, g.len, tot, lane);
    if (!dst || (CBX_DIAG & 16)) return;
#ifndef CBX_U8_DIRECT   // (A/B: each lane's own head / dword / tail stores, g2_store)
    g2_stage_store(dst, ex, tot, op.size, g, true, s_str, lane);
#else
    g2_store(dst + ex, op.size, g, s_str, lane);
#endif
}

__device__ __forceinline__ void str_utf8_fast(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp,
                                              const StrCall& c, const TileCtx& t, const int32_t* s_cnt,
                                              const uint8_t* src, uint32_t rec_addr, const uint32_t* s_lut,
                                              uint8_t* s_str, int lane) {
#ifndef CBX_UTF8_DIRECT   // (A/B: the register read-back + utf8_store_direct for 2-byte pages too)
    if (op.kind == CBX_K_STRING && op.pad == 2) {
        str_utf8_fast2(a, op, opp, c, t, s_cnt, src, rec_addr, s_str, lane);
        return;
    }
#endif
    bool ok;
    u32x4 q[kStrNC];
    const int len = utf8_compose(a, op, opp, t, s_cnt, src, rec_addr, s_lut, s_str, lane, ok, q);
    gp(c.validity)[t.tile] = __ballot(ok);
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32((uint32_t)len, lane, tot);
    CBX_GLOBAL uint8_t* dst = utf8_offsets(a, c, t, utf8_tile_base(c, t), ex, len, tot, lane);
    if (dst && !(CBX_DIAG & 16)) utf8_store_direct(dst + ex, len, op.size * op.pad, q);
}

// Whether two register-path Utf8 elements (size, widest UTF-8 byte count) can be decoded together:
// a tile's payload of each must fit the 16-bit halves of the pair's scan.
__host__ __device__ constexpr bool utf8_pair_fits(int size_a, int w_a, int size_b, int w_b) {
    return kWave * size_a * w_a < 65536 && kWave * size_b * w_b < 65536;
}

// Two register-path elements of the tile (the specialised kernel pairs consecutive ones): composed
// one after the other through the same lane slot, one scan of 16-bit halves, the stores of both.
__device__ __forceinline__ void str_utf8_two(const KernelArgs& a, const StrOp& A, const CBX_CONST StrOp* oppA, const StrCall& ca,
                                             const StrOp& B, const CBX_CONST StrOp* oppB, const StrCall& cb,
                                             const TileCtx& t, const int32_t* s_cnt, const uint8_t* src, uint32_t rec_addr,
                                             const uint32_t* s_lut, uint8_t* s_str, int lane, int64_t base_a, int64_t base_b) {
    bool oka, okb;
    u32x4 qa[kStrNC], qb[kStrNC];
    const int la = utf8_compose(a, A, oppA, t, s_cnt, src, rec_addr, s_lut, s_str, lane, oka, qa);
    const int lb = utf8_compose(a, B, oppB, t, s_cnt, src, rec_addr, s_lut, s_str, lane, okb, qb);
    gp(ca.validity)[t.tile] = __ballot(oka);
    gp(cb.validity)[t.tile] = __ballot(okb);
    uint32_t tot2;
    const uint32_t ex2 = wave_excl_scan32((uint32_t)la | ((uint32_t)lb << 16), lane, tot2);   // a tile's total < 64 KiB
    const uint32_t exa = ex2 & 0xFFFFu, exb = ex2 >> 16, tota = tot2 & 0xFFFFu, totb = tot2 >> 16;
    CBX_GLOBAL uint8_t* da = utf8_offsets(a, ca, t, base_a, exa, la, tota, lane);
    CBX_GLOBAL uint8_t* db = utf8_offsets(a, cb, t, base_b, exb, lb, totb, lane);
    if (CBX_DIAG & 16) return;
    if (da) utf8_store_direct(da + exa, la, A.size * A.pad, qa);
    if (db) utf8_store_direct(db + exb, lb, B.size * B.pad, qb);
}

__device__ __forceinline__ void str_utf8_two(const KernelArgs& a, const StrOp& A, const CBX_CONST StrOp* oppA, const StrCall& ca,
                                             const StrOp& B, const CBX_CONST StrOp* oppB, const StrCall& cb,
                                             const TileCtx& t, const int32_t* s_cnt, const uint8_t* src, uint32_t rec_addr,
                                             const uint32_t* s_lut, uint8_t* s_str, int lane) {
    str_utf8_two(a, A, oppA, ca, B, oppB, cb, t, s_cnt, src, rec_addr, s_lut, s_str, lane, utf8_tile_base(ca, t),
                 utf8_tile_base(cb, t));
}

// Two register-path Utf8 elements of mutually exclusive segment redefines (exp2's STATIC-DETAILS /
// CONTACTS: the same record bytes read as fields of different segments) in one pass, as str_view_pair
// does for views: each lane composes the field of its record's segment, so the tile pays one compose
// for the pair; each column gets its validity word, its int32 offsets (a record of the other segment
// adds 0 bytes: a null value) and the lane's bytes at its place.  One scan of 16-bit halves places both
// columns (utf8_pair_fits).  The specialised kernel pairs them (cbx_jit.h: same kind, trim and code
// page, no OCCURS).
__device__ __forceinline__ void str_utf8_pair(const KernelArgs& a, const StrOp& A, const StrCall& ca, const StrOp& B,
                                              const StrCall& cb, const TileCtx& t, const uint8_t* src, uint32_t rec_addr,
                                              const uint32_t* s_lut, uint8_t* s_str, int lane) {
    const bool sa = t.seg == A.segment;
    const int eo = sa ? A.eo : B.eo, size = sa ? A.size : B.size;
    const int smax = A.size > B.size ? A.size : B.size;
    const int o = a.start_off + eo;
    const bool ok = t.active && (sa || t.seg == B.segment) && o <= t.avail;
    const int n = ok ? (size < t.avail - o ? size : t.avail - o) : 0;
    const bool g2 = A.kind == CBX_K_STRING && A.pad == 2;
    G2 g;
    u32x4 q[kStrNC];
    int len;
    if (g2) {
        g2_prep(A.trim, smax, eo, n, ok, src, rec_addr, g);
        len = g.len;
    } else {
        const int l0 = str_lane_compose(A.kind, A.trim, A.pad, smax, eo, n, ok, src, rec_addr, s_lut, s_str, lane, q, false);
        len = ok ? l0 : 0;
    }
    gp(ca.validity)[t.tile] = __ballot(ok && sa);
    gp(cb.validity)[t.tile] = __ballot(ok && !sa);
    const uint32_t la = sa ? (uint32_t)len : 0u, lb = sa ? 0u : (uint32_t)len;
    uint32_t tot2;
    const uint32_t ex2 = wave_excl_scan32(la | (lb << 16), lane, tot2);   // a tile's total < 64 KiB (utf8_pair_fits)
    const uint32_t exa = ex2 & 0xFFFFu, exb = ex2 >> 16;
    CBX_GLOBAL uint8_t* da = utf8_offsets(a, ca, t, utf8_tile_base(ca, t), exa, (int)la, tot2 & 0xFFFFu, lane);
    CBX_GLOBAL uint8_t* db = utf8_offsets(a, cb, t, utf8_tile_base(cb, t), exb, (int)lb, tot2 >> 16, lane);
    if (CBX_DIAG & 16) return;
    CBX_GLOBAL uint8_t* d = sa ? (da ? da + exa : nullptr) : (db ? db + exb : nullptr);
#ifndef CBX_U8_DIRECT
    if (g2) {   // each column's tile staged and copied out in turn (the lanes of the other segment add nothing)
        if (da) g2_stage_store(da, exa, tot2 & 0xFFFFu, smax, g, sa, s_str, lane);
        if (db) g2_stage_store(db, exb, tot2 >> 16, smax, g, !sa, s_str, lane);
        return;
    }
#endif
    if (!d) return;   // (a column whose region overflowed: reported by utf8_offsets)
    if (g2) g2_store(d, smax, g, s_str, lane);
    else utf8_store_direct(d, len, smax * A.pad, q);
}

// ---- Utf8 count pass (specialised kernels only: CBX_COUNT_LUT) ----
// The count kernel's LDS copy of the code-page LUT keeps, per byte, only what a UTF-8 length needs:
// the trim flag and the UTF-8 length.  A trimmed character maps to <= U+0020, one UTF-8 byte, so a
// value's length is the sum over all its bytes of the lengths, minus its leading and trailing
// trimmable bytes: per byte one LDS read, a funnel shift collecting the trim bits (byte j at bit
// size-1-j) and one add of the entry's low byte (trim * 128 + length: the sum of the lengths of <= 32
// bytes stays below 128).  The count LUT is 256 bytes (trim flag at bit 7, UTF-8 length in bits 0-1), read with ds_read_i8:
// the sign extension puts the trim flag at bit 31 for the funnel-shift collect, and a 256-byte table
// spans 64 dwords -- at most 2 distinct dwords per bank for a wave's random bytes, where the 1 KiB
// table of 4-byte entries put up to 8 on one bank (count kernel SQ_LDS_BANK_CONFLICT / active 2.2).
__device__ __forceinline__ uint8_t count_lut_byte(uint32_t e) {
    return (uint8_t)(((e >> 31) << 7) | ((e >> 24) & 3u));
}

// UTF-8 length of the lane's value of a register-path code-page element whose n bytes are all in
// the record (n == op.size; the caller checks), from the count LUT.
// str_count_lane: the same for a lane whose field is `size` <= smax bytes at eo (a segment-redefine pair
// of fields: each lane counts its record's segment's field; smax the compile-time bound).
__device__ __forceinline__ int str_count_lane(int trim, int smax, int size, int eo, const uint8_t* src, uint32_t rec_addr, bool ok,
                                              const uint32_t* s_lut) {
    uint32_t w[8];
    img_bytes32(src, rec_addr + (ok ? (uint32_t)eo : 0u), smax, w);
    uint32_t acc = 0, tm = 0;
    const uint32_t lut8 = lds_addr(s_lut);   // count_lut_byte entries
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++) {
        if (j < smax) {
            const uint32_t idx = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t e = (uint32_t)(int32_t)lds_ld<int8_t>(lut8 + idx);
            tm = __builtin_amdgcn_alignbit(tm, e, 31);   // (tm << 1) | trim bit
            acc += j < size ? (e & 0xFFu) : 0u;          // trim * 128 + UTF-8 length
        }
    }
    const uint32_t keep = ~__builtin_bitreverse32(tm << (32 - smax)) & bits_below(size);
    const int total = (int)(acc & 127u);
    const bool tl = trim == CBX_TRIM_LEFT || trim == CBX_TRIM_BOTH;
    const bool tr = trim == CBX_TRIM_RIGHT || trim == CBX_TRIM_BOTH;
    if (!ok) return 0;
    if (!keep) return (tl || tr) ? 0 : total;
    const int lead = (int)ctz32(keep), trail = size - (32 - (int)clz32(keep));
    return total - (tl ? lead : 0) - (tr ? trail : 0);
}

__device__ __forceinline__ int str_count_fast(const StrOp& op, const uint8_t* src, uint32_t rec_addr, bool ok,
                                              const uint32_t* s_lut) {
    uint32_t w[8];
    img_bytes32(src, rec_addr + (ok ? (uint32_t)op.eo : 0u), op.size, w);
    uint32_t acc = 0;
    const uint32_t lut8 = lds_addr(s_lut);   // count_lut_byte entries
    const int size = op.size;
#ifndef CBX_COUNT_B64   // one ds_read_i8 per byte (the 256-byte table spans 2 rows of the 32 ds_read_b32 banks)
    uint32_t tm = 0;
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++) {
        if (j < size) {
            const uint32_t idx = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t e = (uint32_t)(int32_t)lds_ld<int8_t>(lut8 + ((CBX_DIAG & 32) ? diag_bank(idx) : idx));
            tm = __builtin_amdgcn_alignbit(tm, e, 31);   // (tm << 1) | trim bit
            acc += e & 0xFFu;                            // trim * 128 + UTF-8 length
        }
    }
    const uint32_t keep = ~__builtin_bitreverse32(tm << (32 - size)) & bits_below(size);
#else
    // (A/B, CBX_JIT_DEFINES=CBX_COUNT_B64) per byte its 8-byte row of the 256-byte table (ds_read_b64:
    // one row of the 64 banks, never a conflict) and a v_perm of its entry; per group of 4 the entries
    // packed into a dword: one v_dot4 adds their (trim * 128 + length), one gathers the trim bits.
    // Measured slower: SYNSTR200 Utf8 10.46 -> 11.03 ms -- the kernel is bound by its VALU issue
    // (+2 VALU per byte) more than by the LDS conflicts it removes.
    uint32_t trimm = 0;
    uint32_t m_row = 0xF8u, m_col = 7u;
    asm volatile("" : "+v"(m_row), "+v"(m_col));   // (VGPR operands of the SDWA ands)
#pragma unroll
    for (int g = 0; 4 * g < kStrFastBytes; g++) {
        if (4 * g >= size) break;
        uint32_t p[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (4 * g + k < size) {
                const uint64_t row = lds_ld<uint64_t>(lut8 + byte_and(w[g], k, m_row));
                p[k] = __builtin_amdgcn_perm((uint32_t)(row >> 32), (uint32_t)row, byte_and(w[g], k, m_col));   // entry in byte 0
            } else {
                p[k] = 0u;
            }
        }
        const uint32_t e4 = __builtin_amdgcn_perm(p[1], p[0], 0x0C0C0400u) | __builtin_amdgcn_perm(p[3], p[2], 0x04000C0Cu);
        acc = __builtin_amdgcn_udot4(e4, 0x01010101u, acc, false);
        trimm |= __builtin_amdgcn_udot4((e4 >> 7) & 0x01010101u, 0x08040201u, 0u, false) << (4 * g);
    }
    const uint32_t keep = ~trimm & bits_below(size);   // bit j: byte j not trimmable
#endif
    const int total = (int)(acc & 127u);
    const bool tl = op.trim == CBX_TRIM_LEFT || op.trim == CBX_TRIM_BOTH;
    const bool tr = op.trim == CBX_TRIM_RIGHT || op.trim == CBX_TRIM_BOTH;
    if (!ok) return 0;
    if (!keep) return (tl || tr) ? 0 : total;
    const int lead = (int)ctz32(keep), trail = size - (32 - (int)clz32(keep));
    return total - (tl ? lead : 0) - (tr ? trail : 0);
}

// The Utf8 count pass over a segment-redefine pair (str_utf8_pair's counterpart): each lane counts its
// record's segment's field with the count LUT, one scan of 16-bit halves gives both tile totals.
// Returns false (nothing written) for a tile with a record ending inside its field or a non-code-page
// pair: the caller counts each element on its own (str_element, mode 1).
__device__ __forceinline__ bool str_count_pair(const KernelArgs& a, const StrOp& A, const StrOp& B, const TileCtx& t,
                                               const uint8_t* src, uint32_t rec_addr, const uint32_t* s_lut, int lane) {
    const bool sa = t.seg == A.segment;
    const int eo = sa ? A.eo : B.eo, size = sa ? A.size : B.size;
    const int smax = A.size > B.size ? A.size : B.size;
    const int o = a.start_off + eo;
    const bool el = t.active && (sa || t.seg == B.segment);
    const bool ok = el && o + size <= t.avail;
    const bool part = el && o <= t.avail && !ok;
    if (A.kind != CBX_K_STRING || __ballot(part)) return false;
    const int len = str_count_lane(A.trim, smax, size, eo, src, rec_addr, ok, s_lut + 256);
    const uint32_t la = sa ? (uint32_t)len : 0u, lb = sa ? 0u : (uint32_t)len;
    uint32_t tot2;
    wave_excl_scan32(la | (lb << 16), lane, tot2);
    if (lane == 0) {
        gp(a.str_tot)[(int64_t)A.seq * a.n_tiles + t.tile] = tot2 & 0xFFFFu;
        gp(a.str_tot)[(int64_t)B.seq * a.n_tiles + t.tile] = tot2 >> 16;
    }
    return true;
}

// One string element of the tile (StringDecoders.decodeEbcdicString / decodeAsciiString):
// span + tile-local scan.
// * Arrow large-string layout (str_view 0): the tile's payload is staged contiguously in LDS and
//   copied with dword stores to the tile's scratch region; the tile-local start of every value and
//   the tile's byte total are recorded for the compaction kernel, which places tiles after a
//   device-wide scan of the totals (two-pass string offsets, no cross-tile waiting).
// * Arrow Utf8 layout (str_view 2): a count pass (this function in mode 1: the tile totals only) and
//   a device scan of the totals ran before the decode, so the tile's place in the slot's region is
//   known here: the int32 offsets and the payload are written once, at their final place -- staged
//   in LDS at the tile-local starts and copied out with 16-byte stores (byte stores at the edges).
template <bool kView, typename Sink = DirectSink>
__device__ __forceinline__ void str_element(const KernelArgs& a, const StrOp& op, const CBX_CONST StrOp* opp,
                                            const StrCall& c, const TileCtx& t, const int32_t* s_cnt,
                                            const uint8_t* src, uint32_t rec_addr, bool global,
                                            const uint32_t* s_lut, uint8_t* s_str, int lane, int i = 0,
                                            Sink* sk = nullptr) {
    const bool fast = sop_fast(op, global);
    if (kView && fast) {
        DirectSink ds;
        if (sk) str_view_fast(a, op, opp, i, c, t, s_cnt, src, rec_addr, s_lut, s_str, lane, *sk);
        else str_view_fast(a, op, opp, i, c, t, s_cnt, src, rec_addr, s_lut, s_str, lane, ds);
        return;
    }
    // (the plan sizes the staging for the lane slots of every register-path element)
    if (!kView && fast && str_layout(a) == 2 && kmode(a) == 0) {
        str_utf8_fast(a, op, opp, c, t, s_cnt, src, rec_addr, s_lut, s_str, lane);
        return;
    }
#ifdef CBX_COUNT_LUT
    // the count kernel of the Utf8 layout: code-page elements whose bytes are all in the record take
    // the count LUT (str_count_fast); the others (short records, ASCII) sop_span with the full entries,
    // which the count kernel keeps in its second LUT copy
    if (!kView && fast && op.kind == CBX_K_STRING) {
        bool el = t.active && (op.segment < 0 || op.segment == t.seg);
        if (op.n_odo) el &= odo_present(opp, op.n_odo, s_cnt, lane);
        const int o = a.start_off + op.eo;
        const bool ok = el && o + op.size <= t.avail;
        const bool part = el && o <= t.avail && !ok;   // a record ending inside the field
        if (!__ballot(part)) {
            uint32_t tot;
            wave_excl_scan32((uint32_t)str_count_fast(op, src, rec_addr, ok, s_lut + 256), lane, tot);
            if (lane == 0) gp(a.str_tot)[(int64_t)op.seq * a.n_tiles + t.tile] = tot;
            return;
        }
    }
#endif
    bool ok;
    uint32_t ev[kStrFastBytes];
    const StrSpan sp = sop_span(a, op, opp, t, s_cnt, lane, src, rec_addr, s_lut, ok, fast, ev);
    if (kView) {   // decode mode only: the view layout has no sizes pre-pass (cbx_string_bound)
        DirectSink ds;
        if (sk) str_view_element(a, op, i, c, t, sp, ok, fast, ev, src + rec_addr + (uint32_t)op.eo, s_lut, s_str, lane, *sk);
        else str_view_element(a, op, i, c, t, sp, ok, fast, ev, src + rec_addr + (uint32_t)op.eo, s_lut, s_str, lane, ds);
        return;
    }
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32((uint32_t)sp.utf8_len, lane, tot);
    if (kmode(a) == 1) {
        if (lane == 0) gp(a.str_tot)[(int64_t)op.seq * a.n_tiles + t.tile] = tot;
        return;
    }
    gp(c.validity)[t.tile] = __ballot(ok);
    auto lutf = [&](uint32_t b) { return str_lut(op.kind, s_lut, b); };
    const uint8_t* sp_src = src + rec_addr + (uint32_t)op.eo;
    // the destination region: Utf8 -- the tile's final place in the slot's region (offsets written
    // here, once); large-string -- the tile's scratch region (tile-local starts for the placement pass)
    const bool packed = str_layout(a) == 2;
    CBX_GLOBAL uint8_t* dst;
    if (packed) {
        const int64_t base = utf8_tile_base(c, t);   // the tile's place in the slot's region
        const int64_t end = base + tot;
        CBX_GLOBAL int32_t* offs = gp((int32_t*)c.local);
        st_out(offs + t.tile * kWave + lane, (int32_t)(base + ex));
        if (t.rec == a.n_rec - 1) {   // the closing offset and the slot's size
            offs[a.n_rec] = (int32_t)(base + ex + sp.utf8_len);
            if (c.size) *gp(c.size) = base + ex + sp.utf8_len;
        }
        if (end > c.tile_cap || end > 0x7fffffffll) {   // the region (or an int32 offset) overflows
            if (lane == 0) atomicOr(a.status, 1);
            return;
        }
        dst = gp(c.scratch + base);
    } else {
        (gp(c.local) + t.tile * kWave)[lane] = ex;
        if (lane == 0) gp(a.str_tot)[(int64_t)op.seq * a.n_tiles + t.tile] = tot;
        dst = gp(c.scratch + t.tile * (int64_t)c.tile_cap);   // 16-byte aligned region
    }
    if ((int)tot <= a.str_stage) {
        // (diagnostic builds, CBX_JIT_DEFINES=CBX_DIAG=8 / 16: without the LDS byte writes / the copy-out)
        if (!(CBX_DIAG & 8)) {
            if (fast) string_write32e(ev, sp, s_str + ex, s_str + a.str_stage + a.dump_stride * lane, op.size, op.pad);
            else if (ok) string_write(op.kind, sp_src, sp, s_str + ex, lutf);
        }
        wave_sync_lds();
        if (packed) {
            if (!(CBX_DIAG & 16)) lds_to_global_any(s_str, dst, tot, lane);
        } else {
            // 16-byte pieces: the staging area and the scratch region are 16-byte aligned and the
            // region (a multiple of 16 bytes >= the tile's bound) holds the rounded-up total
            const u32x4* s128 = (const u32x4*)s_str;
            for (int q = lane; 16 * q < (int)tot; q += kWave) gp((u32x4*)dst)[q] = s128[q];
        }
        wave_sync_lds();
    } else if (ok) {
        if (fast) {
            uint8_t dump[4];
            string_write32e(ev, sp, (uint8_t*)(dst + ex), dump, op.size, op.pad);
        } else {
            string_write(op.kind, sp_src, sp, (uint8_t*)(dst + ex), lutf);
        }
    }
}

// Generated columns of a window (File_Id / Record_Id).  kSel: the call may carry per-record
// Record_Ids (selected variable-length records); the contiguous fixed-length loop never does, and
// must not issue that load (a load behind the prefetched tile makes its wait cover the prefetch).
template <bool kSel = true>
__device__ __forceinline__ void decode_generated(const KernelArgs& a, const Window& w, const TileCtx& t, int lane) {
    if (kmode(a) == 1) return;
    for (int i = w.gen_begin; i < w.gen_end; i++) {
        const GenOp g = ldc(a.gops + i);
        const DevColumn col = ldc(a.cols + g.column);
        // Record_Id: the selection's per-record ids (cbx_decode_selected), else first_record_id + r
        const int64_t rid = (kSel && a.rec_id) ? (t.active ? a.rec_id[t.rec] : 0)
                                               : a.first_record_id + (a.rec_id_base ? *a.rec_id_base : 0) + t.rec;
        Val x{g.kind == CBX_K_RECORD_ID ? (uint64_t)rid : (uint64_t)(int64_t)a.file_id, 0, true};
        if (t.active) store_value(col, g.out_type, t.rec, x);
        const uint64_t m = __ballot(t.active);
        if (lane == 0) gp(col.validity)[t.tile] = m;
    }
}

// Decode one window of the current tile.  src + rec_addr is the record's decode base (LDS
// image, or HBM for the global window).
template <bool kGlobal>
__device__ __forceinline__ void decode_window(const KernelArgs& a, const Window& w, const TileCtx& t, const uint8_t* src,
                                              uint32_t rec_addr, const int32_t* s_cnt, const uint32_t* s_lut,
                                              uint8_t* s_str, int lane) {
    const bool sizes = kmode(a) == 1;
    // ---- strings (tile-local; placed by the compaction kernel)
    for (int i = w.sop_begin; i < w.sop_end; i++) {
        const StrOp op = ldc(a.sops + i);
        const StrCall c = sizes ? StrCall{} : ldc(a.scall + i);
        if (str_layout(a) == 1) str_element<true>(a, op, a.sops + i, c, t, s_cnt, src, rec_addr, kGlobal, s_lut, s_str, lane);
        else str_element<false>(a, op, a.sops + i, c, t, s_cnt, src, rec_addr, kGlobal, s_lut, s_str, lane);
    }
    if (sizes) return;
    decode_generated(a, w, t, lane);
    // ---- numerics (look-back words of earlier tiles land meanwhile), one specialised loop per batch
    for (int bi = w.batch_begin; bi < w.batch_end; bi++) {
        const Batch b = ldc(a.batches + bi);
        if (kGlobal) {
            if (b.odo) num_batch<V_GENERIC, 8, true, true>(a, b, t, src, rec_addr, s_cnt, lane);
            else num_batch<V_GENERIC, 8, false, true>(a, b, t, src, rec_addr, s_cnt, lane);
            continue;
        }
        if (b.runs) {  // OCCURS runs: one generic-width loop per variant
#define CBX_RUNS(ODO)                                                                                 \
            switch (b.variant) {                                                                      \
            case V_BCD8: run_batch<V_BCD8, 0, ODO>(a, b, t, src, rec_addr, s_cnt, lane); break;       \
            case V_BCD16: run_batch<V_BCD16, 0, ODO>(a, b, t, src, rec_addr, s_cnt, lane); break;     \
            case V_BIN8: run_batch<V_BIN8, 0, ODO>(a, b, t, src, rec_addr, s_cnt, lane); break;       \
            case V_ZONED16: run_batch<V_ZONED16, 0, ODO>(a, b, t, src, rec_addr, s_cnt, lane); break; \
            case V_FP: run_batch<V_FP, 0, ODO>(a, b, t, src, rec_addr, s_cnt, lane); break;           \
            default: run_batch<V_GENERIC, 0, ODO>(a, b, t, src, rec_addr, s_cnt, lane); break;        \
            }
            if (b.odo) { CBX_RUNS(true) } else { CBX_RUNS(false) }
#undef CBX_RUNS
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
// fetched with 16-byte loads (consecutive lanes on consecutive chunks, 1 KiB per
// wave-instruction) and written to LDS rows of cpitch bytes (odd dword count when padding pays).
// The loads of tile t + stride are issued before tile t is decoded, KP per lane, ALL of them
// unconditionally through a range-checked buffer descriptor over [a0, end of input): chunks past
// the span get an out-of-range offset (no memory access, zero data), and nothing past the input
// is read.  The range check is per dword (a chunk straddling the end of the input returns its
// in-range dwords), and the records end on a dword boundary (stride and base are multiples of 4),
// so every byte of the last tile arrives -- tests/test_gpu_parity.py decodes batches whose input
// ends 8 bytes into a chunk.  Loads
// that are always issued and always overwrite the same registers leave the compiler no reason to
// copy the buffer (a copy would wait for the loads, the whole prefetch) anywhere in the loop.
// KP: chunks per lane -- exact for the specialised kernel (ceil(chunks per span / 64)), the plan
// limit (kPre) for the table-driven one.
constexpr int kPre = 16;   // 16-byte chunks per lane: a 16 KiB tile span (plan limit for contig)
// cache policy of the staging loads (the input is read once): 0, or with CBX_NT_LOADS (A/B) the
// gfx940+ nontemporal bit (CPol::NT)
#ifdef CBX_NT_LOADS
constexpr int kStageCpol = 2;
#else
constexpr int kStageCpol = 0;
#endif

// Chunks per lane that cover any tile span of records of stride_dw dwords (up to 3 dwords of
// misalignment in front of the first record).
__host__ __device__ constexpr int contig_kp(int stride_dw) {
    return ((3 + kWave * stride_dw + 3) / 4 + kWave - 1) / kWave;
}

struct ContigSpan {
    int64_t a0;      // 16-byte aligned start of the span
    int mis_dw;      // dwords between a0 and the first record
    int span_dw;     // dwords of the tile's records
    int nch;         // 16-byte chunks to load
};

__device__ __forceinline__ ContigSpan contig_span(const KernelArgs& a, int64_t tile) {
    ContigSpan sp;
    const int64_t t0b = a.base_shift + tile * kWave * (int64_t)a.stride;
    const int64_t left = a.n_rec - tile * kWave;
    const int nrec_tile = left < kWave ? (left > 0 ? (int)left : 0) : kWave;   // 0 past the last tile
    sp.a0 = t0b & ~(int64_t)15;
    sp.mis_dw = (int)((t0b - sp.a0) >> 2);
    sp.span_dw = nrec_tile * a.stride_dw;
    sp.nch = (sp.mis_dw + sp.span_dw + 3) >> 2;
    return sp;
}

// Issue the KP loads of a span (no wait); chunks outside the input read as zeros.  The descriptor is built from wave-uniform values made
// provably uniform (readfirstlane), so no waterfall loop wraps the loads.
template <int KP>
__device__ __forceinline__ void contig_issue(const KernelArgs& a, const ContigSpan& sp, int lane, uint4 (&buf)[KP]) {
    int64_t left = a.data_len - sp.a0;
    left = left < 0 ? 0 : (left > (1 << 20) ? (1 << 20) : left);
    const uint64_t base = (uint64_t)(a.data + sp.a0);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane((int)left);
    const int nch = __builtin_amdgcn_readfirstlane(sp.nch);
    void* bp = (void*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(bp, (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int u = 0; u < KP; u++) {
        const int c = u * kWave + lane;
        const int off = c < nch ? 16 * c : 0x7ffffff0;   // past the descriptor's range: no access
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kStageCpol);
        buf[u] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// Chunk c (16 bytes at a0 + 16c) into the LDS rows.
__device__ __forceinline__ void contig_put(const KernelArgs& a, const ContigSpan& sp, int c, uint4 v, uint8_t* s_img) {
    if (a.cpitch == 4 * a.stride_dw) {
        *(uint4*)(s_img + 16 * c) = v;
        return;
    }
    uint32_t* img32 = (uint32_t*)s_img;
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int d = 4 * c + k - sp.mis_dw;
        if (d >= 0 && d < sp.span_dw) {
            const int r = (int)(((float)d + 0.5f) * a.inv_stride_dw);
            img32[d + sp.mis_dw + r] = wv[k];
        }
    }
}

template <int KP>
__device__ __forceinline__ void contig_store(const KernelArgs& a, const ContigSpan& sp, int lane, const uint4 (&buf)[KP],
                                             uint8_t* s_img) {
    // opaque lane index: keeps the compiler from computing the LDS addresses when the loads
    // are issued (a tile earlier) and holding them in registers across the decode
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int u = 0; u < KP; u++) {
        const int c = u * kWave + lane;
        if (u * kWave < sp.nch && c < sp.nch) contig_put(a, sp, c, buf[u], s_img);
    }
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
        int64_t ga[8];
        bool slow = a.data_len < 16;
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
            ga[u] = (gb & ~(int64_t)15) + 16 * (int64_t)k;
            slow |= ld[u] && !(ga[u] >= 0 && ga[u] + 16 <= a.data_len);
        }
        // loads of a round issue back to back (unconditional; idle lanes read chunk 0) unless a
        // chunk crosses the end of the input (wave-uniform choice)
        if (__ballot(slow) == 0) {
#pragma unroll
            for (int u = 0; u < 8; u++) buf[u] = *(const uint4*)(a.data + (ld[u] ? ga[u] : 0));
        } else {
#pragma unroll
            for (int u = 0; u < 8; u++) buf[u] = ld[u] ? load16_guarded(a.data, ga[u], a.data_len) : make_uint4(0, 0, 0, 0);
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

// Per-lane tile context: record index, base offset and available bytes.  kFramed: the call may
// carry framed records (rec_off / rec_len); the contiguous loop never does, and must not issue
// those loads (their wait would cover the prefetched tile).
template <bool kFramed = true>
__device__ __forceinline__ TileCtx tile_ctx(const KernelArgs& a, int64_t tile, int lane) {
    TileCtx t;
    t.tile = tile;
    t.rec = tile * kWave + lane;
    t.active = t.rec < a.n_rec;
    t.base = a.base_shift;
    t.avail = 0;
    t.seg = -1;
    if (kFramed && a.rec_off) {
        if (t.active) { t.base += a.rec_off[t.rec]; t.avail = a.rec_len[t.rec]; }
    } else if (t.active) {
        t.base += t.rec * (int64_t)a.stride;
        t.avail = a.stride;
    }
    return t;
}

// Per-record prologue: segment-redefine selection and OCCURS DEPENDING ON element counts
// (their count columns written here), reading the record at rp (the LDS image in contiguous
// mode -- no HBM loads in that loop besides the staging loads -- or HBM).
// kSeg / kArr: the plan may have a segment map / OCCURS DEPENDING ON arrays (the specialised
// kernel compiles only the parts its plan has).
template <bool kSel = true, bool kSeg = true, bool kArr = true>
__device__ __forceinline__ void tile_prologue(const KernelArgs& a, TileCtx& t, const uint8_t* rp, int lane,
                                              const uint32_t* s_lut, int32_t* s_cnt) {
    // ---- segment redefine selection
    if (kSel && a.rec_seg) t.seg = t.active ? a.rec_seg[t.rec] : -1;   // selected records: segment known
    else if (kSeg && a.segmap && t.active) t.seg = segment_of(a, s_lut, rp, t.avail);
    if (kSeg && kmode(a) == 0 && a.seg_col >= 0) {
        const DevColumn c = ldc(a.cols + a.seg_col);
        if (t.active) gp((int32_t*)c.values)[t.rec] = t.seg;
        const uint64_t m = __ballot(t.active);
        if (lane == 0) gp(c.validity)[t.tile] = m;
    }

    // ---- OCCURS DEPENDING ON element counts (extractArray, RecordExtractors.scala:66-114)
    for (int ai = 0; kArr && ai < a.n_arrays; ai++) {
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
        if (a.odo_count && t.active && t.rec < a.odo_pitch) {
            // the caller's count (hierarchical records: the dependee registered by an earlier segment
            // of the record, extractHierarchicalRecord's shared dependFields)
            const int32_t oc = a.odo_count[(int64_t)ai * a.odo_pitch + t.rec];
            if (oc >= 0) cnt = oc;
        }
        s_cnt[ai * kWave + lane] = cnt;
        if (ar.offsets_column >= 0 && kmode(a) == 0) {
            // list layout: the record's present elements (none when the array's segment is not the
            // record's) get a run of the tile's child region starting at a multiple of 64; the
            // list kernel decodes them from these starts and lengths
            const int len = t.active && (ar.segment < 0 || ar.segment == t.seg) ? cnt : 0;
            uint32_t tot;
            const uint32_t ex = wave_excl_scan32(((uint32_t)len + 63u) & ~63u, lane, tot);
            const DevColumn c = ldc(a.cols + ar.offsets_column);
            const int64_t mpad = (int64_t)((ar.max_count + 63) & ~63);
            (gp((int64_t*)c.values) + t.tile * kWave)[lane] = t.tile * kWave * mpad + ex;
            (gp(a.list_len + (int64_t)ai * a.pitch) + t.tile * kWave)[lane] = len;
            const uint64_t m = __ballot(t.active);
            if (lane == 0) gp(c.validity)[t.tile] = m;
        }
        if (kmode(a) == 0 && ar.count_column >= 0) {
            const DevColumn c = ldc(a.cols + ar.count_column);
            const bool ok = t.active && (ar.segment < 0 || ar.segment == t.seg);
            if (t.active) gp((int32_t*)c.values)[t.rec] = cnt;
            const uint64_t m = __ballot(ok);
            if (lane == 0) gp(c.validity)[t.tile] = m;
        }
    }
}

// Diagnostic build only (-DCBX_STAMPS, tools/stamps.py): s_memtime stamps between the segments
// of the contiguous tile loop, summed per segment over all waves.  The product build has none.
struct Stamps {
#ifdef CBX_STAMPS
    uint64_t acc[8];
    unsigned long long last;
    __device__ __forceinline__ void init() {
        for (int k = 0; k < 8; k++) acc[k] = 0;
        last = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    __device__ __forceinline__ void mark(int k) {
        __builtin_amdgcn_sched_barrier(0);
        unsigned long long t;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        acc[k] += t - last;
        last = t;
    }
    __device__ __forceinline__ void flush(const KernelArgs& a, int lane) {
        if (lane == 0 && a.stamps) {
            for (int k = 0; k < 6; k++) atomicAdd((unsigned long long*)a.stamps + k, (unsigned long long)acc[k]);
            atomicAdd((unsigned long long*)a.stamps + 7, 1ull);
        }
    }
#else
    __device__ __forceinline__ void init() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(const KernelArgs&, int) {}
#endif
};

// LDS carve-up of a decode workgroup: the code page LUT, then one region per wave.
struct WaveLds {
    uint32_t* lut;
    uint8_t* img;       // record image (after the front guard)
    int32_t* cnt;       // OCCURS element counts
    uint8_t* str;       // string payload staging
    int wid;            // the wave in its workgroup (coop_loop: which part of the tile's ops it runs)
};

// The kernels' only LDS is the dynamic area (extern smem, no static __shared__), which starts at LDS
// address 0: the LUT at its front is at LDS address 0, where the string paths read it through integer
// LDS addresses (lds_ld: the byte * 4 itself, no add, no pointer conversion).  lds_base_ok checks
// the assumption on the device.  (A pointer built from the constant address 0 is the LDS null pointer
// to the compiler: torch's hipRTC dropped the fill's store to entry 0 through one.)
__device__ __forceinline__ bool lds_base_ok(const uint8_t* smem) {
    return (uint32_t)(size_t)(__attribute__((address_space(3))) const uint8_t*)smem == 0u;
}

__device__ __forceinline__ WaveLds wave_lds(const KernelArgs& a, uint8_t* smem, int wid) {
    WaveLds l;
    l.lut = (uint32_t*)smem;
    uint8_t* wbase = smem + kLutLds + wid * a.lds_wave;
    l.img = wbase + kGuard;
    l.cnt = (int32_t*)(wbase + a.lds_rows);
    l.str = wbase + a.lds_rows + a.lds_counts;
    l.wid = wid;
    return l;
}

// LDS carve-up of a cooperative workgroup (coop_loop): the LUT, ONE record image for the
// workgroup's tile, then each wave's counts / string staging / dump area (lds_wave - lds_rows).
__device__ __forceinline__ WaveLds coop_lds(const KernelArgs& a, uint8_t* smem, int wid) {
    WaveLds l;
    l.lut = (uint32_t*)smem;
    // the image offset opaque (an SGPR): with the constant address torch's bundled hipRTC (the one a
    // product process resolves libhiprtc.so.7 to) crashed compiling the kernel (tests/test_jit_rtc.py)
    int img_off = kLutLds + kGuard;
    asm volatile("" : "+s"(img_off));
    l.img = smem + img_off;
    uint8_t* wbase = smem + kLutLds + a.lds_rows + wid * (a.lds_wave - a.lds_rows);
    l.cnt = (int32_t*)wbase;
    l.str = wbase + a.lds_counts;
    l.wid = wid;
    return l;
}

// Fixed-length records, the whole tile span staged once per tile, its loads issued one tile
// ahead.  Nothing else in this loop loads from HBM (prologue and decode read the LDS image), so
// no wait on the staging loads or on earlier stores sits in the decode.  `body` decodes one
// staged tile in two parts, body.pre and body.post (img, rec_addr, lds, lane, stamps).  kLate:
// the next tile's loads are issued between the two parts instead of before both -- the
// specialised kernel puts a layout's string elements in `pre` when it also has numerics, so the
// string phase's register peak does not stack on the prefetch registers.
// Tile order of a wave: grid-stride over single tiles, or -- for a body that gathers its words
// over runs (Body::kWords > 0, VWords) -- over runs of kVRun consecutive tiles.
template <typename Body>
__device__ __forceinline__ int64_t first_tile(int64_t wave) { return Body::kWords > 0 ? wave * kVRun : wave; }
template <typename Body>
__device__ __forceinline__ int64_t next_tile(int64_t tile, int64_t tstep) {
    if (Body::kWords == 0) return tile + tstep;
    return ((tile + 1) % kVRun) ? tile + 1 : tile + 1 + (tstep - 1) * kVRun;
}
// end of the tile's run: the body's gathered words go out
template <typename Body>
__device__ __forceinline__ void run_end(const KernelArgs& a, Body& body, int64_t tile, int lane) {
    if (Body::kWords > 0 && (((tile + 1) % kVRun) == 0 || tile + 1 >= a.n_tiles)) body.flush(a, tile - tile % kVRun, lane);
}

template <int KP, int kPro, bool kLate, typename Body>
__device__ __forceinline__ void contig_loop(const KernelArgs& a, const WaveLds& l, int64_t tile, int64_t tstep,
                                            int lane, Body body) {
    uint4 buf[KP];
    tile = first_tile<Body>(tile);
    if (tile < a.n_tiles) contig_issue<KP>(a, contig_span(a, tile), lane, buf);
    Stamps st;
    st.init();
    while (tile < a.n_tiles) {
        const ContigSpan sp = contig_span(a, tile);
        contig_store<KP>(a, sp, lane, buf, l.img);
        wave_sync_lds();
        st.mark(0);   // staging: wait for the prefetched loads + LDS writes
        const int64_t next = next_tile<Body>(tile, tstep);
        body.begin(tile);
        // issued even past the last tile (a span of no chunks: every offset out of range, no
        // access), so the buffer is always redefined here and never live across the decode
        if (!kLate) contig_issue<KP>(a, contig_span(a, next), lane, buf);
        st.mark(1);   // prefetch issue
        TileCtx t = tile_ctx<false>(a, tile, lane);
        const uint32_t rec0 = (uint32_t)(lane * a.cpitch + 4 * sp.mis_dw);   // record start in the image
        tile_prologue<false, (kPro & 1) != 0, (kPro & 2) != 0>(a, t, l.img + rec0, lane, l.lut, l.cnt);
        st.mark(2);   // prologue
        body.pre(a, t, (const uint8_t*)l.img, rec0 + (uint32_t)a.start_off, l, lane, st);
        if (kLate) contig_issue<KP>(a, contig_span(a, next), lane, buf);
        body.post(a, t, (const uint8_t*)l.img, rec0 + (uint32_t)a.start_off, l, lane, st);
        run_end(a, body, tile, lane);
        wave_sync_lds();
        st.mark(5);   // end of tile
        tile = next;
    }
    st.flush(a, lane);
}

// Cooperative tiles: the kWavesPerBlock waves of a workgroup decode ONE tile together -- each
// stages its share of the span's chunks into the workgroup's image and runs its part of the
// tile's ops (the specialised kernel splits them by cost, body.pre / body.post dispatch on
// l.wid).  The image (64 records) is shared, so a wave's LDS is its string staging only: on
// SYNSTR200 (12.8 KB of records per tile) twice the resident waves of contig_loop, whose waves
// each hold their own tile's image -- string-heavy layouts, whose decode waits on LDS round
// trips (LUT reads, slot writes and read-backs), want the waves.  Two workgroup barriers per tile
// (image complete; image read before it is overwritten).  Plans without segment selection,
// OCCURS arrays and run-gathered words only (the prologue writes nothing, every op's output is
// its own).  Chunk row u (chunks u * 64 + lane) is staged by wave u % kWavesPerBlock.
template <int KP>
__device__ __forceinline__ void coop_issue(const KernelArgs& a, const ContigSpan& sp, int wid, int lane,
                                           uint4 (&buf)[(KP + kWavesPerBlock - 1) / kWavesPerBlock]) {
    constexpr int KH = (KP + kWavesPerBlock - 1) / kWavesPerBlock;
    int64_t left = a.data_len - sp.a0;
    left = left < 0 ? 0 : (left > (1 << 20) ? (1 << 20) : left);
    const uint64_t base = (uint64_t)(a.data + sp.a0);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane((int)left);
    const int nch = __builtin_amdgcn_readfirstlane(sp.nch);
    void* bp = (void*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(bp, (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int v = 0; v < KH; v++) {
        const int c = (v * kWavesPerBlock + wid) * kWave + lane;
        const int off = c < nch ? 16 * c : 0x7ffffff0;   // past the descriptor's range: no access
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kStageCpol);
        buf[v] = make_uint4(x[0], x[1], x[2], x[3]);
    }
}

// Chunk rows of the wave's share (coop_issue's buf) into the workgroup's image; waits for the loads.
template <int KP>
__device__ __forceinline__ void coop_put(const KernelArgs& a, const ContigSpan& sp, int wid, int lane,
                                         const uint4 (&buf)[(KP + kWavesPerBlock - 1) / kWavesPerBlock], uint8_t* s_img) {
    constexpr int KH = (KP + kWavesPerBlock - 1) / kWavesPerBlock;
    int ln = lane;
    asm volatile("" : "+v"(ln));   // (contig_store: no LDS addresses held across the decode)
#pragma unroll
    for (int v = 0; v < KH; v++) {
        const int c = (v * kWavesPerBlock + wid) * kWave + ln;
        if (c < sp.nch) contig_put(a, sp, c, buf[v], s_img);
    }
}

// The next tile's image is written at the END of a tile (after the barrier that retires the image),
// not at the top of the next one: its loads, issued at the top, are then followed in the same
// iteration by the tile's value stores, and the wait for them is a counted vmcnt(N) that leaves those
// stores in flight.  (At the loop top the wait merged the loop entry -- loads with nothing behind
// them -- and became vmcnt(6..0): every tile waited for all of the previous tile's stores to be
// acknowledged, in issue order, before staging.)  The first tile is loaded and staged before the loop.
// kW: the wave (the kernel runs one instantiation per wave), so the wave's part of the tile
// (body.part<kW>) is straight-line code between the loads and the wait for them.
template <int KP, int kW, typename Body>
__device__ __forceinline__ void coop_loop(const KernelArgs& a, const WaveLds& l, int64_t tile, int64_t tstep,
                                          int lane, Body body) {
    constexpr int KH = (KP + kWavesPerBlock - 1) / kWavesPerBlock;
    uint4 buf[KH];
    constexpr int wid = kW;
    body.wid = wid;
#ifndef CBX_NO_COOP_PRIO
    // the tile's second wave at issue priority 1 for the whole loop (no per-segment flips): the
    // younger wave of a pair otherwise loses every VALU arbitration to the older one and the tile's
    // barriers wait on it (MI355X_MICROARCH.md, two waves per SIMD, item 4).  SYN200 decode 3.83 ->
    // 3.72 ms, three same-box pairs (profiles/r05_ab/coop_prio.log)
    if (wid == 1) __builtin_amdgcn_s_setprio(1);
#endif
    tile = first_tile<Body>(tile);   // (the workgroup's tiles: runs of kVRun with run-gathered words)
    if (tile >= a.n_tiles) return;
    coop_issue<KP>(a, contig_span(a, tile), wid, lane, buf);
    coop_put<KP>(a, contig_span(a, tile), wid, lane, buf, l.img);
    Stamps st;
    st.init();
    while (true) {
        __syncthreads();   // the tile's image complete
        st.mark(0);
        const ContigSpan sp = contig_span(a, tile);
        const int64_t next = next_tile<Body>(tile, tstep);
        body.begin(tile);
        // issued even past the last tile (a span of no chunks: every offset out of range, no access)
        coop_issue<KP>(a, contig_span(a, next), wid, lane, buf);
        st.mark(1);
        TileCtx t = tile_ctx<false>(a, tile, lane);
        const uint32_t rec0 = (uint32_t)(lane * a.cpitch + 4 * sp.mis_dw);
        st.mark(2);
        body.template part<kW>(a, t, (const uint8_t*)l.img, rec0 + (uint32_t)a.start_off, l, lane, st);
        run_end(a, body, tile, lane);
        __syncthreads();   // every wave done with the image
        st.mark(5);
        tile = next;
        if (tile >= a.n_tiles) break;
        coop_put<KP>(a, contig_span(a, tile), wid, lane, buf, l.img);
    }
    st.flush(a, lane);
}

// ---- variable-length records staged by byte span ----
// cbx_decode_var over records that lie close together in the input (RDW / text framing): a tile's
// byte span [min payload offset, max(offset + max(length, span_ext))) that fits KP 16-byte chunks
// per lane is staged like a fixed-length tile -- buffer loads issued one tile ahead, nothing else
// loaded from HBM in the decode -- and lane r decodes its record at (offset - span start) in the
// image.  The record offsets / lengths themselves are loaded two tiles ahead.  A tile whose span
// does not fit (long records, records far apart) is staged record by record over [0, span_ext)
// (stage_window), like the windowed kernel.  Lanes past n_rec reuse the last record, length 0.
__device__ __forceinline__ void span_recs(const KernelArgs& a, int64_t tile, int lane, int64_t& off, int32_t& len) {
    const int64_t r = tile * kWave + lane;
    const int64_t rc = r < a.n_rec ? r : a.n_rec - 1;   // loads always issued (registers always defined)
    const int64_t o = a.rec_off[rc];
    const int32_t l = a.rec_len[rc];
    off = a.base_shift + o;
    len = r < a.n_rec ? l : 0;
}

__device__ __forceinline__ int64_t wave_min64(int64_t v) {
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) {
        const int64_t o = __shfl_xor(v, m, kWave);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) {
        const int64_t o = __shfl_xor(v, m, kWave);
        v = o > v ? o : v;
    }
    return v;
}

// The span of a tile (nch = 0: past the last tile, or too wide for KP chunks per lane).
template <int KP>
__device__ __forceinline__ ContigSpan span_of(const KernelArgs& a, int64_t tile, int64_t off, int32_t len) {
    const int64_t lo = wave_min64(off);
    const int64_t hi = wave_max64(off + (len > a.span_ext ? len : a.span_ext));
    ContigSpan sp;
    sp.a0 = lo & ~(int64_t)15;
    const int64_t nch = (hi - sp.a0 + 15) >> 4;
    sp.nch = (tile < a.n_tiles && nch <= (int64_t)KP * kWave) ? (int)nch : 0;
    sp.mis_dw = 0;
    sp.span_dw = 0;
    return sp;
}

template <int KP>
__device__ __forceinline__ void span_store(const ContigSpan& sp, int lane, const uint4 (&buf)[KP], uint8_t* s_img) {
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int u = 0; u < KP; u++) {
        const int c = u * kWave + lane;
        if (u * kWave < sp.nch && c < sp.nch) *(uint4*)(s_img + 16 * c) = buf[u];
    }
}

template <int KP, int kPro, bool kLate, typename Body>
__device__ __forceinline__ void span_loop(const KernelArgs& a, const WaveLds& l, int64_t tile, int64_t tstep,
                                          int lane, Body body) {
    tile = first_tile<Body>(tile);
    if (tile >= a.n_tiles) return;
    uint4 buf[KP];
    int64_t off_c, off_n;
    int32_t len_c, len_n;
    span_recs(a, tile, lane, off_c, len_c);
    span_recs(a, next_tile<Body>(tile, tstep), lane, off_n, len_n);
    ContigSpan sp_c = span_of<KP>(a, tile, off_c, len_c);
    contig_issue<KP>(a, sp_c, lane, buf);
    Stamps st;
    st.init();
    while (tile < a.n_tiles) {
        const int64_t next = next_tile<Body>(tile, tstep);
        const ContigSpan sp = sp_c;
        const int64_t off = off_c;
        const int32_t len = len_c;
        if (sp.nch > 0) span_store<KP>(sp, lane, buf, l.img);
        // the next tile's span (its offsets were loaded a tile ago) and the offsets of the one after
        sp_c = span_of<KP>(a, next, off_n, len_n);
        off_c = off_n;
        len_c = len_n;
        span_recs(a, next_tile<Body>(next, tstep), lane, off_n, len_n);
        body.begin(tile);
        TileCtx t;
        t.tile = tile;
        t.rec = tile * kWave + lane;
        t.active = t.rec < a.n_rec;
        t.base = off;
        t.avail = t.active ? len : 0;
        t.seg = -1;
        uint32_t rec_addr;
        if (sp.nch > 0) {
            rec_addr = (uint32_t)(off - sp.a0) + (uint32_t)a.start_off;
        } else {   // record by record: [0, span_ext) of every record's decode base
            Window w{};
            w.lo = 0;
            w.hi = a.span_ext - a.start_off;
            w.pitch = a.span_pitch;
            rec_addr = stage_window(a, w, t, l.img, lane);
        }
        wave_sync_lds();
        st.mark(0);
        if (!kLate) contig_issue<KP>(a, sp_c, lane, buf);
        st.mark(1);
        tile_prologue<false, (kPro & 1) != 0, (kPro & 2) != 0>(a, t, l.img + rec_addr - a.start_off, lane, l.lut, l.cnt);
        st.mark(2);
        body.pre(a, t, (const uint8_t*)l.img, rec_addr, l, lane, st);
        if (kLate) contig_issue<KP>(a, sp_c, lane, buf);
        body.post(a, t, (const uint8_t*)l.img, rec_addr, l, lane, st);
        run_end(a, body, tile, lane);
        wave_sync_lds();
        st.mark(5);
        tile = next;
    }
    st.flush(a, lane);
}

}  // namespace cbx
