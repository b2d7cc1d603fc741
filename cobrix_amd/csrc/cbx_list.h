// OCCURS DEPENDING ON list layout: the element-parallel list kernel (list_kernel, and the copybook-
// specialised cbx_jit_list built from the same loop, cbx_jit.h).
#pragma once
#include "cbx_device.h"

namespace cbx {

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

// Issue the staging DMA of group g0 of record r into buf (kListKP 16-byte chunks per lane, chunk c
// of the group at buf + 16 c; chunks past the group: no access).
__device__ __forceinline__ void list_issue(const KernelArgs& a, const ListRec& r, int elo, int stride, int g0, int gsteps,
                                           int lane, uint8_t* buf) {
    const int s0 = r.bias + a.start_off + elo + g0 * kWave * stride;
    const int s16 = s0 & ~15;
    const int n16 = list_n16(r, s0, s16, g0, gsteps, stride);
#pragma unroll
    for (int u = 0; u < kListKP; u++) {
        const int c = u * kWave + lane;
        lds_dma16(r.rs, c < n16 ? (uint32_t)(s16 + 16 * c) : 0x7ffffff0u, buf + 16 * u * kWave);
    }
}

// ---- the specialised list kernel's field step (cbx_jit.h: cbx_jit_list) ----
// One field of the lanes' elements of one step of a clean group (every present element inside the
// record and its safe range), the field's op a compile-time constant: e = LDS address one past the
// lane's field; cstart: the child index of the step's element 0 (a multiple of 64).  The fast
// decoders of the record kernel at the op's output width; zoned forms they cannot decide raise
// `deferred` (the byte-loop pass list_kernel<true> redoes them), as list_item does.
__device__ __forceinline__ uint64_t le64_ending_ptr(const uint8_t* e) {
    const uint8_t* s = e - 8;
    const uint32_t sh = (uint32_t)(size_t)s & 3u;
    const uint32_t* p = (const uint32_t*)(s - sh);
    const uint32_t r0 = p[0], r1 = p[1], r2 = p[2];
    return ((uint64_t)align_bytes(r2, r1, sh) << 32) | align_bytes(r1, r0, sh);
}
// the 4 bytes ending at e in the high half (fields of <= 4 bytes: the decoders mask the rest)
__device__ __forceinline__ uint64_t le32_ending_ptr(const uint8_t* e) {
    const uint8_t* s = e - 4;
    const uint32_t sh = (uint32_t)(size_t)s & 3u;
    const uint32_t* p = (const uint32_t*)(s - sh);
    return (uint64_t)align_bytes(p[1], p[0], sh) << 32;
}

// The lane's element bytes as whole aligned 8-byte words: ds_read_b64 of lanes 8 bytes apart
// (an 8-byte element stride) covers one 256-byte bank row per 32 lanes -- no bank conflict, where
// the per-field dword reads of lanes 8 bytes apart put two lanes on every ds_read_b32 bank (C5's
// list kernel: SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS 4.0) and read each dword once per field.
// Words K0 .. K0 + NW - 1 around el's 8-byte aligned address (K0 <= 0: bytes before the element);
// ph: el's byte phase in its word.  d holds 2 NW dwords + 2 zero dwords (selects past the end).
template <int K0, int NW>
__device__ __forceinline__ void list_words(const uint8_t* el, uint32_t& ph, uint32_t (&d)[2 * NW + 2]) {
    const uint32_t a = lds_addr(el);
    ph = a & 7u;
    const uint32_t a8 = (a & ~7u) + (uint32_t)(8 * K0);
#pragma unroll
    for (int k = 0; k < NW; k++) {
        // (each word its own ds_read_b64: 2 LDS cycles, conflict-free; the pair merged into one
        // ds_read2_b64 would take 8 -- MI355X_MICROARCH.md LDS table)
        uint32_t ak = a8 + 8u * (uint32_t)k;
        if (k) asm volatile("" : "+v"(ak));
        const uint64_t w = lds_ld<uint64_t>(ak);
        d[2 * k] = (uint32_t)w;
        d[2 * k + 1] = (uint32_t)(w >> 32);
    }
    d[2 * NW] = d[2 * NW + 1] = 0u;
}

// The 8 bytes at window byte C + ph (C: a compile-time offset, ph: the lane's phase 0..7) as a
// little-endian u64: dword j = (C + ph) / 4 is one of three candidates, picked by selects.
template <int C, int NW>
__device__ __forceinline__ uint64_t list_win8(const uint32_t (&d)[2 * NW + 2], uint32_t ph) {
    static_assert(C >= 0 && (C + 7) / 4 + 2 <= 2 * NW + 1, "element window too small");
    constexpr int J = C / 4;
    const uint32_t o = (uint32_t)C + ph;
    const uint32_t j = o >> 2, sh = o & 3u;
    uint32_t x0 = d[J], x1 = d[J + 1], x2 = d[J + 2];
    if (j >= (uint32_t)J + 1) { x0 = d[J + 1]; x1 = d[J + 2]; x2 = d[J + 3 < 2 * NW + 2 ? J + 3 : 2 * NW + 1]; }
    if (j >= (uint32_t)J + 2) { x0 = d[J + 2]; x1 = d[J + 3 < 2 * NW + 2 ? J + 3 : 2 * NW + 1]; x2 = d[J + 4 < 2 * NW + 2 ? J + 4 : 2 * NW + 1]; }
    return ((uint64_t)align_bytes(x2, x1, sh) << 32) | align_bytes(x1, x0, sh);
}

// list_jit_field from the element's words: E = the field's end within the element, K0 the window's
// first word (list_words).
template <int V, int W, bool SMALL, int E, int K0, int NW>
__device__ __forceinline__ void list_jit_field_w(const NumOp& op, const DevColumn& col, const uint32_t (&d)[2 * NW + 2],
                                                 uint32_t ph, int64_t cstart, bool present, int lane, bool& deferred) {
    // SMALL: a field of <= 4 bytes of the BCD8 / BIN8 / FP decoders, its bytes in the high half
    uint64_t r1;
    if constexpr (SMALL) r1 = list_win8<E - 4 - 8 * K0, NW>(d, ph) << 32;
    else r1 = list_win8<E - 8 - 8 * K0, NW>(d, ph);
    uint64_t r0 = 0ull;
    if constexpr (V == V_BCD16 || V == V_ZONED16) r0 = list_win8<E - 16 - 8 * K0, NW>(d, ph);
    bool slow = false;
    Val x;
    if (V == V_BCD8) x = bcd8_raw<W>(op, r1);
    else if (V == V_BCD16) x = bcd16_raw<W>(op, r1, r0);
    else if (V == V_BIN8) x = bin8_raw<W>(op, r1);
    else if (V == V_ZONED16) x = zoned16_raw<W>(op, r1, r0, slow);
    else x = fp_raw(op, r1);
    if (V == V_ZONED16) {
        slow &= present;
        deferred |= __ballot(slow) != 0;
        x.valid &= !slow;
    }
    x.valid &= present;
    store_w<W>(col.values, cstart >> 6, lane, x, op.out_type);
    const uint64_t vm = __ballot(x.valid);
    gp(col.validity)[cstart >> 6] = vm;
}

template <int V, int W>
__device__ __forceinline__ void list_jit_field(const NumOp& op, const DevColumn& col, const uint8_t* e, int64_t cstart,
                                               bool present, int lane, bool& deferred) {
    const bool small = op.size <= 4 && (V == V_BCD8 || V == V_BIN8 || V == V_FP);
    const uint64_t r1 = small ? le32_ending_ptr(e) : le64_ending_ptr(e);
    const uint64_t r0 = (V == V_BCD16 || V == V_ZONED16) ? le64_ending_ptr(e - 8) : 0ull;
    bool slow = false;
    Val x;
    if (V == V_BCD8) x = bcd8_raw<W>(op, r1);
    else if (V == V_BCD16) x = bcd16_raw<W>(op, r1, r0);
    else if (V == V_BIN8) x = bin8_raw<W>(op, r1);
    else if (V == V_ZONED16) x = zoned16_raw<W>(op, r1, r0, slow);
    else x = fp_raw(op, r1);
    if (V == V_ZONED16) {
        slow &= present;
        deferred |= __ballot(slow) != 0;
        x.valid &= !slow;
    }
    x.valid &= present;
    store_w<W>(col.values, cstart >> 6, lane, x, op.out_type);
    const uint64_t vm = __ballot(x.valid);
    gp(col.validity)[cstart >> 6] = vm;
}

// A group body that decodes nothing itself (the table-driven field loop does).
struct ListFieldLoop {
    __device__ __forceinline__ bool group(const KernelArgs&, int, const uint8_t*, const ListRec&, int, int, int, bool&) {
        return false;
    }
};

template <bool kFix, typename Body>
__device__ __forceinline__ void list_run(const KernelArgs& a, const CBX_CONST ListOp* lops, int32_t n_lops, Body& body) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x % kWave;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    // two staging buffers per wave: the next group's DMA lands in one while the other is decoded
    uint8_t* const imgs = smem + wid * 2 * (kGuard + kListStage + kGuard) + kGuard;
    uint8_t* img = imgs;
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
            int buf = 0;
            if (staged) list_issue(a, cur, elo, stride, g0, gsteps, lane, imgs);
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
                // this group's DMA (issued a group ago) and the previous group's stores retire (on every
                // path: the compiler then waits for none of its older loads during the decode), then
                // the next group's DMA goes into the other buffer (its last reads were the previous
                // group's, done) while this group is decoded
                lds_dma_wait(0);
                if (staged) {
                    uint8_t* other = imgs + (buf ^ 1) * (kGuard + kListStage + kGuard);
                    if (more) list_issue(a, nxt, elo, stride, ng0, gsteps, lane, other);
                    img = imgs + buf * (kGuard + kListStage + kGuard);
                    buf ^= 1;
                }
                // field by field (its descriptor loaded once per group), the group's steps -- unless the
                // body decodes the group itself (the specialised list kernel, cbx_jit.h)
                const bool done = !kFix && staged &&
                                  body.group(a, ai, img + (s0 - s16), cur, g0, gn, lane, deferred);
                for (int i = i0; i < i1 && !done; i++) {
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
                if (!more) break;
                cur = nxt;
                g0 = ng0;
            }
            i0 = i1;
        }
        if (!kFix) gp(a.list_flag)[tile] = deferred ? 1 : 0;
    }
}


}  // namespace cbx
