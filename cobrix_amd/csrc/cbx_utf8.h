// cbx_utf8.h -- the Arrow Utf8 layout in ONE pass over the input (cbx_jit_utf8).
//
// The two-pass form (cbx_device.h: a count kernel re-reads the whole batch for the per-tile UTF-8
// totals, a device scan, then the decode) reads the input twice.  Here the decode itself produces
// each tile's totals and resolves the tile's place in every string column with a decoupled
// look-back over the other tiles' totals, in the same launch:
//
// * Workgroup = 4 waves, ONE tile (64 records) per workgroup and round (grid-stride): the tile's
//   record image is staged once into LDS and shared; the tile's string elements (and numerics) are
//   split between the waves by cost (cbx_jit.h: jit_utf8_source).
// * Per string element (a wave, lane = record): the characters' LUT entries, trim range and UTF-8
//   length, a wave scan of the lengths (tile-local starts, the tile's total), then the UTF-8 bytes
//   composed straight into the element's tile-contiguous LDS staging at their tile-local positions
//   -- 4 characters at a time with one v_perm selector per group read from a 81-entry table of
//   width patterns (0, 1 or 2 bytes per character: characters outside the trimmed range have
//   width 0, so nothing lands outside the value) and OR-ed into the zeroed staging (neighbouring
//   values share boundary dwords).  The tile's total is published as soon as it is known.
// * Look-back (StringDecoders' offsets are one running sum per column): tiles in blocks of 64.  A
//   tile sums the totals of the tiles before it in its block, then walks back over the block
//   aggregates (B: a block's total, published by its last tile; P: the inclusive prefix through the
//   block) to the nearest P.  Every value is an 8-byte {value, tag} granule stored and polled with
//   agent-scope (sc1) atomics -- the tag is the launch's epoch, so the arrays are never cleared.
// * Then the element's int32 offsets (place + tile-local start) and ONE coalesced copy of the
//   staged payload to its final place (16-byte stores, byte stores at the two ends).
//
// Forward progress does not depend on workgroup residency: a probe that stays unanswered for
// lb_spin polls recounts the missing totals from the input itself (lb_recount: the same trim and
// UTF-8 rules over HBM bytes) -- slow, never wrong.  Recounts are counted in status[1].
//
// Reference: StringDecoders.decodeEbcdicString / decodeAsciiString + StringTools.trim*
// (CP/parser/decoders/StringDecoders.scala:44-89, CP/utils/StringTools.scala:28-61): the value is
// the trimmed characters' UTF-8 bytes; Arrow Utf8 = int32 offsets + the concatenated payload.
#pragma once
#include "cbx_device.h"

namespace cbx {

constexpr int kLbBlock = 64;            // tiles per look-back block
constexpr int kU8Waves = 4;             // waves per workgroup of the one-pass kernel
constexpr int kU8SelOff = 1024;         // LDS: the 81 width-pattern selectors after the 1 KiB LUT
constexpr int kU8LutLds = 1024 + 8 * 81 + 8;   // LUT + selectors (+8: 16-byte aligned image start)

// Width-pattern selector i (= 3^0 w0 + 3^1 w1 + 3^2 w2 + 3^3 w3, w_k in 0..2 the UTF-8 bytes of
// character k of a group) for v_perm over (U23, U01) -- character k's first byte at source 2k, its
// second at 2k + 1: the bytes of the characters in order, then zero bytes (0x0C).  Dword h of entry i.
__host__ __device__ constexpr uint32_t u8_sel(int i, int h) {
    uint64_t v = 0x0C0C0C0C0C0C0C0Cull;
    int n = 0, x = i;
    for (int k = 0; k < 4; k++) {
        const int w = x % 3;
        x /= 3;
        for (int m = 0; m < w; m++) {
            v = (v & ~(0xFFull << (8 * n))) | ((uint64_t)(2 * k + m) << (8 * n));
            n++;
        }
    }
    return (uint32_t)(v >> (32 * h));
}

// LDS carve-up of the one-pass workgroup: LUT (at LDS 0, lds_ld) + selectors, the tile's record
// image, then the string elements' staging regions (offsets fixed by the specialised kernel).
struct U8Lds {
    uint8_t* img;       // record image (after the front guard)
    uint32_t stage;     // LDS byte address of the first staging region
    const int32_t* cnt; // (no OCCURS arrays on this path: the numeric ops' count table is unused)
    int wid;
};

__device__ __forceinline__ U8Lds u8_lds(const KernelArgs& a, uint8_t* smem, int wid) {
    U8Lds l;
    int img_off = kU8LutLds + kGuard;
    asm volatile("" : "+s"(img_off));   // (opaque: see coop_lds)
    l.img = smem + img_off;
    l.stage = lds_addr(smem) + (uint32_t)(kU8LutLds + a.lds_rows);
    l.cnt = nullptr;
    l.wid = wid;
    return l;
}

__device__ __forceinline__ void u8_lut_fill(const KernelArgs& a, uint32_t* lut) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = a.lut[i];
    for (int i = threadIdx.x; i < 2 * 81; i += blockDim.x) lut[256 + i] = u8_sel(i >> 1, i & 1);
}

// ---- look-back granules: {value (low 32 bits), tag (high 32 bits)}, agent-scope relaxed atomics
__device__ __forceinline__ uint64_t lb_ld(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_st(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_gran(uint32_t tag, uint64_t v) {
    return ((uint64_t)tag << 32) | (v > 0xFFFFFFFFull ? 0xFFFFFFFFull : v);
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v, int lane) {
    uint32_t tot;
    (void)wave_excl_scan32(v, lane, tot);
    return tot;
}

// The UTF-8 bytes of element op in the lane's record of tile `tile`, counted from the input in HBM
// (the look-back's fallback for a total left unpublished): the decode's trim and UTF-8 rules, byte by
// byte.  Inlined once (u8_place's tile-group step): a call would make the kernel's register state
// go through scratch memory in the hot loop.
__device__ __forceinline__ uint32_t lb_recount_lane(const KernelArgs& a, const StrOp& op, int64_t tile, int lane) {
    const int64_t r = tile * kWave + lane;
    uint32_t len = 0;
#ifdef U8_NO_RECOUNT
    if (false) {
#else
    if (r < a.n_rec) {
#endif
        const int o = a.start_off + op.eo;
        const int avail = a.stride;
        if (o <= avail) {
            const int n = op.size < avail - o ? op.size : avail - o;
            const uint8_t* p = a.data + a.base_shift + r * (int64_t)a.stride + o;
            const uint32_t* lut = a.lut;
            const int kind = op.kind;
            len = (uint32_t)string_span(kind, op.trim, p, n, [&](uint32_t b) { return str_lut(kind, lut, b); }).utf8_len;
        }
    }
    return len;
}

// Poll budget: a.lb_spin polls, 16 once some probe of the launch had to recount (a workgroup that
// owns tiles is not running: wait little, recount).
__device__ __forceinline__ int lb_budget(const KernelArgs& a) {
    return __hip_atomic_load(a.status + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 16 : a.lb_spin;
}

// The totals of tiles [t0, t0 + n) (n <= 64, lane j: tile t0 + j) of sequence op.seq, polled up to
// `budget` times; returns the lanes still unpublished.
__device__ __forceinline__ uint64_t lb_probe_tiles(const KernelArgs& a, const StrOp& op, int64_t t0, int n, int lane, int budget,
                                                   uint32_t& val) {
    const uint64_t* p = a.lb_tile + (int64_t)op.seq * a.n_tiles + t0;
    val = 0;
    bool need = lane < n;
    for (int spin = 0; need || __ballot(need); spin++) {
        const uint64_t g = need ? lb_ld(p + lane) : 0ull;
        if (need && (uint32_t)(g >> 32) == a.lb_tag) { val = (uint32_t)g; need = false; }
        if (!__ballot(need) || spin >= budget) break;
        __builtin_amdgcn_s_sleep(2);
    }
    return __ballot(need);
}

// ---- the wave's ring of staged elements ----
// Every composed element waits in its wave's LDS ring until its place is known: an element of tile
// t is flushed while the wave composes its next tile (one round later), when every tile of t's round
// has published its total and the round's block totals B are out (each block's last tile publishes
// its B at the end of its round) -- in the round itself the tiles all reach their look-back at the
// same time and each waited on block totals one hop behind (17.6 ms per 50 M records against 6.0
// ms without a look-back, measured).  An element flushed in its own round (the ring full) sums
// the round's blocks from their tiles' totals instead.  Entries: [16-bit tile-local starts]
// [payload], allocated in order at their exact size; the FIFO of pending entries sits in lanes of
// four VGPRs (slot j in lane j).
struct U8Ring {
    uint32_t rb, rw;       // the wave's ring: LDS byte address, bytes
    uint32_t head, tail;   // next allocation, oldest entry
    int np, first;         // pending entries, FIFO slot of the oldest
    uint32_t f_op, f_tile, f_off, f_tot;
    uint32_t f_base;       // the entry's place when a batched probe resolved it (kU8NoBase: not yet)
};

constexpr uint32_t kU8NoBase = 0xFFFFFFFFu;

__device__ __forceinline__ void u8_ring_init(U8Ring& r, uint32_t rb, uint32_t rw) {
    r.rb = rb; r.rw = rw; r.head = r.tail = 0; r.np = 0; r.first = 0;
    r.f_op = r.f_tile = r.f_off = r.f_tot = 0;
    r.f_base = kU8NoBase;
}

// whether an entry of `need` bytes fits (contiguous: at the head or, wrapping, at the ring start)
__device__ __forceinline__ bool u8_fits(const U8Ring& r, uint32_t need) {
    if (r.np == 0) return need <= r.rw;
    if (r.np >= kWave) return false;
    if (r.head > r.tail) return r.rw - r.head >= need || r.tail >= need;
    if (r.head < r.tail) return r.tail - r.head >= need;
    return false;
}

__device__ __forceinline__ uint32_t u8_alloc(U8Ring& r, uint32_t need) {
    if (r.np == 0) r.head = r.tail = 0;
    else if (r.head > r.tail && r.rw - r.head < need) r.head = 0;
    const uint32_t off = r.head;
    r.head += need;
    return off;
}

__device__ __forceinline__ void u8_push(U8Ring& r, int lane, int op, int64_t tile, uint32_t off, uint32_t tot) {
    const int slot = (r.first + r.np) & (kWave - 1);
    if (lane == slot) { r.f_op = (uint32_t)op; r.f_tile = (uint32_t)tile; r.f_off = off; r.f_tot = tot; r.f_base = kU8NoBase; }
    r.np++;
}

__device__ __forceinline__ int64_t u8_oldest_tile(const U8Ring& r) {
    return (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)r.f_tile, r.first);
}

// ---- compose: one register-path string element of the tile into the wave's ring ----
// Code pages whose characters are 1 or 2 UTF-8 bytes (StrOp.pad <= 2: every EBCDIC page but the
// euro variants, ASCII).  The characters' LUT entries, the trim range and, per group of 4
// characters, the widths of the kept ones (0: outside [b, e)), the selector of that width pattern
// and the group's byte count; a wave scan of the lengths gives the tile-local starts and the tile's
// total.  If the ring lacks the entry's room nothing is written and false returned (the caller
// flushes the oldest entry and tries again).  Else the entry: the starts, the payload OR-ed into
// the zeroed region group by group at its running position; the validity word; the tile's total
// published for the look-back of the tiles after it.
constexpr int kU8NG = (kStrFastBytes + 3) / 4;

__device__ __forceinline__ void u8_or(uint32_t addr, uint32_t v) {
    __hip_atomic_fetch_or((__attribute__((address_space(3))) uint32_t*)(size_t)addr, v, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A ring entry: the lanes' 16-bit tile-local starts, then the payload.
constexpr uint32_t kU8ExBytes = 2 * kWave;

__device__ __forceinline__ bool u8_compose(const KernelArgs& a, const StrOp& op, int op_index, const StrCall& c, const TileCtx& t,
                                           const uint8_t* src, uint32_t rec_addr, U8Ring& r, int lane) {
    const int o = a.start_off + op.eo;
    const bool ok = t.active && o <= t.avail;
    const int n = ok ? (op.size < t.avail - o ? op.size : t.avail - o) : 0;
    const int smax = op.size;
    uint32_t w[8], ev[kStrFastBytes];
    img_bytes32(src, rec_addr + (ok ? (uint32_t)op.eo : 0u), smax, w);
    if (op.kind == CBX_K_STRING) {
#pragma unroll
        for (int j = 0; j < kStrFastBytes; j++) ev[j] = j < smax ? lds_ld<uint32_t>(byte_x4(w[j >> 2], j & 3)) : 0u;
    } else {
        lut_entries32(w, smax, [&](uint32_t b) { return ascii_lut(b); }, ev);
    }
    uint32_t u01[kU8NG], u23[kU8NG], lb[kU8NG];
    uint32_t tm = 0;
#pragma unroll
    for (int g = 0; g < kU8NG; g++) {
        if (4 * g >= smax) break;
        const uint32_t e0 = ev[4 * g], e1 = 4 * g + 1 < smax ? ev[4 * g + 1] : 0u;
        const uint32_t e2 = 4 * g + 2 < smax ? ev[4 * g + 2] : 0u, e3 = 4 * g + 3 < smax ? ev[4 * g + 3] : 0u;
        u01[g] = __builtin_amdgcn_perm(e1, e0, 0x05040100u);
        u23[g] = __builtin_amdgcn_perm(e3, e2, 0x05040100u);
        lb[g] = __builtin_amdgcn_perm(e1, e0, 0x0C0C0703u) | __builtin_amdgcn_perm(e3, e2, 0x07030C0Cu);
        const uint32_t tg = __builtin_amdgcn_udot4(lb[g] & 0x80808080u, 0x08040201u, 0u, false);   // 128 * trim bits
        tm |= 4 * g >= 7 ? tg << (4 * g - 7) : tg >> (7 - 4 * g);
    }
    const uint32_t keep = ~tm & bits_below(n);
    int b = 0, e = n;
    if (op.trim == CBX_TRIM_LEFT || op.trim == CBX_TRIM_BOTH) b = keep ? (int)ctz32(keep) : n;
    if (op.trim == CBX_TRIM_RIGHT || op.trim == CBX_TRIM_BOTH) e = keep ? 32 - (int)clz32(keep) : b;
    const uint32_t bb = (uint32_t)b * 0x01010101u, eb = (uint32_t)e * 0x01010101u + 0x7F7F7F7Fu;
    uint2 sel[kU8NG];
    uint32_t nb[kU8NG];
    uint32_t len = 0;
#pragma unroll
    for (int g = 0; g < kU8NG; g++) {
        if (4 * g >= smax) break;
        const uint32_t pos4 = 0x03020100u + 0x04040404u * (uint32_t)g;
        const uint32_t km = ((pos4 | 0x80808080u) - bb) & (eb - pos4);        // byte MSB: b <= position < e
        const uint32_t mk = __builtin_amdgcn_perm(km << 8, km, 0x090B080Au);   // 0xFF per kept character
        const uint32_t wm = lb[g] & mk & 0x03030303u;
        const uint32_t so = __builtin_amdgcn_udot4(wm, 0xD8481808u, 0u, false);   // 8 * (w0 + 3 w1 + 9 w2 + 27 w3)
        const uint64_t sv = lds_ld<uint64_t>((uint32_t)kU8SelOff + so);
        sel[g] = make_uint2((uint32_t)sv, (uint32_t)(sv >> 32));
        nb[g] = __builtin_amdgcn_udot4(wm, 0x01010101u, 0u, false);
        len += nb[g];
    }
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(len, lane, tot);
    const uint32_t need = kU8ExBytes + ((tot + 8u + 15u) & ~15u);
#ifndef U8_PRECHECK
    if (!u8_fits(r, need)) return false;
#endif
    const uint32_t entry = r.rb + u8_alloc(r, need);
    u8_push(r, lane, op_index, t.tile, entry - r.rb, tot);
    gp(c.validity)[t.tile] = __ballot(ok);
    if (lane == 0) lb_st(a.lb_tile + (int64_t)op.seq * a.n_tiles + t.tile, lb_gran(a.lb_tag, tot));
    *(__attribute__((address_space(3))) uint16_t*)(size_t)(entry + 2u * (uint32_t)lane) = (uint16_t)ex;
    const uint32_t stage = entry + kU8ExBytes;
    for (uint32_t q = (uint32_t)lane; 16u * q < tot + 8u; q += kWave)
        *(__attribute__((address_space(3))) u32x4*)(size_t)(stage + 16u * q) = u32x4{0u, 0u, 0u, 0u};
    uint32_t pos = stage + ex, carry = 0;
#pragma unroll
    for (int g = 0; g < kU8NG; g++) {
#ifdef U8_NO_OR
        break;
#endif
        if (4 * g >= smax) break;
        const uint32_t lo = __builtin_amdgcn_perm(u23[g], u01[g], sel[g].x), hi = __builtin_amdgcn_perm(u23[g], u01[g], sel[g].y);
        const uint32_t k8 = 8u * (pos & 3u);
        const uint64_t v = (((uint64_t)hi << 32) | lo) << k8;
        const uint32_t w0 = (uint32_t)v | carry, w1 = (uint32_t)(v >> 32);
        const uint32_t w2 = (uint32_t)(((uint64_t)hi << k8) >> 32);
        const uint32_t a4 = pos & ~3u;
        u8_or(a4, w0);
        u8_or(a4 + 4u, w1);
        const uint32_t np = pos + nb[g];
        const uint32_t dd = (np >> 2) - (pos >> 2);
        carry = dd == 0u ? w0 : dd == 1u ? w1 : w2;
        pos = np;
    }
    u8_or(pos & ~3u, carry);
    return true;
}

// ---- flush: the element's place (look-back), its offsets and one copy of the staged payload ----
// n bytes of LDS staging (byte address s) to global d at any alignment: the bytes up to d's next
// 16-byte boundary and past the last whole chunk as byte stores (the neighbouring tiles own the
// bytes around), 16-byte stores composed from five LDS dwords and a byte align in between.
__device__ __forceinline__ void u8_copy(uint32_t s, CBX_GLOBAL uint8_t* d, uint32_t n, int lane) {
    const uint32_t mis = (uint32_t)((uint64_t)(size_t)d & 15u);
    uint32_t head = (16u - mis) & 15u;
    if (head > n) head = n;
    const uint32_t body = (n - head) >> 4;
    const uint32_t tail0 = head + 16u * body;
    if ((uint32_t)lane < head) d[lane] = lds_ld<uint8_t>(s + (uint32_t)lane);
    if (tail0 + (uint32_t)lane < n) d[tail0 + lane] = lds_ld<uint8_t>(s + tail0 + (uint32_t)lane);
    const uint32_t sh = head & 3u;
    for (uint32_t q = (uint32_t)lane; q < body; q += kWave) {
        const uint32_t o = head + 16u * q;
        const uint32_t r = s + (o & ~3u);
        const uint32_t w0 = lds_ld<uint32_t>(r), w1 = lds_ld<uint32_t>(r + 4u), w2 = lds_ld<uint32_t>(r + 8u),
                       w3 = lds_ld<uint32_t>(r + 12u), w4 = lds_ld<uint32_t>(r + 16u);
        st_pay((CBX_GLOBAL u32x4*)(d + o), u32x4{align_bytes(w1, w0, sh), align_bytes(w2, w1, sh), align_bytes(w3, w2, sh),
                                                  align_bytes(w4, w3, sh)});
    }
}

// The tile's place in the slot region of element op (tot: the tile's total): the totals of the
// tiles of its block before it, the blocks [sync_blk, blk) from their tiles' totals (an element
// flushed in its own round), then a walk back over the block totals B to the nearest inclusive
// prefix P (64 blocks per step).  Every sum of tile totals -- including a block whose B stayed
// unpublished -- goes through ONE step of the loop, so the recount fallback is inlined once.  A
// block's last tile publishes the block's P (and, flushed in its own round, its B).
__device__ __forceinline__ int64_t u8_place(const KernelArgs& a, const StrOp& op, int64_t tile, int lane, uint32_t tot,
                                            int64_t sync_blk) {
    if (CBX_DIAG & 64) return tile * kWave * op.size * op.pad;   // (diagnostic build: no look-back, every tile at its bound)
    const int64_t blk = tile / kLbBlock;
    const int k = (int)(tile & (kLbBlock - 1));
    const bool blk_last = k == kLbBlock - 1;
    uint64_t* const gb = a.lb_blk + (int64_t)op.seq * a.lb_nblk * 2;
    const int budget = lb_budget(a);
    const int64_t sb = sync_blk < blk ? sync_blk : blk;   // blocks [sb, blk) summed from their tiles
    uint32_t intra = 0;
    uint64_t acc = 0;
    bool own = k > 0;             // the tile's own block still to sum
    int64_t next_b = sb;          // next block of [sb, blk) to sum
    int64_t top = sb - 1;         // the walk: blocks above top are accounted for
    uint64_t miss = 0;            // the walk window's blocks whose B stayed unpublished
    int64_t miss_top = 0;
    for (;;) {
        int64_t t0;
        int n, dest;
        if (own) { t0 = blk * kLbBlock; n = k; dest = 0; own = false; }
        else if (next_b < blk) { t0 = next_b * kLbBlock; n = kLbBlock; dest = 1; next_b++; }
        else if (miss) {
            const int j = (int)__builtin_ctzll(miss);
            miss &= miss - 1;
            t0 = (miss_top - j) * kLbBlock;
            n = a.n_tiles - t0 < kLbBlock ? (int)(a.n_tiles - t0) : kLbBlock;
            dest = 2;
        } else if (top >= 0) {
            // up to 64 blocks (lane j: block top - j): their B and P granules
            const int64_t b = top - lane;
            const bool in = b >= 0;
            uint32_t bv = 0, pv = 0;
            bool has_b = false, has_p = false, need = in;
            int jp = kWave;
            for (int spin = 0;; spin++) {
                if (in && !(a.lb_force & 2)) {
                    if (!has_p) {
                        const uint64_t x = lb_ld(gb + 2 * b + 1);
                        if ((uint32_t)(x >> 32) == a.lb_tag) { has_p = true; pv = (uint32_t)x; }
                    }
                    if (!has_b) {
                        const uint64_t x = lb_ld(gb + 2 * b);
                        if ((uint32_t)(x >> 32) == a.lb_tag) { has_b = true; bv = (uint32_t)x; }
                    }
                }
                const uint64_t pm = __ballot(has_p);
                jp = pm ? (int)__builtin_ctzll(pm) : kWave;
                need = in && lane < jp && !has_b;
                if (!__ballot(need) || spin >= budget || (a.lb_force & 2)) break;
                __builtin_amdgcn_s_sleep(2);
            }
            acc += wave_sum32(in && lane < jp && has_b ? bv : 0u, lane);
            miss = __ballot(need);
            miss_top = top;
            if (jp < kWave) { acc += (uint32_t)__builtin_amdgcn_readlane((int)pv, jp); top = -1; }
            else top -= kWave;
            continue;
        } else {
            break;
        }
        // the totals of tiles [t0, t0 + n): polled, the missing ones recounted from the input
        uint32_t val = 0;
        uint64_t m = (a.lb_force & 1) ? (n >= kWave ? ~0ull : ((1ull << n) - 1)) : lb_probe_tiles(a, op, t0, n, lane, budget, val);
        if (m && lane == 0 && !(a.lb_force & 1)) __hip_atomic_store(a.status + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (m) {
            const int j = (int)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t v = wave_sum32(lb_recount_lane(a, op, t0 + j, lane), lane);
            if (lane == 0) atomicAdd(a.status + 1, 1);
            if (lane == j) val = v;
        }
        const uint32_t v = wave_sum32(val, lane);
        if (dest == 0) intra = v;
        else acc += v;
        if (dest == 2 && lane == 0) lb_st(gb + 2 * (t0 / kLbBlock), lb_gran(a.lb_tag, v));
    }
    if (blk_last && sync_blk <= blk && lane == 0) lb_st(gb + 2 * blk, lb_gran(a.lb_tag, (uint64_t)intra + tot));
    if (blk_last && lane == 0) lb_st(gb + 2 * blk + 1, lb_gran(a.lb_tag, acc + intra + tot));
    return (int64_t)acc + intra;
}

// The places of the oldest entries of one earlier round's tile (up to kU8Batch of the FIFO's head):
// every probe of the batch -- the totals of the tiles before it in its block, the block totals B
// and inclusive prefixes P of the 64 blocks before it -- is issued before any is waited on, so the
// batch costs one memory round trip.  An entry whose answers are complete (every total it needs
// published, a P within the window or the window reaching block 0) gets its place in f_base; the
// others keep kU8NoBase and take the polling look-back (u8_place) when flushed.
constexpr int kU8Batch = 4;

__device__ __forceinline__ void u8_probe_lagged(const KernelArgs& a, U8Ring& r, int lane) {
    const int64_t tile = u8_oldest_tile(r);
    const int64_t blk = tile / kLbBlock;
    const int k = (int)(tile & (kLbBlock - 1));
    const int64_t bq = blk - 1 - lane;   // lane j: block blk - 1 - j
    int seq[kU8Batch];
    int m = 0;
    for (; m < kU8Batch && m < r.np; m++) {
        const int s = (r.first + m) & (kWave - 1);
        if ((uint32_t)__builtin_amdgcn_readlane((int)r.f_tile, s) != (uint32_t)tile) break;
        seq[m] = ldc(a.sops + __builtin_amdgcn_readlane((int)r.f_op, s)).seq;
    }
    uint64_t ga[kU8Batch], gb[kU8Batch], gq[kU8Batch];
#pragma unroll
    for (int e = 0; e < kU8Batch; e++) {
        ga[e] = gb[e] = gq[e] = 0;
        if (e < m) {
            const uint64_t* pt = a.lb_tile + (int64_t)seq[e] * a.n_tiles + blk * kLbBlock;
            const uint64_t* pb = a.lb_blk + (int64_t)seq[e] * a.lb_nblk * 2;
            if (lane < k) ga[e] = lb_ld(pt + lane);
            if (bq >= 0) {
                gb[e] = lb_ld(pb + 2 * bq);
                gq[e] = lb_ld(pb + 2 * bq + 1);
            }
        }
    }
    if (a.lb_force) return;
#pragma unroll
    for (int e = 0; e < kU8Batch; e++) {
        if (e >= m) break;
        const uint32_t tag = a.lb_tag;
        const bool has_p = bq >= 0 && (uint32_t)(gq[e] >> 32) == tag;
        const uint64_t pm = __ballot(has_p);
        const int jp = pm ? (int)__builtin_ctzll(pm) : kWave;
        const bool a_in = lane < k, b_in = bq >= 0 && lane < jp;
        const bool bad = (a_in && (uint32_t)(ga[e] >> 32) != tag) || (b_in && (uint32_t)(gb[e] >> 32) != tag);
        if (__ballot(bad) || (jp == kWave && blk > kWave)) continue;
        const uint32_t v = (a_in ? (uint32_t)ga[e] : 0u) + (b_in ? (uint32_t)gb[e] : 0u);
        const uint64_t base = (uint64_t)wave_sum32(v, lane) + (jp < kWave ? (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)gq[e], jp) : 0u);
        if (base < kU8NoBase && lane == ((r.first + e) & (kWave - 1))) r.f_base = (uint32_t)base;
    }
}

// Flush the oldest pending entry: its place, the element's int32 offsets (place + tile-local start)
// and the payload.  cur_tile: the tile the wave is composing (-1 after its last): an entry of the
// same round looks back in sync mode; an entry of an earlier round first has its batch probed.
__device__ __forceinline__ void u8_flush_oldest(const KernelArgs& a, U8Ring& r, int lane, int64_t cur_tile) {
    const int64_t G = (int64_t)gridDim.x;
    const int64_t tile0 = u8_oldest_tile(r);
    const bool lagged = cur_tile < 0 || tile0 / G != cur_tile / G;
    if (lagged && !(CBX_DIAG & 64) && (uint32_t)__builtin_amdgcn_readlane((int)r.f_base, r.first) == kU8NoBase)
        u8_probe_lagged(a, r, lane);
    const int s = r.first;
    const int i = __builtin_amdgcn_readlane((int)r.f_op, s);
    const int64_t tile = tile0;
    const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)r.f_off, s);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)r.f_tot, s);
    const uint32_t fb = (uint32_t)__builtin_amdgcn_readlane((int)r.f_base, s);
    const StrOp op = ldc(a.sops + i);
    int64_t sync_blk = 0x7fffffffffffffffll;
    if (!lagged) sync_blk = (tile / G) * G / kLbBlock;
    int64_t base;
    if (fb != kU8NoBase) {
        base = fb;
        if ((tile & (kLbBlock - 1)) == kLbBlock - 1 && lane == 0)   // the block's inclusive prefix
            lb_st(a.lb_blk + ((int64_t)op.seq * a.lb_nblk + tile / kLbBlock) * 2 + 1, lb_gran(a.lb_tag, (uint64_t)base + tot));
    } else {
        base = u8_place(a, op, tile, lane, tot, sync_blk);
    }
    const uint32_t entry = r.rb + off;
    const uint32_t ex = lds_ld<uint16_t>(entry + 2u * (uint32_t)lane);
    const StrCall c = ldc(a.scall + i);
    CBX_GLOBAL int32_t* offs = gp((int32_t*)c.local);
    st_out(offs + tile * kWave + lane, (int32_t)(base + ex));
    if (tile == a.n_tiles - 1 && lane == 0) {   // the closing offset and the slot's size
        offs[a.n_rec] = (int32_t)(base + tot);
        if (c.size) *gp(c.size) = base + tot;
    }
    if (base + (int64_t)tot > c.tile_cap || base + (int64_t)tot > 0x7fffffffll) {   // the region (or an int32 offset) overflows
        if (lane == 0) atomicOr(a.status, 1);
    } else {
#ifndef U8_NO_COPY
        u8_copy(entry + kU8ExBytes, gp(c.scratch + base), tot, lane);
#endif
    }
    r.first = (r.first + 1) & (kWave - 1);
    r.np--;
    if (r.np == 0) r.head = r.tail = 0;
    else r.tail = (uint32_t)__builtin_amdgcn_readlane((int)r.f_off, r.first);
}

// At the end of a round: the block totals B of the wave's elements [lo, hi) for the block that the
// workgroup's tile closes -- from the block's tiles' totals (published by this round's composes);
// if some stay unpublished past the poll budget the B is left out (its readers sum the tiles).
__device__ __forceinline__ void u8_publish_b(const KernelArgs& a, int lo, int hi, int64_t tile, int lane) {
    if ((tile & (kLbBlock - 1)) != kLbBlock - 1 || (CBX_DIAG & 64)) return;
    const int64_t b = tile / kLbBlock;
    const int budget = lb_budget(a);
#pragma unroll 1
    for (int i = lo; i < hi; i++) {
        const StrOp op = ldc(a.sops + i);
        uint32_t val;
        if (lb_probe_tiles(a, op, b * kLbBlock, kLbBlock, lane, budget, val)) continue;
        const uint32_t v = wave_sum32(val, lane);
        if (lane == 0) lb_st(a.lb_blk + ((int64_t)op.seq * a.lb_nblk + b) * 2, lb_gran(a.lb_tag, v));
    }
}

// ---- the tile loop ----
// Issue the next tile's staging loads: chunk row u (chunks u * 64 + lane) by wave u % NW.
template <int KP, int NW>
__device__ __forceinline__ void u8_issue(const KernelArgs& a, const ContigSpan& sp, int wid, int lane,
                                         uint4 (&buf)[(KP + NW - 1) / NW]) {
    constexpr int KH = (KP + NW - 1) / NW;
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
        const int c = (v * NW + wid) * kWave + lane;
        const int off = c < nch ? 16 * c : 0x7ffffff0;   // past the descriptor's range: no access
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kStageCpol);
        buf[v] = make_uint4(x[0], x[1], x[2], x[3]);
    }
}

// Fixed-length records, one tile per workgroup and round.  body.range(wid, lo, hi): the wave's
// string elements; body.run(a, t, img, rec_addr, l, lane, ring, cur): composes the tile's elements
// into the ring, runs its numerics and flushes the entries of earlier tiles (cur = -1, no tile:
// flushes everything).  Two workgroup barriers per tile (image complete; image free again).
template <int KP, int NW, typename Body>
__device__ __forceinline__ void u8_loop(const KernelArgs& a, const U8Lds& l, int lane, Body body) {
    constexpr int KH = (KP + NW - 1) / NW;
    uint4 buf[KH];
    const int wid = l.wid;
    int lo = 0, hi = 0;
    body.range(wid, lo, hi);
    U8Ring ring;
    u8_ring_init(ring, l.stage + (uint32_t)wid * (uint32_t)a.lb_ring, (uint32_t)a.lb_ring);
    Stamps st;   // (diagnostic build: 0 stage, 1 barrier + prefetch, 2 compose, 3 flush, 4 block totals, 5 end barrier)
    st.init();
    int64_t tile = (int64_t)blockIdx.x;
    const int64_t tstep = (int64_t)gridDim.x;
    if (tile < a.n_tiles) u8_issue<KP, NW>(a, contig_span(a, tile), wid, lane, buf);
    while (tile < a.n_tiles) {
        const ContigSpan sp = contig_span(a, tile);
        {
            int ln = lane;
            asm volatile("" : "+v"(ln));
#pragma unroll
            for (int v = 0; v < KH; v++) {
                const int c = (v * NW + wid) * kWave + ln;
                if (c < sp.nch) contig_put(a, sp, c, buf[v], l.img);
            }
        }
        st.mark(0);
        __syncthreads();   // the tile's image complete
        const int64_t next = tile + tstep;
        u8_issue<KP, NW>(a, contig_span(a, next), wid, lane, buf);
        st.mark(1);
        TileCtx t = tile_ctx<false>(a, tile, lane);
        const uint32_t rec0 = (uint32_t)(lane * a.cpitch + 4 * sp.mis_dw);
        body.run(a, t, (const uint8_t*)l.img, rec0 + (uint32_t)a.start_off, l, lane, ring, tile, st);
        u8_publish_b(a, lo, hi, tile, lane);
        st.mark(4);
        __syncthreads();   // every wave done with the image
        st.mark(5);
        tile = next;
    }
    // every pending entry (the last round's block totals are out)
#ifndef U8_NO_FINAL
    TileCtx t0 = tile_ctx<false>(a, 0, lane);
    body.run(a, t0, (const uint8_t*)l.img, 0u, l, lane, ring, -1, st);
#endif
    st.flush(a, lane);
}

}  // namespace cbx
