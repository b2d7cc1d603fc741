// cbx_walk.h -- the record walk with data-dependent offsets: RecordExtractors.extractRecord
// restated per lane (CP/reader/extractors/record/RecordExtractors.scala:49-183) for the layouts
// the static-offset kernels cannot express:
//   * variable_size_occurs = true: an OCCURS DEPENDING ON array consumes only its present
//     elements, so every later field moves with the data (:109-113);
//   * DEPENDING ON a field inside an OCCURS (each element carries the count of a nested array);
//   * DEPENDING ON a string field through occurs_mappings (dependingOnHandlers, :70-74);
// and VarOccursRecordExtractor's record lengths (CP/reader/extractors/raw/VarOccursRecordExtractor.scala:30-154).
// Included by cbx_capi.hip.
//
// One lane walks one record through the copybook's node table (cbx_walk_node: DFS order with
// child / sibling links) with an explicit frame stack, keeps the dependFields map as a small
// per-lane table of dependee slots (one per DEPENDING ON name, Left(int) or Right(handler key)),
// decodes each primitive with the byte-loop decoders straight from HBM and writes it to its
// (column, slot, record) place; validity bits are OR-ed in with atomics (lanes of a wave diverge:
// no ballot).  String columns use the string-view layout: a value longer than 12 bytes takes its
// place in its tile's region through a per-(column slot, tile) cursor.  Records are independent,
// so the walk is data-parallel; within a record it is the reference's sequence, which is the point.
#pragma once

namespace cbx {

constexpr int kWalkDepth = 16;     // group / OCCURS nesting levels
constexpr int kWalkDeps = 8;       // DEPENDING ON names (dependee slots)
constexpr int kWalkShortStr = 12;
constexpr int kWalkStageChunks = 8;   // 16-byte chunks a lane stages per tile (stage_cap <= 8 KiB)  // string fields of at most this many bytes: walk_prim_f's register path
// the waves' LDS areas start past LDS address 0: the compiler the specialised walk is built with
// (torch's hipRTC) takes a pointer to LDS address 0 for a null one
constexpr int kWalkLdsBase = 16;
constexpr int kWalkLut = 1024;     // the workgroup's 256-entry code-page table

struct WalkArgs {
    const uint8_t* data;
    int64_t data_len;
    const int64_t* rec_off;           // framed records (nullptr: fixed stride)
    const int32_t* rec_len;
    int64_t n_rec;
    int32_t stride, start_off;
    int64_t first_record_id;
    const int64_t* rec_id_base;       // device int64 added to first_record_id (cbx_plan_set_record_base), nullptr: 0
    const int64_t* rec_id;            // selection: per-record Record_Id
    const int32_t* rec_seg;           // selection: per-record active segment
    int32_t file_id;
    int32_t var_occurs;               // variable_size_occurs
    int64_t n_tiles, pitch;
    const CBX_CONST cbx_walk_node* nodes;
    int32_t root;                     // the AST root node (a group whose children are the records)
    const CBX_CONST cbx_walk_array* warr;
    const CBX_CONST cbx_walk_handler* handlers;
    int32_t n_handlers;
    const CBX_CONST cbx_array* arrays;
    const CBX_CONST Field* fields;
    const CBX_CONST DevColumn* cols;
    const CBX_CONST cbx_segment_map* segmap;
    const uint32_t* lut;
    int32_t seg_col, fid_col, rid_col;
    const int64_t* str_slot_base;     // per column: index of its slot 0 among the string column slots
    uint32_t* cursors;                // [string column slots][n_tiles] payload bytes used in the tile region
    const int64_t* tile_bytes;        // per column: view region bytes per tile, tiles per data buffer
    int32_t* status;
    // per-wave LDS accumulation (vlds != 0): the tile's validity words of every (column, slot) and the
    // string slots' payload cursors, stored once per tile instead of one global atomic per value
    int32_t vlds, wave_lds;           // flag; LDS bytes per wave
    int32_t depth, stack_lds;         // frame stack depth (the copybook's nesting), its LDS bytes per wave
    int32_t stage_cap;                // LDS bytes per wave for the tile's record span (a multiple of 16)
    int32_t n_vslots, n_sslots;       // validity words (all column slots); string column slots
    const int64_t* vslot_base;        // per column: index of its slot 0 among all column slots
    const int32_t* vslot_col;         // per validity word: its column and slot
    const int32_t* vslot_slot;
    // hierarchical records (cbx_plan_set_dep_seed): each row's dependFields as the rows before it in
    // extractHierarchicalRecord's walk left the map -- [kWalkDeps][seed_pitch] int64, kind << 32 | value
    // (kind 0 unseen) -- and the root segment: a child row decodes its own group only (:300-322), so
    // its walk registers no common-header dependee (hier_root < 0: not hierarchical)
    const int64_t* dep_seed;
    int64_t seed_pitch;
    int32_t hier_root;
};

// The wave's LDS area of the tile being walked (vlds): validity words, then string cursors.
typedef __attribute__((address_space(3))) const uint8_t walk_lds_cu8;
typedef __attribute__((address_space(3))) uint32_t walk_lds_u32;
typedef __attribute__((address_space(3))) uint64_t walk_lds_u64;
struct WalkLds {
    walk_lds_u64* vw;          // [n_vslots]
    walk_lds_u32* cur;         // [n_sslots]
    const walk_lds_u32* lut;   // the code page's UTF-8 table, staged per workgroup
};
// A plan table of the walk (read-only for the kernel's lifetime): a scalar load.
__device__ __forceinline__ int64_t walk_tab(const int64_t* t, int64_t i) { return ldc((const CBX_CONST int64_t*)t + i); }

struct WalkFrame {
    int32_t node;     // group (children loop) or OCCURS node (elements loop)
    int32_t elems;    // 1: the elements of node (an OCCURS node), 0: node's children
    int32_t cur;      // group: current child; array: current element
    int32_t cnt;      // array: present elements
    int32_t start;    // offset where the node began
    int32_t off;      // running offset
    int32_t slot;     // slot of the node's values (array: the enclosing slot)
};

// A dependee slot: kind 0 unseen, 1 Left(int), 2 Right(string) -> v = handler key index + 1 (0: a
// string no handler lists)
struct WalkDep { int32_t kind, v; };

// The lane's dependFields in registers: slots are addressed with wave-uniform indices (a node's
// dep_slot), unrolled into selects so the table never goes to scratch.
struct WalkDeps {
    int32_t kind[kWalkDeps], v[kWalkDeps];
    bool common_ok;   // the row registers common-header dependees (not a hierarchical child row)
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < kWalkDeps; i++) { kind[i] = 0; v[i] = 0; }
        common_ok = true;
    }
    __device__ __forceinline__ WalkDep get(int s) const {
        WalkDep d{0, 0};
#pragma unroll
        for (int i = 0; i < kWalkDeps; i++)
            if (i == s) d = WalkDep{kind[i], v[i]};
        return d;
    }
    __device__ __forceinline__ void set(int s, bool on, WalkDep d) {
#pragma unroll
        for (int i = 0; i < kWalkDeps; i++)
            if (i == s && on) { kind[i] = d.kind; v[i] = d.v; }
    }
};

// A row's map at its start: empty, or the hierarchical walk's state before the row (dep_seed).
__device__ __forceinline__ void walk_seed(const WalkArgs& a, WalkDeps& dep, int64_t r, bool act, int seg) {
    dep.clear();
    if (a.hier_root >= 0) dep.common_ok = seg == a.hier_root;
    if (a.dep_seed && act && r < a.seed_pitch) {
#pragma unroll
        for (int i = 0; i < kWalkDeps; i++) {
            const int64_t x = a.dep_seed[(int64_t)i * a.seed_pitch + r];
            dep.kind[i] = (int32_t)(x >> 32);
            dep.v[i] = (int32_t)x;
        }
    }
}

__device__ __forceinline__ uint32_t walk_lut(const WalkArgs& a, const WalkLds& wl, int kind, uint32_t b) {
    return kind == CBX_K_STRING_ASCII ? ascii_lut(b) : wl.lut[b];
}

// Validity of (column, slot) for the tile's lanes with v set (wave-uniform call): one OR of the
// ballot into the tile's LDS word (vlds), else one global atomic per tile.
__device__ __forceinline__ void walk_valid(const WalkArgs& a, const WalkLds& wl, uint64_t* validity, int column, int slot,
                                           int64_t tile, int lane, bool v) {
    const uint64_t m = __ballot(v);
    if (m == 0) return;
    if (lane == 0) {
        if (wl.vw) wl.vw[walk_tab(a.vslot_base, column) + slot] |= m;
        else atomicOr((unsigned long long*)(validity + (int64_t)slot * a.n_tiles + tile), m);
    }
}

// extractArray's element count (:66-81)
__device__ __forceinline__ int walk_count(const WalkArgs& a, int ai, const WalkDeps& dep) {
    const cbx_array ar = ldc(a.arrays + ai);
    const cbx_walk_array wa = ldc(a.warr + ai);
    int v = ar.max_count;
    if (wa.dep_slot >= 0) {
        const WalkDep d = dep.get(wa.dep_slot);
        if (d.kind == 1) v = d.v;
        else if (d.kind == 2) {   // dependingOnHandlers.getOrElse(s, arraySize)
            for (int h = wa.h_begin; h < wa.h_end; h++)
                { const cbx_walk_handler hd = ldc(a.handlers + h); if (hd.key_id + 1 == d.v) { v = hd.value; break; } }
        }
    }
    return (v >= ar.min_count && v <= ar.max_count) ? v : ar.max_count;
}

// A numeric value for the walk: COMP-3 of <= 8 bytes and binary of 1 / 2 / 4 / 8 bytes through the
// record kernels' packed-nibble / byte-swap fast decoders (bcd8_raw, bin8_raw: the same Field-derived
// typing as make_numop, folded to constants in cbx_jit_walk), everything else through the byte-loop
// decoder; both give decode_numeric's value (the fast variants are exact for these fields).
template <typename RP>
__device__ __forceinline__ Val walk_numeric(const Field& f, RP p) {
    const bool bcd = f.kind == CBX_K_BCD && f.variant == V_BCD8;
    const bool bin = f.kind == CBX_K_BINARY && f.variant == V_BIN8;
    if (!bcd && !bin) return decode_numeric(f, p);
    NumOp op{};
    op.variant = (uint8_t)f.variant;
    op.size = (uint8_t)f.size;
    uint32_t fl = 0;
    if (f.flags & CBX_F_SIGNED) fl |= NF_SIGNED;
    if (f.flags & CBX_F_BIG_ENDIAN) fl |= NF_BIG_ENDIAN;
    if (f.fin == 0) fl |= NF_INT;
    op.flags = (uint8_t)fl;
    op.shift = (uint8_t)(64 - 8 * f.size);
    op.mask = low_bytes_mask(f.size);
    uint64_t mul = 1;
    for (int i = 0; i < f.e_mul; i++) mul *= 10u;   // (constants in cbx_jit_walk: the loops fold)
    op.mul = mul;
    U128 lim = u128(1);
    for (int i = 0; i < f.e_lim; i++) (void)u128_muladd(lim, 10, 0);
    op.lim_lo = lim.lo;
    op.lim_hi = lim.hi;
    op.lim64 = lim.hi ? ~0ull : lim.lo;
    // the 8 bytes ending at the field's end, little-endian (the field in the top bytes, zeros below)
    uint64_t r1 = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (i < f.size) r1 |= (uint64_t)(uint8_t)p[i] << (8 * (8 - f.size + i));
    return bcd ? bcd8_raw<0>(op, r1) : bin8_raw<0>(op, r1);
}

// One primitive element at record offset `off` (relative to the decode base) for the lanes with
// `la` (wave-uniform call: the node, its field and slot are the wave's).  `element`: an element of a
// primitive OCCURS -- extractArray decodes those with decodeTypeValue, which never touches
// dependFields (RecordExtractors.scala:96-107), so they update no dependee.  f, size (the node's
// dataSize) and dep_slot come from the node: the table-driven walk loads them, the
// copybook-specialised walk (cbx_jit_walk) passes constants, so its decoders fold to the field's.
template <typename RP>
__device__ __forceinline__ void walk_prim_f(const WalkArgs& a, const WalkLds& wl, const Field& f, int size, int dep_slot, int off,
                                            int slot, RP rec, int avail, int64_t r, int64_t tile, int lane, bool la,
                                            WalkDeps& dep, bool element) {
    const int o = a.start_off + off;
    const RP p = rec + o;
    const bool is_str = f.kind == CBX_K_STRING || f.kind == CBX_K_STRING_ASCII || f.kind == CBX_K_HEX ||
                        f.kind == CBX_K_RAW || f.kind == CBX_K_UTF16_BE || f.kind == CBX_K_UTF16_LE;
    const DevColumn c = ldc(a.cols + f.column);
    if (is_str && (f.kind == CBX_K_STRING || f.kind == CBX_K_STRING_ASCII) && size <= kWalkShortStr &&
        (dep_slot < 0 || element)) {
        // Short single-byte-page strings (every value <= 12 UTF-8 bytes of one wave: an inline view):
        // the bytes' LUT entries once, trim and UTF-8 length as bit operations over per-byte masks, the
        // value composed in three registers -- no byte loops, no private array (the generic path below
        // went through scratch for the inline bytes).  A wave holding a longer value takes that path.
        const bool on = la && o <= avail;
        const int n = on ? (o + size <= avail ? size : avail - o) : 0;
        uint32_t ent[kWalkShortStr];
        uint32_t keep = 0;
#pragma unroll
        for (int i = 0; i < kWalkShortStr; i++) {
            ent[i] = 0;
            if (i < size && i < n) {
                ent[i] = walk_lut(a, wl, f.kind, p[i]);
                if (!(ent[i] >> 31)) keep |= 1u << i;
            }
        }
        const bool tl = f.trim == CBX_TRIM_LEFT || f.trim == CBX_TRIM_BOTH;
        const bool tr = f.trim == CBX_TRIM_RIGHT || f.trim == CBX_TRIM_BOTH;
        // string_span: [b, e) after the left then the right trim (all trimmed: empty)
        const int b = tl ? (keep ? __builtin_ctz(keep) : n) : 0;
        const int e = tr ? (keep ? 32 - __builtin_clz(keep) : b) : n;
        int len = 0;
#pragma unroll
        for (int i = 0; i < kWalkShortStr; i++)
            if (i >= b && i < e) len += (int)((ent[i] >> 24) & 3u);
        if (!__ballot(on && len > 12)) {
            uint64_t lo = 0;
            uint32_t hi = 0;
            int at = 0;
#pragma unroll
            for (int i = 0; i < kWalkShortStr; i++) {
                if (i >= b && i < e) {
                    const uint32_t l = (ent[i] >> 24) & 3u;
                    const uint32_t v = ent[i] & (l >= 3 ? 0xFFFFFFu : l == 2 ? 0xFFFFu : 0xFFu);
                    if (at < 8) lo |= (uint64_t)v << (8 * at);
                    if (at >= 8) hi |= v << (8 * (at - 8));
                    else if (at > 5) hi |= v >> (8 * (8 - at));
                    at += (int)l;
                }
            }
            if (on) *gp((u32x4*)c.values + (int64_t)slot * a.pitch + r) = u32x4{(uint32_t)len, (uint32_t)lo, (uint32_t)(lo >> 32), hi};
            walk_valid(a, wl, c.validity, f.column, slot, tile, lane, on);
            return;
        }
    }
    if (is_str) {
        // Primitive.decodeTypeValue (:102-128): offset past the end -> null, else truncated
        bool ok = la && o <= avail;
        const int n = ok ? (o + size <= avail ? size : avail - o) : 0;
        auto lutf = [&](uint32_t b) { return walk_lut(a, wl, f.kind, b); };
        StrSpan sp{};
        if (ok) sp = string_span(f.kind, f.trim, p, n, lutf);
        const int len = ok ? sp.utf8_len : 0;
        const bool lng = ok && len > 12;
        // a long value's place in its tile's region: a wave scan of the long lengths (vlds), else
        // one atomic per lane on the (slot, tile) cursor
        const int64_t tb = walk_tab(a.tile_bytes, 2 * f.column);
        const int64_t tpb = walk_tab(a.tile_bytes, 2 * f.column + 1);   // a power of two (view_tiles_per_buf)
        const int64_t cs = walk_tab(a.str_slot_base, f.column) + slot;
        uint32_t at = 0;
        if (wl.cur) {
            uint32_t tot = 0;
            const uint32_t ex = wave_excl_scan32(lng ? (uint32_t)len : 0u, lane, tot);
            if (tot) {
                const uint32_t base = wl.cur[cs];
                at = base + ex;
                wave_sync_lds();
                if (lane == 0) wl.cur[cs] = base + tot;
                wave_sync_lds();
            }
        } else if (lng) {
            at = atomicAdd(a.cursors + cs * a.n_tiles + tile, (uint32_t)len);
        }
        if (lng && (int64_t)at + len > tb) { atomicOr(a.status, 1); ok = false; }
        if (ok) {
            u32x4 view;
            view.x = (uint32_t)len;
            if (!lng) {
                uint8_t inl[16] = {0};
                string_write(f.kind, p, sp, inl, lutf);
                view.y = inl[0] | (uint32_t)inl[1] << 8 | (uint32_t)inl[2] << 16 | (uint32_t)inl[3] << 24;
                view.z = inl[4] | (uint32_t)inl[5] << 8 | (uint32_t)inl[6] << 16 | (uint32_t)inl[7] << 24;
                view.w = inl[8] | (uint32_t)inl[9] << 8 | (uint32_t)inl[10] << 16 | (uint32_t)inl[11] << 24;
            } else {
                uint8_t* dst = (uint8_t*)gp(c.data + (int64_t)slot * c.capacity + tile * tb + at);
                string_write(f.kind, p, sp, dst, lutf);
                const CBX_GLOBAL uint8_t* d = gp(dst);
                view.y = d[0] | (uint32_t)d[1] << 8 | (uint32_t)d[2] << 16 | (uint32_t)d[3] << 24;
                view.z = (uint32_t)(tile >> __builtin_ctzll((unsigned long long)tpb));
                view.w = (uint32_t)((tile & (tpb - 1)) * tb + at);
            }
            *gp((u32x4*)c.values + (int64_t)slot * a.pitch + r) = view;
        }
        walk_valid(a, wl, c.validity, f.column, slot, tile, lane, ok);
        if (dep_slot >= 0 && !element) {   // Right(s): the handler key it equals (occurs_mappings)
            int key = 0;
            if (ok && len <= 64) {
                uint8_t buf[64];
                string_write(f.kind, p, sp, buf, lutf);
                for (int h = 0; h < a.n_handlers && key == 0; h++) {
                    const cbx_walk_handler hd = ldc(a.handlers + h);
                    bool eq = hd.key_len == len;
                    for (int i = 0; eq && i < len; i++) eq = hd.key[i] == buf[i];
                    if (eq) key = hd.key_id + 1;
                }
            }
            dep.set(dep_slot, ok && (f.segment >= 0 || dep.common_ok), WalkDep{2, key});
        }
        return;
    }
    bool ok = la && o + size <= avail;   // numeric past the end -> null
    Val x{0, 0, false};
    if (ok) x = walk_numeric(f, p);
    ok = ok && x.valid;                  // null: dependFields keeps its previous entry (:126-134)
    if (ok) {
        const int w = f.out_type == CBX_O_I32 || f.out_type == CBX_O_F32 ? 4 : f.out_type == CBX_O_DEC128 ? 16 : 8;
        const int64_t at = (int64_t)slot * a.pitch + r;
        if (w == 4) *gp((uint32_t*)c.values + at) = (uint32_t)x.lo;
        else if (w == 8) *gp((uint64_t*)c.values + at) = x.lo;
        else *gp((u32x4*)c.values + at) = u32x4{(uint32_t)x.lo, (uint32_t)(x.lo >> 32), (uint32_t)x.hi, (uint32_t)(x.hi >> 32)};
    }
    walk_valid(a, wl, c.validity, f.column, slot, tile, lane, ok);
    if (dep_slot >= 0 && !element) {   // Left(Number.intValue)
        Val dv{0, 0, false};
        if (ok) dv = decode_count_int(f, p);
        dep.set(dep_slot, ok && dv.valid && (f.segment >= 0 || dep.common_ok), WalkDep{1, (int32_t)dv.lo});
    }
}

#ifndef CBX_JIT_WALK
// The table-driven walk's primitive: the node's field from the plan tables.
__device__ void walk_prim(const WalkArgs& a, const WalkLds& wl, const cbx_walk_node& nd, int off, int slot, const uint8_t* rec,
                          int avail, int64_t r, int64_t tile, int lane, bool la, WalkDeps& dep, bool element) {
    if (nd.field < 0) return;   // a FILLER that nothing depends on
    walk_prim_f(a, wl, ldc(a.fields + nd.field), nd.data_size, nd.dep_slot, off, slot, rec, avail, r, tile, lane, la, dep, element);
}

#endif

// A frame's wave-uniform part (the node, the loop position, the slot and the lanes taking part);
// its per-lane part -- start and running offset, the array's element count -- lives in LDS rows
// of 64 lanes beside it.
struct WalkU {
    int32_t node, elems, cur, cmax, slot, pad;
    uint64_t mask;
};

__device__ __forceinline__ int32_t ufl(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ WalkU walk_u(const WalkU* p) {
    const WalkU w = *p;
    WalkU u;
    u.node = ufl(w.node); u.elems = ufl(w.elems); u.cur = ufl(w.cur); u.cmax = ufl(w.cmax); u.slot = ufl(w.slot); u.pad = 0;
    u.mask = (uint64_t)(uint32_t)ufl((int32_t)(uint32_t)w.mask) | (uint64_t)(uint32_t)ufl((int32_t)(uint32_t)(w.mask >> 32)) << 32;
    return u;
}

#ifndef CBX_JIT_WALK
// The walk of the tile's 64 records at once (extractRecord's getGroupValues / extractArray /
// extractValue): every record has the copybook's shape, only its counts, segment and offsets
// differ, so the wave walks the node tree in step -- an OCCURS loop runs to the largest count among
// the lanes, each lane taking part in the elements it has -- and the control flow, the node-table
// loads and the decoder dispatch are the wave's (scalar), the offsets and values the lanes'.
// act: the lane has a record; seg: its active segment redefine (-1 none).
__device__ void walk_tile(const WalkArgs& a, const WalkLds& wl, uint8_t* stk, const uint8_t* rec, int avail, int seg,
                          int64_t r, int64_t tile, int lane, bool act) {
    WalkU* U = (WalkU*)stk;
    int32_t* VS = (int32_t*)(U + a.depth);    // [depth][64] frame start
    int32_t* VO = VS + a.depth * kWave;       // [depth][64] running offset
    int32_t* VC = VO + a.depth * kWave;       // [depth][64] element count (array frames)
    WalkDeps dep;
    walk_seed(a, dep, r, act, seg);
    int sp = 0;
    U[0] = WalkU{a.root, 0, ldc(a.nodes + a.root).child, 0, 0, 0, __ballot(act)};
    VS[lane] = 0;
    VO[lane] = 0;
    int last = 0;   // per lane: size consumed by the frame just popped
    bool popped = false;
    while (sp >= 0) {
        WalkU fr = walk_u(U + sp);
        const cbx_walk_node nd = ldc(a.nodes + fr.node);
        const bool la = (fr.mask >> lane) & 1;
        const int row = sp * kWave + lane;
        int off = VO[row];
        if (fr.elems) {   // the elements of an OCCURS node
            const int cnt = VC[row];
            if (popped) {   // a group element finished
                if (la && fr.cur < cnt) off += last;
                fr.cur++;
                popped = false;
            }
            if (fr.cur < fr.cmax) {
                const int slot = fr.slot * ldc(a.arrays + nd.array).max_count + fr.cur;
                const bool le = la && fr.cur < cnt;
                if (nd.kind == CBX_W_GROUP) {
                    if (sp + 1 >= a.depth) { if (lane == 0) atomicOr(a.status, 2); return; }
                    U[sp].cur = fr.cur;
                    VO[row] = off;
                    U[sp + 1] = WalkU{fr.node, 0, nd.child, 0, slot, 0, __ballot(le)};
                    VS[row + kWave] = off;
                    VO[row + kWave] = off;
                    sp++;
                    continue;
                }
                walk_prim(a, wl, nd, off, slot, rec, avail, r, tile, lane, le, dep, true);
                if (le) off += nd.data_size;
                U[sp].cur = fr.cur + 1;
                VO[row] = off;
                continue;
            }
            // extractArray's consumed size: the lane's elements walked, or the static size (:109-113)
            last = a.var_occurs ? off - VS[row] : nd.actual_size;
            sp--;
            popped = true;
            continue;
        }
        // a group's children (the group node itself, or one element of an OCCURS group)
        if (popped) {   // a child group / array finished: advance by its size (getGroupValues, :144-160)
            const cbx_walk_node ch = ldc(a.nodes + fr.cur);
            if (la && !(ch.flags & CBX_W_REDEFINED)) off += (ch.array < 0 && (ch.flags & CBX_W_REDEFINES)) ? ch.actual_size : last;
            fr.cur = ch.next;
            popped = false;
            U[sp].cur = fr.cur;
            VO[row] = off;
        }
        if (fr.cur < 0) {   // the group is done
            last = off - VS[row];
            sp--;
            popped = true;
            continue;
        }
        const int ci = fr.cur;
        const cbx_walk_node ch = ldc(a.nodes + ci);
        if (ch.array >= 0) {   // an OCCURS node: the lanes' element counts, then the elements
            const int cnt = la ? walk_count(a, ch.array, dep) : 0;
            const int ccol = ldc(a.arrays + ch.array).count_column;
            if (ccol >= 0) {
                const DevColumn c = ldc(a.cols + ccol);
                if (la) ((int32_t*)c.values)[(int64_t)fr.slot * a.pitch + r] = cnt;
                walk_valid(a, wl, c.validity, ccol, fr.slot, tile, lane, la);
            }
            if (sp + 1 >= a.depth) { if (lane == 0) atomicOr(a.status, 2); return; }
            const int cmax = (int)wave_max64(cnt);
            U[sp + 1] = WalkU{ci, 1, 0, cmax, fr.slot, 0, fr.mask};
            VS[row + kWave] = off;
            VO[row + kWave] = off;
            VC[row + kWave] = cnt;
            sp++;
            continue;
        }
        if (ch.kind == CBX_W_GROUP) {
            // a segment redefine of another segment: null, full size (:119-121) -- its lanes skip the
            // group, and its start is set one size back so that popping it consumes that size
            const bool on = la && (ch.segment < 0 || ch.segment == seg);
            const uint64_t m = __ballot(on);
            if (m == 0) {
                last = ch.actual_size;
                popped = true;
                continue;
            }
            if (sp + 1 >= a.depth) { if (lane == 0) atomicOr(a.status, 2); return; }
            U[sp + 1] = WalkU{ci, 0, ch.child, 0, fr.slot, 0, m};
            VS[row + kWave] = on ? off : off - ch.actual_size;
            VO[row + kWave] = off;
            sp++;
            continue;
        }
        walk_prim(a, wl, ch, off, fr.slot, rec, avail, r, tile, lane, la, dep, false);
        if (la && !(ch.flags & CBX_W_REDEFINED)) off += ch.actual_size;
        U[sp].cur = ch.next;
        VO[row] = off;
    }
}
#endif

// The tiles of a walk launch (one wave per tile of 64 records, lane = record): the tile's span
// staged in LDS, the generated columns, body(a, wl, area, rec, avail, seg, r, tile, lane, act) for the
// copybook's fields (the table-driven walk_tile, or the copybook-specialised walk of cbx_jit_walk),
// then the tile's LDS validity words.
template <typename Body>
__device__ __forceinline__ void walk_tiles(const WalkArgs& a, uint8_t* wsm, const Body& body) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // the workgroup's code-page table, then per wave: the frame stack, the tile's record bytes, then
    // (vlds) the tile's words and cursors
    walk_lds_u32* lut = (walk_lds_u32*)((__attribute__((address_space(3))) uint8_t*)wsm + kWalkLdsBase);
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = a.lut[i];
    __syncthreads();
    uint8_t* area = wsm + kWalkLdsBase + kWalkLut + wid * a.wave_lds;
    uint8_t* stage = area + a.stack_lds;
    __attribute__((address_space(3))) uint8_t* stage_l = (__attribute__((address_space(3))) uint8_t*)wsm + kWalkLdsBase +
                                                        kWalkLut + wid * a.wave_lds + a.stack_lds;
    WalkLds wl{nullptr, nullptr, lut};
    if (a.vlds) {
        wl.vw = (walk_lds_u64*)(stage_l + a.stage_cap);
        wl.cur = (walk_lds_u32*)(stage_l + a.stage_cap + 8 * a.n_vslots);
        for (int i = lane; i < a.n_vslots; i += kWave) wl.vw[i] = 0;
        for (int i = lane; i < a.n_sslots; i += kWave) wl.cur[i] = 0;
        wave_sync_lds();
    }
    // one wave per tile of 64 records (lane = record): every lane of the wave takes part in the
    // walk and in the tile's flush of the LDS words, records past the batch included
    for (int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid; tile < a.n_tiles; tile += (int64_t)gridDim.x * (blockDim.x >> 6)) {
        const int64_t r = tile * kWave + lane;
        const bool act = r < a.n_rec;
        int64_t base = 0;
        int avail = 0;
        if (act) {
            if (a.rec_off) { base = *gp(a.rec_off + r); avail = *gp(a.rec_len + r); }
            else { base = r * (int64_t)a.stride; avail = a.stride; }
        }
        const uint8_t* rec = a.data + base;
        // the tile's records are one byte span of the file: staged in LDS with 16-byte loads (the
        // decoders' byte reads then hit LDS, not HBM), unless it is wider than the stage
        int stage_at = -1;   // the lane's record in the stage
        {
            const int64_t lo = wave_min64(act ? base : 0x7fffffffffffffffll);
            const int64_t hi = wave_max64(act ? base + avail : 0);
            if (hi > lo) {
                const uint64_t g0 = (uint64_t)(size_t)(a.data + lo);
                const int mis = (int)(g0 & 15);
                const int64_t span = hi - lo + mis;
                if (span <= a.stage_cap) {
                    // every 16-byte chunk's global load issued before the first LDS store (one latency per
                    // tile; the stage is at most 8 KiB: 8 chunks a lane), typed pointers -- generic ones made
                    // each chunk a flat load waited for before its flat store
                    const CBX_GLOBAL u32x4* src = (const CBX_GLOBAL u32x4*)(size_t)(g0 - mis);
                    __attribute__((address_space(3))) u32x4* dst = (__attribute__((address_space(3))) u32x4*)stage_l;
                    const int nq = (int)((span + 15) >> 4);
                    u32x4 v[kWalkStageChunks];
#pragma unroll
                    for (int j = 0; j < kWalkStageChunks; j++)
                        if (lane + kWave * j < nq) v[j] = src[lane + kWave * j];
#pragma unroll
                    for (int j = 0; j < kWalkStageChunks; j++)
                        if (lane + kWave * j < nq) dst[lane + kWave * j] = v[j];
                    wave_sync_lds();
                    stage_at = act ? mis + (int)(base - lo) : 0;
                    rec = stage + stage_at;
                }
            }
        }
        int seg = -1;
        if (act) {
            if (a.rec_seg) seg = *gp(a.rec_seg + r);
            else if (a.segmap) {
                const int k = segment_key(a.segmap, a.lut, a.fields, rec, avail, a.start_off);
                if (k >= 0) seg = a.segmap->key_segment[k];
            }
        }
        if (a.seg_col >= 0) {
            const DevColumn c = ldc(a.cols + a.seg_col);
            if (act) *gp((int32_t*)c.values + r) = seg;
            walk_valid(a, wl, c.validity, a.seg_col, 0, tile, lane, act);
        }
        if (a.fid_col >= 0) {
            const DevColumn c = ldc(a.cols + a.fid_col);
            if (act) *gp((int32_t*)c.values + r) = a.file_id;
            walk_valid(a, wl, c.validity, a.fid_col, 0, tile, lane, act);
        }
        if (a.rid_col >= 0) {
            const DevColumn c = ldc(a.cols + a.rid_col);
            if (act) *gp((int64_t*)c.values + r) = a.rec_id ? *gp(a.rec_id + r) : a.first_record_id + (a.rec_id_base ? *gp(a.rec_id_base) : 0) + r;
            walk_valid(a, wl, c.validity, a.rid_col, 0, tile, lane, act);
        }
        // the copybook's fields, reading the record through a typed pointer: LDS (ds_read) when
        // staged, global otherwise -- a generic one would make every byte read wait for the tile's
        // outstanding stores
        if (!Body::kTyped) body(a, wl, area, rec, avail, seg, r, tile, lane, act);
        else if (__builtin_amdgcn_readfirstlane(stage_at) >= 0) body(a, wl, area, (walk_lds_cu8*)stage_l + stage_at, avail, seg, r, tile, lane, act);
        else body(a, wl, area, gp(a.data) + base, avail, seg, r, tile, lane, act);
        wave_sync_lds();
        if (a.vlds) {   // the tile's words: one plain store each (this wave owns them), then cleared
            for (int i = lane; i < a.n_vslots; i += kWave) {
                const DevColumn c = ldc(a.cols + *gp(a.vslot_col + i));
                *gp(c.validity + (int64_t)*gp(a.vslot_slot + i) * a.n_tiles + tile) = wl.vw[i];
                wl.vw[i] = 0;
            }
            for (int i = lane; i < a.n_sslots; i += kWave) wl.cur[i] = 0;
            wave_sync_lds();
        }
    }
}

// VarOccursRecordExtractor's string dependee (extractVarOccursRecordBytes, :88-101): the zero-filled
// bytes decoded as a string, registered as the occurs_mappings key id + 1 it equals (0: none) --
// walk_length's and the specialised framing's (jit_chain_source) step.
__device__ __forceinline__ void walk_len_str_dep(const WalkArgs& a, const Field& f, const uint8_t* zb, int size, int slot,
                                                 WalkDeps& dep) {
    auto lutf = [&](uint32_t b) { return f.kind == CBX_K_STRING_ASCII ? ascii_lut(b) : a.lut[b]; };
    const StrSpan s = string_span(f.kind, f.trim, zb, size, lutf);
    uint8_t buf[64];
    int key = 0;
    if (s.utf8_len <= 64) {
        string_write(f.kind, zb, s, buf, lutf);
        for (int h = 0; h < a.n_handlers && key == 0; h++) {
            const cbx_walk_handler hd = ldc(a.handlers + h);
            bool eq = hd.key_len == s.utf8_len;
            for (int i = 0; eq && i < s.utf8_len; i++) eq = hd.key[i] == buf[i];
            if (eq) key = hd.key_id + 1;
        }
    }
    dep.set(slot, true, WalkDep{2, key});
}

#ifndef CBX_JIT_WALK
struct TableWalk {
    static constexpr bool kTyped = false;   // one instantiation, generic record pointer
    template <typename RP>
    __device__ __forceinline__ void operator()(const WalkArgs& a, const WalkLds& wl, uint8_t* area, RP rec, int avail,
                                               int seg, int64_t r, int64_t tile, int lane, bool act) const {
        walk_tile(a, wl, area, (const uint8_t*)rec, avail, seg, r, tile, lane, act);
    }
};

__global__ __launch_bounds__(256) void walk_kernel(WalkArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
    walk_tiles(a, wsm, TableWalk{});
}

// ---- hierarchical records: a string DEPENDING ON field's registration per row ----
// extractValue's Right(s) (RecordExtractors.scala:285-292) as the walk keeps it (walk_prim_f): the
// occurs_mappings key id + 1 the decoded string equals (0: no handler lists it), registered whenever
// the field starts within the row (a null string -- offset past the end -- registers nothing).  One
// thread per row; validity one ballot word per 64 rows (cbx_hier_dependee_values).
__global__ __launch_bounds__(64) void hier_dep_str_kernel(const uint8_t* data, int64_t n_bytes, const int64_t* rec_off,
                                                         const int32_t* rec_len, int64_t n, int32_t start_off,
                                                         const CBX_CONST Field* fp, const uint32_t* lut,
                                                         const CBX_CONST cbx_walk_handler* handlers, int32_t n_handlers,
                                                         int64_t* values, uint64_t* validity) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const Field f = ldc(fp);
    bool ok = false;
    int key = 0;
    if (x < n) {
        const int64_t base = rec_off[x];
        const int avail = rec_len[x];
        const int o = start_off + f.offset;
        ok = o <= avail && base + o <= n_bytes;
        if (ok) {
            int m = o + f.size <= avail ? f.size : avail - o;
            if (base + o + m > n_bytes) m = (int)(n_bytes - base - o);
            const uint8_t* p = data + base + o;
            auto lutf = [&](uint32_t b) { return f.kind == CBX_K_STRING_ASCII ? ascii_lut(b) : lut[b]; };
            const StrSpan sp = string_span(f.kind, f.trim, p, m, lutf);
            const int len = sp.utf8_len;
            if (len <= 64) {
                uint8_t buf[64];
                string_write(f.kind, p, sp, buf, lutf);
                for (int h = 0; h < n_handlers && key == 0; h++) {
                    const cbx_walk_handler hd = ldc(handlers + h);
                    bool eq = hd.key_len == len;
                    for (int i = 0; eq && i < len; i++) eq = hd.key[i] == buf[i];
                    if (eq) key = hd.key_id + 1;
                }
            }
        }
        values[x] = key;
    }
    const uint64_t mm = __ballot(ok);
    if (threadIdx.x == 0 && x < n) validity[x >> 6] = mm;
}

// ---- VarOccursRecordExtractor: record lengths by walking each record's dependees ----
// extractVarOccursRecordBytes (:52-136): a walk with no decoding besides the dependees, every
// non-redefined field advancing by its walked size; the record is the walked prefix of the stream
// (a short read at the end is zero-filled: the record may reach past n_bytes).  The stream's framing
// from these lengths is chunk-parallel (cbx_chain.h: VarOccursStep).
__device__ int walk_length(const WalkArgs& a, const uint8_t* rec, int avail) {
    WalkFrame st[kWalkDepth];
    WalkDeps dep;
    dep.clear();
    int sp = 0;
    st[0] = WalkFrame{a.root, 0, ldc(a.nodes + a.root).child, 0, 0, 0, 0};
    int last_size = 0;
    bool popped = false;
    uint8_t zb[64];
    while (sp >= 0) {
        WalkFrame& fr = st[sp];
        const cbx_walk_node nd = ldc(a.nodes + fr.node);
        if (fr.elems) {
            if (popped) { fr.off += last_size; fr.cur++; popped = false; }
            if (fr.cur < fr.cnt) {
                if (nd.kind == CBX_W_GROUP) {
                    if (sp + 1 >= kWalkDepth) return -1;
                    st[sp + 1] = WalkFrame{fr.node, 0, nd.child, 0, fr.off, fr.off, 0};
                    sp++;
                    continue;
                }
                fr.off += nd.data_size * (fr.cnt - fr.cur);   // primitive elements: dataSize * count
                fr.cur = fr.cnt;
                continue;
            }
            last_size = fr.off - fr.start;
            sp--;
            popped = true;
            continue;
        }
        if (popped) {   // extractGroup (:111-131): every non-redefined field advances by its walked size
            const cbx_walk_node ch = ldc(a.nodes + fr.cur);
            if (!(ch.flags & CBX_W_REDEFINED)) fr.off += last_size;
            fr.cur = ch.next;
            popped = false;
        }
        if (fr.cur < 0) { last_size = fr.off - fr.start; sp--; popped = true; continue; }
        const int ci = fr.cur;
        const cbx_walk_node ch = ldc(a.nodes + ci);
        if (ch.array >= 0) {
            const int cnt = walk_count(a, ch.array, dep);
            if (sp + 1 >= kWalkDepth) return -1;
            st[sp + 1] = WalkFrame{ci, 1, 0, cnt, fr.off, fr.off, 0};
            sp++;
            continue;
        }
        if (ch.kind == CBX_W_GROUP) {
            if (sp + 1 >= kWalkDepth) return -1;
            st[sp + 1] = WalkFrame{ci, 0, ch.child, 0, fr.off, fr.off, 0};
            sp++;
            continue;
        }
        if (ch.dep_slot >= 0 && ch.field >= 0) {   // a dependee: decoded from the (zero-filled) bytes
            const Field f = ldc(a.fields + ch.field);
            const int size = ch.actual_size < 64 ? ch.actual_size : 64;
            for (int i = 0; i < size; i++) zb[i] = fr.off + i < avail ? rec[fr.off + i] : 0;
            if (f.kind == CBX_K_STRING || f.kind == CBX_K_STRING_ASCII) {
                walk_len_str_dep(a, f, zb, size, ch.dep_slot, dep);
            } else {
                const Val dv = decode_count_int(f, zb);
                dep.set(ch.dep_slot, dv.valid, WalkDep{1, (int32_t)dv.lo});
            }
        }
        if (!(ch.flags & CBX_W_REDEFINED)) fr.off += ch.actual_size;
        fr.cur = ch.next;
    }
    return last_size;
}

#endif  // CBX_JIT_WALK

}  // namespace cbx
