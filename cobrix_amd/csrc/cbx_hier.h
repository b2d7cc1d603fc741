// cbx_hier.h -- hierarchical records (`segment-children`): VarLenHierarchicalIterator + the
// structure walk of RecordExtractors.extractHierarchicalRecord as passes over the framed records
// (CP/reader/iterator/VarLenHierarchicalIterator.scala:43-162,
//  CP/reader/extractors/record/RecordExtractors.scala:211-385).  Included by cbx_capi.hip.
//
// The reference accumulates the records of one root segment (a new root closes the previous
// hierarchical record; records before the first root are dropped) and walks them recursively:
// the children of type C of a parent instance p are the records of type C after p up to the first
// record whose segment id is p's or one of p's ancestors' (extractChildren, :298-322).  With one
// segment id per non-leaf segment (checked by the host) that rule is static per type: record x of
// type S with parent type P belongs to
//   * the group's root record, when P is the root segment (every record of the group lies before the
//     next root);
//   * else p = the last record of type P before x in the group, provided p itself belongs to the
//     tree and no record of a type that is a strict (non-root) ancestor of P lies between p and x;
// otherwise x is in no list (the reference never reaches it).  Every quantity is a "last position of
// type k" -- a prefix maximum of a vector of positions -- so the passes are:
//   type (segment id -> segment) -> last positions per 4096-record block -> scan over blocks ->
//   per record: parent candidate + static check -> chase to the root (depth <= segments) ->
//   per-table compaction (table 0: roots = hierarchical records, table 1 + s: segment s) ->
//   parent rows -> (per child segment) list offsets by binary search over the parent rows.
// Tables hold rows in record order, so each child list is a contiguous run of its table.
#pragma once

namespace cbx {

constexpr int kHierMaxSeg = 16;
constexpr int kHierThreads = 256;
constexpr int kHierPer = 16;
constexpr int kHierTile = kHierThreads * kHierPer;   // records per block of the last-position passes

struct HierArgs {
    const uint8_t* data;
    const int64_t* rec_off;
    const int32_t* rec_len;
    int64_t n;
    const CBX_CONST cbx_segment_map* m;
    const uint32_t* lut;
    const CBX_CONST Field* fields;
    int32_t n_seg;                    // segment types (<= kHierMaxSeg)
    int32_t start_off;                // record_start_offset (segment ids are read past it)
    int32_t root;                     // the root segment
    int32_t parent[kHierMaxSeg];      // parent segment, -1 for the root / unused
    uint32_t anc[kHierMaxSeg];        // strict non-root ancestors of the parent of each segment (bits)
    int8_t* type;                     // per record: segment, -1 none
    int8_t* key;                      // per record: segment id key, -1 none (the general walk only; may be null)
    int8_t* st;                       // per record: 0 not in the tree, 1 root, 2 child candidate
    int8_t* tab;                      // per record: table, -1 none
    int64_t* par;                     // per record: parent record (candidates)
    int64_t* row_of;                  // per record: row in the output, -1 none
};

// segment id -> segment of the record (VRLRecordReader.getSegmentId + segmentRedefineMap)
__global__ void hier_type_kernel(HierArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int k = segment_key(a.m, a.lut, a.fields, a.data + a.rec_off[i], a.rec_len[i], a.start_off);
    int s = -1;
    if (k >= 0) s = a.m->key_segment[k];
    a.type[i] = (int8_t)(s >= 0 && s < a.n_seg ? s : -1);
    if (a.key) a.key[i] = (int8_t)(s >= 0 && s < a.n_seg ? k : -1);
}

// mode 0: last position of every type in the block -> blk_lp[block][k].
// mode 1: from the block's incoming vector (blk_lp after the scan), every record's parent
// candidate and its static check -> st / par.
__global__ __launch_bounds__(kHierThreads) void hier_last_kernel(HierArgs a, int mode, int64_t* blk_lp) {
    __shared__ int64_t s_lp[kHierThreads][kHierMaxSeg];
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int64_t i0 = b * kHierTile + (int64_t)t * kHierPer;
    for (int k = 0; k < kHierMaxSeg; k++) s_lp[t][k] = -1;
    for (int j = 0; j < kHierPer; j++) {
        const int64_t i = i0 + j;
        if (i >= a.n) break;
        const int s = a.type[i];
        if (s >= 0) s_lp[t][s] = i;
    }
    __syncthreads();
    if (mode == 0) {
        if (t < a.n_seg) {
            int64_t mx = -1;
            for (int u = 0; u < kHierThreads; u++) mx = s_lp[u][t] > mx ? s_lp[u][t] : mx;
            blk_lp[b * kHierMaxSeg + t] = mx;
        }
        return;
    }
    if (t < a.n_seg) {   // exclusive prefix maximum over the block's threads, from the block's incoming value
        int64_t run = blk_lp[b * kHierMaxSeg + t];
        for (int u = 0; u < kHierThreads; u++) {
            const int64_t x = s_lp[u][t];
            s_lp[u][t] = run;
            run = x > run ? x : run;
        }
    }
    __syncthreads();
    for (int j = 0; j < kHierPer; j++) {
        const int64_t i = i0 + j;
        if (i >= a.n) break;
        const int s = a.type[i];
        int8_t state = 0;
        int64_t p = -1;
        if (s == a.root) {
            state = 1;
        } else if (s >= 0 && a.parent[s] >= 0) {
            const int P = a.parent[s];
            const int64_t g0 = s_lp[t][a.root];   // the group's root record
            bool ok = g0 >= 0;
            if (P == a.root) {
                p = g0;
            } else {
                p = s_lp[t][P];
                ok = ok && p > g0;
                for (uint32_t bits = a.anc[s]; ok && bits; bits &= bits - 1)
                    ok = s_lp[t][__builtin_ctz(bits)] < p;
            }
            if (ok) state = 2; else p = -1;
        }
        a.st[i] = state;
        a.par[i] = p;
        if (s >= 0) s_lp[t][s] = i;
    }
}

// Exclusive prefix maximum of the block vectors, in place (one workgroup: contiguous chunks per
// thread, chunk totals scanned by thread 0, chunks rewritten).
__global__ __launch_bounds__(kHierThreads) void hier_lp_scan_kernel(int64_t* blk_lp, int64_t n_blk, int32_t n_seg) {
    __shared__ int64_t s_tot[kHierThreads][kHierMaxSeg];
    const int t = threadIdx.x;
    const int64_t per = (n_blk + kHierThreads - 1) / kHierThreads;
    const int64_t c0 = t * per, c1 = c0 + per < n_blk ? c0 + per : n_blk;
    int64_t acc[kHierMaxSeg];
#pragma unroll
    for (int k = 0; k < kHierMaxSeg; k++) acc[k] = -1;
    for (int64_t c = c0; c < c1; c++)
#pragma unroll
        for (int k = 0; k < kHierMaxSeg; k++) {
            const int64_t x = k < n_seg ? blk_lp[c * kHierMaxSeg + k] : -1;
            acc[k] = x > acc[k] ? x : acc[k];
        }
#pragma unroll
    for (int k = 0; k < kHierMaxSeg; k++) s_tot[t][k] = acc[k];
    __syncthreads();
    if (t < n_seg) {
        int64_t run = -1;
        for (int u = 0; u < kHierThreads; u++) {
            const int64_t x = s_tot[u][t];
            s_tot[u][t] = run;
            run = x > run ? x : run;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kHierMaxSeg; k++) acc[k] = s_tot[t][k];
    for (int64_t c = c0; c < c1; c++)
#pragma unroll
        for (int k = 0; k < kHierMaxSeg; k++) {
            if (k >= n_seg) continue;
            const int64_t x = blk_lp[c * kHierMaxSeg + k];
            blk_lp[c * kHierMaxSeg + k] = acc[k];
            acc[k] = x > acc[k] ? x : acc[k];
        }
}

// A candidate belongs to the tree when every parent up its chain does (depth <= n_seg).
__global__ void hier_chase_kernel(HierArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int s0 = a.st[i];
    int tb = -1;
    if (s0 == 1) {
        tb = 0;
    } else if (s0 == 2) {
        bool ok = true;
        int64_t y = i;
        for (int d = 0; d <= a.n_seg; d++) {
            const int64_t p = a.par[y];
            if (a.type[p] == a.root) break;
            if (a.st[p] != 2) { ok = false; break; }
            y = p;
        }
        if (ok) tb = 1 + a.type[i];
    }
    a.tab[i] = (int8_t)tb;
}

// Stable compaction by table, one record per thread, 4 waves per block.  mode 0: per-(table,
// block) counts -> cnt[table * n_blk + block]; mode 1: rows from the scanned bases.
__global__ __launch_bounds__(256) void hier_emit_kernel(HierArgs a, int mode, int64_t n_blk, uint32_t* cnt,
                                                        const int64_t* base, int64_t first_id, cbx_selection out) {
    __shared__ uint32_t s_cnt[4][kHierMaxSeg + 1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int T = a.n_seg + 1;
    for (int k = threadIdx.x; k < 4 * (kHierMaxSeg + 1); k += blockDim.x) (&s_cnt[0][0])[k] = 0;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int j = i < a.n ? a.tab[i] : -1;
    uint32_t rank = 0;
    uint64_t rem = __ballot(j >= 0);
    while (rem) {   // one ballot per table present in the wave
        const int lead = __builtin_ctzll(rem);
        const int tj = __builtin_amdgcn_readlane(j, lead);
        const uint64_t mm = __ballot(j == tj);
        if (j == tj) rank = (uint32_t)__builtin_popcountll(mm & ((1ull << lane) - 1ull));
        if (lane == 0) s_cnt[w][tj] = (uint32_t)__builtin_popcountll(mm);
        rem &= ~mm;
    }
    __syncthreads();
    if (mode == 0) {
        if ((int)threadIdx.x < T) {
            const int k = threadIdx.x;
            cnt[(int64_t)k * n_blk + blockIdx.x] = s_cnt[0][k] + s_cnt[1][k] + s_cnt[2][k] + s_cnt[3][k];
        }
        return;
    }
    if (i >= a.n) return;
    if (j < 0) { a.row_of[i] = -1; return; }
    uint32_t before = 0;
    for (int u = 0; u < w; u++) before += s_cnt[u][j];
    const int64_t row = base[(int64_t)j * n_blk + blockIdx.x] + before + rank;
    a.row_of[i] = row;
    out.rec_off[row] = a.rec_off[i];
    out.rec_len[row] = a.rec_len[i];
    out.segment[row] = a.type[i];
    if (j == 0) {   // the hierarchical record's Record_Id: the index of the next root (or the end)
        const int64_t n_roots = base[n_blk];   // table 1 starts after every root row
        if (row > 0) out.record_id[row - 1] = first_id + i;
        if (row == n_roots - 1) out.record_id[row] = first_id + a.n;
    } else {
        out.record_id[row] = first_id + i;
    }
}

__global__ void hier_parent_kernel(HierArgs a, int64_t* parent_row) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int j = a.tab[i];
    if (j < 0) return;
    parent_row[a.row_of[i]] = j == 0 ? -1 : a.row_of[a.par[i]];
}

// offsets[k] = first child row (relative to child_begin) whose parent row is >= parent_begin + k
__global__ void hier_offsets_kernel(const int64_t* parent_row, int64_t child_begin, int64_t n_child, int64_t parent_begin,
                                    int64_t n_parent, int32_t* offsets) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > n_parent) return;
    const int64_t target = parent_begin + k;
    int64_t lo = 0, hi = n_child;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (parent_row[child_begin + mid] < target) lo = mid + 1; else hi = mid;
    }
    offsets[k] = (int32_t)lo;
}

// ---- the general walk (segments with children mapped from several segment ids) ----
// extractChildren breaks a parent's child list at a record whose segment ID is the parent's own or
// one of its ancestors' -- ids, not segments: with several ids per segment a record of the parent's
// segment under another id does not end the list, and one child record then sits under several
// parents (RecordExtractors.scala:298-322).  One thread per hierarchical record (its root to the next
// root) runs that recursion as the reference does, an explicit stack of (record, row, segment, child
// type, scan position); mode 0 counts the rows per table, mode 1 writes them at the scanned bases
// (cnt / base: [table][group]).  Rows of a table come out grouped by parent row in parent order.
__global__ void hier_walk_kernel(HierArgs a, const int64_t* root_pos, int64_t G, int mode, uint32_t* cnt,
                                 const int64_t* base, int64_t first_id, cbx_selection out, int64_t* parent_row) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const int64_t r0 = root_pos[g], r1 = g + 1 < G ? root_pos[g + 1] : a.n;
    const int T = a.n_seg + 1;
    int64_t nxt[kHierMaxSeg + 1];
    for (int t = 0; t < T; t++) nxt[t] = mode ? base[(int64_t)t * G + g] : 0;
    auto emit = [&](int t, int64_t rec, int64_t prow) -> int64_t {
        const int64_t row = nxt[t]++;
        if (mode) {
            out.rec_off[row] = a.rec_off[rec];
            out.rec_len[row] = a.rec_len[rec];
            out.segment[row] = a.type[rec];
            out.record_id[row] = first_id + (t == 0 ? r1 : rec);   // a root: the index of the next root (or the end)
            parent_row[row] = prow;
        }
        return row;
    };
    int64_t f_rec[kHierMaxSeg + 1], f_row[kHierMaxSeg + 1], f_j[kHierMaxSeg + 1];
    int f_seg[kHierMaxSeg + 1], f_c[kHierMaxSeg + 1], f_key[kHierMaxSeg + 1];
    int d = 0;
    f_rec[0] = r0; f_row[0] = emit(0, r0, -1); f_seg[0] = a.root; f_c[0] = -1; f_j[0] = r1; f_key[0] = a.key[r0];
    while (d >= 0) {
        const int c = f_c[d];
        bool pushed = false;
        if (c >= 0) {
            for (int64_t j = f_j[d]; j < r1; j++) {
                if (a.type[j] == c) {   // a child of this type: its row, then its own subtree
                    f_j[d] = j + 1;
                    const int64_t row = emit(1 + c, j, f_row[d]);
                    if (d + 1 <= kHierMaxSeg) {
                        d++;
                        f_rec[d] = j; f_row[d] = row; f_seg[d] = c; f_c[d] = -1; f_j[d] = r1; f_key[d] = a.key[j];
                    }
                    pushed = true;
                    break;
                }
                const int kj = a.key[j];
                bool brk = false;
                for (int u = 0; u <= d; u++) brk |= kj >= 0 && kj == f_key[u];
                if (brk) break;
            }
        }
        if (pushed) continue;
        // the next child segment of the frame's segment (segment order = copybook order)
        int nc = -1;
        for (int s = c + 1; s < a.n_seg; s++)
            if (a.parent[s] == f_seg[d]) { nc = s; break; }
        if (nc < 0) { d--; continue; }
        f_c[d] = nc;
        f_j[d] = f_rec[d] + 1;
    }
    if (!mode)
        for (int t = 0; t < T; t++) cnt[(int64_t)t * G + g] = (uint32_t)nxt[t];
}

// the root records' indices (excl: the exclusive scan of the root flags)
__global__ void hier_root_flag_kernel(HierArgs a, uint32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) flag[i] = a.type[i] == a.root ? 1u : 0u;
    if (i == a.n) flag[i] = 0u;
}
__global__ void hier_root_pos_kernel(HierArgs a, const int64_t* excl, int64_t* root_pos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n && a.type[i] == a.root) root_pos[excl[i]] = i;
}

// ---- dependee values of the rows (cbx_hier_dependee_values) ----
// One thread per row: the field decoded from the row's bytes as Primitive.decodeTypeValue does
// (RecordExtractors.extractValue, :276-292) -- null past the row's end or when malformed -- as the
// integer its registration keeps (Number.intValue).  Independent of the row's segment: the root record
// decodes every segment group from its own bytes (getGroupValues over the record group, :365-372).
// Validity: one ballot word per 64 rows.
__global__ __launch_bounds__(64) void hier_dep_values_kernel(const uint8_t* data, int64_t n_bytes, const int64_t* rec_off,
                                                            const int32_t* rec_len, int64_t n, int32_t start_off,
                                                            const CBX_CONST Field* fp, int64_t* values, uint64_t* validity) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const Field f = ldc(fp);
    bool ok = false;
    int64_t v = 0;
    if (x < n) {
        const int64_t base = rec_off[x];
        const int64_t o = base + start_off + f.offset;
        if (f.offset + start_off + f.size <= rec_len[x] && o >= 0 && o + f.size <= n_bytes) {
            const Val dv = decode_count_int(f, data + o);
            ok = dv.valid;
            v = (int64_t)dv.lo;
        }
        values[x] = v;
    }
    const uint64_t m = __ballot(ok);
    if (threadIdx.x == 0 && x < n) validity[x >> 6] = m;
}

// ---- the shared dependFields map (cbx_hier_dependee_counts) ----
// One thread per hierarchical record (root row r): the reference's recursive walk as an explicit
// stack of (row, segment, child-type cursor, child-row range), each row's events replayed in field
// order -- registrations into the thread's map (value + known bit per dependee), resolutions into
// the counts.  Trees are small (a root and its children): the walk is a few dependent loads per row.
static_assert(kHierMaxSeg == CBX_HIER_MAX_SEG, "hierarchical segment limit");

struct HierDepArgs {
    cbx_hier_walk w;
    cbx_hier_dependee dep[CBX_HIER_MAX_DEPS];
    cbx_hier_odo_array arr[CBX_HIER_MAX_DEPS];
    int32_t n_deps, n_arrays;
};

// The record walk's dependee slots (cbx_hier_walk.seeds): kind << 32 | value per slot.
constexpr int kHierWalkSlots = 8;
struct HierSlots {
    int64_t s[kHierWalkSlots];
};

__device__ __forceinline__ void hier_dep_events(const HierDepArgs& a, int ev_row, int64_t x, bool root, int32_t* regv,
                                                uint32_t& regok, int32_t* counts, int64_t pitch, int32_t* changed,
                                                HierSlots& sl) {
    for (int k = 0; k < CBX_HIER_MAX_EVENTS; k++) {
        const int e = a.w.events[ev_row][k];
        if (e == -32768) break;
        if (e >= 0) {
            const cbx_hier_dependee& d = a.dep[e];
            if (!((d.validity[x >> 6] >> (x & 63)) & 1ull)) continue;   // a null value registers nothing
            int32_t v;
            if (d.out_type == CBX_O_I32) v = ((const int32_t*)d.values)[x];
            else if (d.out_type == CBX_O_I64 || d.out_type == CBX_O_STRING) v = (int32_t)((const int64_t*)d.values)[x];
            else v = (int32_t)((const int64_t*)d.values)[2 * x];   // DEC128: the low 64 bits (intValue)
            regv[e] = v;
            regok |= 1u << e;
            if (d.walk_slot >= 0 && d.walk_slot < kHierWalkSlots)   // Left(int) / Right(key id + 1)
                sl.s[d.walk_slot] = (int64_t)(d.out_type == CBX_O_STRING ? 2 : 1) << 32 | (uint32_t)v;
        } else {
            const cbx_hier_odo_array& A = a.arr[-e - 1];
            const int dd = A.dependee;
            const int32_t v = regv[dd];
            const int32_t c = ((regok >> dd) & 1u) && v >= A.min_count && v <= A.max_count ? v : A.max_count;
            counts[(int64_t)A.out_row * pitch + x] = c;
            if (A.first_counts && A.first_counts[x] != c) *changed = 1;
        }
    }
}

__device__ __forceinline__ void hier_put_seed(const HierDepArgs& a, int64_t x, int64_t pitch, const HierSlots& sl) {
    if (!a.w.seeds) return;
#pragma unroll
    for (int i = 0; i < kHierWalkSlots; i++) a.w.seeds[(int64_t)i * pitch + x] = sl.s[i];
}

__global__ void hier_dep_kernel(HierDepArgs a, int32_t* counts, int64_t pitch, int32_t* changed) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.w.table_rows[0]) return;
    int32_t regv[CBX_HIER_MAX_DEPS];
    uint32_t regok = 0;
    for (int k = 0; k < CBX_HIER_MAX_DEPS; k++) regv[k] = 0;
    HierSlots sl;
    for (int k = 0; k < kHierWalkSlots; k++) sl.s[k] = 0;
    // stack frames: row, segment, next child type (index into children[seg]), child rows [lo, hi)
    int64_t f_row[kHierMaxSeg + 1], f_lo[kHierMaxSeg + 1], f_hi[kHierMaxSeg + 1];
    int f_seg[kHierMaxSeg + 1], f_ci[kHierMaxSeg + 1];
    const int root = a.w.root_segment;
    hier_dep_events(a, CBX_HIER_MAX_SEG, r, true, regv, regok, counts, pitch, changed, sl);
    hier_put_seed(a, r, pitch, sl);   // (the root's walk registers its own groups' dependees itself)
    hier_dep_events(a, root, r, true, regv, regok, counts, pitch, changed, sl);
    int d = 0;
    f_row[0] = r; f_seg[0] = root; f_ci[0] = -1; f_lo[0] = f_hi[0] = 0;
    while (d >= 0) {
        if (f_lo[d] < f_hi[d]) {   // the next child row of the current type: visit it, then its subtree
            const int c = a.w.children[f_seg[d]][f_ci[d]];
            const int64_t x = a.w.table_base[1 + c] + f_lo[d]++;
            hier_put_seed(a, x, pitch, sl);
            hier_dep_events(a, c, x, false, regv, regok, counts, pitch, changed, sl);
            if (d + 1 <= kHierMaxSeg) {
                d++;
                f_row[d] = x; f_seg[d] = c; f_ci[d] = -1; f_lo[d] = f_hi[d] = 0;
            }
            continue;
        }
        // the next child type of the row
        const int s = f_seg[d];
        const int ci = ++f_ci[d];
        const int c = ci < kHierMaxSeg ? a.w.children[s][ci] : -1;
        if (c < 0) { d--; continue; }
        // the row's index in its own table (the child's list offsets run over it)
        const int64_t pt = s == root ? 0 : 1 + s;
        const int64_t k = f_row[d] - a.w.table_base[pt];
        f_lo[d] = a.w.child_offsets[c][k];
        f_hi[d] = a.w.child_offsets[c][k + 1];
    }
}

}  // namespace cbx
