// cbx_select.h -- variable-length record streams after framing: record selection with Seg_IdN
// accumulation (VarLenNestedIterator + SegmentIdAccumulator), the Seg_IdN string columns, and
// the sparse index (IndexGenerator).  Included by cbx_capi.hip after cbx_kernels.hip.
//
// The reference walks records one at a time per index entry; here every per-record quantity is a
// scan over the framed records:
//   * key pass: each record's segment id -> key index of the plan's segment map (one thread per
//     record, the bytes read from HBM);
//   * Seg_IdN state: a state machine over the records (SegmentIdAccumulator.acquiredSegmentId) is
//     a scan with an associative "run summary" operator: a run that contains an entry start or a
//     level-0 record resets the state (absolute), any other run adds level counters and may set
//     the current level (relative).  Runs of kSelRun records are summarised in parallel, the run
//     summaries scanned by one workgroup, and every run re-walked from its incoming state;
//   * selection: keep flags (root reached, segment_filter) -> per-run counts -> device scan ->
//     compacted outputs (payload offset / length, Record_Id, active segment, Seg_IdN state).
//   * sparse index: the split chain over the framed records, in closed form where the reference's
//     rule allows it (non-hierarchical record counts; size splits with the split size subtracted)
//     and as one wave walking the candidate list otherwise.
#pragma once

namespace cbx {

constexpr int kSelRun = 64;          // records per run (one thread walks a run)
constexpr int kSelScanThreads = 256;

struct SelArgs {
    const uint8_t* data;
    int64_t n_bytes;
    const int64_t* rec_off;
    const int32_t* rec_len;
    int64_t n;
    int32_t start_off;
    int32_t L;                             // segment levels
    const CBX_CONST cbx_segment_map* m;    // nullptr: no segment field
    const uint32_t* lut;
    const CBX_CONST Field* fields;
    const int64_t* ent_first;              // first record of each entry (ascending)
    const int64_t* ent_rid;                // record_index of each entry
    const int64_t* ent_end;                // offset_to of each entry (-1: to the end of the file)
    int32_t n_ent;
    int32_t footer;                        // file_end_offset
    int8_t* key;                           // per record: key index, -1 none
};

// Seg_IdN state / run summary.  As a state: level = SegmentIdAccumulator.currentLevel, root = the
// record id of the current root (-1: currentRootId == ""), cnt[l] = segmentIdAccumulator(l).  As a
// run summary: reset != 0 -> the state after the run does not depend on the state before it;
// else level is the last level seen (-1 none) and cnt[] are increments.
struct SegSum {
    int32_t reset, level;
    int64_t root;
    int64_t cnt[CBX_MAX_SEG_LEVELS];
};

__device__ __forceinline__ SegSum seg_identity() {
    SegSum s;
    s.reset = 0; s.level = -1; s.root = -1;
    for (int l = 0; l < CBX_MAX_SEG_LEVELS; l++) s.cnt[l] = 0;
    return s;
}

// a then b
__device__ __forceinline__ SegSum seg_compose(const SegSum& a, const SegSum& b, int L) {
    if (b.reset) return b;
    SegSum r = a;
    if (b.level >= 0) r.level = b.level;
    for (int l = 1; l < L; l++) r.cnt[l] += b.cnt[l];
    return r;
}

__device__ __forceinline__ int sel_entry(const SelArgs& a, int64_t i) {
    int lo = 0, hi = a.n_ent - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.ent_first[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// One record through the accumulator (VarLenNestedIterator.getSegmentLevelIds ->
// SegmentIdAccumulator.acquiredSegmentId; a new index entry starts a fresh accumulator).
__device__ __forceinline__ void seg_apply(const SelArgs& a, SegSum& s, int64_t i, int e, int k) {
    if (a.ent_first[e] == i) {
        s.reset = 1; s.level = -1; s.root = -1;
        for (int l = 0; l < CBX_MAX_SEG_LEVELS; l++) s.cnt[l] = 0;
    }
    const int lv = (k >= 0 && a.L > 0) ? a.m->key_level[k] : -1;
    if (lv == 0) {
        s.reset = 1; s.level = 0;
        s.root = a.ent_rid[e] + (i - a.ent_first[e]);
        for (int l = 0; l < CBX_MAX_SEG_LEVELS; l++) s.cnt[l] = 0;
    } else if (lv > 0) {
        s.cnt[lv] += 1;
        s.level = lv;
    }
}

// FileStreamer bounds an entry's stream to offset_to (size = min(file size, offset_to)) and
// RecordHeaderParser*.getRecordMetadata takes a header whose remaining bytes up to that size are
// within file_end_offset for the file footer: such records at the end of a bounded entry are not
// returned (SC/source/streaming/FileStreamer.scala:40, RecordHeaderParserRDW.scala:47-48).
__device__ __forceinline__ bool sel_footer(const SelArgs& a, int64_t i, int e) {
    return a.footer > 0 && a.ent_end[e] > 0 && a.ent_end[e] - a.rec_off[i] <= a.footer;
}

__global__ void sel_key_kernel(SelArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    int k = -1;
    if (a.m) k = segment_key(a.m, a.lut, a.fields, a.data + a.rec_off[i], a.rec_len[i], a.start_off);
    a.key[i] = (int8_t)k;
}

__global__ void sel_sum_kernel(SelArgs a, SegSum* sums, int64_t n_runs) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_runs) return;
    const int64_t i0 = t * kSelRun, i1 = i0 + kSelRun < a.n ? i0 + kSelRun : a.n;
    SegSum s = seg_identity();
    int e = sel_entry(a, i0);
    for (int64_t i = i0; i < i1; i++) {
        while (e + 1 < a.n_ent && a.ent_first[e + 1] <= i) e++;
        if (sel_footer(a, i, e)) continue;
        seg_apply(a, s, i, e, a.key[i]);
    }
    sums[t] = s;
}

// Exclusive scan of the run summaries in place (one workgroup): each thread folds a contiguous
// chunk, thread 0 scans the chunk totals, each thread rewrites its chunk with incoming states.
__global__ __launch_bounds__(kSelScanThreads) void sel_scan_kernel(SegSum* sums, int64_t n_runs, int32_t L) {
    __shared__ SegSum s_tot[kSelScanThreads];
    const int64_t per = (n_runs + kSelScanThreads - 1) / kSelScanThreads;
    const int64_t c0 = threadIdx.x * per, c1 = c0 + per < n_runs ? c0 + per : n_runs;
    SegSum acc = seg_identity();
    for (int64_t t = c0; t < c1; t++) acc = seg_compose(acc, sums[t], L);
    s_tot[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        SegSum run = seg_identity();
        for (int j = 0; j < kSelScanThreads; j++) {
            const SegSum x = s_tot[j];
            s_tot[j] = run;
            run = seg_compose(run, x, L);
        }
    }
    __syncthreads();
    SegSum in = s_tot[threadIdx.x];
    for (int64_t t = c0; t < c1; t++) {
        const SegSum x = sums[t];
        sums[t] = in;
        in = seg_compose(in, x, L);
    }
}

// kept = root reached (no levels, or level-0 id non-null) && segment_filter admits the id
// (VarLenNestedIterator.isSegmentMatchesTheFilter, :138-147)
__device__ __forceinline__ bool sel_keep(const SelArgs& a, const SegSum& s, int k) {
    if (a.L > 0 && s.level < 0) return false;
    if (a.m && a.m->has_filter) return k >= 0 && a.m->key_in_filter[k];
    return true;
}

// pass 0 counts kept records per run; pass 1 writes them at the run's scanned base.
__global__ void sel_emit_kernel(SelArgs a, const SegSum* in_state, int64_t n_runs, int pass, uint32_t* counts,
                                const int64_t* base, cbx_selection out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_runs) return;
    const int64_t i0 = t * kSelRun, i1 = i0 + kSelRun < a.n ? i0 + kSelRun : a.n;
    SegSum s = in_state[t];
    int e = sel_entry(a, i0);
    int64_t o = pass ? base[t] : 0;
    uint32_t c = 0;
    for (int64_t i = i0; i < i1; i++) {
        while (e + 1 < a.n_ent && a.ent_first[e + 1] <= i) e++;
        if (sel_footer(a, i, e)) continue;
        const int k = a.key[i];
        seg_apply(a, s, i, e, k);
        if (!sel_keep(a, s, k)) continue;
        c++;
        if (!pass) continue;
        out.rec_off[o] = a.rec_off[i];
        out.rec_len[o] = a.rec_len[i];
        out.record_id[o] = a.ent_rid[e] + (i - a.ent_first[e]);
        out.segment[o] = (k >= 0 && a.m) ? a.m->key_segment[k] : -1;
        if (out.seg_state && a.L > 0) {
            int64_t* st = out.seg_state + o * (int64_t)(1 + a.L);
            st[0] = s.root;
            for (int l = 0; l < a.L; l++) st[1 + l] = l <= s.level ? (l == 0 ? 0 : s.cnt[l]) : -2;
        }
        o++;
    }
    if (!pass) counts[t] = c;
}

// first record of each entry: the records whose payload lies before the entry's offset_from
__global__ void sel_entry_first_kernel(const int64_t* rec_off, int64_t n, const int64_t* ent_from, int32_t n_ent,
                                       int64_t* ent_first) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_ent) return;
    const int64_t f = ent_from[e];
    int64_t lo = 0, hi = n;   // first i with rec_off[i] >= f
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (rec_off[mid] < f) lo = mid + 1; else hi = mid;
    }
    ent_first[e] = lo;
}

// ------------------------------------------------------------------------------------------
// Seg_IdN strings (SegmentIdAccumulator.getSegmentLevelId, :54-64):
//   level 0: currentRootId = prefix_fileId_rootRecordId ("" before any root of the entry)
//   level l: currentRootId _L<l>_<counter>;  null above the current level.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int dec_digits(int64_t v) {
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    int d = 1;
    while (u >= 10) { u /= 10; d++; }
    return d + (v < 0 ? 1 : 0);
}

__device__ __forceinline__ int put_dec(uint8_t* p, int64_t v) {
    const int n = dec_digits(v);
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    for (int i = n - 1; i >= (v < 0 ? 1 : 0); i--) { p[i] = (uint8_t)('0' + u % 10); u /= 10; }
    if (v < 0) p[0] = '-';
    return n;
}

struct SegIdArgs {
    const int64_t* state;    // [n][1 + L]
    int64_t n;
    int32_t L, level;
    int32_t file_id;
    int32_t prefix_len;
    const CBX_CONST cbx_segment_map* m;
};

__device__ __forceinline__ uint32_t segid_len(const SegIdArgs& a, int64_t r, bool& valid) {
    const int64_t* st = a.state + r * (int64_t)(1 + a.L);
    const int64_t v = st[1 + a.level];
    valid = v != -2;
    if (!valid) return 0;
    const int64_t root = st[0];
    uint32_t n = root >= 0 ? (uint32_t)(a.prefix_len + 1 + dec_digits(a.file_id) + 1 + dec_digits(root)) : 0u;
    if (a.level > 0) n += 2 + dec_digits(a.level) + 1 + dec_digits(v);
    return n;
}

__global__ void segid_len_kernel(SegIdArgs a, uint32_t* len) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > a.n) return;
    bool valid;
    len[r] = r < a.n ? segid_len(a, r, valid) : 0u;
}

// The Seg_Id text of record r at p (segid_len bytes).
__device__ __forceinline__ void segid_emit(const SegIdArgs& a, int64_t r, uint8_t* p) {
    const int64_t* st = a.state + r * (int64_t)(1 + a.L);
    if (st[0] >= 0) {
        for (int i = 0; i < a.prefix_len; i++) *p++ = a.m->prefix[i];
        *p++ = '_';
        p += put_dec(p, a.file_id);
        *p++ = '_';
        p += put_dec(p, st[0]);
    }
    if (a.level > 0) {
        *p++ = '_'; *p++ = 'L';
        p += put_dec(p, a.level);
        *p++ = '_';
        p += put_dec(p, st[1 + a.level]);
    }
}

__global__ void segid_write_kernel(SegIdArgs a, int64_t* offsets, uint8_t* data, int64_t capacity, uint64_t* validity,
                                   int32_t* status) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = r < a.n;
    bool valid = false;
    uint32_t n = act ? segid_len(a, r, valid) : 0u;
    const uint64_t m = __ballot(act && valid);
    if ((threadIdx.x & 63) == 0 && r < a.n + 63) validity[r / 64] = m;
    if (!act || !valid) return;
    const int64_t o = offsets[r];
    if (o + n > capacity) { atomicOr(status, 1); return; }
    segid_emit(a, r, data + o);
}

// String-view layout of a Seg_Id column (one thread per record, 256-thread blocks: a wave is a
// tile): every value is written into its tile's region of the data buffer (wave scan) and its
// view built from the bytes just written (inline when at most 12 bytes).
__global__ __launch_bounds__(256) void segid_view_kernel(SegIdArgs a, u32x4* views, uint8_t* data, int64_t tile_bytes,
                                                         int64_t tiles_per_buf, uint64_t* validity, int64_t pitch) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool act = r < a.n;
    bool valid = false;
    const uint32_t n = act ? segid_len(a, r, valid) : 0u;
    const uint64_t m = __ballot(act && valid);
    if (lane == 0 && r < pitch) validity[r / 64] = m;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(n, lane, tot);
    if (r >= pitch) return;
    const int64_t tile = r / 64;
    uint8_t* p = data + tile * tile_bytes + ex;
    if (act && valid) segid_emit(a, r, p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // read back this lane's own bytes
    uint32_t w[3] = {0u, 0u, 0u};
    const uint32_t k = n > 12 ? 4u : n;
#pragma unroll
    for (uint32_t j = 0; j < 12; j++)
        if (j < k) w[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
    u32x4 v{n, w[0], w[1], w[2]};
    if (n > 12) {
        const int64_t tb = tile >> __builtin_ctzll((unsigned long long)tiles_per_buf);   // a power of two
        v.z = (uint32_t)tb;
        v.w = (uint32_t)((tile - tb * tiles_per_buf) * tile_bytes + ex);
    }
    views[r] = v;
}

// ------------------------------------------------------------------------------------------
// Sparse index (IndexGenerator.sparseIndexGenerator, :61-120) over framed records.
// Record c in the reference's numbering (every header read counts, the file header too) is a
// split candidate when it is valid, the stream is not at its end after reading it, and (when
// hierarchical) its segment id is a root id.  With s_k the k-th entry's first record:
//   records:          s_{k+1} = first candidate >= s_k + N
//   size, subtract:   s_{k+1} = first candidate > s_k with prefix(c) >= (k + 1) S
//   size, reset:      s_{k+1} = first candidate > s_k with prefix(c) - prefix(s_k) >= S
// (prefix(c) = byte offset of c's header).  In candidate ranks the subtract rule is
// rank_{k+1} = max(rank_k + 1, r_{k+1}), r_j = first rank with prefix >= jS, i.e.
// rank_k = k + max(rank_0, max_{j<=k} (r_j - j)): a prefix maximum.  Non-hierarchical record
// splits are s_k = kN.  Hierarchical record splits and reset-mode size splits are a chain walked
// by one wave (64 candidates per probe).
// ------------------------------------------------------------------------------------------
struct IdxArgs {
    const int64_t* rec_off;
    const int32_t* rec_len;
    int64_t n;
    int64_t n_bytes;
    int32_t header_bytes;
    int32_t has_header;      // record numbering offset
    const int8_t* key;       // per record key (root test), nullptr: every valid record is a root
    const CBX_CONST cbx_segment_map* m;
};

__device__ __forceinline__ bool idx_candidate(const IdxArgs& a, int64_t i) {
    if (a.rec_off[i] + a.rec_len[i] >= a.n_bytes) return false;   // isEndOfStream after reading it
    if (a.key) {
        const int k = a.key[i];
        return k >= 0 && a.m->key_level[k] == 0;
    }
    return true;
}

__global__ void idx_flag_kernel(IdxArgs a, uint32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > a.n) return;
    flag[i] = i < a.n && idx_candidate(a, i) ? 1u : 0u;
}

// cand[rank] = framed index of each candidate
__global__ void idx_compact_kernel(IdxArgs a, const uint32_t* flag, const int64_t* excl, int64_t* cand) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    if (flag[i]) cand[excl[i]] = i;
}

__device__ __forceinline__ int64_t idx_prefix(const IdxArgs& a, int64_t i) { return a.rec_off[i] - a.header_bytes; }

// subtract mode: r_j = first candidate rank with prefix >= j*S - rho, for j = 1..K (binary search);
// rho: bytesInChunk at the first record (IndexGenerator.scala:88-127, a piece of a file that starts at
// one of its entries carries that entry's residual)
__global__ void idx_size_kernel(IdxArgs a, const int64_t* cand, int64_t n_cand, int64_t S, int64_t K, int64_t rho, int64_t* rj) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (j > K) return;
    const int64_t target = j * S - rho;
    int64_t lo = 0, hi = n_cand;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (idx_prefix(a, cand[mid]) < target) lo = mid + 1; else hi = mid;
    }
    rj[j - 1] = lo - j;    // r_j - j
}

// One wave walks the split chain over the candidate list: from rank `cur`, the next split is the
// first rank whose candidate satisfies the target; probes of 64 ranks, galloping then 64-ary search.
// mode 0: records (target index s + N);  mode 2: size-reset (target prefix(s) + S; the first entry's
// bytesInChunk starts at rho).  out[k] = framed index of split k (k >= 1); *n_out = number of splits.
__global__ __launch_bounds__(64) void idx_walk_kernel(IdxArgs a, const int64_t* cand, int64_t n_cand, int mode,
                                                      int64_t N, int64_t S, int64_t rho, int64_t* out, int64_t cap, int64_t* n_out) {
    const int lane = threadIdx.x;
    // entry 0 starts at record 0 (numbering position 0); its "position" for the targets:
    int64_t pos_num = 0;                       // record number of the current split
    int64_t pos_prefix = -rho;                 // its header offset (less the bytes it starts with)
    int64_t cur = -1;                          // candidate rank of the current split (-1: entry 0)
    int64_t k = 0;
    auto ok = [&](int64_t r) -> bool {         // candidate r satisfies the target (monotone in r)
        const int64_t i = cand[r];
        if (mode == 0) return i + a.has_header >= pos_num + N;
        return idx_prefix(a, i) - pos_prefix >= S;
    };
    while (true) {
        // first rank > cur with ok(rank): gallop
        int64_t lo = cur + 1;              // ok(lo - 1) false or lo = cur + 1
        if (lo >= n_cand) break;
        int64_t step = 1, hi = -1;
        while (hi < 0) {
            const int64_t r = lo + (int64_t)lane * step;
            const bool good = r < n_cand && ok(r);
            const bool past = r >= n_cand;
            const uint64_t m = __ballot(good || past);
            if (m) {
                const int f = __builtin_ctzll(m);
                hi = lo + (int64_t)f * step;          // ok at or beyond
                if (f > 0) lo = lo + (int64_t)(f - 1) * step + 1;
                break;
            }
            lo = lo + 63 * step + 1;          // every rank up to lo + 63 step was probed and missed
            if (lo >= n_cand) { hi = n_cand; break; }
            step *= 64;
        }
        if (hi > n_cand) hi = n_cand;
        // 64-ary search in [lo, hi]: probes at lo + lane * st with st = ceil(span / 63), so lane 63
        // probes at or past hi and the ballot is never empty (with ceil(span / 64) a match in the
        // last stride left it empty, and ctz(0) sent the search backwards)
        while (lo < hi) {
            const int64_t span = hi - lo;
            const int64_t st = (span + 62) / 63;
            const int64_t r = lo + (int64_t)lane * st;
            const bool good = r >= hi || ok(r);
            const uint64_t m = __ballot(good);
            const int f = __builtin_ctzll(m);
            const int64_t rf = lo + (int64_t)f * st;
            if (f == 0) { hi = lo; break; }
            lo = lo + (int64_t)(f - 1) * st + 1;
            hi = rf < hi ? rf : hi;
        }
        if (lo >= n_cand) break;
        cur = lo;
        const int64_t i = cand[cur];
        pos_num = i + a.has_header;
        pos_prefix = idx_prefix(a, i);
        if (lane == 0 && k < cap) out[k] = i;
        k++;
    }
    if (lane == 0) *n_out = k;
}

}  // namespace cbx
