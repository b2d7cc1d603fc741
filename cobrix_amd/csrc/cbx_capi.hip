// cbx_capi.hip -- C ABI of libcobrix_hip.so (include/cobrix_hip.h): plan building, launches.
//
// The plan turns the flattened copybook (cbx_field / cbx_array tables produced by the JVM or
// the Python host from the Cobrix AST) into the device layout the kernels walk:
//   * per-field constants (decoder variant, 10^precision bounds, slot counts, string sequences),
//   * two window sets: one window holding every field (contiguous fixed-length staging) and a
//     greedy packing of every field element [offset, offset + size) into byte ranges of at most
//     `window_bytes` (windowed staging), each grouped into (field, slot range) runs so a
//     window's decode loop is wave-uniform,
//   * the UTF-8 code-page LUT and the segment-redefine keys.
// Every decode call is asynchronous on the caller's stream: the decode kernel, the fixup kernel
// for deferred values, and for string columns a scan of per-tile payload totals plus the
// placement kernel; device-side data errors are reported by cbx_plan_check.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "cbx_kernels.hip"
#include "cbx_select.h"
#include "cbx_text.h"
#include "cbx_hier.h"
#include "cbx_walk.h"
#include "cbx_chain.h"

using namespace cbx;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_CHECK(x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return fail(CBX_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct cbx_plan {
    std::vector<cbx_field> hfields;
    std::vector<Field> dfields_h;
    std::vector<cbx_array> harrays;
    // window sets (contiguous fixed-length staging: one window / windowed staging), each with
    // its own op tables in window order
    struct OpSet {
        std::vector<Window> win;
        std::vector<NumOp> nops;
        std::vector<Batch> batches;
        std::vector<StrOp> sops;
        std::vector<GenOp> gops;
        Window* d_win = nullptr;
        NumOp* d_nops = nullptr;
        Batch* d_batches = nullptr;
        StrOp* d_sops = nullptr;
        GenOp* d_gops = nullptr;
        int max_str_items = 0;   // string elements in the fullest window
        bool has_runs = false;   // some op stands for a run of OCCURS elements
    } cset, wset;
    bool contig_ok = true;       // every string element fits the single contiguous window
    int str_stage = 16;          // LDS payload staging bytes per wave
    bool view_staged = false;    // view layout: some string field takes the staged byte-loop path
    cbx_plan_options opts;
    int n_columns = 0;
    int seg_col = -1;
    int max_pitch = 0;           // widest row of the windowed set
    int n_seq = 0;               // string sequences (column, slot)
    std::vector<DeferSeq> hdefer;        // deferral sequences (numeric field, slot)
    std::vector<int32_t> col_is_string;   // per column: 1 if string/binary
    std::vector<int32_t> col_slots;       // per column: slots
    std::vector<int32_t> col_max_bytes;   // per column: max payload bytes per value
    bool view = false;                    // string columns in the string-view layout
    bool packed = false;                  // string columns in the Arrow Utf8 layout (count pass + one decode pass)
    std::vector<int32_t> segid_cols;      // segment levels with a Seg_Id column
    std::vector<ListOp> lops;             // list-layout fields (list_kernel), grouped by array
    ListOp* d_lops = nullptr;
    int32_t* d_list_len = nullptr;  int64_t list_len_cap = 0;
    int32_t* d_list_flag = nullptr; int64_t list_flag_cap = 0;
    // device copies
    Field* d_fields = nullptr;
    DeferSeq* d_defer = nullptr;
    uint64_t* d_defer_bits = nullptr;
    int64_t defer_bits_cap = 0;
    cbx_array* d_arrays = nullptr;
    cbx_segment_map* d_segmap = nullptr;
    uint32_t* d_lut = nullptr;
    DevColumn* d_cols = nullptr;
    std::vector<DevColumn> h_cols;         // host staging of the per-call column table
    std::vector<NumCall> h_ncall;          // per-call op address tables (host staging)
    std::vector<StrCall> h_scall;
    NumCall* d_ncall = nullptr;
    StrCall* d_scall = nullptr;
    size_t ncall_cap = 0, scall_cap = 0;
    // string workspace (two-pass placement): per (sequence, tile) totals and their exclusive
    // scan, tile-local value starts, per-tile payload scratch regions, per-sequence call table
    std::vector<int32_t> seq_field, seq_slot;   // sequence -> (field, slot)
    std::vector<int64_t> seq_tile_cap;          // bytes per tile region
    std::vector<SeqCall> h_seqcall;
    std::vector<int64_t> h_seq_scratch;         // per-call scratch offset of each sequence
    SeqCall* d_seqcall = nullptr;
    uint32_t* d_str_tot = nullptr;  int64_t str_tot_cap = 0;
    int64_t* d_str_excl = nullptr;  int64_t str_excl_cap = 0;
    int64_t* d_block_sums = nullptr; int64_t block_sums_cap = 0;
    uint32_t* d_local = nullptr;    int64_t local_cap = 0;
    uint8_t* d_scratch = nullptr;   int64_t scratch_cap = 0;
    uint64_t* d_stamps = nullptr;   // diagnostic build only
    // copybook-specialised kernel (cbx_jit.h), built on the first large contiguous decode
    int64_t jit_min = 262144;
    // specialised kernels: [0] windowed op set, [kp] contiguous op set with kp chunks per lane,
    // [kPre + 1 + kp] the contiguous op set over variable-length spans (span_loop)
    // specialised kernels: [0, kPre] contiguous decode by prefetch depth, kPre + 1 + kp span decode,
    // 2 (kPre + 1) + kp / 3 (kPre + 1) + kp the Utf8 layout's contiguous / span count pass
    // + [4 (kPre + 1)] the specialised list kernel
    bool jit_tried[4 * kPre + 5] = {};
    hipFunction_t jit_fn[4 * kPre + 5] = {};
    // the cooperative-tile decision each specialised kernel was compiled with (jit_coop_of reads env
    // knobs: launches reuse the compile-time answer, never re-derive it)
    bool jit_coop[4 * kPre + 5] = {};
    int rec_extent = 0;          // bytes past the decode base that any field (any OCCURS element) reaches
    std::string jit_error;
    int last_kind = 0;
    int32_t* d_status = nullptr;
    int num_cus = 256;
    // record walk (cbx_plan_set_walk, cbx_walk.h)
    bool walk = false;
    int32_t walk_root = 0, walk_var = 0, walk_n_handlers = 0, walk_depth = 1, walk_max_rec = 0;
    cbx_walk_node* d_wnodes = nullptr;
    std::vector<cbx_walk_node> h_wnodes;   // host copies: the copybook-specialised walk's source
    std::vector<cbx_walk_array> h_warr;
    bool walk_jit_tried = false;
    hipFunction_t walk_jit_fn = nullptr;
    bool chain_jit_tried = false;            // the specialised var-occurs framing (jit_chain_source)
    hipFunction_t chain_jit_fn[5] = {};      // sample, spec, fix, settle, write
    bool last_chain_jit = false;             // the last cbx_frame_var_occurs used them
    cbx_walk_array* d_warr = nullptr;
    cbx_walk_handler* d_whand = nullptr;
    int64_t* d_wslot_base = nullptr;    // per column: first string-slot index
    int64_t* d_wtile_bytes = nullptr;   // per column: view tile bytes
    const int64_t* d_rec_base = nullptr;   // caller's device Record_Id base (cbx_plan_set_record_base)
    const int32_t* d_odo = nullptr;        // caller's OCCURS DEPENDING ON counts (cbx_plan_set_odo_counts)
    int64_t odo_pitch = 0;
    const int64_t* d_dep_seed = nullptr;   // the record walk's per-row dependFields seeds (cbx_plan_set_dep_seed)
    int64_t seed_pitch = 0;
    int32_t seed_root = -1;
    int64_t n_str_slots = 0;
    uint32_t* d_wcursor = nullptr; int64_t wcursor_cap = 0;
    int64_t* d_wvbase = nullptr;        // per column: first validity-word index among all column slots
    int32_t* d_wvcol = nullptr;         // per validity word: column, slot
    int32_t* d_wvslot = nullptr;
    int32_t n_vslots = 0;
    int32_t fid_col = -1, rid_col = -1;
    // cbx_plan_pipeline: Utf8 batches of two plans on two streams, one plan's count pass beside the
    // other's decode (each call waits for the peer's last count pass before its own, and marks its own)
    cbx_plan* pipe_peer = nullptr;
    hipEvent_t pipe_done = nullptr;
    int pipe_count_bpc = 0, pipe_decode_bpc = 0;
    // profiling: HIP events around the decode kernel and the post passes of every call (no sync)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;     // free events
    struct CallEvents { hipEvent_t e[3]; };
    std::vector<CallEvents> ev_calls;    // recorded, not yet read
};

#include "cbx_jit.h"

// grow a device buffer to at least `need` elements (contents not preserved)
template <typename T>
static int grow(T** p, int64_t* cap, int64_t need, hipStream_t st) {
    if (need <= *cap) return CBX_OK;
    HIP_CHECK(hipStreamSynchronize(st));
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_CHECK(hipMalloc((void**)p, sizeof(T) * std::max<int64_t>(need, 1)));
    *cap = need;
    return CBX_OK;
}

static hipEvent_t take_event(cbx_plan* P) {
    if (!P->ev_pool.empty()) { hipEvent_t e = P->ev_pool.back(); P->ev_pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

extern "C" int32_t cbx_abi_version(void) { return CBX_ABI_VERSION; }
extern "C" const char* cbx_last_error(void) { return g_err.c_str(); }

static bool is_string_out(int t) { return t == CBX_O_STRING || t == CBX_O_BINARY; }

template <typename T>
static int upload(T** dst, const T* src, size_t n) {
    size_t bytes = std::max<size_t>(1, n) * sizeof(T);
    HIP_CHECK(hipMalloc((void**)dst, bytes));
    if (n) HIP_CHECK(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return CBX_OK;
}

static bool is_generated(const Field& d) { return d.variant == V_RECORD_ID || d.variant == V_FILE_ID; }
// elements of list-layout arrays are decoded by the list kernel, not from the staged windows
static bool is_list(const Field& d) { return (d.flags & CBX_F_LIST) != 0; }

// One element (slot) of a field: static offset and its OCCURS DEPENDING ON conditions.
struct Elem {
    int field, slot, eo, size;
    bool str;
    int n_odo;
    int16_t odo_arr[CBX_MAX_DIMS], odo_idx[CBX_MAX_DIMS];
};

static std::vector<Elem> field_elements(const cbx_plan* P, int fi) {
    const Field& d = P->dfields_h[fi];
    std::vector<Elem> out;
    out.reserve(d.n_slots);
    for (int s = 0; s < d.n_slots; s++) {
        Elem e{};
        e.field = fi; e.slot = s; e.size = d.size; e.str = is_string_out(d.out_type);
        int eo = d.offset, rem = s;
        int idx[CBX_MAX_DIMS] = {0, 0, 0, 0};
        for (int k = d.n_dims - 1; k >= 0; k--) { idx[k] = rem % d.dim_count[k]; rem /= d.dim_count[k]; eo += idx[k] * d.dim_stride[k]; }
        e.eo = eo;
        for (int k = 0; k < d.n_dims; k++) {
            const cbx_array& ar = P->harrays[d.dim_array[k]];
            if (ar.dependee >= 0) { e.odo_arr[e.n_odo] = (int16_t)d.dim_array[k]; e.odo_idx[e.n_odo] = (int16_t)idx[k]; e.n_odo++; }
        }
        out.push_back(e);
    }
    return out;
}

static StrOp make_strop(const Field& d, const Elem& e) {
    StrOp o{};
    o.eo = e.eo; o.size = d.size; o.kind = (uint8_t)d.kind; o.trim = (uint8_t)d.trim; o.n_odo = (uint8_t)e.n_odo;
    o.pad = (uint8_t)d.max_utf8;
    o.column = d.column; o.slot = e.slot; o.seq = d.seq + e.slot; o.segment = d.segment;
    for (int j = 0; j < CBX_MAX_DIMS; j++) { o.odo_arr[j] = e.odo_arr[j]; o.odo_idx[j] = e.odo_idx[j]; }
    return o;
}

// Append one window holding `els` (any order) to set S.
static int out_width(int out_type) {
    return out_type == CBX_O_I32 || out_type == CBX_O_F32 ? 4 : out_type == CBX_O_DEC128 ? 16 : 8;
}

static void push_window(cbx_plan* P, cbx_plan::OpSet& S, std::vector<Elem> els, int lo, int hi, bool global,
                        const std::vector<int>& gen) {
    // numerics grouped by (variant, output width) so each batch runs a specialised loop;
    // inside a batch, field then slot order (ascending record offsets, output columns)
    auto key = [&](const Elem& e) {
        const Field& d = P->dfields_h[e.field];
        return (e.n_odo > 0 ? 1024 : 0) + (global ? 0 : d.variant * 32 + out_width(d.out_type));
    };
    std::stable_sort(els.begin(), els.end(), [&](const Elem& a, const Elem& b) {
        const int ka = key(a), kb = key(b);
        if (ka != kb) return ka < kb;
        return a.field != b.field ? a.field < b.field : a.slot < b.slot;
    });
    Window w{};
    w.lo = lo; w.hi = hi; w.global = global ? 1 : 0;
    w.nop_begin = (int)S.nops.size();
    w.sop_begin = (int)S.sops.size();
    std::vector<NumOp> wn;
    std::vector<int> wf;   // field of each numeric op
    for (const Elem& e : els) {
        const Field& d = P->dfields_h[e.field];
        if (e.str) S.sops.push_back(make_strop(d, e));
        else { wn.push_back(make_numop(d, e.slot, e.eo, e.odo_arr, e.odo_idx, e.n_odo)); wf.push_back(e.field); }
    }
    // OCCURS runs (staged windows): consecutive elements of a field along its innermost dimension
    // become one op -- the kernel walks the run with the element stride, so wide arrays cost one
    // op record per run instead of one per element
    for (size_t i = 0; i < wn.size();) {
        NumOp o = wn[i];
        const Field& d = P->dfields_h[wf[i]];
        size_t run = 1;
        if (!global && d.n_dims > 0) {
            const int stride = d.dim_stride[d.n_dims - 1];
            const bool inner_odo = o.n_odo > 0 && o.odo_arr[o.n_odo - 1] == d.dim_array[d.n_dims - 1];
            while (i + run < wn.size() && run < 255 && wf[i + run] == wf[i]) {
                const NumOp& n = wn[i + run];
                bool same = n.slot == o.slot + (int)run && n.eo == o.eo + (int)run * stride && n.n_odo == o.n_odo &&
                            n.defer == (o.defer >= 0 ? o.defer + (int)run : -1);
                for (int j = 0; same && j < o.n_odo; j++) {
                    const bool last = j == o.n_odo - 1 && inner_odo;
                    same = n.odo_arr[j] == o.odo_arr[j] && n.odo_idx[j] == o.odo_idx[j] + (last ? (int)run : 0);
                }
                if (!same) break;
                run++;
            }
            o.run_stride = stride;
            o.run_odo = inner_odo ? 1 : 0;
        }
        o.run = (uint8_t)run;
        S.nops.push_back(o);
        i += run;
    }
    w.nop_end = (int)S.nops.size();
    w.sop_end = (int)S.sops.size();
    w.batch_begin = (int)S.batches.size();
    for (int i = w.nop_begin; i < w.nop_end;) {
        const int v = global ? (int)V_GENERIC : S.nops[i].variant, wd = out_width(S.nops[i].out_type);
        const bool odo = S.nops[i].n_odo > 0;
        int j = i + 1;
        while (j < w.nop_end && (global || S.nops[j].variant == v) && out_width(S.nops[j].out_type) == wd &&
               (S.nops[j].n_odo > 0) == odo)
            j++;
        int runs = 0;
        for (int k = i; k < j; k++) runs |= S.nops[k].run > 1;
        S.batches.push_back(Batch{v, wd, i, j, odo ? 1 : 0, runs});
        S.has_runs |= runs != 0;
        i = j;
    }
    w.batch_end = (int)S.batches.size();
    w.gen_begin = (int)S.gops.size();
    for (int fi : gen) {
        const Field& d = P->dfields_h[fi];
        S.gops.push_back(GenOp{d.kind, d.column, d.out_type, 0});
    }
    w.gen_end = (int)S.gops.size();
    int nch = (hi - lo + 15 + 15) >> 4;
    w.pitch = global ? 0 : 16 * nch + 4;   // 4 * nch + 1 dwords: odd
    S.max_str_items = std::max(S.max_str_items, w.sop_end - w.sop_begin);
    if (global) P->max_pitch = P->max_pitch;  // global windows are never staged
    else if (&S == &P->wset) P->max_pitch = std::max(P->max_pitch, w.pitch);
    S.win.push_back(w);
}

// Contiguous set: one window holding every element + a global window with generated columns.
static void build_contig(cbx_plan* P) {
    std::vector<Elem> els;
    std::vector<int> gen;
    int items = 0;
    for (int i = 0; i < (int)P->dfields_h.size(); i++) {
        if (is_generated(P->dfields_h[i])) { gen.push_back(i); continue; }
        if (is_list(P->dfields_h[i])) continue;
        for (const Elem& e : field_elements(P, i)) { items += e.str; els.push_back(e); }
    }
    if (items > kMaxStrItems) P->contig_ok = false;
    if (!els.empty()) push_window(P, P->cset, els, 0, 0, false, {});
    if (!gen.empty()) push_window(P, P->cset, {}, 0, 0, true, gen);
}

// Windowed set: every element [eo, eo + size) sorted by offset, cut into byte ranges of at most
// wmax (and at most kMaxStrItems string elements); oversized fields and generated columns go
// to the global window.
static void build_windowed(cbx_plan* P, int wmax) {
    std::vector<Elem> els, big;
    std::vector<int> gen;
    for (int i = 0; i < (int)P->dfields_h.size(); i++) {
        const Field& d = P->dfields_h[i];
        if (is_generated(d)) { gen.push_back(i); continue; }
        if (is_list(d)) continue;
        std::vector<Elem> fe = field_elements(P, i);
        if (d.size > wmax) big.insert(big.end(), fe.begin(), fe.end());
        else els.insert(els.end(), fe.begin(), fe.end());
    }
    std::stable_sort(els.begin(), els.end(), [](const Elem& a, const Elem& b) { return a.eo < b.eo; });
    size_t e0 = 0;
    while (e0 < els.size()) {
        int lo = els[e0].eo, hi = els[e0].eo + els[e0].size;
        int items = els[e0].str ? 1 : 0;
        size_t e1 = e0 + 1;
        while (e1 < els.size() && std::max(hi, els[e1].eo + els[e1].size) - lo <= wmax && items + (els[e1].str ? 1 : 0) <= kMaxStrItems) {
            hi = std::max(hi, els[e1].eo + els[e1].size);
            items += els[e1].str ? 1 : 0;
            e1++;
        }
        push_window(P, P->wset, std::vector<Elem>(els.begin() + e0, els.begin() + e1), lo, hi, false, {});
        e0 = e1;
    }
    if (!big.empty() || !gen.empty()) push_window(P, P->wset, big, 0, 0, true, gen);
}

template <typename T>
static int upload_vec(T** dst, const std::vector<T>& v) { return upload(dst, v.data(), v.size()); }

static int upload_set(cbx_plan::OpSet& S) {
    int r;
    if ((r = upload_vec(&S.d_win, S.win)) || (r = upload_vec(&S.d_nops, S.nops)) || (r = upload_vec(&S.d_batches, S.batches)) ||
        (r = upload_vec(&S.d_sops, S.sops)) ||
        (r = upload_vec(&S.d_gops, S.gops)))
        return r;
    return CBX_OK;
}

static void free_set(cbx_plan::OpSet& S) {
    (void)hipFree(S.d_win); (void)hipFree(S.d_nops); (void)hipFree(S.d_batches); (void)hipFree(S.d_sops); (void)hipFree(S.d_gops);
}

extern "C" int cbx_plan_create(const cbx_field* fields, int32_t n_fields, const cbx_array* arrays,
                               int32_t n_arrays, const cbx_plan_options* opts, cbx_plan** out_plan) {
    if (!fields || n_fields <= 0 || !opts || !out_plan || n_arrays < 0 || (n_arrays > 0 && !arrays))
        return fail(CBX_E_ARGUMENT, "cbx_plan_create: invalid arguments");
    cbx_plan* P = new cbx_plan();
    P->opts = *opts;
    P->jit_min = opts->jit_min_records < 0 ? -1 : (opts->jit_min_records == 0 ? 262144 : opts->jit_min_records);
    if (const char* e = getenv("CBX_JIT"))
        if (e[0] == '0') P->jit_min = -1;   // operator switch: table-driven kernel only
    P->n_columns = opts->n_columns;
    if (opts->string_views < 0 || opts->string_views > 2)
        { delete P; return fail(CBX_E_ARGUMENT, "cbx_plan_create: string_views must be 0, 1 or 2"); }
    P->view = opts->string_views == 1;
    P->packed = opts->string_views == 2;
    if (P->n_columns <= 0) { delete P; return fail(CBX_E_ARGUMENT, "cbx_plan_create: n_columns must be positive"); }
    P->hfields.assign(fields, fields + n_fields);
    if (n_arrays) P->harrays.assign(arrays, arrays + n_arrays);
    P->col_is_string.assign(P->n_columns, 0);
    P->col_slots.assign(P->n_columns, 1);
    P->col_max_bytes.assign(P->n_columns, 0);

    // widest UTF-8 expansion of the code page
    int lut_max = 1;
    for (int i = 0; i < 256; i++) lut_max = std::max(lut_max, (int)((opts->lut[i] >> 24) & 3));

    // ---- fields
    for (int i = 0; i < n_fields; i++) {
        const cbx_field& f = fields[i];
        const std::string fi = "field " + std::to_string(i);
        if (f.n_dims < 0 || f.n_dims > CBX_MAX_DIMS) { delete P; return fail(CBX_E_ARGUMENT, fi + ": bad n_dims"); }
        for (int k = 0; k < f.n_dims; k++)
            if (f.dim_count[k] <= 0 || f.dim_array[k] < 0 || f.dim_array[k] >= n_arrays) {
                delete P; return fail(CBX_E_ARGUMENT, fi + ": bad dimension");
            }
        Field d = make_field(f);
        if (f.column < 0 || f.column >= P->n_columns) { delete P; return fail(CBX_E_ARGUMENT, fi + ": bad column"); }
        if (!is_generated(d) && (f.size <= 0 || f.offset < 0)) { delete P; return fail(CBX_E_ARGUMENT, fi + ": bad offset/size"); }
        if (!(f.kind >= CBX_K_STRING && f.kind <= CBX_K_UTF16_LE)) { delete P; return fail(CBX_E_ARGUMENT, fi + ": unknown kind"); }
        if (f.kind == CBX_K_BINARY && f.size > 16) { delete P; return fail(CBX_E_UNSUPPORTED, fi + ": binary wider than 16 bytes"); }
        if (f.kind == CBX_K_ASCII_NUM && (f.size > kAsciiNumMax || f.scale < 0 || f.scale > 100 || f.scale_factor < -100 ||
                                          f.scale_factor > 100)) {
            delete P; return fail(CBX_E_UNSUPPORTED, fi + ": ASCII DISPLAY number wider than 64 bytes");
        }
        if ((f.out_type == CBX_O_DEC64 || f.out_type == CBX_O_DEC128) && (f.out_precision < 1 || f.out_precision > 38)) {
            delete P; return fail(CBX_E_UNSUPPORTED, fi + ": decimal precision outside 1..38");
        }
        if (d.variant == V_STRING) {
            if (f.kind == CBX_K_STRING) d.max_utf8 = lut_max;
            d.seq = P->n_seq;
            P->n_seq += d.n_slots;
            for (int sl = 0; sl < d.n_slots; sl++) {
                P->seq_field.push_back(i);
                P->seq_slot.push_back(sl);
                P->seq_tile_cap.push_back(((int64_t)kWave * f.size * d.max_utf8 + 15) & ~(int64_t)15);
            }
            P->col_max_bytes[f.column] = f.size * d.max_utf8;
        } else if ((d.variant == V_ZONED16 || d.variant == V_GENERIC) && !(f.flags & CBX_F_LIST)) {
            d.defer = (int)P->hdefer.size();
            for (int s = 0; s < d.n_slots; s++) P->hdefer.push_back(DeferSeq{i, s});
        }
        P->dfields_h.push_back(d);
        P->col_is_string[f.column] = is_string_out(f.out_type);
        P->col_slots[f.column] = d.n_slots;
    }
    for (int ai = 0; ai < n_arrays; ai++) {
        const cbx_array& ar = arrays[ai];
        if (ar.dependee >= n_fields || ar.max_count <= 0) { delete P; return fail(CBX_E_ARGUMENT, "array " + std::to_string(ai) + ": bad descriptor"); }
        if (ar.offsets_column >= P->n_columns || (ar.offsets_column >= 0 && (ar.dependee < 0 || ar.n_dims != 0)))
            { delete P; return fail(CBX_E_ARGUMENT, "array " + std::to_string(ai) + ": list layout needs a top-level OCCURS DEPENDING ON"); }
        if (ar.dependee >= 0) {
            const cbx_field& df = fields[ar.dependee];
            if (!(df.flags & CBX_F_INTEGRAL) || df.n_dims != 0 || df.precision > 18)
                { delete P; return fail(CBX_E_UNSUPPORTED, "array " + std::to_string(ai) + ": DEPENDING ON source must be a non-array integral field"); }
        }
    }
    for (int ai = 0; ai < n_arrays; ai++)   // list-layout elements: numeric, one level, the array's segment
        for (int i = 0; i < n_fields; i++) {
            const cbx_field& f = fields[i];
            if (!(f.flags & CBX_F_LIST) || (f.n_dims == 1 && f.dim_array[0] != ai)) continue;
            if (f.n_dims != 1 || arrays[ai].offsets_column < 0 || is_string_out(f.out_type) || f.segment != arrays[ai].segment)
                { delete P; return fail(CBX_E_ARGUMENT, "field " + std::to_string(i) + ": CBX_F_LIST needs a numeric element of a list-layout array in its segment"); }
            ListOp lo{};
            const int16_t none[CBX_MAX_DIMS] = {0, 0, 0, 0};
            lo.op = make_numop(P->dfields_h[i], 0, f.offset, none, none, 0);
            lo.field = i;
            lo.array = ai;
            lo.stride = f.dim_stride[0];
            P->lops.push_back(lo);
        }
    for (ListOp& lo : P->lops) {   // elements are staged from the array's first field byte
        lo.elem_lo = lo.op.eo;
        for (const ListOp& o : P->lops)
            if (o.array == lo.array) lo.elem_lo = std::min(lo.elem_lo, o.op.eo);
    }
    if ((int)P->lops.size() != (int)std::count_if(fields, fields + n_fields, [](const cbx_field& f) { return (f.flags & CBX_F_LIST) != 0; }))
        { delete P; return fail(CBX_E_ARGUMENT, "CBX_F_LIST field outside a list-layout array"); }
    P->seg_col = opts->segment_column;
    if (P->seg_col >= P->n_columns) { delete P; return fail(CBX_E_ARGUMENT, "bad segment column"); }

    // ---- window sets + op tables
    int wmax = opts->window_bytes > 0 ? opts->window_bytes : 256;
    if (wmax > kMaxWindowBytes) wmax = kMaxWindowBytes;
    build_contig(P);
    build_windowed(P, wmax);
    // string staging per wave: the byte-loop / large-string paths stage a tile's payload (kWave *
    // size * max_utf8, capped); the register path of the view and Utf8 layouts (str_view_fast,
    // str_utf8_fast) composes multi-byte code pages in lane slots and single-byte ones in registers
    // (no LDS at all), and stores the values from registers
    int slots = 0;
    if (P->view || P->packed) P->str_stage = 0;
    for (const Field& d : P->dfields_h) {
        if (d.variant != V_STRING) continue;
        const bool fast = d.size <= kStrFastBytes && (d.kind == CBX_K_STRING || d.kind == CBX_K_STRING_ASCII);
        if ((P->view || P->packed) && fast) {
            // (env CBX_STR_NO_SHIFT: single-byte pages through the slots too -- A/B runs; the
            // specialised kernel then compiles the slot path for them, cbx_jit.h)
            if (d.max_utf8 > 1 || getenv("CBX_STR_NO_SHIFT")) slots = std::max(slots, kWave * str_lane_slot(d.size, d.max_utf8));
        } else {
            P->str_stage = std::max(P->str_stage, kWave * d.size * d.max_utf8);
            P->view_staged |= P->view;
        }
    }
    P->str_stage = std::min(P->str_stage, kStrStageBytes);
    for (const cbx_field& f : P->hfields) {
        if (f.flags & CBX_F_LIST) continue;   // the list kernel reads those
        int64_t e = (int64_t)f.offset + f.size;
        for (int k = 0; k < f.n_dims; k++) e += (int64_t)(f.dim_count[k] - 1) * f.dim_stride[k];
        if (f.kind != CBX_K_RECORD_ID && f.kind != CBX_K_FILE_ID)
            P->rec_extent = std::max(P->rec_extent, (int)std::min<int64_t>(e, 1 << 30));
    }
    P->str_stage = std::max(P->str_stage, slots);

    // ---- segment map: keys to UTF-8, Seg_IdN string columns
    cbx_segment_map sm = opts->segments;
    if (opts->has_segments) {
        if (sm.n_keys < 0 || sm.n_keys > CBX_MAX_SEG_KEYS || sm.n_levels < 0 || sm.n_levels > CBX_MAX_SEG_LEVELS ||
            sm.prefix_len < 0 || sm.prefix_len > CBX_MAX_SEG_PREFIX || (sm.field_is_int && (sm.field < 0 || sm.field >= n_fields))) {
            delete P; return fail(CBX_E_ARGUMENT, "cbx_plan_create: bad segment map");
        }
        if (sm.field_is_int && !(fields[sm.field].flags & CBX_F_INTEGRAL)) {
            delete P; return fail(CBX_E_UNSUPPORTED, "segment field must be a string or an integral field");
        }
        for (int l = 0; l < sm.n_levels; l++) {
            const int c = sm.level_column[l];
            if (c < 0) continue;
            if (c >= P->n_columns) { delete P; return fail(CBX_E_ARGUMENT, "cbx_plan_create: bad Seg_Id column"); }
            P->col_is_string[c] = 1;
            P->col_slots[c] = 1;
            P->col_max_bytes[c] = sm.prefix_len + 64;   // prefix _ fileId _ rootId _L<l> _ counter
            P->segid_cols.push_back(l);
        }
        for (int k = 0; k < sm.n_keys; k++) {
            std::string u8;
            for (int j = 0; j < opts->segments.key_len[k]; j++) {
                uint32_t c = opts->segments.key[k][j];
                if (c < 0x80) u8 += (char)c;
                else if (c < 0x800) { u8 += (char)(0xC0 | (c >> 6)); u8 += (char)(0x80 | (c & 63)); }
                else { u8 += (char)(0xE0 | (c >> 12)); u8 += (char)(0x80 | ((c >> 6) & 63)); u8 += (char)(0x80 | (c & 63)); }
            }
            if ((int)u8.size() > CBX_MAX_SEG_KEY_LEN) { delete P; return fail(CBX_E_UNSUPPORTED, "segment key too long"); }
            for (size_t j = 0; j < u8.size(); j++) sm.key[k][j] = (uint8_t)u8[j];
            sm.key_len[k] = (int)u8.size();
        }
    }

    int r;
    if ((r = upload(&P->d_fields, P->dfields_h.data(), P->dfields_h.size())) ||
        (r = upload_set(P->cset)) || (r = upload_set(P->wset)) ||
        (r = upload(&P->d_arrays, P->harrays.data(), P->harrays.size())) ||
        (r = upload(&P->d_defer, P->hdefer.data(), P->hdefer.size())) ||
        (r = upload(&P->d_lops, P->lops.data(), P->lops.size())) ||
        (r = upload(&P->d_lut, opts->lut, 256))) {
        cbx_plan_destroy(P);
        return r;
    }
    if (opts->has_segments && (r = upload(&P->d_segmap, &sm, 1))) { cbx_plan_destroy(P); return r; }
    if (hipMalloc((void**)&P->d_cols, sizeof(DevColumn) * P->n_columns) != hipSuccess ||
        hipMalloc((void**)&P->d_seqcall, sizeof(SeqCall) * std::max(1, P->n_seq)) != hipSuccess ||
        hipMalloc((void**)&P->d_status, 64) != hipSuccess ||
        hipMemset(P->d_status, 0, 64) != hipSuccess) {
        cbx_plan_destroy(P);
        return fail(CBX_E_HIP, "cbx_plan_create: device allocation failed");
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) P->num_cus = prop.multiProcessorCount;
    *out_plan = P;
    return CBX_OK;
}

extern "C" void cbx_plan_destroy(cbx_plan* P) {
    if (!P) return;
    (void)hipFree(P->d_fields); (void)hipFree(P->d_defer); (void)hipFree(P->d_defer_bits);
    free_set(P->cset); free_set(P->wset); (void)hipFree(P->d_arrays);
    (void)hipFree(P->d_ncall); (void)hipFree(P->d_scall);
    (void)hipFree(P->d_segmap); (void)hipFree(P->d_lut); (void)hipFree(P->d_cols);
    (void)hipFree(P->d_seqcall); (void)hipFree(P->d_str_tot); (void)hipFree(P->d_str_excl); (void)hipFree(P->d_block_sums);
    (void)hipFree(P->d_local); (void)hipFree(P->d_scratch); (void)hipFree(P->d_status); (void)hipFree(P->d_stamps);
    (void)hipFree(P->d_lops); (void)hipFree(P->d_list_len); (void)hipFree(P->d_list_flag);
    (void)hipFree(P->d_wnodes); (void)hipFree(P->d_warr); (void)hipFree(P->d_whand); (void)hipFree(P->d_wslot_base);
    (void)hipFree(P->d_wtile_bytes); (void)hipFree(P->d_wcursor);
    (void)hipFree(P->d_wvbase); (void)hipFree(P->d_wvcol); (void)hipFree(P->d_wvslot);
    for (auto& e : P->ev_pool) (void)hipEventDestroy(e);
    for (auto& c : P->ev_calls) for (auto& e : c.e) if (e) (void)hipEventDestroy(e);
    if (P->pipe_peer) P->pipe_peer->pipe_peer = nullptr;
    if (P->pipe_done) (void)hipEventDestroy(P->pipe_done);
    delete P;
}

// String-view layout: bytes of a slot region owned by one tile (the tile's payload bound, 16-aligned)
// and tiles per Arrow data buffer (buffers of at most 1 GiB, a whole number of tiles each).
// a tile's region: 64 payloads of the column's widest value, each at a 4-byte-aligned position
// KernelArgs.str_view / CBX_STR_LAYOUT: 0 Arrow large-string, 1 string views, 2 Arrow Utf8
static int str_layout_of(const cbx_plan* P) { return P->view ? 1 : P->packed ? 2 : 0; }
static int64_t view_tile_bytes(const cbx_plan* P, int c) { return ((int64_t)kWave * ((P->col_max_bytes[c] + 3) & ~3) + 15) & ~(int64_t)15; }
// whole tiles per data buffer: the largest power of two fitting 1 GiB (the kernels split a tile
// index into buffer and position by a shift)
// (CBX_VIEW_BUFFER_BYTES lowers the 1 GiB cap: tests of multi-buffer regions on small inputs;
// reader.view_geometry reads the same variable)
static int64_t view_buffer_cap() {
    const char* e = getenv("CBX_VIEW_BUFFER_BYTES");
    const int64_t v = e ? atoll(e) : 0;
    return v >= 16 && v < (int64_t(1) << 30) ? v : (int64_t(1) << 30);
}
static int64_t view_tiles_per_buf(int64_t tile_bytes) {
    const int64_t n = std::max<int64_t>(1, view_buffer_cap() / std::max<int64_t>(16, tile_bytes));
    return int64_t(1) << (63 - __builtin_clzll((unsigned long long)n));
}

extern "C" int cbx_string_bound(const cbx_plan* P, int64_t n_rec, int64_t* out_bytes) {
    if (!P || n_rec < 0 || !out_bytes) return fail(CBX_E_ARGUMENT, "cbx_string_bound: invalid arguments");
    const int64_t n_tiles = (n_rec + kWave - 1) / kWave;
    for (int c = 0; c < P->n_columns; c++)
        out_bytes[c] = !P->col_is_string[c] ? 0 : P->view ? n_tiles * view_tile_bytes(P, c) : n_rec * (int64_t)P->col_max_bytes[c];
    return CBX_OK;
}

extern "C" int cbx_string_view_geometry(const cbx_plan* P, int64_t* tile_bytes, int64_t* buffer_bytes) {
    if (!P || !tile_bytes || !buffer_bytes) return fail(CBX_E_ARGUMENT, "cbx_string_view_geometry: invalid arguments");
    for (int c = 0; c < P->n_columns; c++) {
        const int64_t tb = P->col_is_string[c] ? view_tile_bytes(P, c) : 0;
        tile_bytes[c] = tb;
        buffer_bytes[c] = tb ? view_tiles_per_buf(tb) * tb : 0;
    }
    return CBX_OK;
}

// Exclusive scan (int64) of the per-(sequence, tile) payload totals, sequences concatenated.
static int string_scan(cbx_plan* P, int64_t n_tiles, hipStream_t st) {
    const int64_t n = (int64_t)P->n_seq * n_tiles;
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    int r;
    if ((r = grow(&P->d_str_excl, &P->str_excl_cap, n, st)) || (r = grow(&P->d_block_sums, &P->block_sums_cap, nb, st)))
        return r;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, (const uint32_t*)P->d_str_tot, n,
                       P->d_block_sums);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, P->d_block_sums, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, (const uint32_t*)P->d_str_tot, n,
                       (const int64_t*)P->d_block_sums, P->d_str_excl);
    HIP_CHECK(hipGetLastError());
    return CBX_OK;
}

struct CallShape {
    const uint8_t* data; int64_t data_len; const int64_t* rec_off; const int32_t* rec_len;
    int64_t n_rec; int32_t stride; int32_t start_off; int64_t first_record_id;
    const int64_t* rec_id = nullptr;    // selected records: per-record Record_Id
    const int32_t* rec_seg = nullptr;   // selected records: per-record active segment
    int32_t file_id = -1;               // File_Id of the batch (-1: the plan's)
};

// Prologue parts the plan needs (contig_loop's kPro): segment map 1, OCCURS DEPENDING ON arrays 2.
static int jit_pro(const cbx_plan* P) { return (P->opts.has_segments ? 1 : 0) | (P->harrays.empty() ? 0 : 2); }

static int launch(cbx_plan* P, const CallShape& c, const cbx_column* columns, int mode, hipStream_t st) {
    const int64_t n_tiles = (c.n_rec + kWave - 1) / kWave;
    KernelArgs a{};
    uintptr_t addr = (uintptr_t)c.data;
    a.base_shift = (int64_t)(addr & 15);
    a.data = (const uint8_t*)(addr & ~(uintptr_t)15);
    a.data_len = c.data_len + a.base_shift;
    a.rec_off = c.rec_off;
    a.rec_len = c.rec_len;
    a.n_rec = c.n_rec;
    a.n_tiles = n_tiles;
    a.pitch = n_tiles * kWave;
    a.stride = c.stride;
    a.start_off = c.start_off;
    a.first_record_id = c.first_record_id;
    a.rec_id_base = P->d_rec_base;
    a.rec_id = c.rec_id;
    a.rec_seg = c.rec_seg;
    a.odo_count = P->d_odo;
    a.odo_pitch = P->odo_pitch;
    a.file_id = c.file_id >= 0 ? c.file_id : P->opts.file_id;
    a.mode = mode;
    a.str_view = str_layout_of(P);
    // staging mode
    const int sdw = c.stride / 4;
    const bool contig = !c.rec_off && P->contig_ok && c.stride > 0 && c.stride % 4 == 0 && a.base_shift % 4 == 0 &&
                        contig_kp(sdw) <= kPre;
    a.contig = contig ? 1 : 0;
    // variable-length records through the specialised span kernel (span_loop): decode calls over
    // framed records (not a selection, whose per-record ids / segments stay on the windowed
    // kernel), a layout whose single window spans at most 1/64 of the span staging
    const int span_ext = c.start_off + P->rec_extent;
    const int span_kp = (int)std::min<int64_t>(kPre, ((int64_t)kWave * (span_ext + 8) + 32 + 1023) / 1024);
    hipFunction_t span_fn = nullptr;
    if (c.rec_off && !c.rec_id && !c.rec_seg && P->contig_ok && mode == 0 && P->jit_min >= 0 && c.n_rec >= P->jit_min &&
        (int64_t)kWave * span_ext <= 16 * 1024 && !getenv("CBX_NO_SPAN")) {
        const int k = kPre + 1 + span_kp;
        if (!P->jit_tried[k]) {
            P->jit_tried[k] = true;
            P->jit_fn[k] = jit_get(jit_source(true, span_kp, jit_pro(P), str_layout_of(P), P->cset.win, P->cset.nops, P->cset.batches,
                                              P->cset.sops, true), &P->jit_error);
        }
        span_fn = P->jit_fn[k];
    }
    const bool span = span_fn != nullptr;
    const cbx_plan::OpSet& S = (contig || span) ? P->cset : P->wset;
    if (span) {
        a.span_ext = span_ext;
        const int nch = (P->rec_extent + 15 + 15) >> 4;
        a.span_pitch = 16 * nch + 4;   // as a staged window's rows (push_window)
        a.lds_rows = kGuard + std::max(span_kp * 1024 + 64, kWave * a.span_pitch) + kGuard;
    } else if (contig) {
        a.stride_dw = sdw;
        // pad rows to an odd dword count only when the plain stride would give >= 4-way bank
        // conflicts on the per-lane dword reads (gcd(stride_dw, 32) >= 4); 2-way is cheaper
        // than the dword scatter padding costs
        const int g = std::__gcd(sdw, 32);
        a.cpitch = 4 * ((g >= 4 || (g == 2 && getenv("CBX_PAD_ROWS"))) ? ((sdw & 1) ? sdw : sdw + 1) : sdw);   // env: A/B
        a.inv_stride_dw = 1.0f / (float)sdw;
        a.lds_rows = kGuard + kWave * a.cpitch + 16 + kGuard;
    } else {
        a.lds_rows = kGuard + kWave * std::max(P->max_pitch, 16) + kGuard;
    }
    a.windows = (const CBX_CONST Window*)S.d_win;
    a.n_windows = (int)S.win.size();
    a.nops = (const CBX_CONST NumOp*)S.d_nops;
    a.batches = (const CBX_CONST Batch*)S.d_batches;
    a.sops = (const CBX_CONST StrOp*)S.d_sops;
    a.gops = (const CBX_CONST GenOp*)S.d_gops;
    a.lds_rows = (a.lds_rows + 15) & ~15;
    a.lds_counts = ((int)P->harrays.size() * kWave * 4 + 15) & ~15;   // OCCURS element counts
    // string-view layout: the inline slots (16 bytes per short value) share the area with the long
    // payloads, which it holds for any tile as long as it is at least 16 bytes per lane
    a.str_stage = S.max_str_items > 0 ? (P->view && mode == 0 && P->view_staged ? std::max(P->str_stage, 16 * kWave) : P->str_stage) : 0;
    // per-lane dump slots for the branch-free string stores (a shared slot serialises the wave's
    // LDS stores) -- unless the extra 4 * kWave bytes per wave cost a resident workgroup per CU
    // (wide windowed layouts sit close to the LDS limit; C5 decode 49.7 -> 62.1 ms with them)
    const int lds_base = a.lds_rows + a.lds_counts + a.str_stage;
    auto lds_blocks = [](int per_wave) {
        return (160 * 1024) / (kLutLds + kWavesPerBlock * ((per_wave + 15) & ~15));
    };
    const bool lane_dump = a.str_stage > 0 && lds_blocks(lds_base + 4 * kWave) >= lds_blocks(lds_base + 16);
    a.dump_stride = lane_dump ? 4 : 0;
    a.lds_wave = (lds_base + (lane_dump ? 4 * kWave : 16) + 15) & ~15;
    a.fields = (const CBX_CONST Field*)P->d_fields;
    a.arrays = (const CBX_CONST cbx_array*)P->d_arrays;
    a.n_arrays = (int)P->harrays.size();
    a.seg_col = P->seg_col;
    a.segmap = P->opts.has_segments ? (const CBX_CONST cbx_segment_map*)P->d_segmap : nullptr;
    a.lut = P->d_lut;
    a.cols = (const CBX_CONST DevColumn*)P->d_cols;
    a.n_seq = P->n_seq;
    a.status = P->d_status;
#ifdef CBX_STAMPS
    if (!P->d_stamps) {
        HIP_CHECK(hipMalloc((void**)&P->d_stamps, 8 * sizeof(uint64_t)));
        HIP_CHECK(hipMemset(P->d_stamps, 0, 8 * sizeof(uint64_t)));
    }
    a.stamps = P->d_stamps;
#endif
    if (n_tiles == 0) return CBX_OK;

    // column table + per-op address tables: stream-ordered uploads from pageable host memory
    // (staged by the runtime, so the host vectors are free again when the call returns)
    const int n_defer_seq = (int)P->hdefer.size();
    if (mode == 0 && P->n_seq > 0 && P->packed) {   // the count pass's scan target, before the call tables point at it
        const int64_t n = (int64_t)P->n_seq * n_tiles;
        int rr;
        if ((rr = grow(&P->d_str_excl, &P->str_excl_cap, n, st)) ||
            (rr = grow(&P->d_block_sums, &P->block_sums_cap, (n + kScanTile - 1) / kScanTile, st)))
            return rr;
    }
    if (mode == 0 && P->n_seq > 0 && !P->view && !P->packed) {
        int rr;
        P->h_seq_scratch.resize(P->n_seq);
        int64_t scratch = 0;
        for (int q = 0; q < P->n_seq; q++) { P->h_seq_scratch[q] = scratch; scratch += n_tiles * P->seq_tile_cap[q]; }
        if ((rr = grow(&P->d_local, &P->local_cap, (int64_t)P->n_seq * a.pitch, st)) ||
            (rr = grow(&P->d_scratch, &P->scratch_cap, scratch + 64, st)))   // +64: placement reads up to 20 bytes past a payload end
            return rr;
    }
    if (mode == 0) {
        P->h_cols.resize(P->n_columns);
        for (int i = 0; i < P->n_columns; i++) {
            DevColumn d{};
            d.values = columns[i].values;
            d.validity = columns[i].validity;
            d.offsets = columns[i].offsets;
            d.data = columns[i].data;
            d.capacity = columns[i].data_capacity;
            d.sizes = columns[i].data_sizes;
            P->h_cols[i] = d;
        }
        HIP_CHECK(hipMemcpyAsync(P->d_cols, P->h_cols.data(), sizeof(DevColumn) * P->n_columns, hipMemcpyHostToDevice, st));
        if (n_defer_seq > 0) {
            const int64_t need = n_tiles * (int64_t)n_defer_seq;
            if (need > P->defer_bits_cap) {
                HIP_CHECK(hipStreamSynchronize(st));
                (void)hipFree(P->d_defer_bits);
                P->d_defer_bits = nullptr;
                HIP_CHECK(hipMalloc((void**)&P->d_defer_bits, sizeof(uint64_t) * need));
                P->defer_bits_cap = need;
            }
        }
        P->h_ncall.resize(S.nops.size());
        for (size_t i = 0; i < S.nops.size(); i++) {
            const NumOp& op = S.nops[i];
            const cbx_column& col = columns[op.column];
            NumCall nc{};
            nc.values = (uint8_t*)col.values + (int64_t)op.slot * a.pitch * out_width(op.out_type);
            nc.validity = col.validity + (int64_t)op.slot * n_tiles;
            nc.defer = op.defer >= 0 ? P->d_defer_bits + (int64_t)op.defer * n_tiles : nullptr;
            P->h_ncall[i] = nc;
        }
        P->h_scall.resize(S.sops.size());
        for (size_t i = 0; i < S.sops.size(); i++) {
            const StrOp& op = S.sops[i];
            const cbx_column& col = columns[op.column];
            StrCall sc{};
            sc.validity = col.validity + (int64_t)op.slot * n_tiles;
            if (P->view) {   // the caller's buffers: views + the slot's region, tile_bytes per tile
                sc.tile_cap = view_tile_bytes(P, op.column);
                sc.scratch = col.data + (int64_t)op.slot * col.data_capacity;
                sc.views = (uint8_t*)col.values + (int64_t)op.slot * a.pitch * 16;
                sc.tiles_per_buf = view_tiles_per_buf(sc.tile_cap);
            } else if (P->packed) {   // Arrow Utf8: int32 offsets (pitch + 1 per slot) + the slot's region
                sc.local = (uint32_t*)((int32_t*)col.offsets + (int64_t)op.slot * (a.pitch + 1));
                sc.scratch = col.data + (int64_t)op.slot * col.data_capacity;
                sc.tile_cap = col.data_capacity;
                sc.excl = P->d_str_excl + (int64_t)op.seq * n_tiles;
                sc.size = col.data_sizes ? col.data_sizes + op.slot : nullptr;
            } else {
                sc.local = P->d_local + (int64_t)op.seq * a.pitch;
                sc.scratch = P->d_scratch + P->h_seq_scratch[op.seq];
                sc.tile_cap = P->seq_tile_cap[op.seq];
            }
            P->h_scall[i] = sc;
        }
        P->h_seqcall.resize(P->view || P->packed ? 0 : P->n_seq);   // placement pass only in the large-string layout
        for (int q = 0; q < (int)P->h_seqcall.size(); q++) {
            const Field& d = P->dfields_h[P->seq_field[q]];
            const cbx_column& col = columns[d.column];
            const int sl = P->seq_slot[q];
            SeqCall sq{};
            sq.offsets = col.offsets + (int64_t)sl * (a.pitch + 1);
            sq.region = (int64_t)sl * col.data_capacity;
            sq.data = col.data + sq.region;
            sq.local = P->d_local + (int64_t)q * a.pitch;
            sq.scratch = P->d_scratch + P->h_seq_scratch[q];
            sq.size = col.data_sizes ? col.data_sizes + sl : nullptr;
            sq.capacity = col.data_capacity;
            sq.tile_cap = (int32_t)P->seq_tile_cap[q];
            P->h_seqcall[q] = sq;
        }
        if (P->n_seq > 0 && !P->view && !P->packed)
            HIP_CHECK(hipMemcpyAsync(P->d_seqcall, P->h_seqcall.data(), sizeof(SeqCall) * P->n_seq, hipMemcpyHostToDevice, st));
        if (P->h_ncall.size() > P->ncall_cap) {
            HIP_CHECK(hipStreamSynchronize(st));
            (void)hipFree(P->d_ncall);
            P->d_ncall = nullptr;
            HIP_CHECK(hipMalloc((void**)&P->d_ncall, sizeof(NumCall) * P->h_ncall.size()));
            P->ncall_cap = P->h_ncall.size();
        }
        if (P->h_scall.size() > P->scall_cap) {
            HIP_CHECK(hipStreamSynchronize(st));
            (void)hipFree(P->d_scall);
            P->d_scall = nullptr;
            HIP_CHECK(hipMalloc((void**)&P->d_scall, sizeof(StrCall) * P->h_scall.size()));
            P->scall_cap = P->h_scall.size();
        }
        if (!P->h_ncall.empty())
            HIP_CHECK(hipMemcpyAsync(P->d_ncall, P->h_ncall.data(), sizeof(NumCall) * P->h_ncall.size(), hipMemcpyHostToDevice, st));
        if (!P->h_scall.empty())
            HIP_CHECK(hipMemcpyAsync(P->d_scall, P->h_scall.data(), sizeof(StrCall) * P->h_scall.size(), hipMemcpyHostToDevice, st));
    }
    a.ncall = (const CBX_CONST NumCall*)P->d_ncall;
    a.scall = (const CBX_CONST StrCall*)P->d_scall;
    // string workspace: per (sequence, tile) totals (written by the decode kernel for every tile)
    int r;
    if (P->n_seq > 0 && (r = grow(&P->d_str_tot, &P->str_tot_cap, (int64_t)P->n_seq * n_tiles, st))) return r;
    a.str_tot = P->d_str_tot;
    const bool lists = mode == 0 && !P->lops.empty();
    if (lists && ((r = grow(&P->d_list_len, &P->list_len_cap, (int64_t)P->harrays.size() * a.pitch, st)) ||
                  (r = grow(&P->d_list_flag, &P->list_flag_cap, n_tiles, st))))
        return r;
    a.list_len = P->d_list_len;
    a.list_flag = P->d_list_flag;
    const int n_defer = n_defer_seq;
    a.defer_bits = P->d_defer_bits;
    const size_t lds_own = kLutLds + (size_t)kWavesPerBlock * a.lds_wave;
    if (lds_own > 160 * 1024) return fail(CBX_E_UNSUPPORTED, "record window does not fit in LDS");
    // resident blocks per CU: the LDS bound and the runtime's occupancy (registers)
    // copybook-specialised kernel for large contiguous batches (cbx_jit.h)
    hipFunction_t jfn = span_fn;
    int jk = -1;   // jit_fn slot of jfn (-1: the span kernel or none -- never cooperative)
    if (!span && mode == 0 && P->jit_min >= 0 && c.n_rec >= P->jit_min) {
        const int k = contig ? contig_kp(sdw) : 0;
        if (!P->jit_tried[k]) {
            P->jit_tried[k] = true;
            // the specialised kernel is straight-line code per op: wide layouts (thousands of
            // OCCURS slots) would take minutes in hipRTC and blow the instruction cache -- they
            // stay on the table-driven kernel, whose op loop is the same arithmetic
            size_t elems = S.sops.size();
            for (const NumOp& o : S.nops) elems += o.run > 1 ? o.run : 1;
            if (elems > (size_t)kJitMaxOps || S.win.size() > (size_t)kJitMaxWindows)
                P->jit_error = "layout has " + std::to_string(elems) + " elements in " + std::to_string(S.win.size()) +
                               " windows, above the specialised-kernel limits (" + std::to_string(kJitMaxOps) + ", " +
                               std::to_string(kJitMaxWindows) + ")";
            else {
                CoopSplit cs;
                P->jit_coop[k] = jit_coop_of(contig, span, jit_pro(P), str_layout_of(P), S.win, S.nops, S.batches, S.sops, false, &cs);
                P->jit_fn[k] = jit_get(jit_source(contig, k, jit_pro(P), str_layout_of(P), S.win, S.nops, S.batches, S.sops, false), &P->jit_error);
            }
        }
        jfn = P->jit_fn[k];
        jk = k;
    }
    P->last_kind = jfn ? 1 : 0;
    // cooperative tiles (cbx_jit.h jit_coop, cbx_device.h coop_loop): one image per workgroup,
    // one tile per workgroup
    const bool coop = jfn && jk >= 0 && P->jit_coop[jk];
    const size_t lds = coop ? kLutLds + (size_t)a.lds_rows + (size_t)kWavesPerBlock * (a.lds_wave - a.lds_rows) : lds_own;
    if (lds > 160 * 1024) return fail(CBX_E_UNSUPPORTED, "record window does not fit in LDS");
    int blocks_per_cu = (int)std::max<size_t>(1, std::min<size_t>(16, (160 * 1024) / lds));
    int occ = 0;
    const hipError_t oe = jfn ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&occ, jfn, kWave * kWavesPerBlock, lds)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, decode_kernel, kWave * kWavesPerBlock, lds);
    if (oe == hipSuccess && occ > 0) blocks_per_cu = std::min(blocks_per_cu, occ);
    // string-dominated contiguous layouts run best at 4 workgroups (8 waves) per CU: SYNSTR200 (10 x
    // X(20)) decodes in 8.7 ms at 4, 13.4 ms at 5 and 11.6 ms at 3, while SYN200 (1 string, 27
    // numerics) and the windowed C4/C5 layouts gain from every extra resident workgroup
    if (!coop && contig && S.sops.size() >= S.nops.size() && S.sops.size() > 0) blocks_per_cu = std::min(blocks_per_cu, 4);
    if (const char* e = getenv("CBX_MAX_BLOCKS_PER_CU")) blocks_per_cu = std::max(1, std::min(blocks_per_cu, atoi(e)));   // tuning
    const bool piped = P->pipe_peer && mode == 0 && P->packed && P->n_seq > 0;
    if (piped && P->pipe_decode_bpc > 0) blocks_per_cu = std::min(blocks_per_cu, P->pipe_decode_bpc);
    const int64_t blocks_needed = coop ? n_tiles : (n_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t grid = std::min<int64_t>(blocks_needed, (int64_t)P->num_cus * blocks_per_cu);
    const bool prof = P->profiling && mode == 0;
    cbx_plan::CallEvents ce{{nullptr, nullptr, nullptr}};
    // pipelined with a peer plan: this call's count pass follows the peer's last one (so it runs beside
    // the peer's decode), before the timing starts
    if (piped && P->pipe_peer->pipe_done) HIP_CHECK(hipStreamWaitEvent(st, P->pipe_peer->pipe_done, 0));
    if (prof) {
        for (auto& e : ce.e) if (!(e = take_event(P))) return fail(CBX_E_HIP, "hipEventCreate failed");
        HIP_CHECK(hipEventRecord(ce.e[0], st));
    }
    // Arrow Utf8 layout: the count pass (tile payload totals) and their scan, so the decode writes
    // every offset and payload byte once, at its final place (timed with the decode).  Contiguous and
    // span-staged batches count with a specialised kernel of the same staging; windowed ones (and a
    // failed specialisation) with a mode-1 call of the table-driven kernel.
    hipFunction_t cfn = nullptr;
    int ck = 0;
    if (mode == 0 && P->packed && P->n_seq > 0 && (contig || span) && P->jit_min >= 0 && c.n_rec >= P->jit_min) {
        const int kp = contig ? contig_kp(sdw) : span_kp;
        const int k = (contig ? 2 : 3) * (kPre + 1) + kp;
        if (!P->jit_tried[k]) {
            P->jit_tried[k] = true;
            std::string err;
            CoopSplit cs;
            P->jit_coop[k] = jit_coop_of(true, span, jit_pro(P), 2, S.win, S.nops, S.batches, S.sops, true, &cs);
            P->jit_fn[k] = jit_get(jit_source(true, kp, jit_pro(P), 2, S.win, S.nops, S.batches, S.sops, span, true),
                                   &err, "cbx_jit_count");
        }
        cfn = P->jit_fn[k];
        ck = k;
    }
    if (mode == 0 && P->packed && P->n_seq > 0 && !cfn && !contig) {
        const int kind = P->last_kind;
        if ((r = launch(P, c, columns, 1, st))) return r;
        P->last_kind = kind;
        if (piped) HIP_CHECK(hipEventRecord(P->pipe_done, st));
    } else if (mode == 0 && P->packed && P->n_seq > 0) {
        KernelArgs ac = a;
        ac.mode = 1;
        // the specialised count kernel: no string staging per wave (it only scans lengths), two LUT
        // copies in front (full + count_lut_byte)
        size_t clds = lds_own;
        const bool ccoop = cfn && P->jit_coop[ck];
        if (cfn) {
            ac.lds_wave = (a.lds_rows + a.lds_counts + 16 + 15) & ~15;
            clds = 1024 + kLutLds + (ccoop ? (size_t)a.lds_rows + (size_t)kWavesPerBlock * (ac.lds_wave - a.lds_rows)
                                           : (size_t)kWavesPerBlock * ac.lds_wave);
        }
        int cocc = 0;
        const hipError_t ce2 = cfn ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&cocc, cfn, kWave * kWavesPerBlock, clds)
                                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&cocc, decode_kernel, kWave * kWavesPerBlock, clds);
        int cbpc = (int)std::max<size_t>(1, std::min<size_t>(16, (160 * 1024) / clds));
        if (ce2 == hipSuccess && cocc > 0) cbpc = std::min(cbpc, cocc);
        if (const char* e = getenv("CBX_MAX_BLOCKS_PER_CU")) cbpc = std::max(1, std::min(cbpc, atoi(e)));   // tuning
        if (piped && P->pipe_count_bpc > 0) cbpc = std::min(cbpc, P->pipe_count_bpc);
        const int64_t cneeded = ccoop ? n_tiles : (n_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
        const int64_t cgrid = std::min<int64_t>(cneeded, (int64_t)P->num_cus * cbpc);
        if (cfn) {
            void* kargs[] = {&ac};
            HIP_CHECK(hipModuleLaunchKernel(cfn, (unsigned)cgrid, 1, 1, kWave * kWavesPerBlock, 1, 1, (unsigned)clds, st, kargs, nullptr));
        } else {
            hipLaunchKernelGGL(decode_kernel, dim3((unsigned)cgrid), dim3(kWave * kWavesPerBlock), clds, st, ac);
            HIP_CHECK(hipGetLastError());
        }
        if ((r = string_scan(P, n_tiles, st))) return r;
        if (piped) HIP_CHECK(hipEventRecord(P->pipe_done, st));
    }
    if (jfn) {
        void* kargs[] = {&a};
        HIP_CHECK(hipModuleLaunchKernel(jfn, (unsigned)grid, 1, 1, kWave * kWavesPerBlock, 1, 1, (unsigned)lds, st, kargs, nullptr));
    } else {
        hipLaunchKernelGGL(decode_kernel, dim3((unsigned)grid), dim3(kWave * kWavesPerBlock), lds, st, a);
        HIP_CHECK(hipGetLastError());
    }
    if (lists) {   // child elements of list-layout arrays, from the lengths and starts the prologue wrote
        const int64_t lgrid = std::min<int64_t>((n_tiles + kListWaves - 1) / kListWaves, (int64_t)P->num_cus * 8);
        const size_t llds = kListWaves * 2 * (2 * kGuard + kListStage);   // two staging buffers per wave (cbx_list.h)
        // the copybook-specialised list kernel for large batches (cbx_jit.h: jit_list_source)
        hipFunction_t lfn = nullptr;
        if (P->jit_min >= 0 && c.n_rec >= P->jit_min) {
            const int k = 4 * (kPre + 1);
            if (!P->jit_tried[k]) {
                P->jit_tried[k] = true;
                const std::string src = jit_list_source(P->lops);
                std::string err;
                if (!src.empty()) P->jit_fn[k] = jit_get(src, &err, "cbx_jit_list");
            }
            lfn = P->jit_fn[k];
        }
        const CBX_CONST ListOp* d_lops = (const CBX_CONST ListOp*)P->d_lops;
        int32_t n_lops = (int32_t)P->lops.size();
        if (lfn) {
            void* kargs[] = {&a, &d_lops, &n_lops};
            HIP_CHECK(hipModuleLaunchKernel(lfn, (unsigned)lgrid, 1, 1, kWave * kListWaves, 1, 1, (unsigned)llds, st, kargs, nullptr));
        } else {
            hipLaunchKernelGGL(list_kernel<false>, dim3((unsigned)lgrid), dim3(kWave * kListWaves), llds, st, a, d_lops, n_lops);
        }
        // byte-loop pass over the tiles the first one flagged (deferred zoned forms, wide fields)
        hipLaunchKernelGGL(list_kernel<true>, dim3((unsigned)lgrid), dim3(kWave * kListWaves), llds, st, a,
                           (const CBX_CONST ListOp*)P->d_lops, (int32_t)P->lops.size());
        HIP_CHECK(hipGetLastError());
    }
    if (prof) HIP_CHECK(hipEventRecord(ce.e[1], st));
    if (mode == 0 && n_defer > 0) {
        const unsigned gy = (unsigned)std::min<int64_t>(n_defer, 65535);
        hipLaunchKernelGGL(fixup_kernel, dim3((unsigned)((n_tiles + 4 * kWave - 1) / (4 * kWave)), gy), dim3(4 * kWave), 0, st, a,
                           (const CBX_CONST DeferSeq*)P->d_defer, n_defer);
        HIP_CHECK(hipGetLastError());
    }
    if (P->n_seq > 0 && !((P->view || P->packed) && mode == 0)) {
        if ((r = string_scan(P, n_tiles, st))) return r;
        if (mode == 0) {
            const unsigned gx = (unsigned)((n_tiles + kPlaceWaves * kPlaceTiles - 1) / (kPlaceWaves * kPlaceTiles));
            hipLaunchKernelGGL(str_place_kernel, dim3(gx, (unsigned)std::min<int64_t>(P->n_seq, 65535)), dim3(kWave * kPlaceWaves), 0, st,
                               (const CBX_CONST SeqCall*)P->d_seqcall, (const uint32_t*)P->d_str_tot,
                               (const int64_t*)P->d_str_excl, n_tiles, c.n_rec, P->n_seq, P->d_status);
            HIP_CHECK(hipGetLastError());
        }
    }
    if (prof) {
        HIP_CHECK(hipEventRecord(ce.e[2], st));
        P->ev_calls.push_back(ce);
    }
    return CBX_OK;
}

// ---- the copybook-specialised record walk (cbx_jit_walk) ----
// The node tree unrolled into code: a group's children in sequence, an OCCURS as a loop to the
// largest count among the tile's lanes (each lane in the elements it has), every primitive a call of
// walk_prim_f with its Field as a constant (the decoder dispatch folds away), offsets and masks as
// per-lane registers -- the frame stack, the node-table loads and the generic decoders of the
// table-driven walk (walk_tile) are gone.  Same semantics, statement for statement:
// extractRecord's getGroupValues / extractArray / extractValue (RecordExtractors.scala:49-183).
static std::string field_literal(const Field& f) {
    std::ostringstream o;
    auto arr = [&](const int32_t* v) { o << "{" << v[0] << "," << v[1] << "," << v[2] << "," << v[3] << "}"; };
    o << "{" << f.kind << "," << f.out_type << "," << f.offset << "," << f.size << "," << f.precision << "," << f.scale << ","
      << f.sf << "," << f.out_p << "," << f.out_s << "," << f.flags << "," << f.trim << "," << f.n_dims << ",";
    arr(f.dim_count); o << ","; arr(f.dim_stride); o << ","; arr(f.dim_array);
    o << "," << f.segment << "," << f.column << "," << f.n_slots << "," << f.variant << "," << f.seq << "," << f.max_utf8 << ","
      << f.defer << "," << f.fin << "," << f.plus_null << "," << f.e_mul << "," << f.e_lim << "," << f.lim_lo << "ull," << f.lim_hi
      << "ull}";
    return o.str();
}

struct WalkGen {
    const cbx_plan* P;
    std::ostringstream o;
    int uid = 0, prims = 0;
    bool ok = true;

    void line(int ind, const std::string& t) { o << std::string(2 * ind, ' ') << t << "\n"; }

    void prim(const cbx_walk_node& n, const std::string& off, const std::string& slot, const std::string& m, bool element, int ind) {
        if (n.field < 0) return;   // a FILLER that nothing depends on
        if (++prims > kJitMaxOps) { ok = false; return; }   // (hipRTC time grows with the unrolled code)
        line(ind, "{ constexpr Field f = " + field_literal(P->dfields_h[n.field]) + ";");
        line(ind + 1, "walk_prim_f(a, wl, f, " + std::to_string(n.data_size) + ", " + std::to_string(n.dep_slot) + ", " + off + ", " +
                          slot + ", rec, avail, r, tile, lane, " + m + ", dep, " + (element ? "true" : "false") + "); }");
    }

    // the children of group g: running offset variable `off`, slot expression, lane-mask variable m
    void body(int g, const std::string& off, const std::string& slot, const std::string& m, int ind, int depth) {
        if (depth > 64) { ok = false; return; }
        const std::vector<cbx_walk_node>& N = P->h_wnodes;
        for (int c = N[g].child, guard = 0; c >= 0 && ok && guard < (int)N.size(); c = N[c].next, guard++) {
            const cbx_walk_node& n = N[c];
            const std::string K = std::to_string(uid++);
            const bool adv = !(n.flags & CBX_W_REDEFINED);
            if (n.array >= 0) {   // extractArray (:66-114)
                const cbx_array& ar = P->harrays[n.array];
                line(ind, "{   // OCCURS (node " + std::to_string(c) + ")");
                line(ind + 1, "const int cnt" + K + " = " + m + " ? walk_count(a, " + std::to_string(n.array) + ", dep) : 0;");
                if (ar.count_column >= 0) {
                    const std::string cc = std::to_string(ar.count_column);
                    line(ind + 1, "{ const DevColumn cc = ldc(a.cols + " + cc + "); if (" + m + ") *gp((int32_t*)cc.values + (int64_t)(" + slot +
                                      ") * a.pitch + r) = cnt" + K + "; walk_valid(a, wl, cc.validity, " + cc + ", " + slot +
                                      ", tile, lane, " + m + "); }");
                }
                line(ind + 1, "const int cmax" + K + " = (int)wave_max64(cnt" + K + ");");
                line(ind + 1, "int eo" + K + " = " + off + ";");
                line(ind + 1, "for (int e" + K + " = 0; e" + K + " < cmax" + K + "; e" + K + "++) {");
                line(ind + 2, "const bool le" + K + " = " + m + " && e" + K + " < cnt" + K + ";");
                line(ind + 2, "const int s" + K + " = (" + slot + ") * " + std::to_string(std::max(1, ar.max_count)) + " + e" + K + ";");
                if (n.kind == CBX_W_GROUP) {
                    line(ind + 2, "int go" + K + " = eo" + K + ";");
                    body(c, "go" + K, "s" + K, "le" + K, ind + 2, depth + 1);
                    line(ind + 2, "if (le" + K + ") eo" + K + " = go" + K + ";");
                } else {
                    prim(n, "eo" + K, "s" + K, "le" + K, true, ind + 2);
                    line(ind + 2, "if (le" + K + ") eo" + K + " += " + std::to_string(n.data_size) + ";");
                }
                line(ind + 1, "}");
                // the consumed size: the lane's elements walked, or the static size (:109-113)
                if (adv)
                    line(ind + 1, "if (" + m + ") " + off + " += " + (P->walk_var ? "eo" + K + " - " + off : std::to_string(n.actual_size)) + ";");
                line(ind, "}");
                continue;
            }
            if (n.kind == CBX_W_GROUP) {   // getGroupValues (:144-160); a segment redefine of another segment: null, full size (:119-121)
                const std::string on = n.segment >= 0 ? m + " && seg == " + std::to_string(n.segment) : m;
                line(ind, "{   // group (node " + std::to_string(c) + ")");
                line(ind + 1, "const bool on" + K + " = " + on + ";");
                line(ind + 1, "int last" + K + " = " + std::to_string(n.actual_size) + ";");
                line(ind + 1, "if (__ballot(on" + K + ")) {");
                line(ind + 2, "int go" + K + " = " + off + ";");
                body(c, "go" + K, slot, "on" + K, ind + 2, depth + 1);
                line(ind + 2, "if (on" + K + ") last" + K + " = go" + K + " - " + off + ";");
                line(ind + 1, "}");
                if (adv) {
                    if (n.flags & CBX_W_REDEFINES) line(ind + 1, "if (" + m + ") " + off + " += " + std::to_string(n.actual_size) + ";");
                    else line(ind + 1, "if (" + m + ") " + off + " += last" + K + ";");
                }
                line(ind, "}");
                continue;
            }
            prim(n, off, slot, m, false, ind);
            if (adv) line(ind, "if (" + m + ") " + off + " += " + std::to_string(n.actual_size) + ";");
        }
    }
};

// The specialised walk's source, or "" when the copybook is beyond the unrolled form's limits.
static std::string jit_walk_source(const cbx_plan* P) {
    WalkGen g{P};
    g.o << "#define CBX_STR_LAYOUT 1\n#define CBX_MODE 0\n#define CBX_JIT_WALK 1\n#include \"cbx_device.h\"\n#include \"cbx_walk.h\"\n"
           "namespace cbx {\nstruct JitWalk {\n"
           "  static constexpr bool kTyped = true;\n"
           "  template <typename RP>\n"
           "  __device__ __forceinline__ void operator()(const WalkArgs& a, const WalkLds& wl, uint8_t* area, RP rec,\n"
           "      int avail, int seg, int64_t r, int64_t tile, int lane, bool act) const {\n"
           "    WalkDeps dep;\n    walk_seed(a, dep, r, act, seg);\n    int off0 = 0;\n";
    g.body(P->walk_root, "off0", "0", "act", 2, 0);
    g.o << "  }\n};\n}  // namespace cbx\n"
           "extern \"C\" __global__ __launch_bounds__(256) void cbx_jit_walk(cbx::WalkArgs a) {\n"
           "  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];\n"
           "  cbx::walk_tiles(a, wsm, cbx::JitWalk{});\n}\n";
    return g.ok ? g.o.str() : std::string();
}

// ---- the copybook-specialised var-occurs framing (cbx_frame_var_occurs) ----
// walk_length (cbx_walk.h: VarOccursRecordExtractor.extractVarOccursRecordBytes, :52-136) unrolled like
// cbx_jit_walk: a group's children in sequence, an OCCURS of groups a loop over its elements, every
// dependee decoded with its Field as a constant from the zero-filled record bytes; subtrees without
// OCCURS or dependees fold to their static walked size.  One lane per record (the chain's step), so no
// ballots: the lanes of a wave walk different records of different chunks.  The five chain passes
// (cbx_chain.h) are wrapped as extern "C" kernels of one module around that step.
struct LenGen {
    const cbx_plan* P;
    std::ostringstream o;
    int uid = 0, prims = 0;
    bool ok = true;

    void line(int ind, const std::string& t) { o << std::string(2 * ind, ' ') << t << "\n"; }

    // the walked size of group g's children when it depends on no data (no OCCURS, no dependee), else -1
    int static_size(int g, int depth) const {
        if (depth > 64) return -1;
        const std::vector<cbx_walk_node>& N = P->h_wnodes;
        int sum = 0;
        for (int c = N[g].child, guard = 0; c >= 0 && guard < (int)N.size(); c = N[c].next, guard++) {
            const cbx_walk_node& n = N[c];
            if (n.array >= 0) return -1;
            int w = n.actual_size;
            if (n.kind == CBX_W_GROUP) {
                if ((w = static_size(c, depth + 1)) < 0) return -1;
            } else if (n.dep_slot >= 0 && n.field >= 0) {
                return -1;
            }
            if (!(n.flags & CBX_W_REDEFINED)) sum += w;
        }
        return sum;
    }

    // walk_length's frames: the table walk fails (-1) past kWalkDepth frames; the unrolled form is only
    // generated for copybooks that never get there (sp = the frame index of group g's children)
    void body(int g, const std::string& off, int ind, int sp) {
        if (sp >= 48) { ok = false; return; }
        const std::vector<cbx_walk_node>& N = P->h_wnodes;
        for (int c = N[g].child, guard = 0; c >= 0 && ok && guard < (int)N.size(); c = N[c].next, guard++) {
            const cbx_walk_node& n = N[c];
            const std::string K = std::to_string(uid++);
            const bool adv = !(n.flags & CBX_W_REDEFINED);
            if (n.array >= 0) {   // an OCCURS: its present elements, walked (:109-113)
                if (sp + 1 >= kWalkDepth) { ok = false; return; }
                line(ind, "{   // OCCURS (node " + std::to_string(c) + ")");
                line(ind + 1, "const int cnt" + K + " = walk_count(a, " + std::to_string(n.array) + ", dep);");
                if (n.kind == CBX_W_GROUP) {
                    if (sp + 2 >= kWalkDepth) { ok = false; return; }
                    const int S = static_size(c, 0);
                    if (S >= 0) {
                        line(ind + 1, "const int w" + K + " = cnt" + K + " * " + std::to_string(S) + ";");
                    } else {
                        line(ind + 1, "int eo" + K + " = " + off + ";");
                        line(ind + 1, "for (int e" + K + " = 0; e" + K + " < cnt" + K + "; e" + K + "++) {");
                        body(c, "eo" + K, ind + 2, sp + 2);
                        line(ind + 1, "}");
                        line(ind + 1, "const int w" + K + " = eo" + K + " - " + off + ";");
                    }
                } else {
                    line(ind + 1, "const int w" + K + " = cnt" + K + " * " + std::to_string(n.data_size) + ";");
                }
                if (adv) line(ind + 1, off + " += w" + K + ";");
                line(ind, "}");
                continue;
            }
            if (n.kind == CBX_W_GROUP) {   // every non-redefined field advances by its walked size (:111-131)
                if (sp + 1 >= kWalkDepth) { ok = false; return; }
                const int S = static_size(c, 0);
                if (S >= 0) {
                    if (adv && S) line(ind, off + " += " + std::to_string(S) + ";");
                    continue;
                }
                line(ind, "{   // group (node " + std::to_string(c) + ")");
                line(ind + 1, "int go" + K + " = " + off + ";");
                body(c, "go" + K, ind + 1, sp + 1);
                if (adv) line(ind + 1, off + " = go" + K + ";");
                line(ind, "}");
                continue;
            }
            if (n.dep_slot >= 0 && n.field >= 0) {   // a dependee: decoded from the (zero-filled) bytes
                if (++prims > kJitMaxOps) { ok = false; return; }
                const Field& f = P->dfields_h[n.field];
                const int size = std::min(n.actual_size, 64);
                const bool str = f.kind == CBX_K_STRING || f.kind == CBX_K_STRING_ASCII;
                line(ind, "{   // dependee (node " + std::to_string(c) + ")");
                line(ind + 1, "constexpr Field f = " + field_literal(f) + ";");
                line(ind + 1, "uint8_t zb[64];");
                line(ind + 1, "if (" + off + " + " + std::to_string(size) + " <= avail) {");
                line(ind + 2, "for (int i = 0; i < " + std::to_string(size) + "; i++) zb[i] = rec[" + off + " + i];");
                line(ind + 1, "} else {");
                line(ind + 2, "for (int i = 0; i < " + std::to_string(size) + "; i++) zb[i] = " + off + " + i < avail ? rec[" + off +
                                  " + i] : 0;");
                line(ind + 1, "}");
                if (str) line(ind + 1, "walk_len_str_dep(a, f, zb, " + std::to_string(size) + ", " + std::to_string(n.dep_slot) + ", dep);");
                else line(ind + 1, "{ const Val dv = decode_count_int(f, zb); dep.set(" + std::to_string(n.dep_slot) +
                                       ", dv.valid, WalkDep{1, (int32_t)dv.lo}); }");
                line(ind, "}");
            }
            if (adv && n.actual_size) line(ind, off + " += " + std::to_string(n.actual_size) + ";");
        }
    }
};

// The specialised framing's source, or "" when the copybook is beyond the unrolled form's limits.
static std::string jit_chain_source(const cbx_plan* P) {
    LenGen g{P};
    g.o << "#define CBX_STR_LAYOUT 1\n#define CBX_MODE 0\n#define CBX_JIT_WALK 1\n#include \"cbx_device.h\"\n"
           "#include \"cbx_walk.h\"\n#include \"cbx_chain.h\"\n"
           "namespace cbx {\n"
           "__device__ __forceinline__ int jit_walk_length(const WalkArgs& a, const CBX_GLOBAL uint8_t* rec, int avail) {\n"
           "  WalkDeps dep;\n  dep.clear();\n  int off0 = 0;\n";
    g.body(P->walk_root, "off0", 1, 0);
    g.o << "  return off0;\n}\n"
           "struct JitVarOccursStep {   // VarOccursStep's layout and semantics\n"
           "  WalkArgs a;\n  int64_t n_bytes;\n"
           "  __device__ __forceinline__ ChainStep at(int64_t pos) const {\n"
           "    ChainStep s{kChainStop, 0, 0};\n"
           "    if (pos >= n_bytes) return s;\n"
           "    const int64_t left = n_bytes - pos;\n"
           "    const int len = jit_walk_length(a, gp(a.data) + pos, left < 0x7fffffff ? (int)left : 0x7fffffff);\n"
           "    if (len <= 0) return s;\n"
           "    s.len = len;\n    s.next = pos + len;\n    return s;\n  }\n};\n"
           "}  // namespace cbx\n"
           "using cbx::JitVarOccursStep;\nusing cbx::ChainArgs;\n"
           "extern \"C\" __global__ void cbx_jit_chain_sample(JitVarOccursStep s, ChainArgs c, int n_max) { cbx::chain_sample_run(s, c, n_max); }\n"
           "extern \"C\" __global__ __launch_bounds__(256) void cbx_jit_chain_spec(JitVarOccursStep s, ChainArgs c) { cbx::chain_spec_run(s, c); }\n"
           "extern \"C\" __global__ __launch_bounds__(256) void cbx_jit_chain_fix(JitVarOccursStep s, ChainArgs c, const int64_t* ex_in, int64_t* ex_out) {\n"
           "  cbx::chain_fix_run(s, c, ex_in, ex_out);\n}\n"
           "extern \"C\" __global__ void cbx_jit_chain_settle(JitVarOccursStep s, ChainArgs c, int64_t* ex) { cbx::chain_settle_run(s, c, ex); }\n"
           "extern \"C\" __global__ __launch_bounds__(256) void cbx_jit_chain_write(JitVarOccursStep s, ChainArgs c, const int64_t* base, int64_t capacity,\n"
           "                                                  int64_t* rec_off, int32_t* rec_len) {\n"
           "  cbx::chain_write_run(s, c, base, capacity, rec_off, rec_len);\n}\n";
    return g.ok ? g.o.str() : std::string();
}

// The record walk (cbx_walk.h): one lane per record, data-dependent offsets.
static int walk_launch(cbx_plan* P, const CallShape& c, cbx_column* columns, hipStream_t st) {
    const int64_t n_tiles = (c.n_rec + kWave - 1) / kWave;
    for (int i = 0; i < P->n_columns; i++) {
        if (!P->col_is_string[i] || c.n_rec == 0) continue;
        const int64_t need = n_tiles * view_tile_bytes(P, i);
        if (!columns[i].values || !columns[i].data || columns[i].data_capacity < need)
            return fail(CBX_E_CAPACITY, "column " + std::to_string(i) + ": string-view buffers of cbx_string_bound required");
    }
    if (c.n_rec == 0) return CBX_OK;
    P->h_cols.resize(P->n_columns);
    for (int i = 0; i < P->n_columns; i++) {
        DevColumn d{};
        d.values = columns[i].values; d.validity = columns[i].validity; d.offsets = columns[i].offsets;
        d.data = columns[i].data; d.capacity = columns[i].data_capacity; d.sizes = columns[i].data_sizes;
        P->h_cols[i] = d;
    }
    HIP_CHECK(hipMemcpyAsync(P->d_cols, P->h_cols.data(), sizeof(DevColumn) * P->n_columns, hipMemcpyHostToDevice, st));
    int r;
    const int64_t nc = std::max<int64_t>(1, P->n_str_slots * n_tiles);
    if ((r = grow(&P->d_wcursor, &P->wcursor_cap, nc, st))) return r;
    HIP_CHECK(hipMemsetAsync(P->d_wcursor, 0, sizeof(uint32_t) * nc, st));
    WalkArgs a{};
    a.data = c.data; a.data_len = c.data_len; a.rec_off = c.rec_off; a.rec_len = c.rec_len; a.n_rec = c.n_rec;
    a.stride = c.stride; a.start_off = c.start_off; a.first_record_id = c.first_record_id; a.rec_id_base = P->d_rec_base;
    a.rec_id = c.rec_id; a.rec_seg = c.rec_seg; a.file_id = c.file_id >= 0 ? c.file_id : P->opts.file_id;
    a.var_occurs = P->walk_var; a.n_tiles = n_tiles; a.pitch = n_tiles * kWave;
    a.dep_seed = P->d_dep_seed; a.seed_pitch = P->seed_pitch; a.hier_root = P->seed_root;
    a.nodes = (const CBX_CONST cbx_walk_node*)P->d_wnodes; a.root = P->walk_root;
    a.warr = (const CBX_CONST cbx_walk_array*)P->d_warr;
    a.handlers = (const CBX_CONST cbx_walk_handler*)P->d_whand; a.n_handlers = P->walk_n_handlers;
    a.arrays = (const CBX_CONST cbx_array*)P->d_arrays; a.fields = (const CBX_CONST Field*)P->d_fields;
    a.cols = (const CBX_CONST DevColumn*)P->d_cols;
    a.segmap = P->opts.has_segments ? (const CBX_CONST cbx_segment_map*)P->d_segmap : nullptr;
    a.lut = P->d_lut; a.seg_col = P->seg_col; a.fid_col = P->fid_col; a.rid_col = P->rid_col;
    a.str_slot_base = P->d_wslot_base; a.cursors = P->d_wcursor; a.tile_bytes = P->d_wtile_bytes; a.status = P->d_status;
    // per-wave LDS words (validity of every column slot, string cursors) when they fit 8 KiB a wave
    a.n_vslots = P->n_vslots;
    a.n_sslots = (int32_t)P->n_str_slots;
    // per wave: the frame stack (uniform part + three 64-lane rows per level), the tile's record
    // bytes, then the tile's validity words and string cursors when they fit 8 KiB
    a.depth = P->walk_depth;
    // the copybook-specialised walk for large batches (cbx_jit_walk), else the table-driven one
    hipFunction_t jfn = nullptr;
    if (P->jit_min >= 0 && c.n_rec >= P->jit_min && !getenv("CBX_NO_JIT_WALK")) {
        if (!P->walk_jit_tried) {
            P->walk_jit_tried = true;
            const std::string src = jit_walk_source(P);
            if (!src.empty()) P->walk_jit_fn = jit_get(src, &P->jit_error, "cbx_jit_walk");
        }
        jfn = P->walk_jit_fn;
    }
    // the table-driven walk's frame stack (the specialised walk keeps its frames in registers)
    a.stack_lds = jfn ? 0 : (int32_t)((a.depth * (sizeof(WalkU) + 3 * sizeof(int32_t) * kWave) + 15) & ~(size_t)15);
    const int32_t words = (int32_t)((8 * (int64_t)P->n_vslots + 4 * P->n_str_slots + 15) & ~15ll);
    a.vlds = P->n_vslots > 0 && words <= 8192 && !getenv("CBX_WALK_GLOBAL_ATOMICS") ? 1 : 0;
    // the tile's record bytes: 64 records of the copybook's largest form + 8 bytes of framing each
    // (RDW headers, line ends), at most 8 KiB -- the resident waves per CU are LDS-bound; a wider
    // tile reads its records from HBM
    a.stage_cap = getenv("CBX_WALK_NO_STAGE")
                      ? 0
                      : (int32_t)std::min<int64_t>(8192, (kWave * (int64_t)(P->walk_max_rec + c.start_off + 8) + 31) & ~15ll);
    a.wave_lds = a.stack_lds + a.stage_cap + (a.vlds ? words : 0);
    a.vslot_base = P->d_wvbase; a.vslot_col = P->d_wvcol; a.vslot_slot = P->d_wvslot;
    const size_t wlds = kWalkLdsBase + kWalkLut + 4 * (size_t)a.wave_lds;
    const int64_t grid = std::min<int64_t>((n_tiles + 3) / 4, (int64_t)P->num_cus * 8);
    // kernel timing (cbx_plan_set_profiling): the walk is the decode; it has no post passes
    cbx_plan::CallEvents ce{{nullptr, nullptr, nullptr}};
    if (P->profiling) {
        for (auto& e : ce.e) if (!(e = take_event(P))) return fail(CBX_E_HIP, "hipEventCreate failed");
        HIP_CHECK(hipEventRecord(ce.e[0], st));
    }
    if (jfn) {
        void* kargs[] = {&a};
        HIP_CHECK(hipModuleLaunchKernel(jfn, (unsigned)grid, 1, 1, 256, 1, 1, (unsigned)wlds, st, kargs, nullptr));
    } else {
        hipLaunchKernelGGL(walk_kernel, dim3((unsigned)grid), dim3(256), wlds, st, a);
        HIP_CHECK(hipGetLastError());
    }
    if (P->profiling) {
        HIP_CHECK(hipEventRecord(ce.e[1], st));
        HIP_CHECK(hipEventRecord(ce.e[2], st));
        P->ev_calls.push_back(ce);
    }
    P->last_kind = jfn ? 3 : 2;
    return CBX_OK;
}

static int decode_common(cbx_plan* P, const CallShape& c, cbx_column* columns, int64_t* sizes_only, hipStream_t st) {
    if (!P || !c.data || c.n_rec < 0 || c.start_off < 0) return fail(CBX_E_ARGUMENT, "invalid decode arguments");
    if (!sizes_only && !columns) return fail(CBX_E_ARGUMENT, "columns required");
    if (sizes_only) {
        for (int i = 0; i < P->n_columns; i++) sizes_only[i] = 0;
        if (P->n_seq == 0 || c.n_rec == 0) return CBX_OK;
        if (P->view) return cbx_string_bound(P, c.n_rec, sizes_only);   // the layout's capacity is per tile
        int r = launch(P, c, nullptr, 1, st);
        if (r) return r;
        // sequence total = excl[last tile] + tot[last tile] - excl[first tile]
        const int64_t n_tiles = (c.n_rec + kWave - 1) / kWave;
        std::vector<int64_t> e0(P->n_seq), e1(P->n_seq);
        std::vector<uint32_t> t1(P->n_seq);
        for (int q = 0; q < P->n_seq; q++) {
            HIP_CHECK(hipMemcpyAsync(&e0[q], P->d_str_excl + (int64_t)q * n_tiles, 8, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipMemcpyAsync(&e1[q], P->d_str_excl + (int64_t)q * n_tiles + n_tiles - 1, 8, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipMemcpyAsync(&t1[q], P->d_str_tot + (int64_t)q * n_tiles + n_tiles - 1, 4, hipMemcpyDeviceToHost, st));
        }
        HIP_CHECK(hipStreamSynchronize(st));
        for (int q = 0; q < P->n_seq; q++) {
            const int col = P->dfields_h[P->seq_field[q]].column;
            sizes_only[col] = std::max(sizes_only[col], e1[q] + (int64_t)t1[q] - e0[q]);
        }
        return CBX_OK;
    }
    if (P->walk) return walk_launch(P, c, columns, st);
    for (int i = 0; i < P->n_columns; i++) {
        if (!P->col_is_string[i] || c.n_rec == 0) continue;
        if (P->view) {
            const int64_t need = (c.n_rec + kWave - 1) / kWave * view_tile_bytes(P, i);
            if (!columns[i].values || !columns[i].data)
                return fail(CBX_E_ARGUMENT, "column " + std::to_string(i) + ": string-view buffers (values, data) required");
            if (columns[i].data_capacity < need)
                return fail(CBX_E_CAPACITY, "column " + std::to_string(i) + ": string-view data_capacity " +
                                                std::to_string(columns[i].data_capacity) + " < " + std::to_string(need) +
                                                " (cbx_string_bound)");
        } else if (!columns[i].offsets || (!columns[i].data && columns[i].data_capacity > 0)) {
            return fail(CBX_E_ARGUMENT, "column " + std::to_string(i) + ": string buffers required");
        }
    }
    return launch(P, c, columns, 0, st);
}

extern "C" int cbx_plan_check(cbx_plan* P, void* stream) {
    if (!P) return fail(CBX_E_ARGUMENT, "null plan");
    hipStream_t st = (hipStream_t)stream;
    int32_t status = 0;
    HIP_CHECK(hipMemcpyAsync(&status, P->d_status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (status != 0) {
        HIP_CHECK(hipMemset(P->d_status, 0, sizeof(int32_t)));
        if (status & 4)   // (cbx_device.h: lds_base_ok)
            return fail(CBX_E_HIP, "specialised kernel: dynamic LDS does not start at address 0 (its outputs are invalid)");
        if (status & 2)   // (cbx_walk.h: the table-driven walk's frame stack)
            return fail(CBX_E_STATE, "record walk: copybook nesting exceeded the walk's frame stack");
        return fail(CBX_E_CAPACITY, "a string column's payload exceeded its data_capacity (size it with cbx_string_bound or cbx_string_sizes_*)");
    }
    return CBX_OK;
}

extern "C" int cbx_plan_set_record_base(cbx_plan* P, const int64_t* d_base) {
    if (!P) return fail(CBX_E_ARGUMENT, "cbx_plan_set_record_base: invalid plan");
    P->d_rec_base = d_base;
    return CBX_OK;
}

extern "C" int cbx_plan_set_dep_seed(cbx_plan* P, const int64_t* d_seed, int64_t pitch, int32_t root_segment) {
    if (!P || pitch < 0 || (d_seed && (pitch == 0 || root_segment < 0)))
        return fail(CBX_E_ARGUMENT, "cbx_plan_set_dep_seed: invalid arguments");
    if (d_seed && !P->walk) return fail(CBX_E_STATE, "cbx_plan_set_dep_seed: the plan has no record walk (cbx_plan_set_walk)");
    P->d_dep_seed = d_seed;
    P->seed_pitch = d_seed ? pitch : 0;
    P->seed_root = d_seed ? root_segment : -1;
    return CBX_OK;
}

extern "C" int cbx_plan_set_odo_counts(cbx_plan* P, const int32_t* d_counts, int64_t pitch) {
    if (!P || pitch < 0 || (d_counts && pitch == 0)) return fail(CBX_E_ARGUMENT, "cbx_plan_set_odo_counts: invalid arguments");
    if (d_counts && P->walk) return fail(CBX_E_UNSUPPORTED, "cbx_plan_set_odo_counts: the record walk reads its counts itself");
    P->d_odo = d_counts;
    P->odo_pitch = d_counts ? pitch : 0;
    return CBX_OK;
}

extern "C" int cbx_plan_pipeline(cbx_plan* A, cbx_plan* B, int32_t count_blocks_per_cu, int32_t decode_blocks_per_cu) {
    if (!A || A == B || count_blocks_per_cu < 0 || decode_blocks_per_cu < 0)
        return fail(CBX_E_ARGUMENT, "cbx_plan_pipeline: invalid arguments");
    if (A->pipe_peer) { A->pipe_peer->pipe_peer = nullptr; A->pipe_peer = nullptr; }
    A->pipe_count_bpc = A->pipe_decode_bpc = 0;
    if (!B) return CBX_OK;
    if (B->pipe_peer) { B->pipe_peer->pipe_peer = nullptr; B->pipe_peer = nullptr; }
    for (cbx_plan* P : {A, B}) {
        if (!P->pipe_done) HIP_CHECK(hipEventCreateWithFlags(&P->pipe_done, hipEventDisableTiming));
        P->pipe_count_bpc = count_blocks_per_cu;
        P->pipe_decode_bpc = decode_blocks_per_cu;
    }
    A->pipe_peer = B;
    B->pipe_peer = A;
    return CBX_OK;
}

extern "C" int cbx_plan_set_profiling(cbx_plan* P, int32_t enable) {
    if (!P) return fail(CBX_E_ARGUMENT, "null plan");
    P->profiling = enable != 0;
    return CBX_OK;
}

#ifdef CBX_STAMPS
// Diagnostic build only: per-segment s_memtime sums of the contiguous decode loop since the
// last call (out[0..5] segments, out[7] waves), then reset.
extern "C" int cbx_debug_stamps(cbx_plan* P, uint64_t* out) {
    if (!P || !out) return fail(CBX_E_ARGUMENT, "cbx_debug_stamps: invalid arguments");
    if (!P->d_stamps) { memset(out, 0, 8 * sizeof(uint64_t)); return CBX_OK; }
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(out, P->d_stamps, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemset(P->d_stamps, 0, 8 * sizeof(uint64_t)));
    return CBX_OK;
}
#endif

extern "C" int cbx_plan_specialize(cbx_plan* P, char* source, int64_t source_cap, int64_t* source_len, int32_t compile) {
    if (!P) return fail(CBX_E_ARGUMENT, "cbx_plan_specialize: invalid arguments");
    const cbx_plan::OpSet& S = P->contig_ok ? P->cset : P->wset;
    const std::string src = jit_source(P->contig_ok, P->contig_ok ? kPre : 0, jit_pro(P), str_layout_of(P), S.win, S.nops, S.batches, S.sops, false);
    if (source_len) *source_len = (int64_t)src.size();
    if (source && source_cap > 0) {
        const size_t n = std::min<size_t>(src.size(), (size_t)source_cap - 1);
        memcpy(source, src.data(), n);
        source[n] = 0;
    }
    if (compile) {
        std::vector<char> code;
        std::string err;
        if (!jit_compile(src, &code, &err)) return fail(CBX_E_HIP, err);
        if (P->packed && P->contig_ok && P->n_seq > 0 &&   // the Utf8 layout's count pass too
            !jit_compile(jit_source(true, kPre, jit_pro(P), 2, S.win, S.nops, S.batches, S.sops, false, true), &code, &err))
            return fail(CBX_E_HIP, err);
    }
    return CBX_OK;
}

extern "C" int cbx_plan_kernel_kind(cbx_plan* P, int32_t* kind) {
    if (!P || !kind) return fail(CBX_E_ARGUMENT, "cbx_plan_kernel_kind: invalid arguments");
    *kind = P->last_kind;
    if (!P->last_kind && !P->jit_error.empty()) g_err = P->jit_error;
    return CBX_OK;
}

extern "C" int cbx_plan_frame_kind(cbx_plan* P, int32_t* kind) {
    if (!P || !kind) return fail(CBX_E_ARGUMENT, "cbx_plan_frame_kind: invalid arguments");
    *kind = P->last_chain_jit ? 1 : 0;
    return CBX_OK;
}

extern "C" int cbx_plan_kernel_times(cbx_plan* P, float* decode_ms, float* fixup_ms, int32_t max_calls, int32_t* n_calls) {
    if (!P || !n_calls || max_calls < 0) return fail(CBX_E_ARGUMENT, "cbx_plan_kernel_times: invalid arguments");
    int n = 0;
    for (auto& c : P->ev_calls) {
        HIP_CHECK(hipEventSynchronize(c.e[2]));
        if (n < max_calls) {
            float d = 0, f = 0;
            HIP_CHECK(hipEventElapsedTime(&d, c.e[0], c.e[1]));
            HIP_CHECK(hipEventElapsedTime(&f, c.e[1], c.e[2]));
            if (decode_ms) decode_ms[n] = d;
            if (fixup_ms) fixup_ms[n] = f;
            n++;
        }
        for (auto& e : c.e) P->ev_pool.push_back(e);
    }
    P->ev_calls.clear();
    *n_calls = n;
    return CBX_OK;
}

extern "C" int cbx_string_sizes_fixed(cbx_plan* P, const uint8_t* d_records, int64_t n_rec, int32_t rec_stride,
                                      int32_t start_offset, int64_t* out_sizes, void* stream) {
    if (!out_sizes) return fail(CBX_E_ARGUMENT, "out_sizes required");
    if (rec_stride <= 0) return fail(CBX_E_ARGUMENT, "record stride must be positive");
    CallShape c{d_records, n_rec * (int64_t)rec_stride, nullptr, nullptr, n_rec, rec_stride, start_offset, 0};
    return decode_common(P, c, nullptr, out_sizes, (hipStream_t)stream);
}

extern "C" int cbx_decode_fixed(cbx_plan* P, const uint8_t* d_records, int64_t n_rec, int32_t rec_stride,
                                int32_t start_offset, int64_t first_record_id, cbx_column* columns, void* stream) {
    if (rec_stride <= 0) return fail(CBX_E_ARGUMENT, "record stride must be positive");
    CallShape c{d_records, n_rec * (int64_t)rec_stride, nullptr, nullptr, n_rec, rec_stride, start_offset, first_record_id};
    return decode_common(P, c, columns, nullptr, (hipStream_t)stream);
}

extern "C" int cbx_decode_var(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                              const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset, int64_t first_record_id,
                              cbx_column* columns, void* stream) {
    if (!d_rec_off || !d_rec_len || n_bytes < 0) return fail(CBX_E_ARGUMENT, "record offsets/lengths required");
    CallShape c{d_data, n_bytes, d_rec_off, d_rec_len, n_rec, 0, start_offset, first_record_id};
    return decode_common(P, c, columns, nullptr, (hipStream_t)stream);
}

extern "C" int cbx_string_sizes_var(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                                    const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset,
                                    int64_t* out_sizes, void* stream) {
    if (!d_rec_off || !d_rec_len || !out_sizes || n_bytes < 0) return fail(CBX_E_ARGUMENT, "invalid arguments");
    CallShape c{d_data, n_bytes, d_rec_off, d_rec_len, n_rec, 0, start_offset, 0};
    return decode_common(P, c, nullptr, out_sizes, (hipStream_t)stream);
}

// The stream-ordered pool of the current device keeps what it holds (release threshold: no limit):
// cbx_frame_rdw's staging (gigabytes for a 10 GB file) is then reused from call to call instead of
// being unmapped at every synchronisation and mapped again by the next call's hipMallocAsync.
static void keep_pool_memory() {
    static std::mutex mu;
    static std::vector<int> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(mu);
    for (int d : done) if (d == dev) return;
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
        uint64_t thr = ~0ull;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
    done.push_back(dev);
}

namespace cbx {
// The async walk's outcome (cbx_frame_rdw_async): count, first header error, capacity flag.
__global__ void rdw_state_kernel(const unsigned long long* res, int64_t capacity, int64_t* state) {
    if (threadIdx.x == 0) {
        const int64_t total = (int64_t)res[1];
        state[0] = total;
        state[1] = (int64_t)res[0];
        state[2] = total > capacity ? 1 : 0;
    }
}
}  // namespace cbx

// Host -> device copy of a small host array with no host wait: a ring of pinned buffers, each
// reused once the copy that last read it has completed (one event per slot; long done in practice).
static int upload_no_wait(const void* src, size_t n, void* dst, hipStream_t st) {
    struct Slot { void* p = nullptr; size_t cap = 0; hipEvent_t ev = nullptr; int dev = -1; };
    static thread_local Slot ring[4];
    static thread_local int next = 0;
    Slot& sl = ring[next];
    next = (next + 1) % 4;
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    // the copy that last read the slot's buffer must be done before it is overwritten or freed --
    // also when it ran on another device (then the slot starts over with an event of this one)
    if (sl.ev) HIP_CHECK(hipEventSynchronize(sl.ev));
    if (sl.ev && sl.dev != dev) {
        (void)hipEventDestroy(sl.ev);
        sl.ev = nullptr;
    }
    if (sl.cap < n) {
        if (sl.p) HIP_CHECK(hipHostFree(sl.p));
        sl.p = nullptr;
        sl.cap = 0;
        HIP_CHECK(hipHostMalloc(&sl.p, n, hipHostMallocDefault));
        sl.cap = n;
    }
    if (!sl.ev) {
        HIP_CHECK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
        sl.dev = dev;
    }
    memcpy(sl.p, src, n);
    HIP_CHECK(hipMemcpyAsync(dst, sl.p, n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipEventRecord(sl.ev, st));
    return CBX_OK;
}

static int rdw_error(unsigned long long first_err) {
    const long long off = (long long)(first_err >> 2);
    char msg[200];
    if ((first_err & 3) == 2) snprintf(msg, sizeof msg, "RDW headers should never be zero. Found zero size record at %lld.", off);
    else snprintf(msg, sizeof msg, "RDW headers too big (length > %lld) at %lld.", 100ll * 1024 * 1024, off);
    return fail(CBX_E_STATE, msg);
}

// The walk of cbx_frame_rdw (d_state == nullptr: host waits for the settle check and the count) and of
// cbx_frame_rdw_async (d_state: max_rounds parallel fix rounds + the settle pass enqueued without waiting,
// the outcome on the device).
static int frame_rdw_impl(const uint8_t* d_data, int64_t n_bytes, const int64_t* seeds, int32_t n_seeds,
                          const cbx_rdw_params* params, int64_t* d_rec_off, int32_t* d_rec_len, int64_t capacity,
                          int64_t* n_records, int64_t* d_state, int32_t max_rounds, hipStream_t st) {
    const bool async = d_state != nullptr;
    keep_pool_memory();
    // seed ranges cut into chunks (rdw_wave_kernel: speculation + walk, fix rounds; rdw_place_kernel)
    // 256 KiB chunks: every chunk pays one speculated entry, so C5's 16 KB records want few of them
    // (framing 21.1 / 2.30 / 1.59 / 1.23 / 1.10 ms at 16 / 64 / 128 / 256 / 512 KiB), while C4's
    // 65-byte records walk ~4,000 per chunk at no loss (4.02 / 3.97 / 3.96 / 4.11 ms at 64 / 128 /
    // 256 / 512 KiB; same-box runs, tools/gpu.sh A/B)
    int64_t chunk = 256 * 1024;
    if (const char* e = getenv("CBX_RDW_CHUNK_BYTES")) chunk = std::max<int64_t>(8, atoll(e));   // tests: many chunks
    std::vector<int64_t> hs;
    if (n_seeds <= 0) hs.push_back(0);
    else hs.assign(seeds, seeds + n_seeds);
    // seed ranges (the chunk table is computed on the device from them)
    std::vector<RdwRange> ranges(hs.size());
    int64_t n = 0;
    for (size_t k = 0; k < hs.size(); k++) {
        const int64_t r0 = hs[k], r1 = k + 1 < hs.size() ? hs[k + 1] : n_bytes;
        if (r0 < 0 || r0 > n_bytes || r1 < r0) return fail(CBX_E_ARGUMENT, "cbx_frame_rdw: seeds must be increasing offsets");
        ranges[k] = RdwRange{r0, r1, n};
        n += std::max<int64_t>(1, (r1 - r0 + chunk - 1) / chunk);
    }
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    // one device block: entry, exit x2, err, base (int64 x n) | first_err, total, changed | block sums |
    // ranges | count (u32 x n)
    // staging: chunk bytes / 40 records per chunk (C4's ~65-byte records use ~60 % of it; chunks of
    // shorter records are walked again by the placement pass)
    // (a multiple of 64: the wave walk stores whole rows of 64 records)
    const int64_t stage_cap = (std::max<int64_t>(64, chunk / 40) + 63) & ~(int64_t)63;
    // + one changed flag per fix round (rounds <= n + 1)
    const size_t bytes = sizeof(int64_t) * (5 * n + 4 + nb) + sizeof(RdwRange) * ranges.size() + sizeof(uint32_t) * n +
                         sizeof(int32_t) * (n + 2) + 64;
    const size_t stage_bytes = (size_t)n * stage_cap * (sizeof(uint32_t) + sizeof(int32_t));
    uint8_t* blk = nullptr;
    uint8_t* stage = nullptr;
    HIP_CHECK(hipMallocAsync((void**)&blk, bytes, st));
    if (hipMallocAsync((void**)&stage, stage_bytes, st) != hipSuccess) {
        (void)hipFreeAsync(blk, st);
        return fail(CBX_E_HIP, "cbx_frame_rdw: staging allocation of " + std::to_string(stage_bytes) + " bytes failed");
    }
    int64_t* d64 = (int64_t*)blk;
    RdwChunkArgs c{};
    c.entry = d64;
    c.err = d64 + 3 * n;
    int64_t* d_base = d64 + 4 * n;
    unsigned long long* d_first_err = (unsigned long long*)(d64 + 5 * n);   // [0] first error, [1] total
    int64_t* d_block_sums = d64 + 5 * n + 4;
    RdwRange* d_ranges = (RdwRange*)(d_block_sums + nb);
    c.count = (uint32_t*)(d_ranges + ranges.size());
    c.changed = (int32_t*)(c.count + n);   // [round]
    c.ranges = d_ranges; c.n_ranges = (int32_t)ranges.size(); c.chunk = chunk; c.n = n;
    c.stage_off = (uint32_t*)stage;
    c.stage_len = (int32_t*)(stage + (size_t)n * stage_cap * sizeof(uint32_t));
    c.stage_cap = stage_cap;
    if (async) {
        const int r = upload_no_wait(ranges.data(), sizeof(RdwRange) * ranges.size(), d_ranges, st);
        if (r) return r;
    } else {
        HIP_CHECK(hipMemcpyAsync(d_ranges, ranges.data(), sizeof(RdwRange) * ranges.size(), hipMemcpyHostToDevice, st));
    }
    HIP_CHECK(hipMemsetAsync(d_first_err, 0xFF, sizeof(unsigned long long), st));
    RdwArgs a{};
    a.data = d_data; a.n_bytes = n_bytes; a.p = *params;
    c.exit_in = nullptr; c.exit_out = d64 + n;   // exits, updated in place by the fix rounds
    HIP_CHECK(hipMemsetAsync(c.changed, 0, sizeof(int32_t) * (n + 2), st));
    const unsigned wblocks = (unsigned)((n + kRdwWaves - 1) / kRdwWaves);
    // speculation, then the lane-per-chunk walk of chunks of long records (C5's 16 KB roots: 64 chains
    // in flight per wave), then the wave walk of the chunks it hands back (dense ones: C4); env
    // CBX_RDW_LANE_WALK=0: speculation and wave walk in one pass (A/B)
    const char* lw = getenv("CBX_RDW_LANE_WALK");
    const bool lane_walk = !lw || atoi(lw) != 0;
    if (lane_walk) {
        if (getenv("CBX_RDW_SPEC_IN_WAVE")) hipLaunchKernelGGL(rdw_wave_kernel<false>, dim3(wblocks), dim3(kWave * kRdwWaves), 0, st, a, c, 1);
        else hipLaunchKernelGGL(rdw_spec_kernel, dim3(wblocks), dim3(kWave * kRdwWaves), 0, st, a, c);
        hipLaunchKernelGGL(rdw_lane_walk_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, c);
        hipLaunchKernelGGL(rdw_wave_kernel<false>, dim3(wblocks), dim3(kWave * kRdwWaves), 0, st, a, c, 2);
    } else {
        hipLaunchKernelGGL(rdw_wave_kernel<false>, dim3(wblocks), dim3(kWave * kRdwWaves), 0, st, a, c, 0);
    }
    HIP_CHECK(hipGetLastError());
    std::vector<int64_t> dbg_spec;   // env CBX_RDW_DEBUG: speculated vs settled entries (diagnostic)
    if (!async && getenv("CBX_RDW_DEBUG")) {
        dbg_spec.resize(n);
        HIP_CHECK(hipMemcpyAsync(dbg_spec.data(), c.entry, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    // fix rounds until one changes no entry (each round validates at least the next chunk of every
    // range: bounded by the chunk count).  The first kAsyncRounds (async: max_rounds) go out without
    // waiting: a round after one that changed nothing returns at once on the device.
    const int64_t async_rounds = std::min<int64_t>(async && max_rounds > 0 ? max_rounds : 3, n + 1);
    int64_t round = 0;
    hipLaunchKernelGGL(rdw_check_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c);
    for (; round < async_rounds && round <= n; round++)
        hipLaunchKernelGGL(rdw_wave_kernel<true>, dim3(wblocks), dim3(kWave * kRdwWaves), 0, st, a, c, (int32_t)round);
    HIP_CHECK(hipGetLastError());
    if (async) {   // whatever the parallel rounds left unsettled, settled on the device in one pass
        hipLaunchKernelGGL(rdw_settle_kernel, dim3(1), dim3(kWave), 0, st, a, c, (int32_t)(round - 1));
        HIP_CHECK(hipGetLastError());
    } else {
        int32_t last_changed = 0;
        HIP_CHECK(hipMemcpyAsync(&last_changed, c.changed + round - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        for (; last_changed && round <= n + 1; round++) {
            hipLaunchKernelGGL(rdw_wave_kernel<true>, dim3(wblocks), dim3(kWave * kRdwWaves), 0, st, a, c, (int32_t)round);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyAsync(&last_changed, c.changed + round, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
        }
    }
    if (!dbg_spec.empty()) {
        std::vector<int64_t> fin(n);
        HIP_CHECK(hipMemcpyAsync(fin.data(), c.entry, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        int64_t bad = 0;
        for (int64_t k = 0; k < n; k++)
            if (fin[k] != dbg_spec[k] && bad++ < 5)
                fprintf(stderr, "cbx rdw debug: chunk %lld speculated %lld settled %lld\n", (long long)k, (long long)dbg_spec[k],
                        (long long)fin[k]);
        fprintf(stderr, "cbx rdw debug: %lld of %lld speculated entries wrong, %lld rounds\n", (long long)bad, (long long)n,
                (long long)round);
    }
    // record counts -> bases: device exclusive scan of the chunk counts
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, (const uint32_t*)c.count, n,
                       d_block_sums);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, d_block_sums, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, (const uint32_t*)c.count, n,
                       (const int64_t*)d_block_sums, d_base);
    hipLaunchKernelGGL(rdw_place_kernel, dim3((unsigned)((n + kRdwPlaceWaves - 1) / kRdwPlaceWaves)), dim3(kWave * kRdwPlaceWaves),
                       0, st, a, c, (const int64_t*)d_base, d_rec_off, d_rec_len, capacity, d_first_err);
    HIP_CHECK(hipGetLastError());
    if (async) {
        hipLaunchKernelGGL(rdw_state_kernel, dim3(1), dim3(kWave), 0, st, (const unsigned long long*)d_first_err,
                           capacity, d_state);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipFreeAsync(stage, st));
        HIP_CHECK(hipFreeAsync(blk, st));
        return CBX_OK;
    }
    unsigned long long res[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(res, d_first_err, sizeof(res), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipFreeAsync(stage, st));
    HIP_CHECK(hipFreeAsync(blk, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const unsigned long long first_err = res[0];
    const int64_t total = (int64_t)res[1];
    if (first_err != ~0ull) return rdw_error(first_err);
    *n_records = total;
    if (total > capacity) return fail(CBX_E_CAPACITY, "record capacity " + std::to_string(capacity) + " < " + std::to_string(total));
    return CBX_OK;
}

extern "C" int cbx_frame_rdw(const uint8_t* d_data, int64_t n_bytes, const int64_t* seeds, int32_t n_seeds,
                             const cbx_rdw_params* params, int64_t* d_rec_off, int32_t* d_rec_len,
                             int64_t capacity, int64_t* n_records, void* stream) {
    if (!d_data || n_bytes < 0 || !params || !n_records || (n_seeds > 0 && !seeds))
        return fail(CBX_E_ARGUMENT, "cbx_frame_rdw: invalid arguments");
    *n_records = 0;
    return frame_rdw_impl(d_data, n_bytes, seeds, n_seeds, params, d_rec_off, d_rec_len, capacity, n_records, nullptr, 0,
                          (hipStream_t)stream);
}

extern "C" int cbx_frame_rdw_async(const uint8_t* d_data, int64_t n_bytes, const int64_t* seeds, int32_t n_seeds,
                                   const cbx_rdw_params* params, int64_t* d_rec_off, int32_t* d_rec_len,
                                   int64_t capacity, int64_t* d_state, int32_t max_rounds, void* stream) {
    if (!d_data || n_bytes < 0 || !params || !d_state || (n_seeds > 0 && !seeds) || max_rounds < 0)
        return fail(CBX_E_ARGUMENT, "cbx_frame_rdw_async: invalid arguments");
    return frame_rdw_impl(d_data, n_bytes, seeds, n_seeds, params, d_rec_off, d_rec_len, capacity, nullptr, d_state,
                          max_rounds, (hipStream_t)stream);
}

extern "C" int cbx_frame_rdw_state(const int64_t* d_state, int64_t* n_records, void* stream) {
    if (!d_state || !n_records) return fail(CBX_E_ARGUMENT, "cbx_frame_rdw_state: invalid arguments");
    hipStream_t st = (hipStream_t)stream;
    int64_t s[3] = {0, 0, 0};
    HIP_CHECK(hipMemcpyAsync(s, d_state, sizeof(s), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    *n_records = s[0];
    if ((unsigned long long)s[1] != ~0ull) return rdw_error((unsigned long long)s[1]);
    if (s[2] & 1) return fail(CBX_E_CAPACITY, "record capacity < " + std::to_string(s[0]));
    return CBX_OK;
}

namespace {
struct AsyncBlock {   // one hipMallocAsync block, freed (stream-ordered) when the scope ends
    void* p = nullptr;
    hipStream_t st;
    explicit AsyncBlock(hipStream_t s) : st(s) {}
    ~AsyncBlock() { if (p) (void)hipFreeAsync(p, st); }
};
}  // namespace

// Text framing (is_text): cbx_text.h.  Needs d_data readable up to n_bytes; records past n_bytes
// (the reference's zero fill, cbx_text.h) require the caller's buffer to hold zeros up to
// *virtual_bytes (at most n_bytes + record_size + 2).
extern "C" int cbx_frame_text(const uint8_t* d_data, int64_t n_bytes, int32_t record_size, int64_t* d_rec_off,
                              int32_t* d_rec_len, int64_t capacity, int64_t* n_records, int64_t* virtual_bytes,
                              void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!d_data || n_bytes < 0 || record_size < 1 || !n_records || !virtual_bytes || capacity < 0)
        return fail(CBX_E_ARGUMENT, "cbx_frame_text: invalid arguments");
    *n_records = 0;
    *virtual_bytes = 0;
    if (n_bytes == 0) return CBX_OK;   // hasNext is false on an empty stream (TextRecordExtractor.scala:33)
    const int64_t M = (int64_t)record_size + 2;   // maxRecordSize (TextRecordExtractor.scala:28)
    if (record_size > INT32_MAX - 2 || n_bytes / M >= (int64_t)UINT32_MAX - 2)   // per-segment counts are 32-bit
        return fail(CBX_E_ARGUMENT, "cbx_frame_text: record_size too large or too many records per line for one call");
    const int64_t nch = (n_bytes + kTextChunk - 1) / kTextChunk;
    // pass 1: LF counts -> bases -> positions
    auto scan = [&](uint32_t* cnt, int64_t n, int64_t* out, int64_t* sums) {
        const int64_t nb = (n + kScanTile - 1) / kScanTile;
        hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, (const uint32_t*)cnt, n, sums);
        hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, sums, nb);
        hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, (const uint32_t*)cnt, n,
                           (const int64_t*)sums, out);
    };
    auto sums_len = [](int64_t n) { return (n + kScanTile - 1) / kScanTile; };
    // stream-ordered temporaries, each released when its scope ends (every return path)
    AsyncBlock b_cnt(st), b_base(st), b_sums(st), b_lf(st), b_eol(st), b_scnt(st), b_sbase(st), b_big(st), b_sums2(st);
    HIP_CHECK(hipMallocAsync(&b_cnt.p, sizeof(uint32_t) * (nch + 1), st));
    HIP_CHECK(hipMallocAsync(&b_base.p, sizeof(int64_t) * (nch + 1), st));
    HIP_CHECK(hipMallocAsync(&b_sums.p, sizeof(int64_t) * sums_len(nch + 1), st));
    uint32_t* d_cnt = (uint32_t*)b_cnt.p;
    int64_t* d_base = (int64_t*)b_base.p;
    int64_t* d_sums = (int64_t*)b_sums.p;
    HIP_CHECK(hipMemsetAsync(d_cnt + nch, 0, sizeof(uint32_t), st));
    const unsigned cblocks = (unsigned)((nch + 3) / 4);   // 4 waves per block, one chunk each
    hipLaunchKernelGGL(text_lf_kernel, dim3(cblocks), dim3(256), 0, st, d_data, n_bytes, nch, 0, d_cnt,
                       (const int64_t*)nullptr, (int64_t*)nullptr);
    scan(d_cnt, nch + 1, d_base, d_sums);
    int64_t n_lf = 0;
    HIP_CHECK(hipMemcpyAsync(&n_lf, d_base + nch, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipMallocAsync(&b_lf.p, sizeof(int64_t) * (n_lf + 1), st));
    int64_t* d_lf = (int64_t*)b_lf.p;
    hipLaunchKernelGGL(text_lf_kernel, dim3(cblocks), dim3(256), 0, st, d_data, n_bytes, nch, 1, d_cnt,
                       (const int64_t*)d_base, d_lf);
    HIP_CHECK(hipGetLastError());
    // line-ending length before every segment (scan of per-segment maps, cbx_text.h)
    const int64_t n_eol_tiles = (n_lf + 1 + kEolTile - 1) / kEolTile;
    HIP_CHECK(hipMallocAsync(&b_eol.p, n_eol_tiles + n_lf + 1 + 16, st));
    uint8_t* d_eol = (uint8_t*)b_eol.p;   // [n_eol_tiles] tile maps | [n_lf + 1] f before each segment
    uint8_t* d_fb = d_eol + n_eol_tiles;
    hipLaunchKernelGGL(text_eol_kernel, dim3((unsigned)n_eol_tiles), dim3(kEolThreads), 0, st, d_data, (const int64_t*)d_lf,
                       n_lf, M, 0, d_eol, (const uint8_t*)nullptr, (uint8_t*)nullptr);
    hipLaunchKernelGGL(text_eol_scan_kernel, dim3(1), dim3(1), 0, st, d_eol, n_eol_tiles);
    hipLaunchKernelGGL(text_eol_kernel, dim3((unsigned)n_eol_tiles), dim3(kEolThreads), 0, st, d_data, (const int64_t*)d_lf,
                       n_lf, M, 2, (uint8_t*)nullptr, (const uint8_t*)d_eol, d_fb);
    HIP_CHECK(hipGetLastError());
    // pass 2: records per segment (n_lf line-ended segments + the tail) -> bases -> records
    const int64_t nseg = n_lf + 1;
    HIP_CHECK(hipMallocAsync(&b_scnt.p, sizeof(uint32_t) * (nseg + 1), st));
    HIP_CHECK(hipMallocAsync(&b_sbase.p, sizeof(int64_t) * (nseg + 2), st));
    HIP_CHECK(hipMallocAsync(&b_big.p, sizeof(unsigned long long) * (1 + kBigSegCap), st));
    HIP_CHECK(hipMallocAsync(&b_sums2.p, sizeof(int64_t) * sums_len(nseg + 1), st));
    uint32_t* d_scnt = (uint32_t*)b_scnt.p;
    int64_t* d_sbase = (int64_t*)b_sbase.p;   // [nseg + 1] bases, then the tail's final start
    unsigned long long* d_big = (unsigned long long*)b_big.p;   // [0] count of segments with many forced records, [1..] their indices
    d_sums = (int64_t*)b_sums2.p;
    HIP_CHECK(hipMemsetAsync(d_big, 0, sizeof(unsigned long long), st));
    HIP_CHECK(hipMemsetAsync(d_scnt + nseg, 0, sizeof(uint32_t), st));
    const unsigned sblocks = (unsigned)((nseg + 255) / 256);
    hipLaunchKernelGGL(text_seg_kernel, dim3(sblocks), dim3(256), 0, st, d_data, n_bytes, (const int64_t*)d_lf, n_lf,
                       M, 0, d_scnt, (const int64_t*)nullptr, (int64_t*)nullptr, (int32_t*)nullptr, d_sbase + nseg + 1,
                       d_big, 0, (const uint8_t*)d_fb);
    scan(d_scnt, nseg + 1, d_sbase, d_sums);
    int64_t hv[2] = {0, 0};   // body records, tail final start
    unsigned long long n_big = 0;
    HIP_CHECK(hipMemcpyAsync(hv, d_sbase + nseg, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(&n_big, d_big, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const int32_t big_ok = n_big > 0 && n_big <= kBigSegCap;
    const int64_t body = hv[0], tail_start = hv[1];
    int rc = CBX_OK;
    if (body > capacity) {
        *n_records = body;   // required size (at least; the tail record may add one)
        rc = fail(CBX_E_CAPACITY, "record capacity " + std::to_string(capacity) + " < " + std::to_string(body));
    } else {
        hipLaunchKernelGGL(text_seg_kernel, dim3(sblocks), dim3(256), 0, st, d_data, n_bytes, (const int64_t*)d_lf, n_lf,
                           M, 1, d_scnt, (const int64_t*)d_sbase, d_rec_off, d_rec_len, (int64_t*)nullptr, d_big, big_ok,
                           (const uint8_t*)d_fb);
        HIP_CHECK(hipGetLastError());
        if (big_ok) {
            hipLaunchKernelGGL(text_forced_kernel, dim3((unsigned)n_big, 64), dim3(256), 0, st, d_data, n_bytes,
                               (const int64_t*)d_lf, n_lf, M, (const unsigned long long*)d_big, (const int64_t*)d_sbase,
                               d_rec_off, d_rec_len, (const uint8_t*)d_fb);
            HIP_CHECK(hipGetLastError());
        }
    }
    if (rc) { HIP_CHECK(hipStreamSynchronize(st)); return rc; }
    // the virtual length: the window that first reached past the data (record start s_k, the
    // first with s_k + M >= n_bytes) was marked full (ensureBytesRead, :98-107)
    const int64_t k = std::min<int64_t>(body, M + 1);
    std::vector<int64_t> last(k);
    if (k > 0) HIP_CHECK(hipMemcpyAsync(last.data(), d_rec_off + (body - k), sizeof(int64_t) * k, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int64_t s_k = -1;
    for (int64_t i = 0; i < k && s_k < 0; i++)
        if (last[i] + M >= n_bytes && last[i] < n_bytes) s_k = last[i];
    if (s_k < 0 && tail_start < n_bytes && tail_start + M >= n_bytes) s_k = tail_start;
    const int64_t vlen = s_k >= 0 ? std::max(n_bytes, s_k + M) : n_bytes;
    int64_t total = body;
    if (tail_start < vlen) {   // the rest of the stream: the last record (:62-66, hasNext :33)
        if (body + 1 > capacity) {
            *n_records = body + 1;
            return fail(CBX_E_CAPACITY, "record capacity " + std::to_string(capacity) + " < " + std::to_string(body + 1));
        }
        const int64_t h_off = tail_start;
        const int32_t h_len = (int32_t)(vlen - tail_start);
        HIP_CHECK(hipMemcpyAsync(d_rec_off + body, &h_off, sizeof(int64_t), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(d_rec_len + body, &h_len, sizeof(int32_t), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));
        total++;
    }
    *n_records = total;
    *virtual_bytes = vlen;
    return CBX_OK;
}

// ---------------------------------------------------------------------------------------------
// Variable-length record streams: record selection, selected decode (+ Seg_IdN columns), sparse
// index (cbx_select.h).  Temporaries are stream-ordered allocations released on every exit path.
// ---------------------------------------------------------------------------------------------
namespace {

// exclusive scan of n uint32 values into int64 out (cbx_kernels.hip scan passes); sums: nb int64
void device_scan(const uint32_t* in, int64_t n, int64_t* out, int64_t* sums, hipStream_t st) {
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, sums);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, sums, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, (const int64_t*)sums, out);
}

int64_t scan_sums_len(int64_t n) { return (n + kScanTile - 1) / kScanTile; }

unsigned blocks_for(int64_t n, int threads) { return (unsigned)std::max<int64_t>(1, (n + threads - 1) / threads); }
}  // namespace

extern "C" int cbx_select_records(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                                  const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset,
                                  const cbx_index_entry* entries, int32_t n_entries, cbx_selection* out,
                                  int64_t* n_selected, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!P || !out || !n_selected || n_rec < 0 || start_offset < 0 || (n_rec > 0 && (!d_data || !d_rec_off || !d_rec_len)) ||
        (n_entries > 0 && !entries) || n_entries < 0)
        return fail(CBX_E_ARGUMENT, "cbx_select_records: invalid arguments");
    *n_selected = 0;
    const int L = P->opts.has_segments ? P->opts.segments.n_levels : 0;
    if (n_rec > 0 && (!out->rec_off || !out->rec_len || !out->record_id || !out->segment || (L > 0 && !out->seg_state)))
        return fail(CBX_E_ARGUMENT, "cbx_select_records: output arrays required");
    if (n_rec == 0) return CBX_OK;
    std::vector<int64_t> h_from, h_rid, h_end;
    if (n_entries == 0) { h_from.push_back(0); h_rid.push_back(0); h_end.push_back(-1); }
    for (int e = 0; e < n_entries; e++) {
        if (e > 0 && entries[e].offset_from < entries[e - 1].offset_from)
            return fail(CBX_E_ARGUMENT, "cbx_select_records: entries must be in file order");
        h_from.push_back(entries[e].offset_from);
        h_rid.push_back(entries[e].record_index);
        h_end.push_back(entries[e].offset_to);
    }
    const int n_ent = (int)h_from.size();
    const int64_t n_runs = (n_rec + kSelRun - 1) / kSelRun;
    const int64_t nb = scan_sums_len(n_runs + 1);
    // block: ent_from | ent_rid | ent_end | ent_first | base (n_runs + 1) | sums (nb) | SegSum (n_runs) | counts | key (n_rec)
    const size_t off_sum = sizeof(int64_t) * (4 * (size_t)n_ent + (n_runs + 1) + nb);
    const size_t off_cnt = off_sum + sizeof(SegSum) * n_runs;
    const size_t off_key = off_cnt + sizeof(uint32_t) * (n_runs + 1);
    AsyncBlock blk(st);
    HIP_CHECK(hipMallocAsync(&blk.p, off_key + n_rec + 64, st));
    int64_t* d64 = (int64_t*)blk.p;
    int64_t* ent_from = d64;
    int64_t* ent_rid = d64 + n_ent;
    int64_t* ent_end = d64 + 2 * n_ent;
    int64_t* ent_first = d64 + 3 * n_ent;
    int64_t* base = d64 + 4 * n_ent;
    int64_t* sums = base + n_runs + 1;
    SegSum* runs = (SegSum*)((uint8_t*)blk.p + off_sum);
    uint32_t* counts = (uint32_t*)((uint8_t*)blk.p + off_cnt);
    int8_t* key = (int8_t*)((uint8_t*)blk.p + off_key);
    HIP_CHECK(hipMemcpyAsync(ent_from, h_from.data(), sizeof(int64_t) * n_ent, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(ent_rid, h_rid.data(), sizeof(int64_t) * n_ent, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(ent_end, h_end.data(), sizeof(int64_t) * n_ent, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(counts + n_runs, 0, sizeof(uint32_t), st));
    SelArgs a{};
    a.data = d_data; a.n_bytes = n_bytes; a.rec_off = d_rec_off; a.rec_len = d_rec_len; a.n = n_rec;
    a.start_off = start_offset; a.L = L;
    a.m = P->opts.has_segments ? (const CBX_CONST cbx_segment_map*)P->d_segmap : nullptr;
    a.lut = P->d_lut;
    a.fields = (const CBX_CONST Field*)P->d_fields;
    a.ent_first = ent_first; a.ent_rid = ent_rid; a.ent_end = ent_end; a.n_ent = n_ent; a.key = key;
    a.footer = out->footer_bytes;
    hipLaunchKernelGGL(sel_entry_first_kernel, dim3(blocks_for(n_ent, 64)), dim3(64), 0, st, d_rec_off, n_rec,
                       (const int64_t*)ent_from, n_ent, ent_first);
    hipLaunchKernelGGL(sel_key_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(sel_sum_kernel, dim3(blocks_for(n_runs, 256)), dim3(256), 0, st, a, runs, n_runs);
    hipLaunchKernelGGL(sel_scan_kernel, dim3(1), dim3(kSelScanThreads), 0, st, runs, n_runs, L);
    hipLaunchKernelGGL(sel_emit_kernel, dim3(blocks_for(n_runs, 256)), dim3(256), 0, st, a, (const SegSum*)runs, n_runs, 0,
                       counts, (const int64_t*)nullptr, *out);
    device_scan(counts, n_runs + 1, base, sums, st);
    hipLaunchKernelGGL(sel_emit_kernel, dim3(blocks_for(n_runs, 256)), dim3(256), 0, st, a, (const SegSum*)runs, n_runs, 1,
                       counts, (const int64_t*)base, *out);
    HIP_CHECK(hipGetLastError());
    int64_t total = 0;
    HIP_CHECK(hipMemcpyAsync(&total, base + n_runs, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    *n_selected = total;
    return CBX_OK;
}

namespace cbx {
// Utf8 layout: int64 offsets of a scanned column narrowed to Arrow's int32 (overflow -> status)
__global__ void narrow_offsets_kernel(const int64_t* in, int64_t n, int32_t* out, int32_t* status) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t v = in[i];
    if (v > 0x7fffffffll) atomicOr(status, 1);
    out[i] = (int32_t)v;
}
}  // namespace cbx

extern "C" int cbx_decode_selected(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const cbx_selection* sel,
                                   int64_t n_rec, int32_t start_offset, cbx_column* columns, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!P || !sel || (n_rec > 0 && (!sel->rec_off || !sel->rec_len || !sel->record_id || !sel->segment)) || n_bytes < 0)
        return fail(CBX_E_ARGUMENT, "cbx_decode_selected: invalid arguments");
    const int L = P->opts.has_segments ? P->opts.segments.n_levels : 0;
    if (n_rec > 0 && !P->segid_cols.empty() && !sel->seg_state)
        return fail(CBX_E_ARGUMENT, "cbx_decode_selected: seg_state required for Seg_Id columns");
    CallShape c{d_data, n_bytes, sel->rec_off, sel->rec_len, n_rec, 0, start_offset, 0};
    c.rec_id = sel->record_id;
    c.rec_seg = sel->segment;
    c.file_id = sel->file_id;
    int r = decode_common(P, c, columns, nullptr, st);
    if (r) return r;
    // Seg_IdN columns (slot 0 of each string column): lengths -> scanned offsets -> bytes
    for (int l : P->segid_cols) {
        const int ci = P->opts.segments.level_column[l];
        const cbx_column& col = columns[ci];
        if (P->view) {   // views written where the values are made: no scan
            if (n_rec == 0) continue;
            SegIdArgs g{};
            g.state = sel->seg_state; g.n = n_rec; g.L = L; g.level = l; g.file_id = sel->file_id;
            g.prefix_len = P->opts.segments.prefix_len;
            g.m = (const CBX_CONST cbx_segment_map*)P->d_segmap;
            const int64_t tb = view_tile_bytes(P, ci);
            const int64_t pitch = (n_rec + kWave - 1) / kWave * kWave;
            hipLaunchKernelGGL(segid_view_kernel, dim3(blocks_for(pitch, 256)), dim3(256), 0, st, g, (u32x4*)col.values,
                               col.data, tb, view_tiles_per_buf(tb), col.validity, pitch);
            HIP_CHECK(hipGetLastError());
            continue;
        }
        if (n_rec == 0) {
            HIP_CHECK(hipMemsetAsync(col.offsets, 0, P->packed ? sizeof(int32_t) : sizeof(int64_t), st));
            if (col.data_sizes) HIP_CHECK(hipMemsetAsync(col.data_sizes, 0, sizeof(int64_t), st));
            continue;
        }
        AsyncBlock blk(st);
        const int64_t nb = scan_sums_len(n_rec + 1);
        // (Utf8 layout: int64 offsets scanned into the block, narrowed to the column's int32 after)
        const int64_t n64 = P->packed ? n_rec + 1 : 0;
        HIP_CHECK(hipMallocAsync(&blk.p, sizeof(int64_t) * (nb + n64) + sizeof(uint32_t) * (n_rec + 1) + 16, st));
        int64_t* sums = (int64_t*)blk.p;
        int64_t* offs64 = P->packed ? sums + nb : (int64_t*)col.offsets;
        uint32_t* len = (uint32_t*)(sums + nb + n64);
        SegIdArgs g{};
        g.state = sel->seg_state; g.n = n_rec; g.L = L; g.level = l; g.file_id = sel->file_id;
        g.prefix_len = P->opts.segments.prefix_len;
        g.m = (const CBX_CONST cbx_segment_map*)P->d_segmap;
        hipLaunchKernelGGL(segid_len_kernel, dim3(blocks_for(n_rec + 1, 256)), dim3(256), 0, st, g, len);
        device_scan(len, n_rec + 1, offs64, sums, st);
        hipLaunchKernelGGL(segid_write_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, g, offs64,
                           col.data, col.data_capacity, col.validity, P->d_status);
        if (P->packed)
            hipLaunchKernelGGL(narrow_offsets_kernel, dim3(blocks_for(n_rec + 1, 256)), dim3(256), 0, st,
                               (const int64_t*)offs64, n_rec + 1, (int32_t*)col.offsets, P->d_status);
        if (col.data_sizes)
            HIP_CHECK(hipMemcpyAsync(col.data_sizes, offs64 + n_rec, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
        HIP_CHECK(hipGetLastError());
    }
    return CBX_OK;
}

namespace cbx {
__global__ void idx_gather_kernel(const int64_t* idx, int64_t k, const int64_t* rec_off, int32_t header_bytes,
                                  int32_t has_header, int64_t* from, int64_t* recno) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    from[j] = rec_off[idx[j]] - header_bytes;
    recno[j] = idx[j] + has_header;
}
__global__ void idx_rank_kernel(const int64_t* ranks, int64_t k, const int64_t* cand, int64_t* idx) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < k) idx[j] = cand[ranks[j]];
}
}  // namespace cbx

extern "C" int cbx_sparse_index(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                                const int32_t* d_rec_len, int64_t n_rec, const cbx_index_params* prm,
                                cbx_index_entry* entries, int64_t capacity, int64_t* n_entries, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!P || !prm || !n_entries || capacity < 0 || (capacity > 0 && !entries) || n_rec < 0 ||
        (n_rec > 0 && (!d_rec_off || !d_rec_len || !d_data)) || (prm->header_bytes != 0 && prm->header_bytes != 4) ||
        prm->records_per_entry < 0 || (prm->records_per_entry == 0 && prm->bytes_per_entry <= 0) || prm->start_bytes < 0)
        return fail(CBX_E_ARGUMENT, "cbx_sparse_index: invalid arguments");
    const int64_t rho = prm->start_bytes;   // bytesInChunk at the first record (an entry already cut)
    *n_entries = 0;
    bool root_keys = false;   // level-0 keys: segment_id_level0 / segment_id_root, or a hierarchical file's root ids
    for (int k = 0; P->opts.has_segments && k < P->opts.segments.n_keys; k++) root_keys |= P->opts.segments.key_level[k] == 0;
    const bool hier = prm->hierarchical && root_keys;
    if (prm->hierarchical && !hier) return fail(CBX_E_ARGUMENT, "cbx_sparse_index: hierarchical cuts need level-0 segment keys in the plan");
    const int64_t hh = prm->has_file_header ? 1 : 0;
    std::vector<int64_t> from{0}, recno{0};   // the first mandatory entry
    if (n_rec > 0) {
        const int64_t nb = scan_sums_len(n_rec + 1);
        AsyncBlock blk(st);
        // flags (n + 1 u32) | excl (n + 1) | cand (n) | sums (nb) | key (n i8)
        const size_t off_excl = ((sizeof(uint32_t) * (n_rec + 1)) + 15) & ~(size_t)15;
        const size_t off_cand = off_excl + sizeof(int64_t) * (n_rec + 1);
        const size_t off_sums = off_cand + sizeof(int64_t) * n_rec;
        const size_t off_key = off_sums + sizeof(int64_t) * nb;
        HIP_CHECK(hipMallocAsync(&blk.p, off_key + n_rec + 64, st));
        uint8_t* b = (uint8_t*)blk.p;
        uint32_t* flag = (uint32_t*)b;
        int64_t* excl = (int64_t*)(b + off_excl);
        int64_t* cand = (int64_t*)(b + off_cand);
        int64_t* sums = (int64_t*)(b + off_sums);
        int8_t* key = (int8_t*)(b + off_key);
        IdxArgs ia{};
        ia.rec_off = d_rec_off; ia.rec_len = d_rec_len; ia.n = n_rec; ia.n_bytes = n_bytes;
        ia.header_bytes = prm->header_bytes; ia.has_header = (int32_t)hh;
        ia.m = (const CBX_CONST cbx_segment_map*)P->d_segmap;
        if (hier) {
            // IndexGenerator.getSegmentId reads the field without the record start offset (:153-156)
            SelArgs sa{};
            sa.data = d_data; sa.n_bytes = n_bytes; sa.rec_off = d_rec_off; sa.rec_len = d_rec_len; sa.n = n_rec;
            sa.start_off = 0; sa.m = ia.m; sa.lut = P->d_lut; sa.fields = (const CBX_CONST Field*)P->d_fields; sa.key = key;
            hipLaunchKernelGGL(sel_key_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, sa);
            ia.key = key;
        }
        hipLaunchKernelGGL(idx_flag_kernel, dim3(blocks_for(n_rec + 1, 256)), dim3(256), 0, st, ia, flag);
        device_scan(flag, n_rec + 1, excl, sums, st);
        hipLaunchKernelGGL(idx_compact_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, ia, (const uint32_t*)flag,
                           (const int64_t*)excl, cand);
        HIP_CHECK(hipGetLastError());
        int64_t n_cand = 0;
        HIP_CHECK(hipMemcpyAsync(&n_cand, excl + n_rec, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        std::vector<int64_t> split_idx;         // framed index of every split (host list) ...
        int64_t* d_split = nullptr;              // ... or device list of n_split
        int64_t n_split = 0;
        AsyncBlock blk2(st);
        if (n_cand > 0) {
            const int64_t N = prm->records_per_entry, S = prm->bytes_per_entry;
            if (N > 0 && !hier) {
                // every valid record but the stream's last is a candidate: splits at numbers k N
                for (int64_t k = 1;; k++) {
                    const int64_t i = k * N - hh;
                    if (i >= n_cand) break;
                    split_idx.push_back(i);
                }
            } else if (N == 0 && prm->subtract_size) {
                int64_t last = 0;
                HIP_CHECK(hipMemcpyAsync(&last, cand + n_cand - 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
                int64_t last_off = 0, first_cand = 0;
                HIP_CHECK(hipStreamSynchronize(st));
                HIP_CHECK(hipMemcpyAsync(&last_off, d_rec_off + last, sizeof(int64_t), hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipMemcpyAsync(&first_cand, cand, sizeof(int64_t), hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
                // thresholds j S - rho (bytesInChunk = prefix + rho - cuts S), j = 1..K
                const int64_t K = (last_off - prm->header_bytes + rho) / S + 1;
                HIP_CHECK(hipMallocAsync(&blk2.p, sizeof(int64_t) * (2 * K + 2), st));
                int64_t* rj = (int64_t*)blk2.p;
                hipLaunchKernelGGL(idx_size_kernel, dim3(blocks_for(K, 256)), dim3(256), 0, st, ia, (const int64_t*)cand, n_cand,
                                   S, K, rho, rj);
                HIP_CHECK(hipGetLastError());
                std::vector<int64_t> h(K);
                HIP_CHECK(hipMemcpyAsync(h.data(), rj, sizeof(int64_t) * K, hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
                // rank_k = k + max(rank_0, max_{j<=k}(r_j - j)), rank_0 = 0 iff candidate 0 is record number 0
                int64_t mx = (hh == 0 && first_cand == 0) ? 0 : -1;
                std::vector<int64_t> ranks;
                for (int64_t k = 1; k <= K; k++) {
                    mx = std::max(mx, h[k - 1]);
                    const int64_t rk = k + mx;
                    if (rk >= n_cand) break;
                    ranks.push_back(rk);
                }
                n_split = (int64_t)ranks.size();
                if (n_split > 0) {
                    int64_t* d_ranks = rj;                 // reuse: K >= n_split
                    d_split = rj + K + 1;                  // needs n_split <= K + 1 entries
                    HIP_CHECK(hipMemcpyAsync(d_ranks, ranks.data(), sizeof(int64_t) * n_split, hipMemcpyHostToDevice, st));
                    hipLaunchKernelGGL(idx_rank_kernel, dim3(blocks_for(n_split, 256)), dim3(256), 0, st, (const int64_t*)d_ranks,
                                       n_split, (const int64_t*)cand, d_split);
                    HIP_CHECK(hipGetLastError());
                }
            } else {
                // chain walk by one wave: records (hierarchical) or size with the split reset
                HIP_CHECK(hipMallocAsync(&blk2.p, sizeof(int64_t) * (n_cand + 2), st));
                d_split = (int64_t*)blk2.p + 1;
                hipLaunchKernelGGL(idx_walk_kernel, dim3(1), dim3(64), 0, st, ia, (const int64_t*)cand, n_cand, N > 0 ? 0 : 2, N,
                                   S, N > 0 ? 0 : rho, d_split, n_cand, (int64_t*)blk2.p);
                HIP_CHECK(hipGetLastError());
                HIP_CHECK(hipMemcpyAsync(&n_split, blk2.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
            }
        }
        if (!split_idx.empty()) {
            n_split = (int64_t)split_idx.size();
            HIP_CHECK(hipMallocAsync(&blk2.p, sizeof(int64_t) * n_split, st));
            d_split = (int64_t*)blk2.p;
            HIP_CHECK(hipMemcpyAsync(d_split, split_idx.data(), sizeof(int64_t) * n_split, hipMemcpyHostToDevice, st));
        }
        if (n_split > 0) {
            AsyncBlock blk3(st);
            HIP_CHECK(hipMallocAsync(&blk3.p, sizeof(int64_t) * 2 * n_split, st));
            int64_t* d_from = (int64_t*)blk3.p;
            int64_t* d_recno = d_from + n_split;
            hipLaunchKernelGGL(idx_gather_kernel, dim3(blocks_for(n_split, 256)), dim3(256), 0, st, (const int64_t*)d_split,
                               n_split, d_rec_off, prm->header_bytes, (int32_t)hh, d_from, d_recno);
            HIP_CHECK(hipGetLastError());
            from.resize(1 + n_split);
            recno.resize(1 + n_split);
            HIP_CHECK(hipMemcpyAsync(from.data() + 1, d_from, sizeof(int64_t) * n_split, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipMemcpyAsync(recno.data() + 1, d_recno, sizeof(int64_t) * n_split, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
        }
    }
    const int64_t n = (int64_t)from.size();
    *n_entries = n;
    if (n > capacity) return fail(CBX_E_CAPACITY, "index capacity " + std::to_string(capacity) + " < " + std::to_string(n));
    for (int64_t k = 0; k < n; k++) {
        entries[k].offset_from = from[k];
        entries[k].offset_to = k + 1 < n ? from[k + 1] : -1;
        entries[k].record_index = recno[k];
        entries[k].file_id = prm->file_id;
        entries[k].reserved = 0;
    }
    return CBX_OK;
}

// ---------------------------------------------------------------------------------------------
// Hierarchical records (cbx_hier.h): table rows + parent rows, list offsets per child table.
// ---------------------------------------------------------------------------------------------
extern "C" int cbx_hier_select(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                               const int32_t* d_rec_len, int64_t n_rec, const cbx_hier_params* prm, cbx_selection* out,
                               int64_t* d_parent_row, int64_t* table_rows, int64_t* n_rows, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!P || !prm || !out || !n_rows || !table_rows || n_rec < 0 || n_bytes < 0 ||
        (n_rec > 0 && (!d_data || !d_rec_off || !d_rec_len || !d_parent_row || !out->rec_off || !out->rec_len ||
                       !out->record_id || !out->segment)))
        return fail(CBX_E_ARGUMENT, "cbx_hier_select: invalid arguments");
    if (!P->opts.has_segments) return fail(CBX_E_ARGUMENT, "cbx_hier_select: the plan has no segment map");
    const int S = prm->n_segments;
    if (S < 1 || S > kHierMaxSeg) return fail(CBX_E_UNSUPPORTED, "cbx_hier_select: 1 to 16 segments");
    if (prm->root_segment < 0 || prm->root_segment >= S || prm->parent[prm->root_segment] != -1)
        return fail(CBX_E_ARGUMENT, "cbx_hier_select: bad root segment");
    HierArgs a{};
    a.n_seg = S;
    a.start_off = prm->start_offset;
    a.root = prm->root_segment;
    for (int s = 0; s < kHierMaxSeg; s++) { a.parent[s] = -1; a.anc[s] = 0; }
    for (int s = 0; s < S; s++) {
        const int p = prm->parent[s];
        if (s != a.root && (p < 0 || p >= S || p == s)) return fail(CBX_E_ARGUMENT, "cbx_hier_select: bad parent segment");
        a.parent[s] = s == a.root ? -1 : p;
    }
    for (int s = 0; s < S; s++) {   // every chain reaches the root; anc = strict non-root ancestors of the parent
        if (s == a.root) continue;
        int d = 0;
        for (int q = a.parent[s]; q != a.root; q = a.parent[q]) {
            if (q < 0 || ++d > S) return fail(CBX_E_ARGUMENT, "cbx_hier_select: a segment does not reach the root");
            if (q != a.parent[s]) a.anc[s] |= 1u << q;
        }
    }
    *n_rows = 0;
    for (int t = 0; t <= S; t++) table_rows[t] = 0;
    if (n_rec == 0) return CBX_OK;
    if (prm->flags & 1) {
        // the general walk (several segment ids per segment with children): one thread per
        // hierarchical record, rows counted, scanned, then written; a record may sit under several
        // parents, so the rows can outnumber the records -- CBX_E_CAPACITY (with *n_rows and
        // table_rows set) when they do not fit the n_rec rows the outputs hold
        const int T = S + 1;
        const size_t o_key = ((size_t)n_rec + 15) & ~(size_t)15;
        const size_t o_flag = (o_key + (size_t)n_rec + 15) & ~(size_t)15;
        const size_t o_excl = (o_flag + 4 * (size_t)(n_rec + 1) + 15) & ~(size_t)15;
        const size_t o_sums = o_excl + 8 * (size_t)(n_rec + 1);
        const int64_t nb0 = scan_sums_len(n_rec + 1);
        AsyncBlock blk(st);
        HIP_CHECK(hipMallocAsync(&blk.p, o_sums + 8 * (size_t)nb0 + 64, st));
        uint8_t* b = (uint8_t*)blk.p;
        a.data = d_data; a.rec_off = d_rec_off; a.rec_len = d_rec_len; a.n = n_rec;
        a.m = (const CBX_CONST cbx_segment_map*)P->d_segmap;
        a.lut = P->d_lut;
        a.fields = (const CBX_CONST Field*)P->d_fields;
        a.type = (int8_t*)b; a.key = (int8_t*)(b + o_key);
        uint32_t* flag = (uint32_t*)(b + o_flag);
        int64_t* excl = (int64_t*)(b + o_excl);
        hipLaunchKernelGGL(hier_type_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, a);
        hipLaunchKernelGGL(hier_root_flag_kernel, dim3(blocks_for(n_rec + 1, 256)), dim3(256), 0, st, a, flag);
        device_scan(flag, n_rec + 1, excl, (int64_t*)(b + o_sums), st);
        int64_t G = 0;
        HIP_CHECK(hipMemcpyAsync(&G, excl + n_rec, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        if (G == 0) return CBX_OK;   // no root record: no hierarchical record
        const int64_t n_cnt = (int64_t)T * G;
        const int64_t nb = scan_sums_len(n_cnt + 1);
        const size_t o_cnt = ((size_t)8 * G + 15) & ~(size_t)15;
        const size_t o_base = (o_cnt + 4 * (size_t)(n_cnt + 1) + 15) & ~(size_t)15;
        const size_t o_s2 = o_base + 8 * (size_t)(n_cnt + 1);
        AsyncBlock blk2(st);
        HIP_CHECK(hipMallocAsync(&blk2.p, o_s2 + 8 * (size_t)nb + 64, st));
        uint8_t* b2 = (uint8_t*)blk2.p;
        int64_t* root_pos = (int64_t*)b2;
        uint32_t* cnt = (uint32_t*)(b2 + o_cnt);
        int64_t* base = (int64_t*)(b2 + o_base);
        hipLaunchKernelGGL(hier_root_pos_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, a, (const int64_t*)excl, root_pos);
        HIP_CHECK(hipMemsetAsync(cnt + n_cnt, 0, sizeof(uint32_t), st));
        hipLaunchKernelGGL(hier_walk_kernel, dim3(blocks_for(G, 64)), dim3(64), 0, st, a, (const int64_t*)root_pos, G, 0, cnt,
                           (const int64_t*)nullptr, prm->first_record_id, *out, d_parent_row);
        device_scan(cnt, n_cnt + 1, base, (int64_t*)(b2 + o_s2), st);
        std::vector<int64_t> tb(T + 1);
        for (int t = 0; t < T; t++)
            HIP_CHECK(hipMemcpyAsync(&tb[t], base + (int64_t)t * G, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipMemcpyAsync(&tb[T], base + n_cnt, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        for (int t = 0; t < T; t++) table_rows[t] = tb[t + 1] - tb[t];
        *n_rows = tb[T];
        if (tb[T] > (prm->row_capacity > 0 ? prm->row_capacity : n_rec)) return fail(CBX_E_CAPACITY, "cbx_hier_select: the rows (records under several parents) "
                                                       "outnumber the output capacity; call again with n_rows rows");
        hipLaunchKernelGGL(hier_walk_kernel, dim3(blocks_for(G, 64)), dim3(64), 0, st, a, (const int64_t*)root_pos, G, 1, cnt,
                           (const int64_t*)base, prm->first_record_id, *out, d_parent_row);
        HIP_CHECK(hipGetLastError());
        return CBX_OK;
    }
    const int64_t n_blk = (n_rec + kHierTile - 1) / kHierTile;   // last-position blocks
    const int64_t n_eb = (n_rec + 255) / 256;                     // compaction blocks
    const int64_t n_cnt = (int64_t)(S + 1) * n_eb;
    const int64_t nb = scan_sums_len(n_cnt + 1);
    // type, st, tab (n each) | par, row_of (n int64) | blk_lp (n_blk x 16) | cnt (n_cnt + 1 u32) | base (n_cnt + 1) | sums
    const size_t o_par = ((3 * (size_t)n_rec) + 15) & ~(size_t)15;
    const size_t o_row = o_par + 8 * (size_t)n_rec;
    const size_t o_lp = o_row + 8 * (size_t)n_rec;
    const size_t o_cnt = o_lp + 8 * (size_t)n_blk * kHierMaxSeg;
    const size_t o_base = (o_cnt + 4 * (size_t)(n_cnt + 1) + 15) & ~(size_t)15;
    const size_t o_sums = o_base + 8 * (size_t)(n_cnt + 1);
    AsyncBlock blk(st);
    HIP_CHECK(hipMallocAsync(&blk.p, o_sums + 8 * (size_t)nb + 64, st));
    uint8_t* b = (uint8_t*)blk.p;
    a.data = d_data; a.rec_off = d_rec_off; a.rec_len = d_rec_len; a.n = n_rec;
    a.m = (const CBX_CONST cbx_segment_map*)P->d_segmap;
    a.lut = P->d_lut;
    a.fields = (const CBX_CONST Field*)P->d_fields;
    a.type = (int8_t*)b; a.st = (int8_t*)b + n_rec; a.tab = (int8_t*)b + 2 * n_rec;
    a.par = (int64_t*)(b + o_par); a.row_of = (int64_t*)(b + o_row);
    int64_t* blk_lp = (int64_t*)(b + o_lp);
    uint32_t* cnt = (uint32_t*)(b + o_cnt);
    int64_t* base = (int64_t*)(b + o_base);
    int64_t* sums = (int64_t*)(b + o_sums);
    HIP_CHECK(hipMemsetAsync(cnt + n_cnt, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(hier_type_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(hier_last_kernel, dim3((unsigned)n_blk), dim3(kHierThreads), 0, st, a, 0, blk_lp);
    hipLaunchKernelGGL(hier_lp_scan_kernel, dim3(1), dim3(kHierThreads), 0, st, blk_lp, n_blk, (int32_t)S);
    hipLaunchKernelGGL(hier_last_kernel, dim3((unsigned)n_blk), dim3(kHierThreads), 0, st, a, 1, blk_lp);
    hipLaunchKernelGGL(hier_chase_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(hier_emit_kernel, dim3((unsigned)n_eb), dim3(256), 0, st, a, 0, n_eb, cnt, (const int64_t*)nullptr,
                       prm->first_record_id, *out);
    device_scan(cnt, n_cnt + 1, base, sums, st);
    hipLaunchKernelGGL(hier_emit_kernel, dim3((unsigned)n_eb), dim3(256), 0, st, a, 1, n_eb, cnt, (const int64_t*)base,
                       prm->first_record_id, *out);
    hipLaunchKernelGGL(hier_parent_kernel, dim3(blocks_for(n_rec, 256)), dim3(256), 0, st, a, d_parent_row);
    HIP_CHECK(hipGetLastError());
    std::vector<int64_t> tb(S + 2);
    for (int t = 0; t <= S; t++)
        HIP_CHECK(hipMemcpyAsync(&tb[t], base + (int64_t)t * n_eb, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(&tb[S + 1], base + n_cnt, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    for (int t = 0; t <= S; t++) table_rows[t] = tb[t + 1] - tb[t];
    *n_rows = tb[S + 1];
    return CBX_OK;
}

extern "C" int cbx_hier_list_offsets(const int64_t* d_parent_row, int64_t child_begin, int64_t n_child, int64_t parent_begin,
                                     int64_t n_parent, int32_t* d_offsets, void* stream) {
    if (!d_offsets || child_begin < 0 || n_child < 0 || parent_begin < 0 || n_parent < 0 || (n_child > 0 && !d_parent_row))
        return fail(CBX_E_ARGUMENT, "cbx_hier_list_offsets: invalid arguments");
    if (n_child > INT32_MAX) return fail(CBX_E_UNSUPPORTED, "cbx_hier_list_offsets: more than 2^31 - 1 child rows");
    hipLaunchKernelGGL(hier_offsets_kernel, dim3(blocks_for(n_parent + 1, 256)), dim3(256), 0, (hipStream_t)stream,
                       d_parent_row, child_begin, n_child, parent_begin, n_parent, d_offsets);
    HIP_CHECK(hipGetLastError());
    return CBX_OK;
}

// ---- string views -> Arrow Utf8 (cbx_views_to_utf8) ----
__global__ void views_len_kernel(const u32x4* views, int64_t n, uint32_t* len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) len[i] = views[i].x;
    else if (i == n) len[i] = 0;
}

// One value per thread: its int32 offset and its bytes (inline in the view when <= 12, else at buffer
// view.z, offset view.w of the slot's region), dword stores where the destination allows.
__global__ void views_copy_kernel(const u32x4* views, int64_t n, const uint8_t* region, int64_t bb, const int64_t* offs,
                                  int32_t* offs32, uint8_t* out, int64_t cap, int64_t* size, int32_t* status) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const int64_t total = offs[n];
    if (total > cap || total > 0x7fffffffll) {
        if (i == 0) *status = 1;
        return;
    }
    offs32[i] = (int32_t)offs[i];
    if (i == n) { *size = total; return; }
    const u32x4 v = views[i];
    const uint32_t len = v.x;
    const uint8_t* src = len <= 12 ? (const uint8_t*)(views + i) + 4 : region + (int64_t)v.z * bb + v.w;
    uint8_t* dst = out + offs[i];
    for (uint32_t k = 0; k < len; k++) dst[k] = src[k];
}

extern "C" int cbx_views_to_utf8(const uint8_t* d_views, int64_t n, const uint8_t* d_region, int64_t buffer_bytes,
                                 int32_t* d_offsets, uint8_t* d_data, int64_t data_capacity, int64_t* d_size, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (n < 0 || !d_offsets || !d_size || (n > 0 && (!d_views || !d_region || buffer_bytes <= 0)) || data_capacity < 0 ||
        (data_capacity > 0 && !d_data) || ((uintptr_t)d_views & 15))
        return fail(CBX_E_ARGUMENT, "cbx_views_to_utf8: invalid arguments");
    const int64_t nsum = scan_sums_len(n + 1);
    AsyncBlock blk(st);
    const size_t bytes = (size_t)((n + 1) * 4 + 15) / 16 * 16 + (size_t)(n + 1) * 8 + (size_t)nsum * 8 + 16;
    HIP_CHECK(hipMallocAsync(&blk.p, bytes, st));
    uint32_t* len = (uint32_t*)blk.p;
    int64_t* offs = (int64_t*)((uint8_t*)blk.p + (size_t)((n + 1) * 4 + 15) / 16 * 16);
    int64_t* sums = offs + (n + 1);
    int32_t* status = (int32_t*)(sums + nsum);
    HIP_CHECK(hipMemsetAsync(status, 0, 4, st));
    const unsigned g = (unsigned)((n + 1 + 255) / 256);
    hipLaunchKernelGGL(views_len_kernel, dim3(g), dim3(256), 0, st, (const u32x4*)d_views, n, len);
    device_scan(len, n + 1, offs, sums, st);
    hipLaunchKernelGGL(views_copy_kernel, dim3(g), dim3(256), 0, st, (const u32x4*)d_views, n, d_region, buffer_bytes,
                       (const int64_t*)offs, d_offsets, d_data, data_capacity, d_size, status);
    HIP_CHECK(hipGetLastError());
    int32_t h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, status, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h) return fail(CBX_E_CAPACITY, "cbx_views_to_utf8: the payload exceeds data_capacity or an int32 offset");
    return CBX_OK;
}

extern "C" int cbx_hier_dependee_values(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                                        const int32_t* d_rec_len, int64_t n_rows, int32_t start_offset, int32_t field,
                                        int64_t* d_values, uint64_t* d_validity, void* stream) {
    if (!P || n_rows < 0 || n_bytes < 0 || start_offset < 0 || field < 0 || field >= (int32_t)P->hfields.size() ||
        (n_rows > 0 && (!d_data || !d_rec_off || !d_rec_len || !d_values || !d_validity)))
        return fail(CBX_E_ARGUMENT, "cbx_hier_dependee_values: invalid arguments");
    const Field f = P->dfields_h[field];
    const bool str = f.kind == CBX_K_STRING || f.kind == CBX_K_STRING_ASCII;
    if (!(str || f.kind == CBX_K_BCD || f.kind == CBX_K_BINARY || f.kind == CBX_K_ASCII_NUM || f.kind == CBX_K_ZONED) ||
        f.n_dims != 0)
        return fail(CBX_E_UNSUPPORTED, "cbx_hier_dependee_values: the field is not an integral or string DEPENDING ON field");
    if (n_rows > 0 && str) {   // Right(s): the occurs_mappings key it equals (the plan's walk handlers)
        hipLaunchKernelGGL(hier_dep_str_kernel, dim3(blocks_for(n_rows, 64)), dim3(64), 0, (hipStream_t)stream, d_data,
                           n_bytes, d_rec_off, d_rec_len, n_rows, start_offset, (const CBX_CONST Field*)P->d_fields + field,
                           (const uint32_t*)P->d_lut, (const CBX_CONST cbx_walk_handler*)P->d_whand,
                           P->d_whand ? P->walk_n_handlers : 0, d_values, d_validity);
        HIP_CHECK(hipGetLastError());
    } else if (n_rows > 0) {
        hipLaunchKernelGGL(hier_dep_values_kernel, dim3(blocks_for(n_rows, 64)), dim3(64), 0, (hipStream_t)stream, d_data,
                           n_bytes, d_rec_off, d_rec_len, n_rows, start_offset, (const CBX_CONST Field*)P->d_fields + field,
                           d_values, d_validity);
        HIP_CHECK(hipGetLastError());
    }
    return CBX_OK;
}

extern "C" int cbx_hier_dependee_counts(const cbx_hier_walk* walk, const cbx_hier_dependee* deps, int32_t n_deps,
                                        const cbx_hier_odo_array* arrays, int32_t n_arrays, int32_t* d_counts, int64_t pitch,
                                        int32_t* d_changed, void* stream) {
    if (!walk || n_deps < 0 || n_deps > CBX_HIER_MAX_DEPS || n_arrays < 0 || n_arrays > CBX_HIER_MAX_DEPS ||
        (n_deps && !deps) || (n_arrays && !arrays) || !d_changed || pitch < 0 || (n_arrays && !d_counts) ||
        walk->n_segments < 1 || walk->n_segments > CBX_HIER_MAX_SEG || walk->root_segment < 0 ||
        walk->root_segment >= walk->n_segments)
        return fail(CBX_E_ARGUMENT, "cbx_hier_dependee_counts: invalid arguments");
    HierDepArgs a{};
    a.w = *walk;
    a.n_deps = n_deps;
    a.n_arrays = n_arrays;
    for (int i = 0; i < n_deps; i++) {
        const int ot = deps[i].out_type;
        if (!deps[i].values || !deps[i].validity || (ot != CBX_O_I32 && ot != CBX_O_I64 && ot != CBX_O_DEC128 && ot != CBX_O_STRING) ||
            deps[i].walk_slot >= 8)
            return fail(CBX_E_ARGUMENT, "cbx_hier_dependee_counts: a dependee column must be I32, I64, DEC128 or string keys");
        a.dep[i] = deps[i];
    }
    for (int i = 0; i < n_arrays; i++) {
        if (arrays[i].dependee < 0 || arrays[i].dependee >= n_deps)
            return fail(CBX_E_ARGUMENT, "cbx_hier_dependee_counts: array dependee out of range");
        a.arr[i] = arrays[i];
    }
    // every event names a known dependee / array, every child segment has its offsets
    for (int s = 0; s <= CBX_HIER_MAX_SEG; s++)
        for (int k = 0; k < CBX_HIER_MAX_EVENTS; k++) {
            const int e = walk->events[s][k];
            if (e == -32768) break;
            if ((e >= 0 && e >= n_deps) || (e < 0 && -e - 1 >= n_arrays))
                return fail(CBX_E_ARGUMENT, "cbx_hier_dependee_counts: event out of range");
        }
    for (int s = 0; s < walk->n_segments; s++)
        for (int k = 0; k < CBX_HIER_MAX_SEG && walk->children[s][k] >= 0; k++) {
            const int c = walk->children[s][k];
            if (c >= walk->n_segments || !walk->child_offsets[c])
                return fail(CBX_E_ARGUMENT, "cbx_hier_dependee_counts: child segment without list offsets");
        }
    hipStream_t st = (hipStream_t)stream;
    HIP_CHECK(hipMemsetAsync(d_changed, 0, sizeof(int32_t), st));
    const int64_t n = walk->table_rows[0];
    if (n > 0) {
        hipLaunchKernelGGL(hier_dep_kernel, dim3(blocks_for(n, 64)), dim3(64), 0, st, a, d_counts, pitch, d_changed);
        HIP_CHECK(hipGetLastError());
    }
    return CBX_OK;
}

// ---------------------------------------------------------------------------------------------
// The record walk: node tables (cbx_plan_set_walk) and VarOccursRecordExtractor framing.
// ---------------------------------------------------------------------------------------------
extern "C" int cbx_plan_set_walk(cbx_plan* P, const cbx_walk_node* nodes, int32_t n_nodes, int32_t root,
                                 const cbx_walk_array* arrays, const cbx_walk_handler* handlers, int32_t n_handlers,
                                 int32_t variable_size_occurs) {
    if (!P || !nodes || n_nodes <= 0 || root < 0 || root >= n_nodes || n_handlers < 0 || (n_handlers > 0 && !handlers) ||
        (!P->harrays.empty() && !arrays))
        return fail(CBX_E_ARGUMENT, "cbx_plan_set_walk: invalid arguments");
    const int nf = (int)P->dfields_h.size(), na = (int)P->harrays.size();
    for (int i = 0; i < n_nodes; i++) {
        const cbx_walk_node& n = nodes[i];
        if ((n.kind != CBX_W_GROUP && n.kind != CBX_W_PRIM) || n.next >= n_nodes || n.child >= n_nodes || n.field >= nf ||
            n.array >= na || n.dep_slot >= kWalkDeps || (n.kind == CBX_W_PRIM && n.data_size <= 0))
            return fail(CBX_E_ARGUMENT, "cbx_plan_set_walk: bad node " + std::to_string(i));
    }
    for (int i = 0; i < na; i++)
        if (arrays[i].dep_slot >= kWalkDeps || arrays[i].h_begin < 0 || arrays[i].h_end > n_handlers || arrays[i].h_begin > arrays[i].h_end)
            return fail(CBX_E_ARGUMENT, "cbx_plan_set_walk: bad array " + std::to_string(i));
    for (int i = 0; i < n_handlers; i++)
        if (handlers[i].key_len < 0 || handlers[i].key_len > 64) return fail(CBX_E_ARGUMENT, "cbx_plan_set_walk: bad handler");
    if (P->walk) return fail(CBX_E_STATE, "cbx_plan_set_walk: the plan already walks");
    std::vector<int64_t> slot_base(P->n_columns, 0), tile_bytes(2 * (size_t)P->n_columns, 0);   // [tile bytes, tiles per buffer]
    int64_t ns = 0;
    for (int c = 0; c < P->n_columns; c++) {
        if (!P->col_is_string[c]) continue;
        if (!P->view) return fail(CBX_E_UNSUPPORTED, "cbx_plan_set_walk: string columns need the string-view layout");
        slot_base[c] = ns;
        ns += P->col_slots[c];
        tile_bytes[2 * c] = view_tile_bytes(P, c);
        tile_bytes[2 * c + 1] = view_tiles_per_buf(tile_bytes[2 * c]);
    }
    // every column slot's validity word of a tile (the walk accumulates them in LDS per tile); a
    // count column has one slot per element of its array's enclosing arrays
    std::vector<int64_t> cslots(P->n_columns);
    for (int c = 0; c < P->n_columns; c++) cslots[c] = P->col_slots[c];
    for (const cbx_array& ar : P->harrays) {
        if (ar.count_column < 0 || ar.count_column >= P->n_columns) continue;
        int64_t k = 1;
        for (int p = ar.parent, guard = 0; p >= 0 && p < (int)P->harrays.size() && guard < 64; p = P->harrays[p].parent, guard++)
            k *= std::max(1, P->harrays[p].max_count);
        cslots[ar.count_column] = std::max(cslots[ar.count_column], k);
    }
    std::vector<int64_t> vbase(P->n_columns, 0);
    std::vector<int32_t> vcol, vslot;
    for (int c = 0; c < P->n_columns; c++) {
        vbase[c] = (int64_t)vcol.size();
        for (int64_t k = 0; k < cslots[c] && vcol.size() < (1u << 20); k++) { vcol.push_back(c); vslot.push_back((int32_t)k); }
    }
    if (vcol.empty()) { vcol.push_back(0); vslot.push_back(0); }
    int r;
    if ((r = upload(&P->d_wvbase, vbase.data(), vbase.size())) || (r = upload(&P->d_wvcol, vcol.data(), vcol.size())) ||
        (r = upload(&P->d_wvslot, vslot.data(), vslot.size())))
        return r;
    P->n_vslots = P->n_columns > 0 ? (int32_t)vcol.size() : 0;
    if ((r = upload(&P->d_wnodes, nodes, n_nodes)) || (r = upload(&P->d_warr, arrays, na)) ||
        (r = upload(&P->d_whand, handlers, n_handlers)) || (r = upload(&P->d_wslot_base, slot_base.data(), slot_base.size())) ||
        (r = upload(&P->d_wtile_bytes, tile_bytes.data(), tile_bytes.size())))
        return r;
    for (const Field& d : P->dfields_h) {
        if (d.variant == V_FILE_ID) P->fid_col = d.column;
        if (d.variant == V_RECORD_ID) P->rid_col = d.column;
    }
    // the frame stack's depth: the root's frame, one per group level, two per OCCURS group level
    // (the elements' frame and the element's), one per OCCURS of primitives
    std::vector<int> memo(n_nodes, -1);
    std::function<int(int, int)> body = [&](int g, int guard) -> int {   // frames of group g's body
        if (guard > 64) return 1 << 20;
        if (memo[g] >= 0) return memo[g];
        int m = 0;
        for (int c = nodes[g].child, k = 0; c >= 0 && k < n_nodes; c = nodes[c].next, k++) {
            const cbx_walk_node& n = nodes[c];
            const int sub = n.kind == CBX_W_GROUP ? body(c, guard + 1) : 0;
            m = std::max(m, n.array >= 0 ? 1 + sub : sub);
        }
        return memo[g] = 1 + m;
    };
    const int depth = body(root, 0);
    if (depth > kWalkDepth)
        return fail(CBX_E_UNSUPPORTED, "cbx_plan_set_walk: the copybook nests " + std::to_string(depth) + " levels, above " +
                                           std::to_string(kWalkDepth));
    P->walk_depth = depth;
    // the largest record the copybook describes (the root group's children at their static sizes)
    int32_t max_rec = 0;
    for (int c = nodes[root].child, k = 0; c >= 0 && k < n_nodes; c = nodes[c].next, k++) max_rec = std::max(max_rec, nodes[c].actual_size);
    P->walk_max_rec = max_rec;
    P->h_wnodes.assign(nodes, nodes + n_nodes);
    P->h_warr.assign(arrays, arrays + na);
    P->n_str_slots = ns;
    P->walk_root = root;
    P->walk_var = variable_size_occurs != 0;
    P->walk_n_handlers = n_handlers;
    P->walk = true;
    return CBX_OK;
}

namespace {
// Chunk-parallel framing of a record chain (cbx_chain.h) from `first` over [first, n_bytes).
// h: [0] records, [1] the chain's end position, [2] error kind (the step's), [3] error position.
// jf: the specialised passes (sample, spec, fix, settle, write: jit_chain_source's kernels, Step's layout),
// nullptr: the library's templates.
template <typename Step>
int frame_chain(const Step& s, int64_t first, int64_t n_bytes, int64_t capacity, int64_t* d_rec_off, int32_t* d_rec_len,
                hipStream_t st, int64_t h[4], int64_t min_chunk, const hipFunction_t* jf = nullptr) {
    h[0] = 0; h[1] = first; h[2] = 0; h[3] = 0;
    const int64_t span = n_bytes - first;
    if (span <= 0) return CBX_OK;
    // chunks: ~32 k lanes of walkers for a large stream, >= min_chunk bytes each -- enough records per
    // chunk that a speculated chain meets the true one inside it (env CBX_CHAIN_CHUNK: tests force
    // small chunks, so chains cross many of them)
    int64_t chunk = std::min<int64_t>(std::max<int64_t>(65536, min_chunk), std::max<int64_t>(min_chunk, span / 32768));
    if (const char* e = getenv("CBX_CHAIN_CHUNK")) chunk = std::max<int64_t>(32, atoll(e));
    chunk = (chunk + 31) & ~(int64_t)31;
    const int64_t K = (span + chunk - 1) / chunk;
    const int64_t nw = (span + 31) / 32 + 1;
    const int64_t nsum = scan_sums_len(K);
    auto r16 = [](size_t n) { return (n + 15) & ~(size_t)15; };
    const size_t bytes = r16((size_t)nw * 4) + 6 * r16((size_t)K * 8) + r16((size_t)K * 4) + r16((size_t)nsum * 8 + 8) + r16(16 * 8);
    AsyncBlock blk(st);
    HIP_CHECK(hipMallocAsync(&blk.p, bytes, st));
    uint8_t* q = (uint8_t*)blk.p;
    auto take = [&](size_t n) { uint8_t* r = q; q += (n + 15) & ~(size_t)15; return r; };
    ChainArgs c{};
    c.first = first; c.chunk = chunk; c.n_chunks = K; c.n_bits = span;
    c.bits = (uint32_t*)take((size_t)nw * 4);
    c.ent = (int64_t*)take((size_t)K * 8);
    c.spec_exit = (int64_t*)take((size_t)K * 8);
    c.spec_cnt = (int64_t*)take((size_t)K * 8);
    int64_t* ex[2] = {(int64_t*)take((size_t)K * 8), (int64_t*)take((size_t)K * 8)};
    int64_t* base = (int64_t*)take((size_t)K * 8);
    c.cnt = (uint32_t*)take((size_t)K * 4);
    int64_t* sums = (int64_t*)take((size_t)nsum * 8 + 8);
    c.out = (int64_t*)take(16 * 8);
    HIP_CHECK(hipMemsetAsync(c.bits, 0, (size_t)nw * 4, st));
    HIP_CHECK(hipMemsetAsync(c.out, 0, 16 * 8, st));
    const unsigned g = (unsigned)((K + 255) / 256);
    Step sa = s;   // (addressable kernel arguments for the module launches)
    auto mlaunch = [&](hipFunction_t f, unsigned grid, unsigned block, void** args) {
        return hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, 0, st, args, nullptr);
    };
    int n_sample = 256;
    if (jf) {
        void* a0[] = {&sa, &c, &n_sample};
        HIP_CHECK(mlaunch(jf[0], 1, 1, a0));
        void* a1[] = {&sa, &c};
        HIP_CHECK(mlaunch(jf[1], g, 256, a1));
    } else {
        hipLaunchKernelGGL(chain_sample<Step>, dim3(1), dim3(1), 0, st, s, c, n_sample);
        hipLaunchKernelGGL(chain_spec<Step>, dim3(g), dim3(256), 0, st, s, c);
        HIP_CHECK(hipGetLastError());
    }
    HIP_CHECK(hipMemcpyAsync(ex[0], c.spec_exit, (size_t)K * 8, hipMemcpyDeviceToDevice, st));
    int cur = 0;
    bool changed = K > 1;
    for (int r = 0; r < kChainRounds && changed; r++) {
        HIP_CHECK(hipMemsetAsync(c.out + 4, 0, 8, st));
        if (jf) {
            const int64_t* ein = ex[cur];
            int64_t* eout = ex[cur ^ 1];
            void* a2[] = {&sa, &c, &ein, &eout};
            HIP_CHECK(mlaunch(jf[2], g, 256, a2));
        } else {
            hipLaunchKernelGGL(chain_fix<Step>, dim3(g), dim3(256), 0, st, s, c, (const int64_t*)ex[cur], ex[cur ^ 1]);
            HIP_CHECK(hipGetLastError());
        }
        cur ^= 1;
        int64_t flag = 0;
        HIP_CHECK(hipMemcpyAsync(&flag, c.out + 4, 8, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        changed = flag != 0;
    }
    if (changed) {
        if (jf) {
            int64_t* e = ex[cur];
            void* a3[] = {&sa, &c, &e};
            HIP_CHECK(mlaunch(jf[3], 1, 1, a3));
        } else {
            hipLaunchKernelGGL(chain_settle<Step>, dim3(1), dim3(1), 0, st, s, c, ex[cur]);
        }
    }
    device_scan(c.cnt, K, base, sums, st);
    if (jf) {
        const int64_t* b = base;
        void* a4[] = {&sa, &c, &b, &capacity, &d_rec_off, &d_rec_len};
        HIP_CHECK(mlaunch(jf[4], g, 256, a4));
    } else {
        hipLaunchKernelGGL(chain_write<Step>, dim3(g), dim3(256), 0, st, s, c, (const int64_t*)base, capacity, d_rec_off, d_rec_len);
        HIP_CHECK(hipGetLastError());
    }
    HIP_CHECK(hipMemcpyAsync(h, c.out, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return CBX_OK;
}
}  // namespace

extern "C" int cbx_frame_length_field(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, int32_t field,
                                      int32_t start_offset, int32_t end_offset, int32_t adjustment, int64_t* d_rec_off,
                                      int32_t* d_rec_len, int64_t capacity, int64_t* n_records, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!P || !n_records || n_bytes < 0 || start_offset < 0 || end_offset < 0 || capacity < 0 ||
        (n_bytes > 0 && !d_data) || (capacity > 0 && (!d_rec_off || !d_rec_len)) || field < 0 ||
        field >= (int)P->hfields.size())
        return fail(CBX_E_ARGUMENT, "cbx_frame_length_field: invalid arguments");
    const cbx_field& hf = P->hfields[field];
    if (hf.n_dims != 0 || !(hf.flags & CBX_F_INTEGRAL) || is_string_out(hf.out_type) || hf.kind == CBX_K_RECORD_ID ||
        hf.kind == CBX_K_FILE_ID)
        return fail(CBX_E_ARGUMENT, "cbx_frame_length_field: the record length field must be a primitive integral field");
    *n_records = 0;
    LenFieldArgs a{};
    a.data = d_data; a.n_bytes = n_bytes;
    a.field = (const CBX_CONST Field*)P->d_fields + field;
    a.start_off = start_offset; a.end_off = end_offset; a.adjustment = adjustment;
    a.lfb = hf.offset + hf.size;
    int64_t h[4];
    int r;
    if ((r = frame_chain(LenFieldStep{a}, 0, n_bytes, capacity, d_rec_off, d_rec_len, st, h, 1024))) return r;
    *n_records = h[0];
    if (h[2] == 1)
        return fail(CBX_E_STATE, "Record length value of the field at byte " + std::to_string(h[3]) +
                                     " must be an integral type.");
    if (h[0] > capacity) return fail(CBX_E_CAPACITY, "record capacity " + std::to_string(capacity) + " < " + std::to_string(h[0]));
    return CBX_OK;
}

extern "C" int cbx_frame_var_occurs(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, int64_t first_offset,
                                    int64_t* d_rec_off, int32_t* d_rec_len, int64_t capacity, int64_t* n_records,
                                    int64_t* virtual_bytes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!P || !n_records || !virtual_bytes || n_bytes < 0 || first_offset < 0 || capacity < 0 ||
        (n_bytes > 0 && !d_data) || (capacity > 0 && (!d_rec_off || !d_rec_len)))
        return fail(CBX_E_ARGUMENT, "cbx_frame_var_occurs: invalid arguments");
    if (!P->walk) return fail(CBX_E_STATE, "cbx_frame_var_occurs: the plan has no walk tables (cbx_plan_set_walk)");
    *n_records = 0;
    *virtual_bytes = n_bytes;
    if (first_offset >= n_bytes) return CBX_OK;
    WalkArgs a{};
    a.data = d_data;
    a.hier_root = -1;
    a.nodes = (const CBX_CONST cbx_walk_node*)P->d_wnodes; a.root = P->walk_root;
    a.warr = (const CBX_CONST cbx_walk_array*)P->d_warr;
    a.handlers = (const CBX_CONST cbx_walk_handler*)P->d_whand; a.n_handlers = P->walk_n_handlers;
    a.arrays = (const CBX_CONST cbx_array*)P->d_arrays; a.fields = (const CBX_CONST Field*)P->d_fields;
    a.lut = P->d_lut;
    // the copybook-specialised step for large streams (records estimated at the copybook's largest
    // form; cbx_plan_options.jit_min_records, CBX_NO_JIT_WALK as for the walk), else the table walk
    const hipFunction_t* jf = nullptr;
    if (P->jit_min >= 0 && (n_bytes - first_offset) / std::max<int64_t>(1, P->walk_max_rec) >= P->jit_min &&
        !getenv("CBX_NO_JIT_WALK")) {
        if (!P->chain_jit_tried) {
            P->chain_jit_tried = true;
            const std::string src = jit_chain_source(P);
            static const char* const names[5] = {"cbx_jit_chain_sample", "cbx_jit_chain_spec", "cbx_jit_chain_fix",
                                                 "cbx_jit_chain_settle", "cbx_jit_chain_write"};
            bool all = !src.empty();
            for (int i = 0; i < 5 && all; i++) all = (P->chain_jit_fn[i] = jit_get(src, &P->jit_error, names[i])) != nullptr;
            if (!all) for (auto& f : P->chain_jit_fn) f = nullptr;
        }
        if (P->chain_jit_fn[0]) jf = P->chain_jit_fn;
    }
    P->last_chain_jit = jf != nullptr;
    int64_t h[4];
    int r;
    // (a record walked from a wrong start reads its counts from the wrong bytes -- often the maxima --
    // so such chains need more records than length-field ones to land on a true start: 16 KiB chunks)
    if ((r = frame_chain(VarOccursStep{a, n_bytes}, first_offset, n_bytes, capacity, d_rec_off, d_rec_len, st, h, 16384, jf))) return r;
    if (h[2] == 2) return fail(CBX_E_UNSUPPORTED, "cbx_frame_var_occurs: copybook nesting deeper than the walk's frame stack");
    *n_records = h[0];
    *virtual_bytes = std::max(n_bytes, h[1]);
    if (h[0] > capacity) return fail(CBX_E_CAPACITY, "record capacity " + std::to_string(capacity) + " < " + std::to_string(h[0]));
    return CBX_OK;
}
