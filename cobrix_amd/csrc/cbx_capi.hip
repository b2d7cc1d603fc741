// cbx_capi.hip -- C ABI of libcobrix_hip.so (include/cobrix_hip.h): plan building, launches.
//
// The plan turns the flattened copybook (cbx_field / cbx_array tables produced by the JVM or
// the Python host from the Cobrix AST) into the device layout the kernels walk:
//   * per-field constants (10^precision bounds, slot counts),
//   * LDS windows: greedy packing of every field element [offset, offset + size) sorted by
//     offset into byte ranges of at most `window_bytes`, then grouped into (field, slot range)
//     runs so a window's decode loop is wave-uniform,
//   * the UTF-8 code-page LUT and the segment-redefine keys.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cbx_kernels.hip"

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
    std::vector<Window> hwindows, hswindows;   // decode pass / string sizing pass
    std::vector<Run> hruns, hsruns;
    std::vector<int32_t> global_fields;
    cbx_plan_options opts;
    int n_columns = 0;
    int seg_col = -1;
    int max_pitch = 0;
    int n_string_cols = 0;
    std::vector<int32_t> col_is_string;   // per column: 1 if string/binary
    std::vector<int32_t> col_slots;       // per column: slots
    // device copies
    Field* d_fields = nullptr;
    Window* d_windows = nullptr;
    Run* d_runs = nullptr;
    Window* d_swindows = nullptr;
    Run* d_sruns = nullptr;
    cbx_array* d_arrays = nullptr;
    int32_t* d_global_fields = nullptr;
    cbx_segment_map* d_segmap = nullptr;
    uint32_t* d_lut = nullptr;
    DevColumn* d_cols = nullptr;
    int64_t* d_seq_base = nullptr;
    // workspace
    int64_t* d_tile_sums = nullptr;
    int64_t tile_sums_cap = 0;
    int64_t* d_block_sums = nullptr;
    int64_t block_sums_cap = 0;
    int num_cus = 256;
    int contig_max_bytes = 20 * 1024;   // LDS span budget for contiguous fixed-length staging
    // profiling
    bool profiling = false;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    float last_ms[3] = {0, 0, 0};
};

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

// Greedy LDS window packing: every element [offset, offset + size) sorted by offset, cut into
// byte ranges of at most wmax, each window's elements regrouped into (field, slot range) runs.
static void build_windows(cbx_plan* P, int wmax, bool strings_only, std::vector<Window>& wins,
                          std::vector<Run>& runs) {
    struct Elem { int lo, hi, field, slot; };
    std::vector<Elem> els;
    for (int i = 0; i < (int)P->dfields_h.size(); i++) {
        const Field& d = P->dfields_h[i];
        if (d.kind == CBX_K_RECORD_ID || d.kind == CBX_K_FILE_ID || d.size > wmax) continue;
        if (strings_only && !is_string_out(d.out_type)) continue;
        for (int s = 0; s < d.n_slots; s++) {
            int eo = d.offset, rem = s;
            for (int k = d.n_dims - 1; k >= 0; k--) { int idx = rem % d.dim_count[k]; rem /= d.dim_count[k]; eo += idx * d.dim_stride[k]; }
            els.push_back(Elem{eo, eo + d.size, i, s});
        }
    }
    std::stable_sort(els.begin(), els.end(), [](const Elem& a, const Elem& b) { return a.lo < b.lo; });
    size_t e0 = 0;
    while (e0 < els.size()) {
        int lo = els[e0].lo, hi = els[e0].hi;
        size_t e1 = e0 + 1;
        while (e1 < els.size() && std::max(hi, els[e1].hi) - lo <= wmax) { hi = std::max(hi, els[e1].hi); e1++; }
        std::vector<Elem> win(els.begin() + e0, els.begin() + e1);
        std::stable_sort(win.begin(), win.end(), [](const Elem& a, const Elem& b) {
            return a.field != b.field ? a.field < b.field : a.slot < b.slot;
        });
        Window w{};
        w.lo = lo; w.hi = hi;
        w.run_begin = (int)runs.size();
        for (size_t j = 0; j < win.size();) {
            size_t k = j + 1;
            while (k < win.size() && win[k].field == win[j].field && win[k].slot == win[k - 1].slot + 1) k++;
            runs.push_back(Run{win[j].field, win[j].slot, win[k - 1].slot + 1, 0});
            if (is_string_out(P->dfields_h[win[j].field].out_type)) w.has_strings = 1;
            j = k;
        }
        w.run_end = (int)runs.size();
        int nch = (hi - lo + 15 + 15) >> 4;
        w.pitch = 16 * nch + 4;
        wins.push_back(w);
        e0 = e1;
    }
}

extern "C" int cbx_plan_create(const cbx_field* fields, int32_t n_fields, const cbx_array* arrays,
                               int32_t n_arrays, const cbx_plan_options* opts, cbx_plan** out_plan) {
    if (!fields || n_fields <= 0 || !opts || !out_plan || n_arrays < 0 || (n_arrays > 0 && !arrays))
        return fail(CBX_E_ARGUMENT, "cbx_plan_create: invalid arguments");
    cbx_plan* P = new cbx_plan();
    P->opts = *opts;
    P->n_columns = opts->n_columns;
    P->hfields.assign(fields, fields + n_fields);
    if (n_arrays) P->harrays.assign(arrays, arrays + n_arrays);
    P->col_is_string.assign(P->n_columns, 0);
    P->col_slots.assign(P->n_columns, 1);

    // ---- fields
    for (int i = 0; i < n_fields; i++) {
        const cbx_field& f = fields[i];
        if (f.n_dims < 0 || f.n_dims > CBX_MAX_DIMS) { delete P; return fail(CBX_E_ARGUMENT, "field " + std::to_string(i) + ": bad n_dims"); }
        for (int k = 0; k < f.n_dims; k++)
            if (f.dim_count[k] <= 0 || f.dim_array[k] < 0 || f.dim_array[k] >= n_arrays) {
                delete P; return fail(CBX_E_ARGUMENT, "field " + std::to_string(i) + ": bad dimension");
            }
        Field d = make_field(f);
        if (f.column < 0 || f.column >= P->n_columns) { delete P; return fail(CBX_E_ARGUMENT, "field " + std::to_string(i) + ": bad column"); }
        bool generated = f.kind == CBX_K_RECORD_ID || f.kind == CBX_K_FILE_ID;
        if (!generated && f.size <= 0) { delete P; return fail(CBX_E_ARGUMENT, "field " + std::to_string(i) + ": bad size"); }
        if (f.kind == CBX_K_BINARY && f.size > 16) { delete P; return fail(CBX_E_UNSUPPORTED, "field " + std::to_string(i) + ": binary wider than 16 bytes"); }
        if ((f.out_type == CBX_O_DEC64 || f.out_type == CBX_O_DEC128) && (f.out_precision < 1 || f.out_precision > 38)) {
            delete P; return fail(CBX_E_UNSUPPORTED, "field " + std::to_string(i) + ": decimal precision outside 1..38");
        }
        P->dfields_h.push_back(d);
        P->col_is_string[f.column] = is_string_out(f.out_type);
        P->col_slots[f.column] = d.n_slots;
    }
    for (int ai = 0; ai < n_arrays; ai++) {
        const cbx_array& ar = arrays[ai];
        if (ar.dependee >= n_fields || ar.max_count <= 0) { delete P; return fail(CBX_E_ARGUMENT, "array " + std::to_string(ai) + ": bad descriptor"); }
        if (ar.dependee >= 0) {
            const cbx_field& df = fields[ar.dependee];
            if (!(df.flags & CBX_F_INTEGRAL) || df.n_dims != 0 || df.precision > 18)
                { delete P; return fail(CBX_E_UNSUPPORTED, "array " + std::to_string(ai) + ": DEPENDING ON source must be a non-array integral field"); }
        }
    }
    P->seg_col = opts->segment_column;
    if (P->seg_col >= P->n_columns) { delete P; return fail(CBX_E_ARGUMENT, "bad segment column"); }

    // ---- LDS windows: all fields (decode pass) and string fields only (sizing pass)
    int wmax = opts->window_bytes > 0 ? opts->window_bytes : 256;
    if (wmax > kMaxWindowBytes) wmax = kMaxWindowBytes;
    for (int i = 0; i < n_fields; i++) {
        const Field& d = P->dfields_h[i];
        if (d.kind == CBX_K_RECORD_ID || d.kind == CBX_K_FILE_ID || d.size > wmax) P->global_fields.push_back(i);
    }
    build_windows(P, wmax, false, P->hwindows, P->hruns);
    build_windows(P, wmax, true, P->hswindows, P->hsruns);
    for (const Window& w : P->hwindows) P->max_pitch = std::max(P->max_pitch, w.pitch);
    for (const Window& w : P->hswindows) P->max_pitch = std::max(P->max_pitch, w.pitch);

    // ---- string column sequence bases (per column: n_slots * n_tiles entries; filled per call)
    for (int c = 0; c < P->n_columns; c++) P->n_string_cols += P->col_is_string[c];

    // ---- segment map: keys to UTF-8
    cbx_segment_map sm = opts->segments;
    if (opts->has_segments) {
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
        (r = upload(&P->d_windows, P->hwindows.data(), P->hwindows.size())) ||
        (r = upload(&P->d_runs, P->hruns.data(), P->hruns.size())) ||
        (r = upload(&P->d_swindows, P->hswindows.data(), P->hswindows.size())) ||
        (r = upload(&P->d_sruns, P->hsruns.data(), P->hsruns.size())) ||
        (r = upload(&P->d_arrays, P->harrays.data(), P->harrays.size())) ||
        (r = upload(&P->d_global_fields, P->global_fields.data(), P->global_fields.size())) ||
        (r = upload(&P->d_lut, opts->lut, 256))) {
        cbx_plan_destroy(P);
        return r;
    }
    if (opts->has_segments && (r = upload(&P->d_segmap, &sm, 1))) { cbx_plan_destroy(P); return r; }
    if ((r = upload(&P->d_cols, (DevColumn*)nullptr, 0)) != CBX_OK) { cbx_plan_destroy(P); return r; }
    (void)hipFree(P->d_cols);
    P->d_cols = nullptr;
    HIP_CHECK(hipMalloc((void**)&P->d_cols, sizeof(DevColumn) * std::max(1, P->n_columns)));
    HIP_CHECK(hipMalloc((void**)&P->d_seq_base, sizeof(int64_t) * std::max(1, P->n_columns)));
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) P->num_cus = prop.multiProcessorCount;
    *out_plan = P;
    return CBX_OK;
}

extern "C" void cbx_plan_destroy(cbx_plan* P) {
    if (!P) return;
    (void)hipFree(P->d_fields); (void)hipFree(P->d_windows); (void)hipFree(P->d_runs);
    (void)hipFree(P->d_swindows); (void)hipFree(P->d_sruns); (void)hipFree(P->d_arrays);
    (void)hipFree(P->d_global_fields); (void)hipFree(P->d_segmap); (void)hipFree(P->d_lut); (void)hipFree(P->d_cols);
    (void)hipFree(P->d_seq_base); (void)hipFree(P->d_tile_sums); (void)hipFree(P->d_block_sums);
    for (auto& e : P->ev) if (e) (void)hipEventDestroy(e);
    delete P;
}

// Column pointers and string-sequence bases for one call.
static int prepare_call(cbx_plan* P, int64_t n_rec, const cbx_column* columns, hipStream_t st,
                        int64_t* n_seq_out) {
    const int64_t n_tiles = (n_rec + kWave - 1) / kWave;
    std::vector<DevColumn> cols(P->n_columns);
    std::vector<int64_t> seq(P->n_columns, -1);
    int64_t n_seq = 0;
    for (int c = 0; c < P->n_columns; c++) {
        cols[c].values = columns ? columns[c].values : nullptr;
        cols[c].validity = columns ? columns[c].validity : nullptr;
        cols[c].offsets = columns ? columns[c].offsets : nullptr;
        cols[c].data = columns ? columns[c].data : nullptr;
        if (P->col_is_string[c]) {
            seq[c] = n_seq;
            n_seq += (int64_t)P->col_slots[c] * n_tiles;
        }
    }
    HIP_CHECK(hipMemcpyAsync(P->d_cols, cols.data(), sizeof(DevColumn) * P->n_columns, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(P->d_seq_base, seq.data(), sizeof(int64_t) * P->n_columns, hipMemcpyHostToDevice, st));
    if (n_seq > P->tile_sums_cap) {
        HIP_CHECK(hipStreamSynchronize(st));
        (void)hipFree(P->d_tile_sums);
        HIP_CHECK(hipMalloc((void**)&P->d_tile_sums, sizeof(int64_t) * (n_seq + 1)));
        P->tile_sums_cap = n_seq;
        int64_t nb = (n_seq + kScanTile - 1) / kScanTile + 1;
        (void)hipFree(P->d_block_sums);
        HIP_CHECK(hipMalloc((void**)&P->d_block_sums, sizeof(int64_t) * nb));
        P->block_sums_cap = nb;
    }
    *n_seq_out = n_seq;
    return CBX_OK;
}

static KernelArgs make_args(cbx_plan* P, const uint8_t* data, int64_t data_len, const int64_t* rec_off,
                            const int32_t* rec_len, int64_t n_rec, int32_t stride, int32_t start_off,
                            int64_t first_record_id, int mode) {
    KernelArgs a{};
    uintptr_t addr = (uintptr_t)data;
    a.base_shift = (int64_t)(addr & 15);
    a.data = (const uint8_t*)(addr & ~(uintptr_t)15);
    a.data_len = data_len + a.base_shift;
    a.rec_off = rec_off;
    a.rec_len = rec_len;
    a.n_rec = n_rec;
    a.stride = stride;
    a.start_off = start_off;
    a.first_record_id = first_record_id;
    a.file_id = P->opts.file_id;
    a.mode = mode;
    a.fields = P->d_fields;
    a.windows = mode == 1 ? P->d_swindows : P->d_windows;
    a.n_windows = (int)(mode == 1 ? P->hswindows.size() : P->hwindows.size());
    a.runs = mode == 1 ? P->d_sruns : P->d_runs;
    a.arrays = P->d_arrays;
    a.n_arrays = (int)P->harrays.size();
    a.seg_col = P->seg_col;
    a.segmap = P->opts.has_segments ? P->d_segmap : nullptr;
    a.lut = P->d_lut;
    a.cols = P->d_cols;
    a.str_seq_base = P->d_seq_base;
    a.tile_sums = P->d_tile_sums;
    a.n_tiles = (n_rec + kWave - 1) / kWave;
    a.max_pitch = P->max_pitch;
    return a;
}

static int launch_decode(cbx_plan* P, KernelArgs a, hipStream_t st) {
    if (a.n_tiles == 0) return CBX_OK;
    // fixed-length records short enough to stage a whole 64-record span: contiguous mode
    size_t rows = (size_t)kWave * P->max_pitch;
    if (a.mode == 0 && !a.rec_off && a.stride > 0 && (size_t)kWave * a.stride + 32 <= (size_t)P->contig_max_bytes) {
        a.contig = 1;
        rows = std::max(rows, (size_t)kWave * a.stride + 32);
    }
    size_t lds = 1024 + ((a.n_arrays * kWave * 4 + 15) & ~15) + rows + 16;
    if (lds > 160 * 1024) return fail(CBX_E_UNSUPPORTED, "LDS window too large");
    // one wave per block; enough blocks to cover every CU several times, grid-stride the rest
    int per_cu = (int)std::max<size_t>(1, std::min<size_t>(16, (160 * 1024) / std::max<size_t>(lds, 1)));
    int64_t grid = std::min<int64_t>(a.n_tiles, (int64_t)P->num_cus * per_cu * 2);
    if (a.n_windows > 0 || a.n_arrays > 0 || a.seg_col >= 0)
        hipLaunchKernelGGL(decode_kernel, dim3((unsigned)grid), dim3(kWave), lds, st, a);
    if (!P->global_fields.empty())
        hipLaunchKernelGGL(decode_global_kernel, dim3((unsigned)grid), dim3(kWave), 1024, st, a,
                           (const int32_t*)P->d_global_fields, (int32_t)P->global_fields.size());
    HIP_CHECK(hipGetLastError());
    return CBX_OK;
}

static int run_scan(cbx_plan* P, int64_t n, hipStream_t st) {
    if (n <= 0) return CBX_OK;
    int64_t nb = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, P->d_tile_sums, n, P->d_block_sums);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, P->d_block_sums, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, P->d_tile_sums, n, P->d_block_sums);
    HIP_CHECK(hipGetLastError());
    return CBX_OK;
}

static int decode_common(cbx_plan* P, const uint8_t* data, int64_t data_len, const int64_t* rec_off,
                         const int32_t* rec_len, int64_t n_rec, int32_t stride, int32_t start_off,
                         int64_t first_record_id, cbx_column* columns, int64_t* sizes_only, hipStream_t st) {
    if (!P || !data || n_rec < 0 || start_off < 0) return fail(CBX_E_ARGUMENT, "invalid decode arguments");
    if (!sizes_only && !columns) return fail(CBX_E_ARGUMENT, "columns required");
    int64_t n_seq = 0;
    int r = prepare_call(P, n_rec, columns, st, &n_seq);
    if (r) return r;
    const int64_t n_tiles = (n_rec + kWave - 1) / kWave;
    const bool prof = P->profiling && !sizes_only;
    if (prof) HIP_CHECK(hipEventRecord(P->ev[0], st));
    if (n_seq > 0) {
        // pass 1: per-(column, slot, tile) UTF-8 totals, then one device-wide exclusive scan
        KernelArgs a = make_args(P, data, data_len, rec_off, rec_len, n_rec, stride, start_off, first_record_id, 1);
        if ((r = launch_decode(P, a, st))) return r;
        if (prof) HIP_CHECK(hipEventRecord(P->ev[1], st));
        HIP_CHECK(hipMemsetAsync(P->d_tile_sums + n_seq, 0, sizeof(int64_t), st));
        if ((r = run_scan(P, n_seq + 1, st))) return r;
        // column payload sizes = scan[next column start] - scan[column start]
        std::vector<int64_t> idx;
        int64_t acc = 0;
        for (int c = 0; c < P->n_columns; c++)
            if (P->col_is_string[c]) { idx.push_back(acc); acc += (int64_t)P->col_slots[c] * n_tiles; }
        idx.push_back(n_seq);
        std::vector<int64_t> vals(idx.size());
        for (size_t k = 0; k < idx.size(); k++)
            HIP_CHECK(hipMemcpyAsync(&vals[k], P->d_tile_sums + idx[k], sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        size_t k = 0;
        for (int c = 0; c < P->n_columns; c++) {
            if (!P->col_is_string[c]) {
                if (sizes_only) sizes_only[c] = 0;
                continue;
            }
            int64_t tot = vals[k + 1] - vals[k];
            k++;
            if (sizes_only) { sizes_only[c] = tot; continue; }
            if (columns[c].data_capacity < tot)
                return fail(CBX_E_CAPACITY, "column " + std::to_string(c) + " needs " + std::to_string(tot) + " payload bytes");
            columns[c].data_size = tot;
        }
        if (sizes_only) return CBX_OK;
    } else if (sizes_only) {
        for (int c = 0; c < P->n_columns; c++) sizes_only[c] = 0;
        return CBX_OK;
    }
    // pass 2: decode every column
    KernelArgs a = make_args(P, data, data_len, rec_off, rec_len, n_rec, stride, start_off, first_record_id, 0);
    if (prof) {
        if (n_seq <= 0) HIP_CHECK(hipEventRecord(P->ev[1], st));
        HIP_CHECK(hipEventRecord(P->ev[2], st));
    }
    r = launch_decode(P, a, st);
    if (r) return r;
    if (prof) {
        HIP_CHECK(hipEventRecord(P->ev[3], st));
        HIP_CHECK(hipEventSynchronize(P->ev[3]));
        HIP_CHECK(hipEventElapsedTime(&P->last_ms[0], P->ev[0], P->ev[1]));
        HIP_CHECK(hipEventElapsedTime(&P->last_ms[1], P->ev[1], P->ev[2]));
        HIP_CHECK(hipEventElapsedTime(&P->last_ms[2], P->ev[2], P->ev[3]));
    }
    return CBX_OK;
}

extern "C" int cbx_plan_set_profiling(cbx_plan* P, int32_t enable) {
    if (!P) return fail(CBX_E_ARGUMENT, "null plan");
    if (enable && !P->ev[0])
        for (auto& e : P->ev) HIP_CHECK(hipEventCreate(&e));
    P->profiling = enable != 0;
    return CBX_OK;
}

extern "C" int cbx_plan_last_kernel_ms(const cbx_plan* P, float* sizes_ms, float* scan_ms, float* decode_ms) {
    if (!P) return fail(CBX_E_ARGUMENT, "null plan");
    if (sizes_ms) *sizes_ms = P->last_ms[0];
    if (scan_ms) *scan_ms = P->last_ms[1];
    if (decode_ms) *decode_ms = P->last_ms[2];
    return CBX_OK;
}

extern "C" int cbx_string_sizes_fixed(cbx_plan* P, const uint8_t* d_records, int64_t n_rec, int32_t rec_stride,
                                      int32_t start_offset, int64_t* out_sizes, void* stream) {
    if (!out_sizes) return fail(CBX_E_ARGUMENT, "out_sizes required");
    if (rec_stride <= 0) return fail(CBX_E_ARGUMENT, "record stride must be positive");
    return decode_common(P, d_records, n_rec * (int64_t)rec_stride, nullptr, nullptr, n_rec, rec_stride, start_offset,
                         0, nullptr, out_sizes, (hipStream_t)stream);
}

extern "C" int cbx_decode_fixed(cbx_plan* P, const uint8_t* d_records, int64_t n_rec, int32_t rec_stride,
                                int32_t start_offset, int64_t first_record_id, cbx_column* columns, void* stream) {
    if (rec_stride <= 0) return fail(CBX_E_ARGUMENT, "record stride must be positive");
    return decode_common(P, d_records, n_rec * (int64_t)rec_stride, nullptr, nullptr, n_rec, rec_stride, start_offset,
                         first_record_id, columns, nullptr, (hipStream_t)stream);
}

extern "C" int cbx_decode_var(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                              const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset, int64_t first_record_id,
                              cbx_column* columns, void* stream) {
    if (!d_rec_off || !d_rec_len || n_bytes < 0) return fail(CBX_E_ARGUMENT, "record offsets/lengths required");
    return decode_common(P, d_data, n_bytes, d_rec_off, d_rec_len, n_rec, 0, start_offset, first_record_id,
                         columns, nullptr, (hipStream_t)stream);
}

extern "C" int cbx_string_sizes_var(cbx_plan* P, const uint8_t* d_data, int64_t n_bytes, const int64_t* d_rec_off,
                                    const int32_t* d_rec_len, int64_t n_rec, int32_t start_offset,
                                    int64_t* out_sizes, void* stream) {
    if (!d_rec_off || !d_rec_len || !out_sizes || n_bytes < 0) return fail(CBX_E_ARGUMENT, "invalid arguments");
    return decode_common(P, d_data, n_bytes, d_rec_off, d_rec_len, n_rec, 0, start_offset, 0, nullptr,
                         out_sizes, (hipStream_t)stream);
}

extern "C" int cbx_frame_rdw(const uint8_t* d_data, int64_t n_bytes, const int64_t* seeds, int32_t n_seeds,
                             const cbx_rdw_params* params, int64_t* d_rec_off, int32_t* d_rec_len,
                             int64_t capacity, int64_t* n_records, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!d_data || n_bytes < 0 || !params || !n_records || (n_seeds > 0 && !seeds))
        return fail(CBX_E_ARGUMENT, "cbx_frame_rdw: invalid arguments");
    std::vector<int64_t> hseeds;
    if (n_seeds <= 0) hseeds.push_back(0);
    else hseeds.assign(seeds, seeds + n_seeds);
    int ns = (int)hseeds.size();
    int64_t *d_seeds = nullptr, *d_counts = nullptr, *d_err = nullptr;
    HIP_CHECK(hipMalloc((void**)&d_seeds, sizeof(int64_t) * ns));
    HIP_CHECK(hipMalloc((void**)&d_counts, sizeof(int64_t) * ns));
    HIP_CHECK(hipMalloc((void**)&d_err, sizeof(int64_t) * 2));
    HIP_CHECK(hipMemcpyAsync(d_seeds, hseeds.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(d_err, 0, sizeof(int64_t) * 2, st));
    RdwArgs a{};
    a.data = d_data; a.n_bytes = n_bytes; a.seeds = d_seeds; a.n_seeds = ns; a.p = *params;
    a.counts = d_counts; a.rec_off = d_rec_off; a.rec_len = d_rec_len; a.capacity = capacity; a.error = d_err;
    int threads = 64, blocks = (ns + threads - 1) / threads;
    hipLaunchKernelGGL(rdw_walk_kernel, dim3(blocks), dim3(threads), 0, st, a, 0);
    std::vector<int64_t> cnt(ns);
    int64_t err[2];
    HIP_CHECK(hipMemcpyAsync(cnt.data(), d_counts, sizeof(int64_t) * ns, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(err, d_err, sizeof(err), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int rc = CBX_OK;
    if (err[0] != 0) {
        char msg[160];
        snprintf(msg, sizeof msg, "RDW headers %s at %lld.", err[0] == -2 ? "should never be zero" : "too big (> 100 MiB)",
                 (long long)err[1]);
        rc = fail(CBX_E_STATE, msg);
    } else {
        int64_t total = 0;
        for (int k = 0; k < ns; k++) { int64_t c = cnt[k]; cnt[k] = total; total += c; }
        *n_records = total;
        if (total > capacity) {
            rc = fail(CBX_E_CAPACITY, "record capacity " + std::to_string(capacity) + " < " + std::to_string(total));
        } else {
            HIP_CHECK(hipMemcpyAsync(d_counts, cnt.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(rdw_walk_kernel, dim3(blocks), dim3(threads), 0, st, a, 1);
            HIP_CHECK(hipStreamSynchronize(st));
        }
    }
    (void)hipFree(d_seeds); (void)hipFree(d_counts); (void)hipFree(d_err);
    return rc;
}
