// Micro-benchmark of the C2 decode's memory pattern alone (no decoding): per 64-record tile, 12.8 KB of
// 200-byte records read with 16-byte lane loads (prefetched one tile ahead in registers), 24 columns of
// 64 x 8-byte values written (512 B contiguous per column per tile, nontemporal) -- the HBM rate a
// tile-per-wave column writer can reach, by tile order:
//   mode 0: grid-stride single tiles (all waves on neighbouring tiles at once)
//   mode 1: runs of 8 consecutive tiles per wave (the VWords order of the specialised kernel)
//   mode 2: one contiguous block of tiles per wave
// DEPTH: tiles whose loads are in flight per wave (1: the decode kernels' one-tile-ahead prefetch)
// usage: ubench_cols [records] [waves per CU] [depth 1|2]      (diagnostic only; never shipped)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

constexpr int kCols = 24, KP = 13, kStride = 200;

template <int MODE, int DEPTH>
__global__ __launch_bounds__(64) void k(const uint8_t* __restrict__ in, uint64_t* __restrict__ out, int64_t n_tiles, int64_t pitch) {
    const int lane = threadIdx.x;
    const int64_t G = gridDim.x, w = blockIdx.x;
    int64_t per = (n_tiles + G - 1) / G;
    auto tile_of = [&](int64_t i) -> int64_t {
        if (MODE == 0) return w + i * G;
        if (MODE == 1) return (i / 8) * 8 * G + w * 8 + (i % 8);
        return w * per + i;
    };
    auto valid = [&](int64_t i) { return MODE == 2 ? (i < per && tile_of(i) < n_tiles) : tile_of(i) < n_tiles; };
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, 0x7fffffff, 0x00020000);
    uint4 buf[DEPTH][KP];
    auto issue = [&](int64_t t, uint4 (&b)[KP]) {
        const uint64_t base = (uint64_t)(in + t * 64 * kStride);
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 12800, 0x00020000);
#pragma unroll
        for (int u = 0; u < KP; u++) {
            const int c = u * 64 + lane;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, c < 800 ? 16 * c : 0x7ffffff0, 0, 0);
            b[u] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    (void)rs;
    if (!valid(0)) return;
#pragma unroll
    for (int d = 0; d < DEPTH; d++) if (valid(d)) issue(tile_of(d), buf[d]);
    for (int64_t i = 0;; i += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            if (!valid(i + d)) return;
            const int64_t t = tile_of(i + d);
            uint64_t acc[KP];
#pragma unroll
            for (int u = 0; u < KP; u++) acc[u] = ((uint64_t)buf[d][u].x << 32 | buf[d][u].y) ^ ((uint64_t)buf[d][u].z << 7) ^ buf[d][u].w;
            if (valid(i + d + DEPTH)) issue(tile_of(i + d + DEPTH), buf[d]);
#pragma unroll
            for (int c = 0; c < kCols; c++)
                __builtin_nontemporal_store(acc[c % KP] + c, out + (int64_t)c * pitch + t * 64 + lane);
        }
    }
}

int main(int argc, char** argv) {
    const int64_t n_rec = argc > 1 ? atoll(argv[1]) : 50000000;
    const int wpc = argc > 2 ? atoi(argv[2]) : 16;
    const int depth = argc > 3 ? atoi(argv[3]) : 1;
    const int64_t n_tiles = (n_rec + 63) / 64, pitch = n_tiles * 64;
    uint8_t* in; uint64_t* out;
    if (hipMalloc(&in, n_tiles * 64 * kStride + 4096) != hipSuccess || hipMalloc(&out, (size_t)kCols * pitch * 8) != hipSuccess) { puts("oom"); return 1; }
    hipMemset(in, 1, n_tiles * 64 * kStride);
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    const int grid = p.multiProcessorCount * wpc;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const double bytes = (double)n_tiles * 64 * kStride + (double)kCols * pitch * 8;
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 6; rep++) {
            hipEventRecord(a);
            if (depth == 1) {
                if (mode == 0) hipLaunchKernelGGL((k<0, 1>), dim3(grid), dim3(64), 0, 0, in, out, n_tiles, pitch);
                if (mode == 1) hipLaunchKernelGGL((k<1, 1>), dim3(grid), dim3(64), 0, 0, in, out, n_tiles, pitch);
                if (mode == 2) hipLaunchKernelGGL((k<2, 1>), dim3(grid), dim3(64), 0, 0, in, out, n_tiles, pitch);
            } else {
                if (mode == 0) hipLaunchKernelGGL((k<0, 2>), dim3(grid), dim3(64), 0, 0, in, out, n_tiles, pitch);
                if (mode == 1) hipLaunchKernelGGL((k<1, 2>), dim3(grid), dim3(64), 0, 0, in, out, n_tiles, pitch);
                if (mode == 2) hipLaunchKernelGGL((k<2, 2>), dim3(grid), dim3(64), 0, 0, in, out, n_tiles, pitch);
            }
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep >= 4) printf("mode %d waves/CU %d depth %d: %.3f ms  %.0f GB/s\n", mode, wpc, depth, ms, bytes / ms / 1e6);
        }
    }
    return 0;
}
