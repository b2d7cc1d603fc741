// ubench_lut.hip -- LDS cost of a per-byte 256-entry code-page lookup on gfx950 (design probe for the
// Utf8 string path).  Each lane looks up 20 bytes per iteration (one PIC X(20)
// value), the way the string decoders do, with one of these table forms:
//   0  ds_read_b32  1 KiB table of 4-byte entries (the LUT the kernels use today)
//   1  ds_read_u8   256-byte table
//   2  ds_bpermute  the 256-byte table held in ONE VGPR across the wave (+ byte extract)
//   3  ds_read_b32  32 KiB table, 32 copies interleaved so lane l always hits bank l % 32
//   4  ds_read_u16  16 KiB table of 2-byte entries, 32 interleaved copies
//   5  ds_read_u8   8 KiB table of 1-byte entries, 32 interleaved copies
//   8  no lookup (the byte generator + accumulate alone: the VALU floor)
//   9  compose stores: 40 ds_write_b8 into a lane slot (today's multi-byte compose)
//  10  compose stores: 6 ds_write2_b32 into a lane slot (the carry compose)
// Bytes come from a per-lane LCG (no HBM traffic): "uniform" = any byte, "text" = 33-byte alphabet
// 32 letters + ~25 % EBCDIC spaces (SYNSTR200-like).  Output: ns per wave-lookup-instruction
// per CU (LDS cycles = that x clock).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lut tools/ubench_lut.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

template <int V, bool kText>
__global__ __launch_bounds__(256) void lut_kernel(const uint32_t* lut_in, uint32_t* out, int iters, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint32_t lut[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) {
        const uint32_t e = lut_in[(i >> 5) & 255];
        if (V == 3) lut[i] = e;                                    // [b][copy]
        else if (V == 4) ((uint16_t*)lut)[i * 2] = (uint16_t)e, ((uint16_t*)lut)[i * 2 + 1] = (uint16_t)(e >> 8);
        else lut[i] = lut_in[i & 255];
    }
    if (V == 5) {
        __syncthreads();
        for (int i = threadIdx.x; i < 8192; i += 256) {
            // dword (b >> 2) * 32 + copy holds entries 4(b>>2) .. +3 for that copy
            const int q = i >> 5;
            lut[i] = (lut_in[4 * q] & 255) | (lut_in[4 * q + 1] & 255) << 8 | (lut_in[4 * q + 2] & 255) << 16 |
                     (lut_in[4 * q + 3] & 255) << 24;
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t lreg = (lut_in[4 * lane] & 255) | (lut_in[4 * lane + 1] & 255) << 8 | (lut_in[4 * lane + 2] & 255) << 16 |
                          (lut_in[4 * lane + 3] & 255) << 24;
    uint8_t* slot = (uint8_t*)lut + (threadIdx.x >> 6) * 3328 + lane * 52;   // V 9/10: 52-byte lane slots
    uint32_t x = seed ^ ((blockIdx.x * 256 + threadIdx.x) * 2654435761u);
    uint32_t acc = 0, tr = 0;
    for (int it = 0; it < iters; it++) {
        uint32_t w[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            x = x * 1664525u + 1013904223u;
            uint32_t v = x;
            if (kText) {   // 32 letters 0xC0-0xDF, ~25 % EBCDIC spaces (VALU only, no table)
                const uint32_t sp = (v >> 5) & (v >> 6) & 0x01010101u;
                const uint32_t m = sp * 0xFFu;
                v = (((v & 0x1F1F1F1Fu) + 0xC0C0C0C0u) & ~m) | (0x40404040u & m);
            }
            w[k] = v;
        }
        if (V == 9) {
            uint8_t* p = slot;
#pragma unroll
            for (int j = 0; j < 20; j++) {
                const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 255;
                p[0] = (uint8_t)b;
                p[1] = (uint8_t)(b >> 1);
                p += 1 + (b >> 7);
            }
            acc += (uint32_t)(p - slot);
            continue;
        }
        if (V == 10) {
            uint32_t o = 0;
#pragma unroll
            for (int g = 0; g < 5; g++) {
                uint32_t* d = (uint32_t*)(slot + (o & ~3u));
                d[0] = w[g];
                d[1] = w[g] >> 3;
                o += 4 + __builtin_popcount(w[g] & 0x80808080u);
            }
            *(uint32_t*)(slot + (o & ~3u)) = o;
            acc += o;
            continue;
        }
#pragma unroll
        for (int j = 0; j < 20; j++) {
            const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 255;
            uint32_t e;
            if (V == 0) e = lut[b];
            else if (V == 1) e = ((const uint8_t*)lut)[b];
            else if (V == 2) e = ((uint32_t)__builtin_amdgcn_ds_bpermute((int)(b & 0xFCu), (int)lreg) >> ((b & 3) * 8)) & 255u;
            else if (V == 3) e = lut[(b << 5) | (lane & 31)];
            else if (V == 4) e = ((const uint16_t*)lut)[(((b >> 1) << 5) | (lane & 31)) * 2 + (b & 1)];
            else if (V == 5) e = ((const uint8_t*)lut)[((((b >> 2) << 5) | (lane & 31)) << 2) | (b & 3)];
            else e = b * 0x01010101u;
            tr = __builtin_amdgcn_alignbit(tr, e, 31);
            acc += e >> 24 | (e & 3);
        }
    }
    if ((acc ^ tr) == 0x12345678u) out[blockIdx.x] = acc;   // keep the work live
}

template <int V, bool kText>
static float run(const uint32_t* d_lut, uint32_t* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    lut_kernel<V, kText><<<blocks, 256>>>(d_lut, d_out, iters, 1u);   // warm-up
    CK(hipGetLastError());
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; r++) lut_kernel<V, kText><<<blocks, 256>>>(d_lut, d_out, iters, 7u + r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / 5;
}

int main(int argc, char** argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 5;   // 32 KiB LDS per block: 5 blocks (20 waves) per CU
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    std::vector<uint32_t> h(256);
    for (int i = 0; i < 256; i++) h[i] = (uint32_t)((i * 37 + 11) & 255) | (1u << 24) | (i < 0x41 ? 0x80000000u : 0u);
    uint32_t *d_lut, *d_out;
    CK(hipMalloc(&d_lut, 1024));
    CK(hipMalloc(&d_out, blocks * 4));
    CK(hipMemcpy(d_lut, h.data(), 1024, hipMemcpyHostToDevice));
    const double per_cu = (double)blocks * 4 * iters / cus;   // wave-iterations per CU
    struct R { const char* name; float u, t; int n; };
    std::vector<R> rs;
#define RUN(V, name, n) rs.push_back({name, run<V, false>(d_lut, d_out, blocks, iters), run<V, true>(d_lut, d_out, blocks, iters), n})
    RUN(8, "none (VALU floor)", 20);
    RUN(0, "ds_read_b32 1KiB", 20);
    RUN(1, "ds_read_u8 256B", 20);
    RUN(2, "ds_bpermute 1 VGPR", 20);
    RUN(3, "ds_read_b32 32KiB x32", 20);
    RUN(4, "ds_read_u16 16KiB x32", 20);
    RUN(5, "ds_read_u8 8KiB x32", 20);
    RUN(9, "40 x ds_write_b8", 40);
    RUN(10, "6 x ds_write2_b32", 6);
    printf("{\"cus\": %d, \"blocks\": %d, \"iters\": %d, \"results\": [\n", cus, blocks, iters);
    for (size_t i = 0; i < rs.size(); i++) {
        const double nu = rs[i].u * 1e6 / (per_cu * rs[i].n), nt = rs[i].t * 1e6 / (per_cu * rs[i].n);
        printf("  {\"variant\": \"%s\", \"ms_uniform\": %.3f, \"ms_text\": %.3f, \"ns_per_wave_instr_per_cu_uniform\": %.4f, "
               "\"ns_per_wave_instr_per_cu_text\": %.4f}%s\n",
               rs[i].name, rs[i].u, rs[i].t, nu, nt, i + 1 < rs.size() ? "," : "");
    }
    printf("]}\n");
    return 0;
}
