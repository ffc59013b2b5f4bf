// Streaming-store bandwidth probe (MI355X): how fast can HBM absorb the
// hourly planes' write stream?  k_hourly_batt writes 3 f32 planes in
// hour-quad tiles [2190][n][4] (a lane stores 16 B, a wave 1 KB contiguous
// per plane every 4 hours, non-temporal).  This probe writes the same tile
// pattern with no arithmetic: one thread per agent, 2190 quads x 3 planes,
// `nt` vs plain stores, and a flat grid-stride stream for reference.
//   hipcc --offload-arch=gfx950 -O3 -o write_bw write_bw.hip && ./write_bw [n_agents]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(128) k_tiles(char* p0, char* p1, char* p2, long n, int quads) {
    const long i = (long)blockIdx.x * 128 + threadIdx.x;
    if (i >= n) return;
    const unsigned off = (unsigned)i * 16u;
    const size_t row = (size_t)n * 16u;
    f32x4 v = {(float)i, 1.0f, 2.0f, 3.0f};
    size_t q = 0;
    for (int k = 0; k < quads; k++, q += row) {
        v.x += 1.0f;
        if (NT) {
            asm volatile("global_store_dwordx4 %0, %1, %2 nt" :: "v"(off), "v"(v), "s"(p0 + q) : "memory");
            asm volatile("global_store_dwordx4 %0, %1, %2 nt" :: "v"(off), "v"(v), "s"(p1 + q) : "memory");
            asm volatile("global_store_dwordx4 %0, %1, %2 nt" :: "v"(off), "v"(v), "s"(p2 + q) : "memory");
        } else {
            asm volatile("global_store_dwordx4 %0, %1, %2" :: "v"(off), "v"(v), "s"(p0 + q) : "memory");
            asm volatile("global_store_dwordx4 %0, %1, %2" :: "v"(off), "v"(v), "s"(p1 + q) : "memory");
            asm volatile("global_store_dwordx4 %0, %1, %2" :: "v"(off), "v"(v), "s"(p2 + q) : "memory");
        }
    }
}

__global__ void k_flat(f32x4* p, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    f32x4 v = {1.0f, 2.0f, 3.0f, 4.0f};
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n16; k += stride) {
        v.x += 1.0f;
        __builtin_nontemporal_store(v, p + k);
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 200000;
    const int quads = 2190;
    const size_t plane = (size_t)n * 16u * quads;
    char *p0, *p1, *p2;
    CK(hipMalloc(&p0, plane));
    CK(hipMalloc(&p1, plane));
    CK(hipMalloc(&p2, plane));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const dim3 grid((unsigned)((n + 127) / 128)), block(128);
    for (int nt = 0; nt < 2; nt++) {
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(a));
            if (nt) hipLaunchKernelGGL(k_tiles<true>, grid, block, 0, 0, p0, p1, p2, n, quads);
            else hipLaunchKernelGGL(k_tiles<false>, grid, block, 0, 0, p0, p1, p2, n, quads);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("{\"probe\": \"tiles_%s\", \"agents\": %ld, \"bytes\": %zu, \"ms\": %.3f, \"TBps\": %.3f}\n",
                            nt ? "nt" : "plain", n, 3 * plane, ms, 3.0 * plane / ms / 1e9);
        }
    }
    for (int rep = 0; rep < 4; rep++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_flat, dim3(256 * 32), dim3(256), 0, 0, (f32x4*)p0, plane / 16);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep) printf("{\"probe\": \"flat_nt\", \"bytes\": %zu, \"ms\": %.3f, \"TBps\": %.3f}\n", plane, ms,
                        plane / ms / 1e9);
    }
    return 0;
}
