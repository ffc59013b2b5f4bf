// Probe (diagnostic, not product): does an agent-scope acquire fence
// (buffer_inv sc1 on gfx950) lose private-memory (scratch) stores made just
// before it?  Each lane fills a dynamically indexed private array (forced to
// scratch), fences, reads it back and counts mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(64) k_probe(const int* __restrict__ idx, int n, unsigned* bad,
                                              double* sink) {
    volatile double buf[512];
    const int lane = threadIdx.x + blockIdx.x * 64;
    for (int r = 0; r < 8; r++) {
        for (int k = 0; k < 512; k++) buf[idx[(k + r) % n] % 512] = lane * 1000.0 + k + r;
        if (MODE == 1) {
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        } else if (MODE == 2) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        unsigned nb = 0;
        double acc = 0.0;
        for (int k = 0; k < 512; k++) {
            const int j = idx[(k + r) % n] % 512;
            const double v = buf[j];
            acc += v;
            if (v != lane * 1000.0 + k + r) nb++;
        }
        if (nb) atomicAdd(bad, nb);
        sink[lane] = acc;
    }
}

int main() {
    const int n = 512, blocks = 2048;
    int h_idx[512];
    for (int k = 0; k < n; k++) h_idx[k] = k;   // identity: each slot written once per round
    int* d_idx;
    unsigned* d_bad;
    double* d_sink;
    hipMalloc(&d_idx, sizeof(h_idx));
    hipMalloc(&d_bad, sizeof(unsigned) * 3);
    hipMalloc(&d_sink, sizeof(double) * 64 * blocks);
    hipMemcpy(d_idx, h_idx, sizeof(h_idx), hipMemcpyHostToDevice);
    hipMemset(d_bad, 0, sizeof(unsigned) * 3);
    k_probe<0><<<blocks, 64>>>(d_idx, n, d_bad + 0, d_sink);
    k_probe<1><<<blocks, 64>>>(d_idx, n, d_bad + 1, d_sink);
    k_probe<2><<<blocks, 64>>>(d_idx, n, d_bad + 2, d_sink);
    hipError_t e = hipDeviceSynchronize();
    unsigned h_bad[3] = {0, 0, 0};
    hipMemcpy(h_bad, d_bad, sizeof(h_bad), hipMemcpyDeviceToHost);
    printf("status %s; mismatches: no fence %u, waitcnt+acquire %u, acquire %u (of %d reads each)\n",
           hipGetErrorString(e), h_bad[0], h_bad[1], h_bad[2], 8 * 512 * 64 * blocks);
    return 0;
}
