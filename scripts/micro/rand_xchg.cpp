// Random-access ceiling for the Snappy encoder's table traffic (experiment): every lane runs a
// serial chain of K probes into its own 64 KiB table (16 384 u32 entries) in HBM, the next index
// hashed from the value returned.  Modes: 0 = atomic exchange (the encoder's probe), 1 = load then
// store, 2 = load only, 3 = the encoder's mix: an exchange, then (for ~60 % of the steps, as
// Snappy's candidate compares on the bench corpus: 9.7 K per 16.5 K probes) a dependent load at a
// random position of the lane's own 64 KiB input region.  Prints probes/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void __launch_bounds__(256) k_chain(uint32_t* __restrict__ tab, const uint32_t* __restrict__ inp, uint32_t lanes, uint32_t K,
                                               int mode, uint32_t* __restrict__ sink) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= lanes) return;
    uint32_t* t = tab + (size_t)l * 16384;
    const uint32_t* src = inp + (size_t)l * 16384;
    uint32_t h = l * 0x9E3779B1u, acc = 0;
    for (uint32_t i = 0; i < K; ++i) {
        const uint32_t idx = (h * 0x1e35a7bdu) >> 18;
        uint32_t v;
        if (mode == 0) {
            v = __hip_atomic_exchange(&t[idx], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (mode == 1) {
            v = t[idx];
            t[idx] = i;
        } else if (mode == 2) {
            v = __builtin_nontemporal_load(&t[idx]);
        } else {
            v = __hip_atomic_exchange(&t[idx], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (((h >> 7) % 10u) < 6u) v += src[(v * 0x27D4EB2Fu + i) >> 18];
        }
        acc += v;
        h = h * 0x85EBCA77u + v + i;
    }
    sink[l] = acc;
}
int main(int argc, char** argv) {
    const uint32_t K = 16384;
    uint32_t* tab;
    uint32_t* sink;
    uint32_t* inp;
    const uint32_t maxl = 262144;
    if (hipMalloc(&tab, (size_t)maxl * 16384 * 4) != hipSuccess) return 1;
    if (hipMalloc(&inp, (size_t)maxl * 16384 * 4) != hipSuccess) return 1;
    (void)hipMemset(inp, 1, (size_t)maxl * 16384 * 4);
    if (hipMalloc(&sink, maxl * 4) != hipSuccess) return 1;
    (void)hipMemset(tab, 0, (size_t)maxl * 16384 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int mode = 0; mode < 4; ++mode) {
        for (uint32_t lanes : {16384u, 65536u, 131072u, 262144u}) {
            hipLaunchKernelGGL(k_chain, dim3((lanes + 255) / 256), dim3(256), 0, 0, tab, inp, lanes, 256u, mode, sink);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k_chain, dim3((lanes + 255) / 256), dim3(256), 0, 0, tab, inp, lanes, K, mode, sink);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            const double probes = (double)lanes * K;
            printf("mode %d lanes %6u: %.1f ms  %.2f G probes/s  per-lane step %.0f ns\n", mode, lanes, ms, probes / ms / 1e6,
                   ms * 1e6 / K);
        }
    }
    return 0;
}
