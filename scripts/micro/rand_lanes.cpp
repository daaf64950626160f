// Serial chains of dependent random atomic exchanges (the Snappy encoder's table probe) with FEWER
// lanes than the encoder runs, so that all tables fit the 256 MiB Infinity Cache (or the L2s): does
// a cache-resident working set raise the chain rate above the DRAM-bound ~18-21 G exchanges/s that
// 262 144 lanes x 64 KiB reach (rand_footprint.log)?  Mode 1 adds, after each exchange, a dependent
// load of the lane's own input region of 64 KiB (the candidate compare), for 60 % of the steps.
// Usage: rand_lanes  (prints one line per lanes x table size x mode)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void __launch_bounds__(256) k_chain(uint32_t* __restrict__ tab, const uint32_t* __restrict__ inp, uint32_t lanes,
                                               uint32_t K, uint32_t bits, int mode, uint32_t* __restrict__ sink) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= lanes) return;
    uint32_t* t = tab + ((size_t)l << bits);
    const uint32_t* in = inp + ((size_t)l << 14);
    uint32_t h = l * 0x9E3779B1u, acc = 0;
    for (uint32_t i = 0; i < K; ++i) {
        const uint32_t v = __hip_atomic_exchange(&t[(h * 0x1e35a7bdu) >> (32 - bits)], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += v;
        h = h * 0x85EBCA77u + v + i;
        if (mode == 1 && ((h >> 7) % 10u) < 6u) {
            const uint32_t w = in[(h * 0x9E3779B1u) >> 18];
            acc += w;
            h ^= w;
        }
    }
    sink[l] = acc;
}
int main() {
    const uint32_t maxl = 262144, K = 8192;
    uint32_t *tab, *inp, *sink;
    if (hipMalloc(&tab, (size_t)maxl << 16) != hipSuccess) return 1;
    if (hipMalloc(&inp, (size_t)maxl << 16) != hipSuccess) return 1;
    if (hipMalloc(&sink, maxl * 4) != hipSuccess) return 1;
    (void)hipMemset(tab, 0, (size_t)maxl << 16);
    (void)hipMemset(inp, 1, (size_t)maxl << 16);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int mode = 0; mode < 2; ++mode)
        for (uint32_t bits = 13; bits <= 14; ++bits)
            for (uint32_t lanes = 2048; lanes <= maxl; lanes *= 2) {
                hipLaunchKernelGGL(k_chain, dim3(lanes / 256), dim3(256), 0, 0, tab, inp, lanes, 256u, bits, mode, sink);
                (void)hipEventRecord(a);
                hipLaunchKernelGGL(k_chain, dim3(lanes / 256), dim3(256), 0, 0, tab, inp, lanes, K, bits, mode, sink);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                printf("mode %d table %3u KiB/lane lanes %6u (%7.1f MiB tables): %8.2f ms  %6.2f G steps/s  %7.0f ns/step/lane\n", mode,
                       (4u << bits) >> 10, lanes, (double)lanes * (4u << bits) / (1 << 20), ms, (double)lanes * K / ms / 1e6,
                       ms * 1e6 / K);
                fflush(stdout);
            }
    return 0;
}
