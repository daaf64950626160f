// Does the table footprint matter (TLB reach / DRAM page locality)?  262 144 lanes, each a serial
// chain of 8 192 atomic exchanges into its own table of 2^b u32 entries (b = 12..15: 16 KiB .. 128 KiB
// per lane, 4 .. 32 GiB in total), and the same with 16-bit-sized tables addressed as u32 pairs.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void __launch_bounds__(256) k_chain(uint32_t* __restrict__ tab, uint32_t lanes, uint32_t K, uint32_t bits,
                                               uint32_t* __restrict__ sink) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= lanes) return;
    uint32_t* t = tab + ((size_t)l << bits);
    uint32_t h = l * 0x9E3779B1u, acc = 0;
    for (uint32_t i = 0; i < K; ++i) {
        const uint32_t v = __hip_atomic_exchange(&t[(h * 0x1e35a7bdu) >> (32 - bits)], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += v;
        h = h * 0x85EBCA77u + v + i;
    }
    sink[l] = acc;
}
int main() {
    const uint32_t lanes = 262144, K = 8192;
    uint32_t *tab, *sink;
    if (hipMalloc(&tab, (size_t)lanes << 17) != hipSuccess) return 1;
    if (hipMalloc(&sink, lanes * 4) != hipSuccess) return 1;
    (void)hipMemset(tab, 0, (size_t)lanes << 17);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep)
        for (uint32_t bits = 10; bits <= 15; ++bits) {
            hipLaunchKernelGGL(k_chain, dim3(lanes / 256), dim3(256), 0, 0, tab, lanes, 128u, bits, sink);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k_chain, dim3(lanes / 256), dim3(256), 0, 0, tab, lanes, K, bits, sink);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("table %3u KiB/lane (%5.1f GiB total): %.1f ms  %.2f G exchanges/s\n", (4u << bits) >> 10,
                   (double)lanes * (4u << bits) / (1 << 30), ms, (double)lanes * K / ms / 1e6);
        }
    return 0;
}
