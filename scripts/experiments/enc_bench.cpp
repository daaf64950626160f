// Standalone timing harness for the Snappy encoder kernel (experiments only): N text chunks of
// 64 KiB generated on the host (include/netty_amd_textgen.h), encoded R times, kernel ms and the
// output checksum printed.  Variants are selected at compile time with -D flags.
#include "snappy_encode_lds_window.hip"
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
int main(int argc, char** argv) {
    int N = argc > 1 ? atoi(argv[1]) : 4096, R = argc > 2 ? atoi(argv[2]) : 3;
    const int L = 65536;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)N * L);
    for (int i = 0; i < 64 && i < N; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    for (int i = 64; i < N; ++i) memcpy(h.data() + (size_t)i * L, h.data() + (size_t)(i % 64) * L, L);
    const size_t cap = 76496;
    uint8_t *din, *dout;
    uint64_t *ioff, *ooff;
    uint32_t *ilen, *olen;
    int32_t* st;
    hipMalloc(&din, (size_t)N * L); hipMalloc(&dout, (size_t)N * cap);
    hipMalloc(&ioff, 8 * N); hipMalloc(&ooff, 8 * N); hipMalloc(&ilen, 4 * N); hipMalloc(&olen, 4 * N); hipMalloc(&st, 4 * N);
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (int i = 0; i < N; ++i) { io[i] = (uint64_t)i * L; oo[i] = (uint64_t)i * cap; }
    hipMemcpy(din, h.data(), h.size(), hipMemcpyHostToDevice);
    hipMemcpy(ioff, io.data(), 8 * N, hipMemcpyHostToDevice); hipMemcpy(ooff, oo.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(ilen, il.data(), 4 * N, hipMemcpyHostToDevice);
#ifdef NX_ENC_TIMING
    unsigned long long* tim;
    hipMalloc(&tim, 64);
    hipMemset(tim, 0, 64);
    hipMemcpyToSymbol(HIP_SYMBOL(nx::enc::g_tim), &tim, sizeof(tim));
#endif
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < R; ++r) {
        hipEventRecord(a);
        nx_snappy_encode_batch(din, ioff, ilen, dout, ooff, olen, st, N, 0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    std::vector<uint32_t> ol(N);
    std::vector<int32_t> s(N);
    hipMemcpy(ol.data(), olen, 4 * N, hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), st, 4 * N, hipMemcpyDeviceToHost);
    uint64_t tot = 0; int bad = 0;
    for (int i = 0; i < N; ++i) { tot += ol[i]; bad += s[i] != 0; }
    printf("N=%d ms=%.2f per_chunk_us=%.1f GiB/s=%.2f out=%llu bad=%d\n", N, best, best * 1e3 / N * 1024,
           (double)N * L / (best / 1e3) / (1 << 30), (unsigned long long)tot, bad);
#ifdef NX_ENC_TIMING
    unsigned long long t[8];
    hipMemcpy(t, tim, 64, hipMemcpyDeviceToHost);
    printf("windows/chunk %.0f  cycles/window: speculate %.0f  candidates %.0f  walk %.0f  emit+commit %.0f\n", (double)t[4] / N / R,
           (double)t[0] / t[4], (double)t[1] / t[4], (double)t[2] / t[4], (double)t[3] / t[4]);
#endif
    return 0;
}
