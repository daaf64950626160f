// Encoder variant timing (experiments only): the namespace-renamed copy snappy_encode_exp.hip,
// compiled with -D flags, against libnetty_amd's nx_snappy_encode_batch on the same N text chunks
// (byte-identical output required).
#ifndef NX_EXP_SWAP
#define NX_EXP_SWAP true
#endif
#include "snappy_encode_exp.hip"
#include "../../include/netty_amd.h"
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
int main(int argc, char** argv) {
    int N = argc > 1 ? atoi(argv[1]) : 262144, R = argc > 2 ? atoi(argv[2]) : 3;
    const int L = 65536;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)N * L);
    const int distinct = N < 1024 ? N : 1024;
    for (int i = 0; i < distinct; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    for (int i = distinct; i < N; ++i) memcpy(h.data() + (size_t)i * L, h.data() + (size_t)(i % distinct) * L, L);
    const size_t cap = 76496;
    uint8_t *din, *d1, *d2;
    uint64_t *ioff, *ooff;
    uint32_t *ilen, *l1, *l2;
    int32_t *s1, *s2;
    (void)hipMalloc(&din, (size_t)N * L); (void)hipMalloc(&d1, (size_t)N * cap); (void)hipMalloc(&d2, (size_t)N * cap);
    (void)hipMalloc(&ioff, 8 * N); (void)hipMalloc(&ooff, 8 * N); (void)hipMalloc(&ilen, 4 * N);
    (void)hipMalloc(&l1, 4 * N); (void)hipMalloc(&l2, 4 * N); (void)hipMalloc(&s1, 4 * N); (void)hipMalloc(&s2, 4 * N);
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (int i = 0; i < N; ++i) { io[i] = (uint64_t)i * L; oo[i] = (uint64_t)i * cap; }
    (void)hipMemcpy(din, h.data(), h.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(ioff, io.data(), 8 * N, hipMemcpyHostToDevice); (void)hipMemcpy(ooff, oo.data(), 8 * N, hipMemcpyHostToDevice);
    (void)hipMemcpy(ilen, il.data(), 4 * N, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best_ref = 1e30f, best = 1e30f;
    for (int r = 0; r < R; ++r) {
        float ms;
        (void)hipEventRecord(a);
        if (nx_snappy_encode_batch(din, ioff, ilen, d1, ooff, l1, s1, N, 0) != 0) return 2;
        (void)hipEventRecord(b); (void)hipEventSynchronize(b); (void)hipEventElapsedTime(&ms, a, b);
        best_ref = std::min(best_ref, ms);
        (void)hipEventRecord(a);
#if defined(NX_EXP_LDS)
        if (xexp_lds_encode_batch(din, ioff, ilen, d2, ooff, l2, s2, N, 0) != 0) return 2;
#elif defined(NX_EXP_SPREAD)
        if (xexp_spread_encode_batch(din, ioff, ilen, d2, ooff, l2, s2, N, 0) != 0) return 2;
#else
        if (xexp_nx_snappy_encode_batch(din, ioff, ilen, d2, ooff, l2, s2, N, 0) != 0) return 2;
#endif
        (void)hipEventRecord(b); (void)hipEventSynchronize(b); (void)hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
    }
    std::vector<uint32_t> h1(N), h2(N);
    (void)hipMemcpy(h1.data(), l1, 4 * N, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2.data(), l2, 4 * N, hipMemcpyDeviceToHost);
    std::vector<uint8_t> o1((size_t)N * cap), o2((size_t)N * cap);
    (void)hipMemcpy(o1.data(), d1, o1.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(o2.data(), d2, o2.size(), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < N; ++i) bad += h1[i] != h2[i] || memcmp(o1.data() + (size_t)i * cap, o2.data() + (size_t)i * cap, h1[i]) != 0;
    printf("N=%d ref_ms=%.1f variant_ms=%.1f ratio=%.3f mismatched_chunks=%d\n", N, best_ref, best, best / best_ref, bad);
    return bad != 0;
}
