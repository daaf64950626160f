// A/B timing of two builds of the Snappy encoder on one box (experiments only): ENC_SRC is a copy of
// netty_amd/csrc/snappy_encode.hip compiled into this binary.  N text chunks of 64 KiB (1024 distinct,
// repeated), encoded R times with nx_snappy_encode_batch; prints the best kernel ms and an output
// checksum (equal checksums = identical bytes).
#include ENC_SRC
#ifdef ENC_FASTLZ  // level AUTO (1 below 64 KiB), u16 limit = chunk length
static int32_t fastlz_ab(const uint8_t* in, const uint64_t* io, const uint32_t* il, uint8_t* out, const uint64_t* oo, uint32_t* ol,
                         int32_t* st, uint32_t n, void* s) {
    return nx_fastlz_compress_batch(in, io, il, out, oo, ol, nullptr, nullptr, st, n, s);
}
#define ENC_FN fastlz_ab
#endif
#ifndef ENC_FN
#define ENC_FN nx_snappy_encode_batch
#endif
#ifndef ENC_LEN
#define ENC_LEN 65536
#endif
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 262144, R = argc > 2 ? atoi(argv[2]) : 3;
    const int L = ENC_LEN;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    const size_t cap = 76496;
    uint8_t *din, *dout;
    uint64_t *ioff, *ooff;
    uint32_t *ilen, *olen;
    int32_t* st;
    if (hipMalloc(&din, (size_t)N * L) || hipMalloc(&dout, (size_t)N * cap)) return 1;
    hipMalloc(&ioff, 8 * N); hipMalloc(&ooff, 8 * N); hipMalloc(&ilen, 4 * N); hipMalloc(&olen, 4 * N); hipMalloc(&st, 4 * N);
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (int i = 0; i < N; ++i) { io[i] = (uint64_t)i * L; oo[i] = (uint64_t)i * cap; }
    for (int i = 0; i < N; i += 1024) hipMemcpy(din + (size_t)i * L, h.data(), (size_t)std::min(1024, N - i) * L, hipMemcpyHostToDevice);
    hipMemcpy(ioff, io.data(), 8 * N, hipMemcpyHostToDevice); hipMemcpy(ooff, oo.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(ilen, il.data(), 4 * N, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < R; ++r) {
        hipEventRecord(a);
        if (ENC_FN(din, ioff, ilen, dout, ooff, olen, st, N, 0) != 0) return 2;
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    std::vector<uint32_t> ol(N);
    hipMemcpy(ol.data(), olen, 4 * N, hipMemcpyDeviceToHost);
    std::vector<uint8_t> ob(cap);
    unsigned long long sum = 0, tot = 0;
    for (int i = 0; i < 1024 && i < N; ++i) {
        hipMemcpy(ob.data(), dout + (size_t)i * cap, ol[i], hipMemcpyDeviceToHost);
        for (uint32_t k = 0; k < ol[i]; ++k) sum = sum * 1000003ull + ob[k];
    }
    for (int i = 0; i < N; ++i) tot += ol[i];
#ifdef ENC_SEL_DIAG
    printf("  candidates:");
    for (int k = 0; k < g_pn; ++k) printf(" %.3f", g_pms[k]);
    printf("  pick %d\n", g_pick);
#endif
    printf("%s N=%d best %.2f ms  %.1f GiB/s  out %llu B  checksum %016llx\n", ENC_NAME, N, best, (double)N * L / (best / 1e3) / (1 << 30), tot, sum);
    return 0;
}
