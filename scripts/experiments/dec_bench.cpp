// Standalone timing harness for the Snappy decode kernels (experiments only).  N text chunks of
// 64 KiB (include/netty_amd_textgen.h) are encoded with libnetty_amd's nx_snappy_encode_batch, then
// decoded R times with the k_parse / k_expand of DEC_SRC (default: the product source; an A/B copy
// with -D flags for variants), compiled into this binary; per-kernel ms (HIP events) and the identity check are printed.
#ifndef DEC_SRC
#define DEC_SRC "../../netty_amd/csrc/snappy_decode.hip"
#endif
#include DEC_SRC
#include "../../include/netty_amd.h"
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
int main(int argc, char** argv) {
    using namespace nx::dec;
    int N = argc > 1 ? atoi(argv[1]) : 65536, R = argc > 2 ? atoi(argv[2]) : 3, crc = argc > 3 ? atoi(argv[3]) : 1;
    const int L = 65536;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)N * L);
    const int distinct = N < 1024 ? N : 1024;
    for (int i = 0; i < distinct; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    for (int i = distinct; i < N; ++i) memcpy(h.data() + (size_t)i * L, h.data() + (size_t)(i % distinct) * L, L);
    const size_t cap = 76496;
    uint8_t *din, *denc, *ddec;
    uint64_t *ioff, *ooff;
    uint32_t *ilen, *olen, *crcs, *dlen;
    int32_t* st;
    hipMalloc(&din, (size_t)N * L); hipMalloc(&denc, (size_t)N * cap); hipMalloc(&ddec, (size_t)N * L);
    hipMalloc(&ioff, 8 * N); hipMalloc(&ooff, 8 * N); hipMalloc(&ilen, 4 * N); hipMalloc(&olen, 4 * N); hipMalloc(&st, 4 * N);
    hipMalloc(&crcs, 4 * N); hipMalloc(&dlen, 4 * N);
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (int i = 0; i < N; ++i) { io[i] = (uint64_t)i * L; oo[i] = (uint64_t)i * cap; }
    hipMemcpy(din, h.data(), h.size(), hipMemcpyHostToDevice);
    hipMemcpy(ioff, io.data(), 8 * N, hipMemcpyHostToDevice); hipMemcpy(ooff, oo.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(ilen, il.data(), 4 * N, hipMemcpyHostToDevice);
    if (nx_crc32c_masked_batch(din, ioff, ilen, crcs, N, 0) != 0) return 2;
    if (nx_snappy_encode_batch(din, ioff, ilen, denc, ooff, olen, st, N, 0) != 0) return 2;
    hipDeviceSynchronize();
    if (nx::crc_tables_init() != NX_OK) return 2;
    const size_t lds = kTabBytes + kWaves * sizeof(WaveLds);
#ifdef NX_EXP_R8
#define K_EXPAND k_expand8
#else
#define K_EXPAND k_expand
#endif
    hipFuncSetAttribute((const void*)K_EXPAND, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned bpc = (unsigned)(160 * 1024 / lds);
    uint32_t *rec, *nrec;
    hipMalloc(&rec, (size_t)N * kRecCap * 4); hipMalloc(&nrec, 4 * N);
    hipEvent_t e0, e1, e2;
    hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
    float bp = 1e30f, be = 1e30f;
    const unsigned eg = (unsigned)std::min<uint64_t>((N + kWaves - 1) / kWaves, (uint64_t)cus * bpc);
    for (int r = 0; r < R; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_parse, dim3((N + kParseBlock - 1) / kParseBlock), dim3(kParseBlock), 0, 0, denc, ooff, olen, nullptr, rec,
                           nrec, dlen, nullptr, st, (uint32_t)N);
        hipEventRecord(e1);
        hipLaunchKernelGGL(K_EXPAND, dim3(eg), dim3(kWaves * 64), lds, 0, denc, ooff, olen, ddec, ioff, rec, nrec, dlen, st,
                           crc ? crcs : nullptr, nullptr, (uint32_t)N, nx::crc_tables_dev());
        hipEventRecord(e2);
        hipEventSynchronize(e2);
        float a, b;
        hipEventElapsedTime(&a, e0, e1);
        hipEventElapsedTime(&b, e1, e2);
        bp = std::min(bp, a);
        be = std::min(be, b);
    }
    std::vector<uint8_t> out((size_t)N * L);
    std::vector<int32_t> s(N);
    hipMemcpy(out.data(), ddec, out.size(), hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), st, 4 * N, hipMemcpyDeviceToHost);
    int bad = 0, badst = 0;
    for (int i = 0; i < N; ++i) {
        badst += s[i] != 0;
        bad += memcmp(out.data() + (size_t)i * L, h.data() + (size_t)i * L, L) != 0;
    }
    std::vector<uint32_t> ol(N);
    hipMemcpy(ol.data(), olen, 4 * N, hipMemcpyDeviceToHost);
    uint64_t tot = 0;
    for (int i = 0; i < N; ++i) tot += ol[i];
    printf("N=%d lds=%zu grid=%u parse_ms=%.2f expand_ms=%.2f per262k=%.1f+%.1f decGiB/s=%.1f ratio=%.4f badstatus=%d mismatch=%d\n", N, lds,
           eg, bp, be, bp * 262144.0 / N, be * 262144.0 / N, (double)N * L / ((bp + be) / 1e3) / (1 << 30), (double)tot / N / L, badst,
           bad);
#ifdef NX_EXP_COUNT
    unsigned long long c[8];
    hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cnt), sizeof(c));
    const double fr = (double)N * R;
    printf("per frame: passes %.1f rounds %.1f pieces %.1f far %.1f overlap %.1f  rounds/pass %.2f\n", c[0] / fr, c[1] / fr, c[2] / fr,
           c[3] / fr, c[4] / fr, (double)c[1] / c[0]);
#endif
    return 0;
}
