// Parse beside expand (round 6; experiments only).  Can k_parse of one piece of a
// decode call run while k_expand works on the previous piece?  k_expand is issue- and latency-bound
// at three 8-wave workgroups per CU (141.7 KB of LDS), k_parse latency-bound; a 128-lane parse block
// (19 KB, scripts/build_dec_pipe.sh builds the kernels with NX_PARSE_BLOCK=128) fits beside three
// expander workgroups, a 256-lane one beside two.  One TU with the kernel part of snappy_decode.hip,
// linked against libnetty_amd.so (encoder, CRC tables).  Per N frames of 64 KiB text chunks:
//   serial   : parse(N) then expand(N) on one stream (what nx_snappy_decode_batch does)
//   pipe P,X : P pieces; piece 0's parse, then expand(i) on stream A with parse(i+1) on stream B,
//              the expander at X workgroups per CU
// Every run's statuses, lengths and the first 1024 frames' bytes are checked.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "nx_common.hpp"
#include "../../include/netty_amd.h"
#include "../../include/netty_amd_textgen.h"
#include DEC_SRC

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144u, R = argc > 2 ? (uint32_t)atoi(argv[2]) : 3u;
    const uint32_t L = 65536, cap = 76496;
    if (N % 1024) return 1;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    if (nx::crc_tables_init() != 0) return 1;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    uint8_t *din, *enc, *dec;
    uint64_t *ioff, *ooff;
    uint32_t *ilen, *olen, *rec, *nrec, *dlen, *flag;
    int32_t *est, *dst;
    CK(hipMalloc(&din, (size_t)N * L));
    CK(hipMalloc(&enc, (size_t)N * cap));
    CK(hipMalloc(&dec, (size_t)N * L));
    CK(hipMalloc(&rec, (size_t)N * nx::dec::kRecCap * 4));
    CK(hipMalloc(&ioff, 8ull * N));
    CK(hipMalloc(&ooff, 8ull * N));
    for (uint32_t** p : {&ilen, &olen, &nrec, &dlen, &flag}) CK(hipMalloc(p, 4ull * N));
    for (int32_t** p : {&est, &dst}) CK(hipMalloc(p, 4ull * N));
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (uint32_t i = 0; i < N; ++i) {
        io[i] = (uint64_t)i * L;
        oo[i] = (uint64_t)i * cap;
    }
    for (uint32_t i = 0; i < N; i += 1024) CK(hipMemcpy(din + (size_t)i * L, h.data(), (size_t)1024 * L, hipMemcpyHostToDevice));
    CK(hipMemcpy(ioff, io.data(), 8ull * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(ooff, oo.data(), 8ull * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(ilen, il.data(), 4ull * N, hipMemcpyHostToDevice));
    if (nx_snappy_encode_batch(din, ioff, ilen, enc, ooff, olen, est, N, nullptr) != 0) return 3;
    CK(hipDeviceSynchronize());
    printf("parse block %d lanes (%zu B of LDS), expander %zu B per workgroup, %d CUs\n", nx::dec::kParseBlock,
           (size_t)nx::dec::kParseBlock * (nx::dec::ParseWin::kStride + nx::dec::ParseRec::kStride) * 4, (size_t)kExpandLds, cus);
    hipStream_t sA, sB;
    CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
    auto parse = [&](uint32_t base, uint32_t m, hipStream_t s) {
        hipLaunchKernelGGL(nx::dec::k_parse, dim3((m + nx::dec::kParseBlock - 1) / nx::dec::kParseBlock), dim3(nx::dec::kParseBlock), 0, s,
                           (const uint8_t*)enc, (const uint64_t*)ooff + base, (const uint32_t*)olen + base, (const uint32_t*)nullptr,
                           rec + (size_t)base * nx::dec::kRecCap, nrec + base, dlen + base, (uint32_t*)nullptr, dst + base, m, flag);
    };
    auto expand = [&](uint32_t base, uint32_t m, unsigned per_cu, hipStream_t s) {
        const uint64_t need = (m + nx::dec::kExpandWaves - 1) / nx::dec::kExpandWaves, want = (uint64_t)cus * per_cu;
        hipLaunchKernelGGL(nx::dec::k_expand, dim3((unsigned)(need < want ? need : want)), dim3(nx::dec::kExpandWaves * 64), kExpandLds, s,
                           (const uint8_t*)enc, (const uint64_t*)ooff + base, (const uint32_t*)olen + base, dec,
                           (const uint64_t*)ioff + base, (const uint32_t*)rec + (size_t)base * nx::dec::kRecCap,
                           (const uint32_t*)nrec + base, dlen + base, dst + base, (const uint32_t*)nullptr, (uint32_t*)nullptr, m,
                           nx::crc_tables_dev());
    };
    CK(hipFuncSetAttribute((const void*)nx::dec::k_expand, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kExpandLds));
    auto check = [&]() {
        std::vector<int32_t> s(N);
        std::vector<uint32_t> l(N);
        CK(hipMemcpy(s.data(), dst, 4ull * N, hipMemcpyDeviceToHost));
        CK(hipMemcpy(l.data(), dlen, 4ull * N, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < N; ++i)
            if (s[i] != 0 || l[i] != L) return false;
        std::vector<uint8_t> d((size_t)1024 * L);
        CK(hipMemcpy(d.data(), dec, d.size(), hipMemcpyDeviceToHost));
        return memcmp(d.data(), h.data(), d.size()) == 0;
    };
    auto clear = [&]() {
        CK(hipMemset(dec, 0, (size_t)1024 * L));
        CK(hipMemset(dst, 0xFF, 4ull * N));
        CK(hipMemset(flag, 0, 4));
        CK(hipDeviceSynchronize());
    };
    hipEvent_t t0, t1, go;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventCreateWithFlags(&go, hipEventDisableTiming));
    std::vector<hipEvent_t> pev(64);
    for (auto& e : pev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (uint32_t r = 0; r < R; ++r) {
        float ms;
        clear();
        CK(hipEventRecord(t0, sA));
        parse(0, N, sA);
        expand(0, N, 3, sA);
        CK(hipEventRecord(t1, sA));
        CK(hipEventSynchronize(t1));
        CK(hipEventElapsedTime(&ms, t0, t1));
        printf("serial              %8.2f ms  ok %d\n", ms, (int)check());
        for (unsigned P : {2u, 4u, 8u}) {
            for (unsigned X : {3u, 2u}) {
                const uint32_t m = N / P;
                clear();
                CK(hipEventRecord(t0, sA));
                parse(0, m, sA);
                CK(hipEventRecord(go, sA));
                CK(hipStreamWaitEvent(sB, go, 0));
                for (unsigned i = 0; i < P; ++i) {
                    if (i + 1 < P) {  // the next piece's parse beside this piece's expand
                        parse((i + 1) * m, m, sB);
                        CK(hipEventRecord(pev[i + 1], sB));
                    }
                    if (i > 0) CK(hipStreamWaitEvent(sA, pev[i], 0));
                    expand(i * m, m, X, sA);
                }
                CK(hipEventRecord(t1, sA));
                CK(hipEventSynchronize(t1));
                CK(hipEventElapsedTime(&ms, t0, t1));
                printf("pipe P %u X %u/CU    %8.2f ms  ok %d\n", P, X, ms, (int)check());
            }
        }
        fflush(stdout);
    }
    return 0;
}
