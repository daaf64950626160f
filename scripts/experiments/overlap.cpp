// Overlap experiment (round 5; experiments only): can the record expander of one sub-batch run
// under the encoder of the next?  The encoder is bound by random table requests, the expander by
// its own instruction stream, so they might share CUs — if the encoder leaves LDS for an expander
// workgroup (its output stage: STAGE_DW dwords per lane) and registers for its waves.
// One TU with the kernel parts of snappy_encode.hip and snappy_decode.hip (scripts/build_overlap.sh),
// linked against libnetty_amd.so for the CRC tables.  Times, per 262 144 chunks: the encoder alone,
// the expander alone (3 and 1 workgroups per CU), and both at once on two streams.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <vector>
#include "nx_common.hpp"
#include "../../include/netty_amd_textgen.h"
#include ENC_SRC
#include DEC_SRC

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
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
    if (N % 256) return 1;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    if (nx::crc_tables_init() != 0) return 1;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    uint64_t* ws = nullptr;
    nx::PlacementReport rep{};
    CK(nx::alloc_placed_workspace<uint64_t>(N, 14, 0, &ws, &rep));
    printf("placement: %d candidates, pick %d (%.3f ms); stage %d dwords per lane\n", rep.n, rep.pick, rep.n ? rep.ms[rep.pick] : 0.f,
           (int)nx::enc::kStageDw);
    uint8_t *din, *enc1, *enc2, *dec;
    uint64_t *ioff, *ooff, *doff;
    uint32_t *ilen, *olen1, *olen2, *rec, *nrec, *dlen, *dlen0, *expect, *flag;
    int32_t *st1, *st2, *dst, *dst0;
    CK(hipMalloc(&din, (size_t)N * L));
    CK(hipMalloc(&enc1, (size_t)N * cap));
    CK(hipMalloc(&enc2, (size_t)N * cap));
    CK(hipMalloc(&dec, (size_t)N * L));
    CK(hipMalloc(&rec, (size_t)N * nx::dec::kRecCap * 4));
    CK(hipMalloc(&ioff, 8ull * N));
    CK(hipMalloc(&ooff, 8ull * N));
    CK(hipMalloc(&doff, 8ull * N));
    for (uint32_t** p : {&ilen, &olen1, &olen2, &nrec, &dlen, &dlen0, &expect, &flag}) CK(hipMalloc(p, 4ull * N));
    for (int32_t** p : {&st1, &st2, &dst, &dst0}) CK(hipMalloc(p, 4ull * N));
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (uint32_t i = 0; i < N; ++i) {
        io[i] = (uint64_t)i * L;
        oo[i] = (uint64_t)i * cap;
    }
    for (uint32_t i = 0; i < N; i += 1024) CK(hipMemcpy(din + (size_t)i * L, h.data(), (size_t)std::min(1024u, N - i) * L, hipMemcpyHostToDevice));
    CK(hipMemcpy(ioff, io.data(), 8ull * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(doff, io.data(), 8ull * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(ooff, oo.data(), 8ull * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(ilen, il.data(), 4ull * N, hipMemcpyHostToDevice));
    hipStream_t sA, sB;
    CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
    const dim3 egrid(N / 256), eblk(256);
    auto encode = [&](uint8_t* out, uint32_t* ol, int32_t* st, hipStream_t s) {
        hipLaunchKernelGGL((nx::enc::k_snappy_encode<true, false>), egrid, eblk, 0, s, din, ioff, ilen, out, ooff, ol, st, N, ws, 0u);
    };
    const size_t xlds = kExpandLds;
    auto expand = [&](unsigned per_cu, hipStream_t s) {
        hipLaunchKernelGGL(nx::dec::k_expand, dim3(cus * per_cu), dim3(nx::dec::kExpandWaves * 64), xlds, s, (const uint8_t*)enc1,
                           (const uint64_t*)ooff, (const uint32_t*)olen1, dec, (const uint64_t*)doff, (const uint32_t*)rec,
                           (const uint32_t*)nrec, dlen, dst, (const uint32_t*)nullptr, expect, N, nx::crc_tables_dev());
    };
    // the decode input: sub-batch Y encoded once, parsed once (records kept)
    CK(hipMemset(ws, 0, (size_t)N * 16384u * 8u));
    encode(enc1, olen1, st1, 0);
    CK(hipMemset(flag, 0, 4));
    hipLaunchKernelGGL(nx::dec::k_parse, dim3(N / 256), dim3(256), 0, 0, (const uint8_t*)enc1, (const uint64_t*)ooff, (const uint32_t*)olen1,
                       (const uint32_t*)nullptr, rec, nrec, dlen, (uint32_t*)nullptr, dst, N, flag);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(dlen0, dlen, 4ull * N, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(dst0, dst, 4ull * N, hipMemcpyDeviceToDevice));
    auto reset = [&]() {
        CK(hipMemset(ws, 0, (size_t)N * 16384u * 8u));
        CK(hipMemcpy(dlen, dlen0, 4ull * N, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(dst, dst0, 4ull * N, hipMemcpyDeviceToDevice));
        CK(hipDeviceSynchronize());
    };
    auto check = [&]() {  // every frame decoded (status 0) and the first 1024 equal their sources
        std::vector<int32_t> s(N);
        CK(hipMemcpy(s.data(), dst, 4ull * N, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < N; ++i)
            if (s[i] != 0) return false;
        std::vector<uint8_t> d((size_t)1024 * L);
        CK(hipMemcpy(d.data(), dec, d.size(), hipMemcpyDeviceToHost));
        return memcmp(d.data(), h.data(), d.size()) == 0;
    };
    hipEvent_t a0, a1, b0, b1;
    for (hipEvent_t* e : {&a0, &a1, &b0, &b1}) CK(hipEventCreate(e));
    for (uint32_t r = 0; r < R; ++r) {
        float ms;
        reset();
        CK(hipEventRecord(a0, sA));
        encode(enc2, olen2, st2, sA);
        CK(hipEventRecord(a1, sA));
        CK(hipEventSynchronize(a1));
        CK(hipEventElapsedTime(&ms, a0, a1));
        printf("encode alone          %8.2f ms\n", ms);
        for (unsigned per : {3u, 1u}) {
            reset();
            CK(hipEventRecord(b0, sB));
            expand(per, sB);
            CK(hipEventRecord(b1, sB));
            CK(hipEventSynchronize(b1));
            CK(hipEventElapsedTime(&ms, b0, b1));
            printf("expand alone (%u/CU)   %8.2f ms  ok %d\n", per, ms, (int)check());
        }
        for (unsigned per : {1u, 2u}) {
            reset();
            const double t0 = now_ms();
            CK(hipEventRecord(a0, sA));
            encode(enc2, olen2, st2, sA);
            CK(hipEventRecord(a1, sA));
            CK(hipEventRecord(b0, sB));
            expand(per, sB);
            CK(hipEventRecord(b1, sB));
            CK(hipStreamSynchronize(sA));
            CK(hipStreamSynchronize(sB));
            const double wall = now_ms() - t0;
            float me, mx;
            CK(hipEventElapsedTime(&me, a0, a1));
            CK(hipEventElapsedTime(&mx, b0, b1));
            printf("together (%u/CU): encode %8.2f ms, expand %8.2f ms, wall %8.2f ms  ok %d\n", per, me, mx, wall, (int)check());
        }
        for (unsigned per : {1u, 2u}) {  // the expander dispatched first, then the encoder
            reset();
            const double t0 = now_ms();
            CK(hipEventRecord(b0, sB));
            expand(per, sB);
            CK(hipEventRecord(b1, sB));
            CK(hipEventRecord(a0, sA));
            encode(enc2, olen2, st2, sA);
            CK(hipEventRecord(a1, sA));
            CK(hipStreamSynchronize(sA));
            CK(hipStreamSynchronize(sB));
            const double wall = now_ms() - t0;
            float me, mx;
            CK(hipEventElapsedTime(&me, a0, a1));
            CK(hipEventElapsedTime(&mx, b0, b1));
            printf("expand first (%u/CU): encode %8.2f ms, expand %8.2f ms, wall %8.2f ms  ok %d\n", per, me, mx, wall, (int)check());
        }
        fflush(stdout);
    }
    return 0;
}
