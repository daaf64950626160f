// Encoder time against chunks per launch (round 6; experiments only).
// Built by scripts/enc_ab3.sh with MAIN=enc_curve: ENC_A / ENC_B are the kernel parts of two encoder
// sources.  ONE table workspace for the largest count is placed with the product's chooser
// (alloc_placed_workspace), then for every count N of the list and both builds the dense
// k_snappy_encode<true,false> runs once over N chunks (grid N / 256, one chunk per lane) on that same
// workspace, re-zeroed before each launch.  Prints ms per launch (HIP events), µs per chunk and an
// output checksum of the first 1024 chunks per build.
//   enc_curve_<tag> <reps> N1 N2 ...      (every N a multiple of 256)
//   enc_curve_<tag> <reps> loops L K1 K2 ...  (L lanes, each encoding K chunks in turn in one launch:
//   K x L chunks whose inputs and output slots repeat with period L; against K launches of L, it
//   shows what the tail of a launch costs, i.e. what a lane's varying chain time leaves idle)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "nx_common.hpp"
#include "../../include/netty_amd_textgen.h"
namespace va {
#include ENC_A
}
namespace vb {
#include ENC_B
}

// loops mode (see the header)
static int run_loops(uint32_t R, uint32_t Lanes, int nk, char** ks) {
    const uint32_t L = 65536;
    if (Lanes == 0 || Lanes % 256 != 0 || nk <= 0) return 2;
    uint32_t kmax = 1;
    for (int i = 0; i < nk; ++i) kmax = std::max(kmax, (uint32_t)atoi(ks[i]));
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    const size_t cap = 76496;
    uint64_t* ws = nullptr;
    nx::PlacementReport rep{};
    if (nx::alloc_placed_workspace<uint64_t>(Lanes, 14, 0, &ws, &rep) != hipSuccess) return 1;
    printf("placement: %d candidates, pick %d (%.3f ms), workspace %u lanes\n", rep.n, rep.pick, rep.n ? rep.ms[rep.pick] : 0.f, Lanes);
    const size_t N = (size_t)Lanes * kmax;
    uint8_t *din, *dout;
    uint64_t *ioff, *ooff;
    uint32_t *olen, *ilen;
    int32_t* st;
    if (hipMalloc(&din, (size_t)Lanes * L) || hipMalloc(&dout, (size_t)Lanes * cap)) return 1;
    if (hipMalloc(&ioff, 8 * N) || hipMalloc(&ooff, 8 * N) || hipMalloc(&ilen, 4 * N) || hipMalloc(&olen, 4 * N) || hipMalloc(&st, 4 * N))
        return 1;
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (size_t i = 0; i < N; ++i) {
        // chunk i = k * Lanes + t runs on lane t; its input rotates by 331 chunks per k, so a lane meets
        // other text chunks in turn (the 1024 distinct chunks repeat with period 1024)
        io[i] = (uint64_t)((i % Lanes + (i / Lanes) * 331u) % Lanes) * L;
        oo[i] = (uint64_t)(i % Lanes) * cap;
    }
    for (uint32_t i = 0; i < Lanes; i += 1024)
        (void)hipMemcpy(din + (size_t)i * L, h.data(), (size_t)std::min(1024u, Lanes - i) * L, hipMemcpyHostToDevice);
    (void)hipMemcpy(ioff, io.data(), 8 * N, hipMemcpyHostToDevice);
    (void)hipMemcpy(ooff, oo.data(), 8 * N, hipMemcpyHostToDevice);
    (void)hipMemcpy(ilen, il.data(), 4 * N, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (uint32_t r = 0; r < R; ++r) {
        for (int i = 0; i < nk; ++i) {
            const uint32_t K = (uint32_t)atoi(ks[i]);
            for (int mode = 0; mode < 2; ++mode) {  // 0: one launch, K chunks per lane; 1: K launches of one chunk per lane
                (void)hipMemset(ws, 0, (size_t)Lanes * 16384u * 8u);
                (void)hipDeviceSynchronize();
                (void)hipEventRecord(a);
                if (mode == 0) {
                    hipLaunchKernelGGL((vb::nx::enc::k_snappy_encode<true, false>), dim3(Lanes / 256), dim3(256), 0, 0, din, ioff, ilen, dout,
                                       ooff, olen, st, Lanes * K, ws, 0u);
                } else {
                    for (uint32_t k = 0; k < K; ++k)
                        hipLaunchKernelGGL((vb::nx::enc::k_snappy_encode<true, false>), dim3(Lanes / 256), dim3(256), 0, 0, din,
                                           ioff + (size_t)k * Lanes, ilen, dout, ooff + (size_t)k * Lanes, olen, st, Lanes, ws, k);
                }
                (void)hipEventRecord(b);
                if (hipEventSynchronize(b) != hipSuccess) return 3;
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                printf("%s lanes %u K %u  %9.2f ms  %.4f us/chunk\n", mode == 0 ? "one-launch" : "K-launches", Lanes, K, ms,
                       ms * 1e3 / ((double)Lanes * K));
                fflush(stdout);
            }
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s reps N1 [N2 ...]\n", argv[0]);
        return 2;
    }
    const uint32_t R = (uint32_t)atoi(argv[1]);
    std::vector<uint32_t> ns;
    const bool loops = argc > 3 && strcmp(argv[2], "loops") == 0;
    if (loops) return run_loops(R, (uint32_t)atoi(argv[3]), argc - 4, argv + 4);
    for (int i = 2; i < argc; ++i) {
        const uint32_t v = (uint32_t)atoi(argv[i]);
        if (v == 0 || v % 256 != 0) {
            fprintf(stderr, "N must be a positive multiple of 256: %u\n", v);
            return 2;
        }
        ns.push_back(v);
    }
    const uint32_t N = *std::max_element(ns.begin(), ns.end());
    const uint32_t L = 65536;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    const size_t cap = 76496;
    uint64_t* ws = nullptr;
    nx::PlacementReport rep{};
    if (nx::alloc_placed_workspace<uint64_t>(N, 14, 0, &ws, &rep) != hipSuccess) return 1;
    printf("placement: %d candidates, pick %d (%.3f ms), workspace %u lanes\n", rep.n, rep.pick, rep.n ? rep.ms[rep.pick] : 0.f, N);
    uint8_t *din, *dout;
    uint64_t *ioff, *ooff;
    uint32_t *olen, *ilen;
    int32_t* st;
    if (hipMalloc(&din, (size_t)N * L) || hipMalloc(&dout, (size_t)N * cap)) return 1;
    if (hipMalloc(&ioff, 8ull * N) || hipMalloc(&ooff, 8ull * N) || hipMalloc(&ilen, 4ull * N) || hipMalloc(&olen, 4ull * N) ||
        hipMalloc(&st, 4ull * N))
        return 1;
    std::vector<uint64_t> io(N), oo(N);
    std::vector<uint32_t> il(N, L);
    for (uint32_t i = 0; i < N; ++i) {
        io[i] = (uint64_t)i * L;
        oo[i] = (uint64_t)i * cap;
    }
    for (uint32_t i = 0; i < N; i += 1024)
        (void)hipMemcpy(din + (size_t)i * L, h.data(), (size_t)std::min(1024u, N - i) * L, hipMemcpyHostToDevice);
    (void)hipMemcpy(ioff, io.data(), 8ull * N, hipMemcpyHostToDevice);
    (void)hipMemcpy(ooff, oo.data(), 8ull * N, hipMemcpyHostToDevice);
    (void)hipMemcpy(ilen, il.data(), 4ull * N, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto sum = [&]() {
        std::vector<uint32_t> ol(1024);
        (void)hipMemcpy(ol.data(), olen, 4 * 1024, hipMemcpyDeviceToHost);
        std::vector<uint8_t> ob(cap);
        unsigned long long s = 0;
        for (int i = 0; i < 1024; ++i) {
            (void)hipMemcpy(ob.data(), dout + (size_t)i * cap, ol[i], hipMemcpyDeviceToHost);
            for (uint32_t k = 0; k < ol[i]; ++k) s = s * 1000003ull + ob[k];
        }
        return s;
    };
    for (uint32_t r = 0; r < R; ++r) {
        for (uint32_t n : ns) {
            for (int v = 0; v < 2; ++v) {
                (void)hipMemset(ws, 0, (size_t)n * 16384u * 8u);
                (void)hipDeviceSynchronize();
                const dim3 grid(n / 256), blk(256);
                (void)hipEventRecord(a);
                if (v == 0)
                    hipLaunchKernelGGL((va::nx::enc::k_snappy_encode<true, false>), grid, blk, 0, 0, din, ioff, ilen, dout, ooff, olen, st,
                                       n, ws, 0u);
                else
                    hipLaunchKernelGGL((vb::nx::enc::k_snappy_encode<true, false>), grid, blk, 0, 0, din, ioff, ilen, dout, ooff, olen, st,
                                       n, ws, 0u);
                (void)hipEventRecord(b);
                if (hipEventSynchronize(b) != hipSuccess) return 3;
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                printf("%s N %6u  %8.2f ms  %.4f us/chunk  checksum %016llx\n", v == 0 ? "A" : "B", n, ms, ms * 1e3 / n, sum());
                fflush(stdout);
            }
        }
    }
    return 0;
}
