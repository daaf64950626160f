// Encoder time against chunks per launch (round 6; experiments only).
// Built by scripts/enc_ab3.sh with MAIN=enc_curve: ENC_A / ENC_B are the kernel parts of two encoder
// sources.  ONE table workspace for the largest count is placed with the product's chooser
// (alloc_placed_workspace), then for every count N of the list and both builds the dense
// k_snappy_encode<true,false> runs once over N chunks (grid N / 256, one chunk per lane) on that same
// workspace, re-zeroed before each launch.  Prints ms per launch (HIP events), µs per chunk and an
// output checksum of the first 1024 chunks per build.
//   enc_curve_<tag> <reps> N1 N2 ...      (every N a multiple of 256)
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
int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s reps N1 [N2 ...]\n", argv[0]);
        return 2;
    }
    const uint32_t R = (uint32_t)atoi(argv[1]);
    std::vector<uint32_t> ns;
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
