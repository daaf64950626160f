// Placement-controlled A/B of two Snappy encoder KERNEL builds (round 5; experiments only).
// enc_ab2.cpp drove the batch API, which now leases a shared workspace (workspace.hpp); this harness
// instead includes only the kernel part of each source (ENC_A / ENC_B: snappy_encode.hip cut before
// its host entry points, see scripts/enc_ab3.sh), places ONE 32 GiB table workspace with the
// product's own chooser (alloc_placed_workspace, 24 candidates) and launches the dense
// k_snappy_encode<true,false> of each build alternately on it, re-zeroing the workspace before
// every launch.  Prints per-launch ms (HIP events) and an output checksum per build.
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
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144u, R = argc > 2 ? (uint32_t)atoi(argv[2]) : 4u;
    const uint32_t L = 65536;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    const size_t cap = 76496;
    uint64_t* ws = nullptr;
    nx::PlacementReport rep{};
    if (nx::alloc_placed_workspace<uint64_t>(N, 14, 0, &ws, &rep) != hipSuccess) return 1;
    printf("placement: %d candidates, pick %d (%.3f ms)\n", rep.n, rep.pick, rep.n ? rep.ms[rep.pick] : 0.f);
    uint8_t *din, *dout;
    uint64_t *ioff, *ooff;
    uint32_t* olen;
    uint32_t* ilen;
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
    const dim3 grid(N / 256), blk(256);
    for (uint32_t r = 0; r < R; ++r) {
        for (int v = 0; v < 2; ++v) {
            (void)hipMemset(ws, 0, (size_t)N * 16384u * 8u);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(a);
            if (v == 0)
                hipLaunchKernelGGL((va::nx::enc::k_snappy_encode<true, false>), grid, blk, 0, 0, din, ioff, ilen, dout, ooff, olen, st, N,
                                   ws, 0u);
            else
                hipLaunchKernelGGL((vb::nx::enc::k_snappy_encode<true, false>), grid, blk, 0, 0, din, ioff, ilen, dout, ooff, olen, st, N,
                                   ws, 0u);
            (void)hipEventRecord(b);
            if (hipEventSynchronize(b) != hipSuccess) return 3;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("%s %.2f ms  checksum %016llx\n", v == 0 ? "A" : "B", ms, sum());
            fflush(stdout);
        }
    }
    return 0;
}
