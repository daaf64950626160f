// Encoder run-to-run modes (experiments only): ENC_SRC (a copy of snappy_encode.hip) is compiled in,
// so this harness can drop the encoder's hash-table workspace between trials and let the next call
// allocate a fresh one.  Each trial prints the best of R launches and the workspace / buffer
// addresses, to tell placement effects from clock or box effects.
#include ENC_SRC
#include "../../netty_amd/tools/probe_ceiling.hip"
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 262144, R = argc > 2 ? atoi(argv[2]) : 3, T = argc > 3 ? atoi(argv[3]) : 6;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;  // 0: new workspace per trial; 1: also a 1 GiB spacer per trial
    const int L = 65536;
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
    std::vector<void*> spacers;
    for (int t = 0; t < T; ++t) {
        if (mode == 2 || mode == 3) {  // workspace allocated here: 2 = physically contiguous, 3 = default flags
            const size_t bytes = (size_t)262144 * 16384 * 8;
            void* p = nullptr;
            if (hipExtMallocWithFlags(&p, bytes, mode == 2 ? hipDeviceMallocContiguous : hipDeviceMallocDefault) != hipSuccess) {
                printf("alloc failed\n");
                return 5;
            }
            hipMemset(p, 0, bytes);
            g_ws[{0, (hipStream_t)0}] = Workspace{(uint64_t*)p, 262144, 0};
        }
        float best = 1e30f, worst = 0.f;
        for (int r = 0; r < R; ++r) {
            hipEventRecord(a);
            if (nx_snappy_encode_batch(din, ioff, ilen, dout, ooff, olen, st, N, 0) != 0) return 2;
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
            worst = ms > worst ? ms : worst;
        }
        void* wsp = nullptr;
        for (auto& kv : g_ws) wsp = kv.second.ws;
        // the same workspace under the encoder's request pattern without compute (probe_ceiling.hip)
        float pms[2] = {0.f, 0.f};
        for (int k = 0; k < 2; ++k)
            nx_probe_ceiling((uint64_t*)wsp, (const uint32_t*)din, olen, (uint32_t)std::min(N, 262144), k ? 1024u : 256u, k ? 258u : 0u, &pms[k], 0);
        printf("%s trial %d best %.2f worst %.2f ms  probe256(exchanges only) %.3f probe1024(+25.8%% loads) %.3f ms  ws %p in %p out %p\n", ENC_NAME, t, best, worst,
               pms[0], pms[1], wsp, (void*)din, (void*)dout);
        if (mode >= 1) {  // the same probe over each 4 GiB piece of the workspace alone (32 768 lanes)
            printf("   pieces:");
            for (int k = 0; k < 8; ++k) {
                float m = 0.f;
                nx_probe_ceiling((uint64_t*)wsp + (size_t)k * 32768 * 16384, (const uint32_t*)(din + (size_t)k * 32768 * L), olen, 32768u,
                                 512u, 258u, &m, 0);
                printf(" %.3f", m);
            }
            printf("\n");
        }
        fflush(stdout);
        for (auto& kv : g_ws) hipFree(kv.second.ws);
        g_ws.clear();
        if (mode == 1) {
            void* p = nullptr;
            hipMalloc(&p, (size_t)1 << 30);
            spacers.push_back(p);
        }
    }
    return 0;
}
