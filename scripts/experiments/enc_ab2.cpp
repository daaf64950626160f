// Placement-controlled A/B of two Snappy encoder builds (experiments only).  The encoder's time
// depends on where its 32 GiB table workspace lands (profiles/r02/s3/encoder_output_staging.md), so
// both builds are compiled into this one binary (ENC_A / ENC_B, each in its own namespace) and run
// alternately on the SAME workspace and buffers: the workspace is zeroed and both builds' stamp
// counters reset before every launch.  Prints per-launch ms and output checksums.
#include <stdlib.h>
#include <algorithm>
#include <map>
#include <mutex>
#include "../../netty_amd/csrc/nx_common.hpp"
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
#define nx_snappy_encode_batch enc_a_batch
#define nx_snappy_encode_placement enc_a_placement
namespace va {
#include ENC_A
}
#undef nx_snappy_encode_batch
#undef nx_snappy_encode_placement
#define nx_snappy_encode_batch enc_b_batch
#define nx_snappy_encode_placement enc_b_placement
namespace vb {
#include ENC_B
}
#undef nx_snappy_encode_batch
#undef nx_snappy_encode_placement
int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 262144, R = argc > 2 ? atoi(argv[2]) : 4;
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
    // one workspace, allocated by build A's first call, then shared
    if (va::enc_a_batch(din, ioff, ilen, dout, ooff, olen, st, N, 0)) return 2;
    hipDeviceSynchronize();
    uint64_t* ws = nullptr;
    size_t slots = 0;
    for (auto& kv : va::g_ws) { ws = kv.second.ws; slots = kv.second.threads; }
    for (auto& kv : va::g_ws) vb::g_ws[kv.first] = vb::Workspace{ws, slots, 0};
    hipDeviceptr_t wbase = nullptr;
    size_t wbytes = 0;
    if (hipMemGetAddressRange(&wbase, &wbytes, (hipDeviceptr_t)ws) != hipSuccess) return 4;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto sum = [&]() {
        std::vector<uint32_t> ol(1024);
        hipMemcpy(ol.data(), olen, 4 * 1024, hipMemcpyDeviceToHost);
        std::vector<uint8_t> ob(cap);
        unsigned long long s = 0;
        for (int i = 0; i < 1024; ++i) {
            hipMemcpy(ob.data(), dout + (size_t)i * cap, ol[i], hipMemcpyDeviceToHost);
            for (uint32_t k = 0; k < ol[i]; ++k) s = s * 1000003ull + ob[k];
        }
        return s;
    };
    for (int r = 0; r < R; ++r) {
        for (int v = 0; v < 2; ++v) {
            hipMemset(wbase, 0, wbytes);
            for (auto& kv : va::g_ws) kv.second.stamp = 0;
            for (auto& kv : vb::g_ws) kv.second.stamp = 0;
            hipDeviceSynchronize();
            hipEventRecord(a);
            const int rc = v == 0 ? va::enc_a_batch(din, ioff, ilen, dout, ooff, olen, st, N, 0)
                                  : vb::enc_b_batch(din, ioff, ilen, dout, ooff, olen, st, N, 0);
            hipEventRecord(b);
            hipEventSynchronize(b);
            if (rc) return 3;
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%s %.2f ms  checksum %016llx\n", v == 0 ? ENC_A : ENC_B, ms, sum());
            fflush(stdout);
        }
    }
    return 0;
}
