// A/B timing of two builds of the FastLZ or LZF block decoder on one box (experiments only): DEC_SRC
// is a copy of netty_amd/csrc/fastlz.hip or lzf.hip compiled into this binary.  N text chunks of
// 65535 bytes (1024 distinct, repeated) are encoded once with the same build, then decoded R times;
// prints the best decode ms and whether every chunk came back byte-identical.
#include DEC_SRC
#include "../../include/netty_amd_textgen.h"
#include <stdio.h>
#include <string.h>
#include <vector>
int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 262144, R = argc > 2 ? atoi(argv[2]) : 3;
    const int L = 65535;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<uint8_t> h((size_t)1024 * L);
    for (int i = 0; i < 1024; ++i) nx_tg_chunk(&tg, i, h.data() + (size_t)i * L, L);
    const size_t cap = 70016;
    uint8_t *din, *dz, *dout;
    uint64_t *ioff, *zoff;
    uint32_t *ilen, *zlen;
    int32_t* st;
    if (hipMalloc(&din, (size_t)N * L) || hipMalloc(&dz, (size_t)N * cap) || hipMalloc(&dout, (size_t)N * L)) return 1;
    hipMalloc(&ioff, 8 * N); hipMalloc(&zoff, 8 * N); hipMalloc(&ilen, 4 * N); hipMalloc(&zlen, 4 * N); hipMalloc(&st, 4 * N);
    std::vector<uint64_t> io(N), zo(N);
    std::vector<uint32_t> il(N, L);
    for (int i = 0; i < N; ++i) { io[i] = (uint64_t)i * L; zo[i] = (uint64_t)i * cap; }
    for (int i = 0; i < N; i += 1024) hipMemcpy(din + (size_t)i * L, h.data(), (size_t)std::min(1024, N - i) * L, hipMemcpyHostToDevice);
    hipMemcpy(ioff, io.data(), 8 * N, hipMemcpyHostToDevice); hipMemcpy(zoff, zo.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(ilen, il.data(), 4 * N, hipMemcpyHostToDevice);
#ifdef DEC_FASTLZ
    if (nx_fastlz_compress_batch(din, ioff, ilen, dz, zoff, zlen, nullptr, nullptr, st, N, 0)) return 2;
#else
    if (nx_lzf_encode_batch(din, ioff, ilen, dz, zoff, zlen, st, N, 0)) return 2;
    // the decoder takes the compressed body of each ZV block (header 7 bytes; all blocks of text compress)
    std::vector<uint32_t> zl(N);
    hipMemcpy(zl.data(), zlen, 4 * N, hipMemcpyDeviceToHost);
    for (int i = 0; i < N; ++i) { zo[i] += 7; zl[i] -= 7; }
    hipMemcpy(zoff, zo.data(), 8 * N, hipMemcpyHostToDevice); hipMemcpy(zlen, zl.data(), 4 * N, hipMemcpyHostToDevice);
#endif
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < R; ++r) {
        hipMemset(dout, 0, (size_t)N * L);
        hipEventRecord(a);
#ifdef DEC_FASTLZ
        if (nx_fastlz_decompress_batch(dz, zoff, zlen, nullptr, dout, ioff, ilen, st, N, 0)) return 3;
#else
        if (nx_lzf_decode_batch(dz, zoff, zlen, dout, ioff, ilen, st, N, 0)) return 3;
#endif
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    std::vector<uint8_t> o((size_t)1024 * L);
    hipMemcpy(o.data(), dout + (size_t)(N - 1024) * L, o.size(), hipMemcpyDeviceToHost);
    const bool same = memcmp(o.data(), h.data(), o.size()) == 0;
    printf("%s N=%d decode best %.2f ms  %.1f GiB/s  identity %s\n", DEC_NAME, N, best, (double)N * L / (best / 1e3) / (1 << 30), same ? "ok" : "FAIL");
    return same ? 0 : 4;
}
