// textgen.hip — device-side generator for the BASELINE "text-like" chunks (bench/test data only).
// One lane per chunk runs include/netty_amd_textgen.h's nx_tg_chunk; output is assembled in a
// 16-byte register word and stored with 16-byte stores when the destination is aligned.
#include "nx_common.hpp"
#include "../../include/netty_amd_textgen.h"
#include <mutex>

namespace nx {
namespace tg {

__global__ void __launch_bounds__(256) k_textgen(const nx_textgen_tables* __restrict__ t, uint8_t* __restrict__ out, uint64_t first,
                                                 uint32_t n_chunks, uint32_t chunk_len) {
    __shared__ uint32_t s_cdf[NX_TG_WORDS];
    __shared__ uint16_t s_off[NX_TG_WORDS + 1];
    const uint8_t* __restrict__ chars = t->chars;  // 40 KiB: read through L1/L2
    for (int i = threadIdx.x; i < (int)NX_TG_WORDS; i += blockDim.x) s_cdf[i] = t->cdf[i];
    for (int i = threadIdx.x; i <= (int)NX_TG_WORDS; i += blockDim.x) s_off[i] = (uint16_t)t->off[i];
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= n_chunks) return;
    uint8_t* o = out + (size_t)tid * chunk_len;
    const bool al = ((((uintptr_t)o) & 15u) == 0);
    uint64_t s = NX_TG_SEED_XOR ^ (first + tid);
    uint32_t pos = 0;
    uint32_t word[4] = {0, 0, 0, 0};
    uint32_t fill = 0;  // bytes in word[]
    auto emit = [&](uint8_t b) {
        if (pos >= chunk_len) return;
        if (al) {
            word[fill >> 2] |= (uint32_t)b << (8 * (fill & 3));
            if (++fill == 16) {
                *reinterpret_cast<uint4*>(o + pos - 15) = make_uint4(word[0], word[1], word[2], word[3]);
                word[0] = word[1] = word[2] = word[3] = 0;
                fill = 0;
            }
        } else {
            o[pos] = b;
        }
        ++pos;
    };
    while (pos < chunk_len) {
        const uint64_t r = nx_tg_splitmix(&s);
        const uint32_t w = nx_tg_pick(s_cdf, (uint32_t)(r >> 32));
        for (uint32_t c = s_off[w]; c < s_off[w + 1]; ++c) emit(chars[c]);
        if (((uint32_t)(r & 0xFFFFu)) % 10u == 0u) emit('.');
        emit(' ');
    }
    if (al && fill) {
        const uint32_t start = pos - fill;
        for (uint32_t i = 0; i < fill; ++i) o[start + i] = (uint8_t)(word[i >> 2] >> (8 * (i & 3)));
    }
}

}  // namespace tg
}  // namespace nx

namespace {
std::mutex g_mu;
nx_textgen_tables* g_dt = nullptr;
int g_dev = -1;
}  // namespace

extern "C" int32_t nx_textgen_device(uint8_t* out, uint64_t first_chunk, uint32_t n_chunks, uint32_t chunk_len, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n_chunks == 0) return NX_OK;
    if (!out) return NX_ERR_INVALID_ARG;
    int dev = 0;
    NX_HIP_CHECK(hipGetDevice(&dev));
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_dt || g_dev != dev) {
            nx_textgen_tables* h = new nx_textgen_tables;
            nx_textgen_build(h);
            NX_HIP_CHECK(hipMalloc(&g_dt, sizeof(nx_textgen_tables)));
            NX_HIP_CHECK(hipMemcpy(g_dt, h, sizeof(nx_textgen_tables), hipMemcpyHostToDevice));
            delete h;
            g_dev = dev;
        }
    }
    hipLaunchKernelGGL(nx::tg::k_textgen, dim3((n_chunks + 255) / 256), dim3(256), 0, (hipStream_t)stream, g_dt, out, first_chunk,
                       n_chunks, chunk_len);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
