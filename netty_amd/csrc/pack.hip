// pack.hip — gather variable-length chunk outputs from fixed-capacity slots into one contiguous
// stream (dst_off = exclusive scan of the lengths).  This is the device half of handing a batch
// of encoded chunks back to host ByteBufs with ONE D2H copy instead of one per chunk
// (MessageToByteEncoder hands each `out` downstream, MessageToByteEncoder.java:105-117; the frame
// bytes of chunk i follow chunk i-1 in SnappyFrameEncoder's output, SnappyFrameEncoder.java:89-117).
// One wave per chunk; 16-byte loads/stores when source and destination share 16-byte alignment,
// otherwise 4-byte loads through a funnel shift into aligned 4-byte stores.
#include "nx_common.hpp"

namespace nx {
namespace pk {

__global__ void __launch_bounds__(256) k_pack(const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                                              const uint32_t* __restrict__ len, uint8_t* __restrict__ dst,
                                              const uint64_t* __restrict__ dst_off, uint32_t n) {
    const int lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (c >= n) return;
    const uint8_t* s = src + src_off[c];
    uint8_t* d = dst + dst_off[c];
    const uint32_t L = len[c];
    const uint32_t sa = (uint32_t)((uintptr_t)s & 15u), da = (uint32_t)((uintptr_t)d & 15u);
    if (sa == da) {
        // head bytes up to 16-byte alignment, body in 16-byte vectors, tail bytes
        const uint32_t head = da ? (16u - da < L ? 16u - da : L) : 0u;
        if ((uint32_t)lane < head) d[lane] = s[lane];
        const uint32_t nv = (L - head) >> 4;
        const uint4* __restrict__ sv = reinterpret_cast<const uint4*>(s + head);
        uint4* __restrict__ dv = reinterpret_cast<uint4*>(d + head);
        for (uint32_t i = lane; i < nv; i += 64) dv[i] = sv[i];
        const uint32_t t0 = head + (nv << 4);
        if (t0 + (uint32_t)lane < L) d[t0 + lane] = s[t0 + lane];
    } else {
        for (uint32_t i = lane; i < L; i += 64) d[i] = s[i];
    }
}

}  // namespace pk
}  // namespace nx

extern "C" int32_t nx_pack_batch(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint8_t* dst,
                                 const uint64_t* dst_off, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!src || !src_off || !len || !dst || !dst_off) return NX_ERR_INVALID_ARG;
    hipLaunchKernelGGL(nx::pk::k_pack, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, src, src_off, len, dst, dst_off, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
