// snappy_decode_lane.hip — EXPERIMENT: lane-per-frame Snappy decode with 16-byte wide copies
// straight to HBM (no LDS history).  Timing prototype for the decoder design choice; semantics as
// snappy_decode_naive.hip (Snappy.java:315-650), no CRC.
#include "nx_common.hpp"

namespace nx {
namespace lane {

typedef unsigned int v4 __attribute__((ext_vector_type(4)));
typedef v4 v4u __attribute__((aligned(1)));
__device__ __forceinline__ v4 ld16(const uint8_t* p) { return *reinterpret_cast<const v4u*>(p); }
__device__ __forceinline__ void st16(uint8_t* p, v4 v) { *reinterpret_cast<v4u*>(p) = v; }

__global__ void __launch_bounds__(256) k_lane(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                              const uint32_t* __restrict__ in_len_a, uint8_t* __restrict__ out,
                                              const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                              int32_t* __restrict__ status, uint32_t n) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint8_t* s = in + in_off[c];
    uint8_t* o = out + out_off[c];
    const uint32_t in_len = in_len_a[c], cap = 65536u;
    uint32_t ip = 0, op = 0;
    int32_t st = NX_OK;
    uint32_t ulen = 0;
    {
        int bi = 0;
        bool complete = false;
        while (ip < in_len) {
            const uint32_t cur = s[ip++];
            ulen |= (cur & 0x7f) << (bi++ * 7);
            if ((cur & 0x80) == 0) {
                complete = true;
                break;
            }
            if (bi >= 4) break;
        }
        if (!complete) ip = in_len;
    }
    while (ip < in_len) {
        const uint32_t tag = s[ip++];
        const uint32_t type = tag & 3u;
        if (type == 0) {
            const uint32_t code = tag >> 2;
            uint32_t L;
            if (code < 60) {
                L = code + 1;
            } else {
                const uint32_t nb = code - 59;
                uint32_t v = 0;
                for (uint32_t k = 0; k < nb; ++k) v |= (uint32_t)s[ip + k] << (8 * k);
                ip += nb;
                L = v + 1;
            }
            if (in_len - ip < L || op + L > cap) {
                st = -50;
                break;
            }
            const uint32_t L16 = (L + 15u) & ~15u;
            if (ip + L16 <= in_len && op + L16 <= cap) {
                for (uint32_t k = 0; k < L; k += 16) st16(o + op + k, ld16(s + ip + k));
            } else {
                for (uint32_t k = 0; k < L; ++k) o[op + k] = s[ip + k];
            }
            ip += L;
            op += L;
        } else {
            uint32_t L, F;
            if (type == 1) {
                L = 4 + ((tag >> 2) & 7);
                F = ((tag & 0xe0) << 3) | s[ip];
                ip += 1;
            } else if (type == 2) {
                L = 1 + (tag >> 2);
                F = s[ip] | ((uint32_t)s[ip + 1] << 8);
                ip += 2;
            } else {
                L = 1 + (tag >> 2);
                F = s[ip] | ((uint32_t)s[ip + 1] << 8) | ((uint32_t)s[ip + 2] << 16) | ((uint32_t)s[ip + 3] << 24);
                ip += 4;
            }
            if (F == 0 || F > op || op + L > cap) {
                st = -51;
                break;
            }
            const uint32_t L16 = (L + 15u) & ~15u;
            if (F >= 16 && op + L16 <= cap) {
                for (uint32_t k = 0; k < L; k += 16) st16(o + op + k, ld16(o + op - F + k));
            } else {
                for (uint32_t k = 0; k < L; ++k) o[op + k] = o[op + k - F];
            }
            op += L;
        }
    }
    out_len[c] = op;
    status[c] = st;
}

}  // namespace lane
}  // namespace nx

extern "C" int32_t nx_snappy_decode_batch_lane_experiment(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                          uint8_t* out, const uint64_t* out_off, uint32_t* out_len, int32_t* status,
                                                          uint32_t n, void* stream) {
    hipLaunchKernelGGL(nx::lane::k_lane, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, in, in_off, in_len, out, out_off,
                       out_len, status, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
