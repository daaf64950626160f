// lz4_frame.hip — the LZ4 frame codec around the block kernels.
//
//   nx_xxhash32_batch         Lz4XXHash32.update/getValue (Lz4XXHash32.java:37-102) per block: XXH32
//                             as lz4-java 1.8.0 computes it (third-party; restated from the published
//                             algorithm, pinned by Lz4FrameDecoderTest's vector and python-xxhash).
//   nx_lz4_frame_encode_batch Lz4FrameEncoder.flushBufferedData (Lz4FrameEncoder.java:248-284) per
//                             block: 21-byte header + compressed block, or the raw bytes when the
//                             compressed form is not smaller (:270-273).
//   nx_lz4_frame_scan_batch   Lz4FrameDecoder.decode's block walk (Lz4FrameDecoder.java:121-261) over
//                             device-resident cumulations, listing blocks for nx_lz4_decode_batch and
//                             nx_xxhash32_batch.
//
// XXH32 is a serial chain per 16-byte stripe lane (multiply, rotate, multiply), so one block's hash
// cannot be split across lanes and recombined as CRC32C can; the parallelism is across blocks, one
// lane each, with all four stripe accumulators in registers.  A lane streams its block with 16-byte
// loads; at 64 KiB blocks 262144 blocks give 4096 waves, enough to cover every SIMD several times.
#include "nx_common.hpp"
#include "../../include/netty_amd.h"

namespace nx {
namespace lz4f {

constexpr uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
constexpr int kHeader = 21;

typedef uint32_t __attribute__((aligned(1))) u32u;
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_rotateleft32(x, r); }
__device__ __forceinline__ uint32_t round1(uint32_t v, uint32_t w) { return rotl(v + w * P2, 13) * P1; }

__device__ __forceinline__ uint32_t sel4(uint32_t j, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t lo = (j & 1u) ? b : a, hi = (j & 1u) ? d : c;
    return (j & 2u) ? hi : lo;
}
// The four little-endian words at byte offset 4*j + sb of the 32-byte window lo:hi.
__device__ __forceinline__ void window_words(const uint4& lo, const uint4& hi, uint32_t j, uint32_t sb, uint32_t w[4]) {
    const uint32_t D[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t S[5];
#pragma unroll
    for (int m = 0; m < 5; ++m) S[m] = sel4(j, D[m], D[m + 1], D[m + 2], D[m + 3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = __builtin_amdgcn_alignbyte(S[k + 1], S[k], sb);
}

__device__ uint32_t xxh32(const uint8_t* __restrict__ p, uint32_t n, uint32_t seed) {
    uint32_t i = 0, h;
    if (n >= 16u) {
        uint32_t v0 = seed + P1 + P2, v1 = seed + P2, v2 = seed, v3 = seed - P1;
        const bool al16 = ((uintptr_t)p & 15u) == 0;
        if (al16) {
            // 128 bytes (eight 16-byte loads in flight: a whole line per lane, so no line is
            // fetched twice) per step, then single stripes
            for (; i + 16u <= n && (((uintptr_t)(p + i)) & 127u) != 0u; i += 16u) {  // up to a line start
                const uint4 q = *reinterpret_cast<const uint4*>(p + i);
                v0 = round1(v0, q.x);
                v1 = round1(v1, q.y);
                v2 = round1(v2, q.z);
                v3 = round1(v3, q.w);
            }
            for (; i + 128u <= n; i += 128u) {
                uint4 q[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) q[k] = *reinterpret_cast<const uint4*>(p + i + 16u * k);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    v0 = round1(v0, q[k].x);
                    v1 = round1(v1, q[k].y);
                    v2 = round1(v2, q[k].z);
                    v3 = round1(v3, q[k].w);
                }
            }
        }
        else {
            // Misaligned block (raw frame blocks sit at header + 21): aligned 16-byte loads, each
            // stripe's four words cut out of a 32-byte window with alignbyte (branch-free for any
            // offset).  Every granule read holds a byte of the block, so none crosses its page.
            const uint32_t r = (uint32_t)((uintptr_t)p & 15u), j = r >> 2, sb = r & 3u;
            const uint4* a = reinterpret_cast<const uint4*>(p - r);
            uint4 prev = a[0];
            // single stripes until the next granule load starts a 128-byte line, so the 128-byte
            // steps below read whole lines
            while (i + 16u <= n && (((uintptr_t)(a + (i >> 4) + 1u)) & 127u) != 0u) {
                const uint4 q = a[(i >> 4) + 1u];
                uint32_t w[4];
                window_words(prev, q, j, sb, w);
                v0 = round1(v0, w[0]);
                v1 = round1(v1, w[1]);
                v2 = round1(v2, w[2]);
                v3 = round1(v3, w[3]);
                prev = q;
                i += 16u;
            }
            for (; i + 128u <= n; i += 128u) {
                uint4 q[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) q[k] = a[(i >> 4) + 1u + k];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    uint32_t w[4];
                    window_words(prev, q[k], j, sb, w);
                    v0 = round1(v0, w[0]);
                    v1 = round1(v1, w[1]);
                    v2 = round1(v2, w[2]);
                    v3 = round1(v3, w[3]);
                    prev = q[k];
                }
            }
        }
        for (; i + 16u <= n; i += 16u) {
            v0 = round1(v0, ld32(p + i));
            v1 = round1(v1, ld32(p + i + 4));
            v2 = round1(v2, ld32(p + i + 8));
            v3 = round1(v3, ld32(p + i + 12));
        }
        h = rotl(v0, 1) + rotl(v1, 7) + rotl(v2, 12) + rotl(v3, 18);
    } else {
        h = seed + P5;
    }
    h += n;
    for (; i + 4u <= n; i += 4u) h = rotl(h + ld32(p + i) * P3, 17) * P4;
    for (; i < n; ++i) h = rotl(h + p[i] * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

// hdr == nullptr: out[i] = XXH32.  Otherwise the masked value goes little-endian into the checksum
// field of block i's frame header at hdr + hdr_off[i] + 17 (Lz4FrameEncoder.java:250-252, :282).
__global__ void __launch_bounds__(256) k_xxhash32(const uint8_t* __restrict__ in, const uint64_t* __restrict__ off,
                                                  const uint32_t* __restrict__ len, uint32_t seed, uint32_t* __restrict__ out,
                                                  uint8_t* __restrict__ hdr, const uint64_t* __restrict__ hdr_off, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = xxh32(in + off[i], len[i], seed);
    if (hdr == nullptr) {
        out[i] = h;
    } else if (len[i] != 0u) {
        uint8_t* q = hdr + hdr_off[i] + 17;
        const uint32_t m = h & 0x0FFFFFFFu;  // Lz4XXHash32.java:101
        q[0] = (uint8_t)m;
        q[1] = (uint8_t)(m >> 8);
        q[2] = (uint8_t)(m >> 16);
        q[3] = (uint8_t)(m >> 24);
    }
}

// One wave per block: lane 0 writes the header fields other than the checksum; when the compressed
// block is not smaller than the input (:270-273) the wave overwrites it with the raw bytes.
__global__ void __launch_bounds__(256) k_frame_fix(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                   const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                   int32_t* __restrict__ status, uint32_t level, uint32_t n) {
    const uint32_t i = blockIdx.x * (blockDim.x / NX_WAVE) + threadIdx.x / NX_WAVE;
    const uint32_t lane = threadIdx.x % NX_WAVE;
    if (i >= n) return;
    const uint32_t len = in_len[i];
    if (status[i] != NX_OK) return;
    if (len == 0u) {  // flushBufferedData writes nothing for an empty buffer (:249)
        if (lane == 0) out_len[i] = 0;
        return;
    }
    uint32_t clen = out_len[i];  // the block encoder's length (no header)
    uint32_t type = 0x20u;
    uint8_t* o = out + out_off[i];
    if (clen >= len) {
        type = 0x10u;
        clen = len;
        const uint8_t* s = in + in_off[i];
        for (uint32_t k = lane; k < len; k += NX_WAVE) o[kHeader + k] = s[k];
    }
    if (lane == 0) {
        const uint8_t magic[8] = {'L', 'Z', '4', 'B', 'l', 'o', 'c', 'k'};
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = magic[k];
        o[8] = (uint8_t)(type | level);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            o[9 + k] = (uint8_t)(clen >> (8 * k));
            o[13 + k] = (uint8_t)(len >> (8 * k));
        }
        out_len[i] = kHeader + clen;
    }
}

__device__ __forceinline__ int32_t le32s(const uint8_t* p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// One lane per stream, as the Snappy frame scan: each header gives the position of the next block.
__global__ void __launch_bounds__(256) k_frame_scan(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint64_t* __restrict__ in_len, uint32_t* __restrict__ state,
                                                    uint64_t* __restrict__ consumed, int32_t* __restrict__ status,
                                                    uint64_t* __restrict__ data_off, uint32_t* __restrict__ comp_len,
                                                    uint32_t* __restrict__ decomp_len, uint32_t* __restrict__ checksum,
                                                    uint32_t* __restrict__ block_stream, uint32_t* __restrict__ block_seq,
                                                    uint32_t* __restrict__ counts, uint32_t cap, uint32_t n) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint64_t base = in_off[s];
    const uint8_t* b = in + base;
    const uint64_t len = in_len[s];
    const uint32_t st = state[s];
    bool finished = st & 1u, corrupted = (st >> 1) & 1u;
    uint64_t p = 0;
    int32_t res = NX_OK;
    uint32_t seq = 0;
    if (finished || corrupted) {  // FINISHED / CORRUPTED skip everything readable (:251-254)
        p = len;
    } else {
        while (p < len) {
            if (len - p < (uint64_t)kHeader) break;  // :124-126
            const uint8_t* h = b + p;
            if (h[0] != 'L' || h[1] != 'Z' || h[2] != '4' || h[3] != 'B' || h[4] != 'l' || h[5] != 'o' || h[6] != 'c' ||
                h[7] != 'k') {  // :127-130
                res = NX_ERR_LZ4_BAD_MAGIC;
                break;
            }
            const uint32_t token = h[8];
            const uint32_t level = (token & 0x0Fu) + 10u, type = token & 0xF0u;
            const int32_t clen = le32s(h + 9), dlen = le32s(h + 13);
            if (clen < 0 || clen > (1 << 25)) {  // :136-141
                res = NX_ERR_LZ4_COMPRESSED_LENGTH;
                break;
            }
            if (dlen < 0 || (int64_t)dlen > (int64_t(1) << level)) {  // :143-149
                res = NX_ERR_LZ4_DECOMPRESSED_LENGTH;
                break;
            }
            if ((dlen == 0) != (clen == 0) || (type == 0x10u && dlen != clen)) {  // :150-156
                res = NX_ERR_LZ4_LENGTH_MISMATCH;
                break;
            }
            const uint32_t chk = (uint32_t)le32s(h + 17);
            if (dlen == 0) {  // the end block (:158-166)
                if (chk != 0u) {
                    res = NX_ERR_LZ4_END_CHECKSUM;
                    break;
                }
                finished = true;
                p = len;  // callDecode calls decode() again, and FINISHED skips what is left (:251-254)
                break;
            }
            if (len - p - kHeader < (uint64_t)clen) break;  // :180-182 (header re-read next call)
            if (type != 0x10u && type != 0x20u) {           // :209-213
                res = NX_ERR_LZ4_BLOCK_TYPE;
                break;
            }
            if (atomicAdd(&counts[2], 1u) >= cap) {
                res = NX_SCAN_LIST_FULL;
                break;
            }
            const uint32_t k = type == 0x20u ? atomicAdd(&counts[0], 1u) : cap - 1u - atomicAdd(&counts[1], 1u);
            data_off[k] = base + p + kHeader;
            comp_len[k] = (uint32_t)clen;
            decomp_len[k] = (uint32_t)dlen;
            checksum[k] = chk;
            block_stream[k] = s;
            block_seq[k] = seq++;
            p += kHeader + (uint64_t)clen;
        }
    }
    if (res < 0) corrupted = true;  // :257-259
    consumed[s] = p;
    status[s] = res;
    state[s] = (finished ? 1u : 0u) | (corrupted ? 2u : 0u);
}

}  // namespace lz4f
}  // namespace nx

extern "C" int32_t nx_xxhash32_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t seed,
                                     uint32_t* out, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !off || !len || !out) return NX_ERR_INVALID_ARG;
    hipLaunchKernelGGL(nx::lz4f::k_xxhash32, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, in, off, len, seed,
                       out, (uint8_t*)nullptr, (const uint64_t*)nullptr, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}

extern "C" int32_t nx_lz4hc_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                         const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream);

extern "C" int32_t nx_lz4_frame_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                             uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                             int32_t compression_level, int32_t* status, uint32_t n, void* stream) {
    return nx_lz4_frame_encode_batch_ex(in, in_off, in_len, out, out_off, out_len, compression_level, 0, status, n, stream);
}

extern "C" int32_t nx_lz4_frame_encode_batch_ex(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                                int32_t compression_level, int32_t high_compressor, int32_t* status, uint32_t n,
                                                void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status || compression_level < 0 ||
        compression_level > 15)
        return NX_ERR_INVALID_ARG;
    const hipStream_t st = (hipStream_t)stream;
    // block bodies go straight after each slot's header: the same out_off with the base moved by 21
    int32_t rc = (high_compressor ? nx_lz4hc_encode_batch : nx_lz4_encode_batch)(in, in_off, in_len, out + nx::lz4f::kHeader, out_off,
                                                                               out_len, status, n, stream);
    if (rc != NX_OK) return rc;
    hipLaunchKernelGGL(nx::lz4f::k_xxhash32, dim3((n + 255) / 256), dim3(256), 0, st, in, in_off, in_len,
                       0x9747b28cu, (uint32_t*)nullptr, out, out_off, n);
    NX_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(nx::lz4f::k_frame_fix, dim3((n + 3) / 4), dim3(256), 0, st, in, in_off, in_len, out, out_off, out_len,
                       status, (uint32_t)compression_level, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}

extern "C" int32_t nx_lz4_frame_scan_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                           uint32_t* state, uint64_t* consumed, int32_t* status, uint64_t* data_off,
                                           uint32_t* comp_len, uint32_t* decomp_len, uint32_t* checksum,
                                           uint32_t* block_stream, uint32_t* block_seq, uint32_t* counts, uint32_t cap,
                                           uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (!counts || (n && (!in || !in_off || !in_len || !state || !consumed || !status)) ||
        (cap && (!data_off || !comp_len || !decomp_len || !checksum || !block_stream || !block_seq)))
        return NX_ERR_INVALID_ARG;
    const hipStream_t st = (hipStream_t)stream;
    NX_HIP_CHECK(hipMemsetAsync(counts, 0, 3 * sizeof(uint32_t), st));
    if (n == 0) return NX_OK;
    hipLaunchKernelGGL(nx::lz4f::k_frame_scan, dim3((n + 255) / 256), dim3(256), 0, st, in, in_off, in_len, state, consumed,
                       status, data_off, comp_len, decomp_len, checksum, block_stream, block_seq, counts, cap, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
