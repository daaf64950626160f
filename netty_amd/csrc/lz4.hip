// lz4.hip — LZ4 block encoder, one lane per block.
//
// Lz4FrameEncoder compresses each block with lz4-java 1.8.0's LZ4Compressor
// (Lz4FrameEncoder.java:259-275), a third-party dependency absent from the reference, so its exact
// output cannot be pinned here.  This kernel is bit-exact with the oracle's greedy block compressor
// (oracle/netty_oracle.c orc_lz4_compress): a 4096-entry hash of the 4 bytes at each probed position
// (the step over misses grows by one every 64 misses, LZ4's skip acceleration), matches of >= 4
// bytes extended to at most 5 bytes before the end, the last
// 5 bytes always literal and no match starting in the last 12 (the block-format end rules every
// LZ4 decoder relies on).  Its blocks decode with nx_lz4_decode_batch and any LZ4 block decoder.
//
// Like the Snappy encoder, each lane owns a hash table in an HBM workspace; entries carry a 16-bit
// stamp (the lane's chunk counter) above the 16-bit position, so a table is never cleared between
// chunks.
#include <algorithm>
#include <map>
#include <mutex>
#include "nx_common.hpp"

namespace nx {
namespace lz4 {

constexpr int kHashLog = 12;
constexpr int kMinMatch = 4, kLastLiterals = 5, kMfLimit = 12;

typedef uint32_t __attribute__((aligned(1))) u32u;
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }

__device__ __forceinline__ uint32_t put_len(uint8_t* out, uint32_t op, uint32_t v) {  // extension of a length >= 15
    v -= 15u;
    while (v >= 255u) {
        out[op++] = 255u;
        v -= 255u;
    }
    out[op++] = (uint8_t)v;
    return op;
}

// Large == false: blocks of <= 64 KiB, entries = stamp << 16 | position (no clearing).
// Large == true: blocks of up to 32 MiB (Lz4FrameEncoder block sizes above the default), entries =
// position + 1 in a table the lane zeroes before the block and again after it, so no stale entry
// can pass a later small block's stamp check (stamps start at 1).
template <bool Large>
__device__ uint32_t encode_block(const uint8_t* __restrict__ in, int32_t n, uint8_t* __restrict__ out,
                                 uint32_t* __restrict__ table, uint32_t stamp) {
    uint32_t op = 0;
    int32_t anchor = 0, ip = 0, search = 64;
    const int32_t mlimit = n - kMfLimit;
    const uint32_t stag = stamp << 16;
    if (Large)
        for (uint32_t k = 0; k < (1u << kHashLog); ++k) __hip_atomic_store(table + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (n >= kMfLimit + 1 && ip <= mlimit) {
        const uint32_t w = ld32(in + ip);
        const uint32_t h = (w * 2654435761u) >> (32 - kHashLog);
        const uint32_t e = __hip_atomic_exchange(table + h, Large ? (uint32_t)ip + 1u : (stag | (uint32_t)ip), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        const int32_t ref = Large ? (int32_t)e - 1 : ((e & 0xFFFF0000u) == stag ? (int32_t)(e & 0xFFFFu) : -1);
        if (ref < 0 || ip - ref > 65535 || ld32(in + ref) != w) {
            ip += search++ >> 6;  // LZ4's skip acceleration (skipTrigger 6), as the oracle
            continue;
        }
        search = 64;
        int32_t ml = kMinMatch;
        while (ip + ml < n - kLastLiterals && in[ref + ml] == in[ip + ml]) ++ml;
        const uint32_t lit = (uint32_t)(ip - anchor);
        const uint32_t mc = (uint32_t)(ml - kMinMatch);
        out[op++] = (uint8_t)(((lit >= 15u ? 15u : lit) << 4) | (mc >= 15u ? 15u : mc));
        if (lit >= 15u) op = put_len(out, op, lit);
        for (uint32_t k = 0; k < lit; ++k) out[op + k] = in[anchor + k];
        op += lit;
        out[op++] = (uint8_t)((ip - ref) & 255);
        out[op++] = (uint8_t)((ip - ref) >> 8);
        if (mc >= 15u) op = put_len(out, op, mc);
        ip += ml;
        anchor = ip;
    }
    if (Large)
        for (uint32_t k = 0; k < (1u << kHashLog); ++k) __hip_atomic_store(table + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t lit = (uint32_t)(n - anchor);  // last literals
    out[op++] = (uint8_t)((lit >= 15u ? 15u : lit) << 4);
    if (lit >= 15u) op = put_len(out, op, lit);
    for (uint32_t k = 0; k < lit; ++k) out[op + k] = in[anchor + k];
    return op + lit;
}

__global__ void __launch_bounds__(256) k_lz4_encode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                    const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                    int32_t* __restrict__ status, uint32_t n, uint32_t* __restrict__ workspace,
                                                    uint32_t stamp_base) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nthreads = gridDim.x * blockDim.x;
    uint32_t* table = workspace + (size_t)tid * (1u << kHashLog);
    uint32_t iter = 0;
    for (uint32_t c = tid; c < n; c += nthreads, ++iter) {
        const uint32_t len = in_len[c];
        if (len >= (1u << 25)) {
            out_len[c] = 0;
            status[c] = NX_ERR_INVALID_ARG;
            continue;
        }
        out_len[c] = len > 65536u ? encode_block<true>(in + in_off[c], (int32_t)len, out + out_off[c], table, 0u)
                                  : encode_block<false>(in + in_off[c], (int32_t)len, out + out_off[c], table, stamp_base + iter + 1u);
        status[c] = NX_OK;
    }
}

}  // namespace lz4
}  // namespace nx

namespace {
struct Lz4Workspace {
    uint32_t* ws = nullptr;
    size_t threads = 0;
    uint32_t stamp = 0;
};
std::mutex g_lz4_mu;
std::map<std::pair<int, hipStream_t>, Lz4Workspace> g_lz4_ws;
constexpr uint32_t kMaxStamp = 0xFFFFu;
}  // namespace

extern "C" size_t nx_lz4_max_compressed_length(size_t n) { return n + n / 255 + 16; }

// Replaces LZ4Compressor.compress as Lz4FrameEncoder.flushBufferedData calls it for one block
// (Lz4FrameEncoder.java:259-275); in_len[i] <= 65536 (the default block size, :59).
extern "C" int32_t nx_lz4_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                       const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream) {
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    const size_t want = (size_t)cus * 16 * 64;  // 16 waves per CU, as the Snappy encoder
    const size_t threads = n < want ? ((n + 255) / 256) * 256 : want;
    const size_t per = (1u << nx::lz4::kHashLog) * sizeof(uint32_t);
    std::lock_guard<std::mutex> lk(g_lz4_mu);
    Lz4Workspace& W = g_lz4_ws[{dev, st}];
    if (W.ws == nullptr || W.threads < threads) {
        if (W.ws) NX_HIP_CHECK(hipFree(W.ws));
        W.ws = nullptr;
        NX_HIP_CHECK(hipMalloc(&W.ws, threads * per));
        NX_HIP_CHECK(hipMemsetAsync(W.ws, 0, threads * per, st));
        W.threads = threads;
        W.stamp = 0;
    }
    const uint32_t iters = (uint32_t)((n + threads - 1) / threads);
    if (W.stamp + iters >= kMaxStamp) {
        NX_HIP_CHECK(hipMemsetAsync(W.ws, 0, W.threads * per, st));
        W.stamp = 0;
    }
    hipLaunchKernelGGL(nx::lz4::k_lz4_encode, dim3((unsigned)(threads / 256)), dim3(256), 0, st, in, in_off, in_len, out, out_off,
                       out_len, status, n, W.ws, W.stamp);
    NX_HIP_CHECK(hipGetLastError());
    W.stamp += iters;
    return NX_OK;
}
