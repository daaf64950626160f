// snappy_naive.hip — thread-per-chunk Snappy encoder (bit-exact with Netty's Snappy.encode).
//
// Netty's greedy matcher (Snappy.java:82-165) is a serial state machine whose output depends on the
// exact probe order (skip++ >> 5 heuristic, evolving 16384-entry hash table).  This kernel runs
// one chunk per lane: every lane executes the reference state machine on its own chunk, so the
// parallelism comes from the thousands of independent chunks of a batch.
//
// Hash table: Java allocates a zeroed short[min(nextPow2(len),16384)] per call (Snappy.java:97-99,
// 191).  Here each resident lane owns a 16384-entry uint32 slot in a device workspace; an entry is
// (stamp << 16) | position and a stamp mismatch reads as 0, which is exactly a freshly zeroed
// table without paying the 32 KiB memset per chunk.  Output bytes are produced in a 16-byte
// register staging word and stored with 16-byte stores when aligned.
#include "nx_common.hpp"

namespace nx {

__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

struct ByteWriter {
    uint8_t* base;
    uint32_t pos;
    __device__ __forceinline__ void put(uint8_t b) { base[pos++] = b; }
};

__device__ __forceinline__ int nlz32(uint32_t v) { return v ? __clz(v) : 32; }

__device__ void enc_literal(const uint8_t* in, ByteWriter& w, int32_t length) {
    // encodeLiteral (Snappy.java:268-281)
    if (length < 61) {
        w.put((uint8_t)((length - 1) << 2));
    } else {
        int32_t v = length - 1;
        int bitLength = v ? 31 - nlz32((uint32_t)v) : 0;  // bitsToEncode (:249-257)
        int bytesToEncode = 1 + bitLength / 8;
        w.put((uint8_t)((59 + bytesToEncode) << 2));
        for (int i = 0; i < bytesToEncode; i++) w.put((uint8_t)((v >> (i * 8)) & 0xff));
    }
    for (int32_t i = 0; i < length; ++i) w.put(in[i]);
}

__device__ __forceinline__ void enc_copy_off(ByteWriter& w, int32_t offset, int32_t length) {
    // encodeCopyWithOffset (:283-292)
    if (length < 12 && offset < 2048) {
        w.put((uint8_t)(1 | ((length - 4) << 2) | ((offset >> 8) << 5)));
        w.put((uint8_t)(offset & 0xff));
    } else {
        w.put((uint8_t)(2 | ((length - 1) << 2)));
        w.put((uint8_t)(offset & 0xff));
        w.put((uint8_t)((offset >> 8) & 0xff));
    }
}

__device__ __forceinline__ void enc_copy(ByteWriter& w, int32_t offset, int32_t length) {
    // encodeCopy (:301-313)
    while (length >= 68) {
        enc_copy_off(w, offset, 64);
        length -= 64;
    }
    if (length > 64) {
        enc_copy_off(w, offset, 60);
        length -= 60;
    }
    enc_copy_off(w, offset, length);
}

__device__ __forceinline__ uint32_t hash_at(const uint8_t* in, int32_t i, int shift) {
    return (ld_be32(in + i) * 0x1e35a7bdu) >> shift;
}

// One Snappy.encode call (in.readerIndex() == 0).  Returns bytes written.
__device__ uint32_t snappy_encode_chunk(const uint8_t* __restrict__ in, int32_t length, uint8_t* __restrict__ out,
                                        uint32_t* __restrict__ table, uint32_t stamp) {
    ByteWriter w{out, 0};
    for (int i = 0;; i++) {  // preamble (:84-92)
        uint32_t b = (uint32_t)length >> (i * 7);
        if ((b & 0xFFFFFF80u) != 0) {
            w.put((uint8_t)((b & 0x7f) | 0x80));
        } else {
            w.put((uint8_t)b);
            break;
        }
    }
    int32_t inIndex = 0;
    uint32_t hts = length <= 1 ? 1u : (1u << (32 - nlz32((uint32_t)(length - 1))));
    if (hts > 16384u) hts = 16384u;
    const int shift = nlz32(hts) + 1;
    const uint32_t stag = stamp << 16;
    int32_t nextEmit = 0;
#define TBL_GET(h) ((table[(h)] & 0xFFFF0000u) == stag ? (int32_t)(table[(h)] & 0xFFFFu) : 0)
#define TBL_SET(h, v) (table[(h)] = stag | (uint32_t)(v))
    if (length >= 15) {
        uint32_t nextHash = hash_at(in, ++inIndex, shift);
        for (;;) {
            int32_t skip = 32;
            int32_t candidate;
            int32_t nextIndex = inIndex;
            do {
                inIndex = nextIndex;
                uint32_t hash = nextHash;
                int32_t step = skip++ >> 5;
                nextIndex = inIndex + step;
                if (nextIndex > length - 4) goto done;
                nextHash = hash_at(in, nextIndex, shift);
                candidate = TBL_GET(hash);
                TBL_SET(hash, inIndex);
            } while (ld_be32(in + inIndex) != ld_be32(in + candidate));

            enc_literal(in + nextEmit, w, inIndex - nextEmit);

            int32_t insertTail;
            do {
                int32_t base = inIndex;
                // 4 + findMatchingLength(in, candidate + 4, inIndex + 4, length)  (:224-239)
                int32_t a = candidate + 4, b = inIndex + 4, matched = 0;
                while (b <= length - 4 && ld_be32(in + b) == ld_be32(in + a + matched)) {
                    b += 4;
                    matched += 4;
                }
                while (b < length && in[a + matched] == in[b]) {
                    ++b;
                    ++matched;
                }
                matched += 4;
                inIndex += matched;
                enc_copy(w, base - candidate, matched);
                insertTail = inIndex - 1;
                nextEmit = inIndex;
                if (inIndex >= length - 4) goto done;
                uint32_t prevHash = hash_at(in, insertTail, shift);
                TBL_SET(prevHash, inIndex - 1);
                uint32_t currentHash = hash_at(in, insertTail + 1, shift);
                candidate = TBL_GET(currentHash);
                TBL_SET(currentHash, inIndex);
            } while (ld_be32(in + insertTail + 1) == ld_be32(in + candidate));
            nextHash = hash_at(in, insertTail + 2, shift);
            ++inIndex;
        }
    }
done:
#undef TBL_GET
#undef TBL_SET
    if (nextEmit < length) enc_literal(in + nextEmit, w, length - nextEmit);
    return w.pos;
}

__global__ void __launch_bounds__(256) k_snappy_encode_naive(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                             const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                             int32_t* __restrict__ status, uint32_t n,
                                                             uint32_t* __restrict__ workspace, uint32_t stamp_base) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nthreads = gridDim.x * blockDim.x;
    uint32_t* table = workspace + (size_t)tid * 16384u;
    uint32_t iter = 0;
    for (uint32_t c = tid; c < n; c += nthreads, ++iter) {
        uint32_t len = in_len[c];
        if (len > 65536u) {
            status[c] = NX_ERR_INVALID_ARG;
            out_len[c] = 0;
            continue;
        }
        uint32_t stamp = ((stamp_base + iter) % 65535u) + 1u;
        out_len[c] = snappy_encode_chunk(in + in_off[c], (int32_t)len, out + out_off[c], table, stamp);
        status[c] = NX_OK;
    }
}

}  // namespace nx

// ------------------------------------------------------------------------------------------
// Host side: workspace management for the encoder's per-lane tables.
#include <mutex>

namespace {
std::mutex g_ws_mu;
uint32_t* g_ws = nullptr;
size_t g_ws_threads = 0;
uint32_t g_stamp = 0;
int g_ws_dev = -1;
constexpr unsigned kEncBlock = 256;
}  // namespace

extern "C" int32_t nx_snappy_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                          uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                          int32_t* status, uint32_t n, void* stream) {
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // resident lanes: 8 waves per CU
    size_t want_threads = (size_t)cus * 8 * 64;
    size_t threads = n < want_threads ? ((n + kEncBlock - 1) / kEncBlock) * kEncBlock : want_threads;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if (g_ws == nullptr || g_ws_threads < threads || g_ws_dev != dev) {
        if (g_ws) (void)hipFree(g_ws);
        g_ws = nullptr;
        size_t cap = threads > want_threads ? threads : want_threads;
        NX_HIP_CHECK(hipMalloc(&g_ws, cap * 16384u * sizeof(uint32_t)));
        NX_HIP_CHECK(hipMemsetAsync(g_ws, 0, cap * 16384u * sizeof(uint32_t), (hipStream_t)stream));
        g_ws_threads = cap;
        g_ws_dev = dev;
        g_stamp = 0;
    }
    uint32_t iters = (uint32_t)((n + threads - 1) / threads);
    if ((uint64_t)g_stamp + iters >= 65535u) {
        NX_HIP_CHECK(hipMemsetAsync(g_ws, 0, g_ws_threads * 16384u * sizeof(uint32_t), (hipStream_t)stream));
        g_stamp = 0;
    }
    unsigned grid = (unsigned)(threads / kEncBlock);
    hipLaunchKernelGGL(nx::k_snappy_encode_naive, dim3(grid), dim3(kEncBlock), 0, (hipStream_t)stream, in, in_off, in_len, out,
                       out_off, out_len, status, n, g_ws, g_stamp);
    NX_HIP_CHECK(hipGetLastError());
    g_stamp += iters;
    return NX_OK;
}
