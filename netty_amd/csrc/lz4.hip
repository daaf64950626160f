// lz4.hip — LZ4 block encoder, one lane per block.
//
// Lz4FrameEncoder compresses each block with lz4-java 1.8.0's fastCompressor()
// (Lz4FrameEncoder.java:125,163,273), i.e. liblz4's LZ4_compress_default.  This kernel is that
// algorithm, bit-exact with the oracle's restatement (oracle/netty_oracle.c orc_lz4_compress),
// which tests/test_oracle_kat.py pins byte-for-byte against pyarrow's bundled liblz4:
//   * blocks < 65547 bytes (LZ4_64Klimit): the byU16 table, 8192 slots hashed from the 4 bytes at a
//     position (LZ4_hash4), no distance check; longer blocks: the byU32 table, 4096 slots hashed
//     from the low 5 of the 8 bytes at a position (LZ4_hash5), matches farther than 65535 skipped;
//   * a fresh table reads as all zeros = position 0 (a real candidate, as in liblz4);
//   * the search step grows by one every 64 misses (skipTrigger 6), found matches are extended
//     backwards over equal bytes (catch up) and forwards up to 5 bytes before the end, and after a
//     match position ip-2 is inserted and ip is tested at once (a zero-literal sequence).
//
// Each lane owns a 64 KiB table (8192 64-bit entries) in an HBM workspace.  Small blocks store stamp << 16 | index
// (a stamp mismatch reads as the zeroed table), so the table is never cleared between blocks;
// a large block zeroes its 4096 slots before and after itself, so none of its raw indices can pass
// a later small block's stamp check.
#include <algorithm>
#include "nx_common.hpp"
#include "workspace.hpp"

namespace nx {
namespace lz4 {

constexpr int kMinMatch = 4, kLastLiterals = 5, kMfLimit = 12, kMinLength = 13;
constexpr int32_t k64KLimit = 65536 + kMfLimit - 1;
constexpr uint32_t kTableSlots = 8192;  // byU16 slots (the byU32 table uses the first 4096)

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }

template <bool Large>
__device__ __forceinline__ uint32_t hash_at(const uint8_t* p) {
    if (!Large) return (ld32(p) * 2654435761u) >> (32 - 13);                       // LZ4_hash4, byU16
    return (uint32_t)(((ld64(p) << 24) * 889523592379ull) >> (64 - 12));           // LZ4_hash5, byU32
}

template <class O>
__device__ __forceinline__ uint32_t put_len(O& out, uint32_t op, uint32_t v) {  // 255-run of a length >= 15
    for (; v >= 255u; v -= 255u) out.set(op++, 255u);
    out.set(op++, v);
    return op;
}

// Large == false: blocks < 65547 bytes, entries stamp << 16 | index.  Large == true: blocks of up
// to 32 MiB, raw indices in a table the lane zeroes before and after the block.
// Entries are 64-bit: that word in the high half and the 4 bytes at the index in the low half, so
// the candidate's 4-byte check reads no input (an entry that reads as index 0 — stale, zeroed or
// position 0 itself — is checked against the block's first 4 bytes).
template <bool Large, class O>
__device__ uint32_t encode_block(const uint8_t* __restrict__ in, int32_t n, O& out, uint64_t* __restrict__ table, uint32_t stamp) {
    const uint32_t stag = stamp << 16;
#define XCH(h, v) __hip_atomic_exchange(table + (h), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define PUT(h, v) __hip_atomic_store(table + (h), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define ENT(i, w) (((uint64_t)(Large ? (uint32_t)(i) : (stag | (uint32_t)(i))) << 32) | (uint64_t)(w))
    auto idx = [stag](uint64_t e64) -> int32_t {
        const uint32_t e = (uint32_t)(e64 >> 32);
        return Large ? (int32_t)e : ((e & 0xFFFF0000u) == stag ? (int32_t)(e & 0xFFFFu) : 0);
    };
    const uint32_t w_zero = n >= 4 ? ld32(in) : 0u;
    auto bytes_at = [w_zero](uint64_t e64, int32_t i) -> uint32_t { return i == 0 ? w_zero : (uint32_t)e64; };
    if (Large)
        for (uint32_t k = 0; k < 4096u; ++k) PUT(k, 0ull);
    uint32_t op = 0;
    int32_t ip = 0, anchor = 0;
    const int32_t mflimit_plus_one = n - kMfLimit + 1, matchlimit = n - kLastLiterals;
    if (n >= kMinLength) {
        PUT(hash_at<Large>(in), ENT(0, w_zero));  // first byte
        ip = 1;
        uint32_t forward_h = hash_at<Large>(in + 1);
        uint32_t forward_w = ld32(in + 1);
        for (;;) {
            int32_t match;
            {   // find a match
                int32_t forward_ip = ip, step = 1, search_nb = 1 << 6;
                for (;;) {
                    const uint32_t h = forward_h, cw = forward_w;
                    const int32_t current = forward_ip;
                    ip = forward_ip;
                    forward_ip += step;
                    step = search_nb++ >> 6;
                    if (forward_ip > mflimit_plus_one) goto last_literals;
                    forward_h = hash_at<Large>(in + forward_ip);
                    forward_w = ld32(in + forward_ip);
                    const uint64_t e = XCH(h, ENT(current, cw));
                    match = idx(e);
                    if (Large && match + 65535 < current) continue;  // too far
                    if (bytes_at(e, match) == cw) break;
                }
            }
            while (ip > anchor && match > 0 && in[ip - 1] == in[match - 1]) {  // catch up
                --ip;
                --match;
            }
            uint32_t token = op++;
            {
                const uint32_t lit = (uint32_t)(ip - anchor);
                if (lit >= 15u) {
                    out.set(token, 15u << 4);
                    op = put_len(out, op, lit - 15u);
                } else {
                    out.set(token, lit << 4);
                }
                for (uint32_t k = 0; k < lit; ++k) out.set(op + k, in[anchor + k]);
                op += lit;
            }
            for (;;) {  // _next_match
                const uint32_t off = (uint32_t)(ip - match);
                out.set(op++, off & 0xFFu);
                out.set(op++, (off >> 8) & 0xFFu);
                int32_t mc = 0;
                while (ip + kMinMatch + mc + 4 <= matchlimit) {
                    const uint32_t x = ld32(in + ip + kMinMatch + mc) ^ ld32(in + match + kMinMatch + mc);
                    if (x) {
                        mc += __builtin_ctz(x) >> 3;
                        goto counted;
                    }
                    mc += 4;
                }
                while (ip + kMinMatch + mc < matchlimit && in[ip + kMinMatch + mc] == in[match + kMinMatch + mc]) ++mc;
            counted:
                ip += mc + kMinMatch;
                if (mc >= 15) {
                    out.set(token, out.get(token) + 15u);
                    op = put_len(out, op, (uint32_t)(mc - 15));
                } else {
                    out.set(token, out.get(token) + (uint32_t)mc);
                }
                anchor = ip;
                if (ip >= mflimit_plus_one) goto last_literals;
                PUT(hash_at<Large>(in + ip - 2), ENT(ip - 2, ld32(in + ip - 2)));  // fill table
                const uint32_t iw = ld32(in + ip);
                const uint64_t e = XCH(hash_at<Large>(in + ip), ENT(ip, iw));  // test next position
                const int32_t mi = idx(e);
                if ((!Large || mi + 65535 >= ip) && bytes_at(e, mi) == iw) {
                    match = mi;
                    token = op++;
                    out.set(token, 0u);
                    continue;
                }
                break;
            }
            forward_h = hash_at<Large>(in + ++ip);  // prepare next loop
            forward_w = ld32(in + ip);
        }
    }
last_literals:
#undef XCH
#undef PUT
#undef ENT
    if (Large)
        for (uint32_t k = 0; k < 4096u; ++k) __hip_atomic_store(table + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t lit = (uint32_t)(n - anchor);  // last literals
    if (lit >= 15u) {
        out.set(op++, 15u << 4);
        op = put_len(out, op, lit - 15u);
    } else {
        out.set(op++, lit << 4);
    }
    for (uint32_t k = 0; k < lit; ++k) out.set(op + k, in[anchor + k]);
    out.finish((int32_t)(op + lit));
    return op + lit;
}

template <bool SPREAD>
__global__ void __launch_bounds__(256) k_lz4_encode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                    const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                    int32_t* __restrict__ status, uint32_t n, uint64_t* __restrict__ workspace,
                                                    uint32_t stamp_base) {
    uint32_t tid, nthreads;
    if (!chunk_slot<SPREAD>(tid, nthreads)) return;
    uint64_t* table = workspace + (size_t)tid * kTableSlots;
    uint8_t* slot = nullptr;
    if constexpr (!SPREAD) {
        __shared__ __attribute__((aligned(16))) uint8_t stages[256 * kStageStride];
        slot = &stages[threadIdx.x * kStageStride];
    }
    uint32_t iter = 0;
    for (uint32_t c = tid; c < n; c += nthreads, ++iter) {
        const uint32_t len = in_len[c];
        if (len > (1u << 25)) {
            out_len[c] = 0;
            status[c] = NX_ERR_INVALID_ARG;
            continue;
        }
        if ((int32_t)len >= k64KLimit) {
            GOut o{out + out_off[c]};
            out_len[c] = encode_block<true>(in + in_off[c], (int32_t)len, o, table, 0u);
        } else if (SPREAD) {
            GOut o{out + out_off[c]};
            out_len[c] = encode_block<false>(in + in_off[c], (int32_t)len, o, table, stamp_base + iter + 1u);
        } else {
            ByteStage o(slot, out + out_off[c]);  // dense form: whole 128-byte units (nx_common.hpp)
            out_len[c] = encode_block<false>(in + in_off[c], (int32_t)len, o, table, stamp_base + iter + 1u);
        }
        status[c] = NX_OK;
    }
}

}  // namespace lz4
}  // namespace nx

namespace {
constexpr uint32_t kMaxStamp = 0xFFFFu;
static_assert(nx::kWsSpec[(int)nx::WsKind::Lz4Enc].entry_bytes == sizeof(uint64_t) &&
                  (1u << nx::kWsSpec[(int)nx::WsKind::Lz4Enc].lg) == nx::lz4::kTableSlots,
              "LZ4 table geometry");
}  // namespace

extern "C" size_t nx_lz4_max_compressed_length(size_t n) { return n + n / 255 + 16; }

// Replaces LZ4Compressor.compress as Lz4FrameEncoder.flushBufferedData calls it for one block
// (Lz4FrameEncoder.java:259-275); in_len[i] <= 2^25 (MAX_BLOCK_SIZE, Lz4Constants.java / :175-178).
extern "C" int32_t nx_lz4_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                       const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    const size_t per = nx::lz4::kTableSlots * sizeof(uint64_t);
    nx::WsLease lease(nx::WsKind::Lz4Enc, dev, st);
    NX_HIP_CHECK(lease.acquire(nx::ws_want(nx::WsKind::Lz4Enc, n, cus)));
    nx::SharedWs& W = lease.ws();
    const nx::LaneGrid g = nx::ws_grid(nx::WsKind::Lz4Enc, n, cus, W.slots);  // 16 waves per CU, as the Snappy encoder
    uint64_t* ws = static_cast<uint64_t*>(W.p);
    const uint32_t iters = (uint32_t)((n + g.slots - 1) / g.slots);
    if (W.stamp + iters >= kMaxStamp) {
        NX_HIP_CHECK(hipMemsetAsync(ws, 0, W.slots * per, st));
        W.stamp = 0;
    }
    if (g.spread)
        hipLaunchKernelGGL(nx::lz4::k_lz4_encode<true>, dim3(g.grid), dim3(g.block), 0, st, in, in_off, in_len, out, out_off, out_len,
                           status, n, ws, W.stamp);
    else
        hipLaunchKernelGGL(nx::lz4::k_lz4_encode<false>, dim3(g.grid), dim3(g.block), 0, st, in, in_off, in_len, out, out_off, out_len,
                           status, n, ws, W.stamp);
    NX_HIP_CHECK(hipGetLastError());
    W.stamp += iters;
    return NX_OK;
}
