// lzf.hip — LZF chunk encoder/decoder, batched (LzfEncoder.java:218-221 / LzfDecoder.java:205).
//
// The LZF block arithmetic lives in the third-party com.ning:compress-lzf:1.0.3 (pom.xml:941-945),
// which is not in /root/reference.  The decoder is format-exact (liblzf format: ctrl < 32 → literal
// run of ctrl+1; else back-reference of (ctrl>>5)+2 [+ext] bytes at distance ((ctrl&31)<<8)+byte+1,
// looping until outPos == outEnd as ChunkDecoder.decodeChunk does).  The encoder is ChunkEncoder.
// tryCompress (what LzfEncoder.java:161-163,219 runs) as oracle/netty_oracle.c
// orc_lzf_compress_body_ex restates it — hash ((seen * 57321) >> 9) & 16383 of the big-endian int
// of bytes [p-1, p+2], 3-byte candidate check, MAX_OFF 8192, MAX_REF 264, matchEnd-2/-1 inserts —
// byte for byte (PARITY UNPINNED vs the library itself: no reference bytes exist offline).
#include "nx_common.hpp"
#include "records.hpp"

namespace nx {
namespace lzf {

constexpr int HSIZE = 16384;
constexpr int32_t MAX_OFF = 8192;
constexpr int32_t MAX_REF = 264;
constexpr int32_t MAX_LIT = 32;

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }

// ChunkEncoder.hash: Java int multiply (wraps), arithmetic shift
__device__ __forceinline__ uint32_t jhash(int32_t h) { return (uint32_t)(((int32_t)((uint32_t)h * 57321u) >> 9) & (HSIZE - 1)); }
__device__ __forceinline__ int32_t first2(const uint8_t* in, int32_t p) {  // ChunkEncoder.first: (in[p] << 8) + (in[p+1] & 0xFF), in[p] signed
    return (int32_t)((uint32_t)(int32_t)(int8_t)in[p] << 8) + in[p + 1];
}

// Returns body length.  htab entries: (stamp << 16) | (position + 1) in the high word (the bytes at
// the position in the low one, below); a stamp mismatch is the Java zero (position 0).  A fresh table per chunk is exact for Netty's long-lived per-handler encoder
// (LzfEncoder.java:57,161-163,219), whose table keeps earlier chunks' and messages' entries: the first
// occurrence of every trigram in a chunk is written before any probe reads its slot, so a stale entry
// (or a never-written slot) can never pass the 3-byte check (oracle/netty_oracle.c, above
// lzf_try_compress; tests/test_oracle_kat.py::test_lzf_encoder_state_across_messages).
// The body goes to output positions 7.. (after the LZFChunk header, written last).
// Entries are 64-bit: that word in the high half, the 3 bytes at the position in the low one, so the
// candidate check reads no input.
template <class O>
__device__ int32_t compress_body(const uint8_t* __restrict__ in, int32_t n, O& out, uint64_t* __restrict__ htab, uint32_t stamp) {
    const uint32_t stag = stamp << 16;
    const uint32_t tri_zero = (uint32_t)in[0] | ((uint32_t)in[1] << 8) | ((uint32_t)in[2] << 16);  // a stale entry: position 0
#define LENT(pos1, tri) (((uint64_t)(stag | (uint32_t)(pos1)) << 32) | (uint64_t)(tri))
#define LTRI(sv) ((((uint32_t)(sv) >> 16) & 0xFFu) | ((uint32_t)(sv) & 0xFF00u) | (((uint32_t)(sv) & 0xFFu) << 16))
    const int32_t inEnd = n - 4;
    int32_t ip = 0, op = 1, lit = 0;
    int32_t seen = first2(in, 0);
    int32_t pfp = -1;  // the byte at pfp was loaded one step ahead (a literal step moves ip by one)
    uint32_t pfv = 0;
    while (ip < inEnd) {
        const uint32_t p2 = pfp == ip + 2 ? pfv : (uint32_t)in[ip + 2];
        pfv = in[ip + 3];  // ip + 3 < n
        pfp = ip + 3;
        seen = (int32_t)(((uint32_t)seen << 8) + p2);
        const uint32_t h = jhash(seen);
        const uint32_t tri = LTRI(seen);  // bytes ip .. ip+2
        // read the slot and store this position: one atomic exchange
        const uint64_t e64 = __hip_atomic_exchange(htab + h, LENT(ip + 1, tri), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t e = (uint32_t)(e64 >> 32);
        const bool fresh = (e & 0xFFFF0000u) == stag;
        const int32_t ref = fresh ? (int32_t)(e & 0xFFFFu) - 1 : 0;
        const uint32_t rtri = fresh ? (uint32_t)e64 : tri_zero;  // the bytes at ref
        int32_t off = ip - ref;
        if (ref < 0 || ref >= ip || off > MAX_OFF || ((rtri ^ tri) & 0xFFFFFFu) != 0u) {
            out.set(7 + op++, tri & 0xFFu);  // in[ip]
            ip++;
            if (++lit == MAX_LIT) {
                out.set(7 + op - 33, 31);
                lit = 0;
                op++;
            }
            continue;
        }
        int32_t maxLen = inEnd - ip + 2;
        if (maxLen > MAX_REF) maxLen = MAX_REF;
        if (lit == 0) {
            op--;
        } else {
            out.set(7 + op - lit - 1, (uint8_t)(lit - 1));
            lit = 0;
        }
        int32_t len = 3;
        // extend 8 bytes per compare while the words stay inside the chunk, then byte by byte
        while (len < maxLen && ip + len + 8 <= n) {
            const uint64_t x = ld64(in + ref + len) ^ ld64(in + ip + len);
            const int32_t k = x ? (int32_t)(__builtin_ctzll(x) >> 3) : 8;
            len = len + k < maxLen ? len + k : maxLen;
            if (k < 8) break;
        }
        if (len < maxLen && ip + len + 8 > n)
            while (len < maxLen && in[ref + len] == in[ip + len]) len++;
        len -= 2;
        --off;
        if (len < 7) {
            out.set(7 + op++, (uint8_t)((off >> 8) + (len << 5)));
        } else {
            out.set(7 + op++, (uint8_t)((off >> 8) + (7 << 5)));
            out.set(7 + op++, (uint8_t)(len - 7));
        }
        out.set(7 + op++, (uint8_t)off);
        op++;
        ip += len;  // matchEnd - 2 (<= n - 4)
        seen = first2(in, ip);
        seen = (int32_t)(((uint32_t)seen << 8) + in[ip + 2]);
        __hip_atomic_store(htab + jhash(seen), LENT(ip + 1, LTRI(seen)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ++ip;
        seen = (int32_t)(((uint32_t)seen << 8) + in[ip + 2]);
        __hip_atomic_store(htab + jhash(seen), LENT(ip + 1, LTRI(seen)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ++ip;
    }
    while (ip < n) {  // handleTail
        out.set(7 + op++, in[ip++]);
        if (++lit == MAX_LIT) {
            out.set(7 + op - lit - 1, (uint8_t)(lit - 1));
            lit = 0;
            op++;
        }
    }
    if (lit) {
        out.set(7 + op - lit - 1, (uint8_t)(lit - 1));
    } else {
        op--;
    }
#undef LENT
#undef LTRI
    return op;
}

// One LZFChunk.  Writes the compressed body at out+7 first; falls back to a raw block.
template <class O>
__device__ uint32_t encode_chunk(const uint8_t* __restrict__ in, int32_t n, O& out, uint64_t* htab, uint32_t stamp) {
    if (n >= 16) {
        const int32_t clen = compress_body(in, n, out, htab, stamp);
        if (clen + 7 < n + 5) {
            out.set(0, 'Z');
            out.set(1, 'V');
            out.set(2, 1);
            out.set(3, (uint8_t)(clen >> 8));
            out.set(4, (uint8_t)clen);
            out.set(5, (uint8_t)(n >> 8));
            out.set(6, (uint8_t)n);
            out.finish(clen + 7);
            return (uint32_t)clen + 7;
        }
    }
    out.set(0, 'Z');
    out.set(1, 'V');
    out.set(2, 0);
    out.set(3, (uint8_t)(n >> 8));
    out.set(4, (uint8_t)n);
    for (int32_t i = 0; i < n; ++i) out.set(5 + i, in[i]);
    out.finish(n + 5);
    return (uint32_t)n + 5;
}

template <class O>
__device__ int32_t decode_chunk(const uint8_t* __restrict__ in, int32_t in_len, O& out, int32_t out_len) {
    int32_t ip = 0, op = 0;
    do {
        if (ip >= in_len) return NX_ERR_LZF_CORRUPT;
        const int32_t ctrl = in[ip++];
        if (ctrl < 32) {
            const int32_t k = ctrl + 1;
            if (ip + k > in_len || op + k > out_len) return NX_ERR_LZF_CORRUPT;
            for (int32_t i = 0; i < k; ++i) out.set(op + i, in[ip + i]);
            ip += k;
            op += k;
            continue;
        }
        int32_t len = ctrl >> 5;
        int32_t ref = op - ((ctrl & 0x1f) << 8) - 1;
        if (len == 7) {
            if (ip >= in_len) return NX_ERR_LZF_CORRUPT;
            len += in[ip++];
        }
        if (ip >= in_len) return NX_ERR_LZF_CORRUPT;
        ref -= in[ip++];
        len += 2;
        if (ref < 0 || op + len > out_len) return NX_ERR_LZF_CORRUPT;
        for (int32_t i = 0; i < len; ++i) out.set(op + i, out.get(ref + i));
        op += len;
    } while (op < out_len);
    out.finish(op);
    return op == out_len ? NX_OK : NX_ERR_LZF_CORRUPT;
}

template <bool SPREAD>
__global__ void __launch_bounds__(256) k_encode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                int32_t* __restrict__ status, uint32_t n, uint64_t* __restrict__ ws, uint32_t stamp_base) {
    uint32_t tid, nthreads;
    if (!chunk_slot<SPREAD>(tid, nthreads)) return;
    uint64_t* htab = ws + (size_t)tid * HSIZE;
    uint8_t* slot = nullptr;
    if constexpr (!SPREAD) {
        __shared__ __attribute__((aligned(16))) uint8_t stages[256 * kStageStride];
        slot = &stages[threadIdx.x * kStageStride];
    }
    uint32_t iter = 0;
    for (uint32_t c = tid; c < n; c += nthreads, ++iter) {
        const uint32_t len = in_len[c];
        if (len > 65535u) {
            status[c] = NX_ERR_INVALID_ARG;
            out_len[c] = 0;
            continue;
        }
        const uint32_t stamp = ((stamp_base + iter) % 65535u) + 1u;
        if (SPREAD) {
            GOut o{out + out_off[c]};
            out_len[c] = encode_chunk(in + in_off[c], (int32_t)len, o, htab, stamp);
        } else {
            ByteStage o(slot, out + out_off[c]);  // dense form: whole 128-byte units (nx_common.hpp)
            out_len[c] = encode_chunk(in + in_off[c], (int32_t)len, o, htab, stamp);
        }
        status[c] = NX_OK;
    }
}

// After the record path (records.hpp): blocks it left with kNeedSerial run the lane-serial decoder,
// which reports the status; the others decoded exactly out_len bytes (NX_OK, already set).
__global__ void __launch_bounds__(256) k_decode_finish(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                       const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                       const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_len,
                                                       int32_t* __restrict__ status, uint32_t n) {
    // output through 64-byte LDS units (nx_common.hpp ByteStageT; 17 KiB per block keeps 8 blocks/CU)
    __shared__ __attribute__((aligned(16))) uint8_t stages[256 * 68];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n || status[c] != nx::dec::kNeedSerial) return;
    ByteStageT<64> o(&stages[threadIdx.x * 68], out + out_off[c]);
    status[c] = decode_chunk(in + in_off[c], (int32_t)in_len[c], o, (int32_t)out_len[c]);
}

}  // namespace lzf
}  // namespace nx

#include "workspace.hpp"
static_assert(nx::kWsSpec[(int)nx::WsKind::LzfEnc].entry_bytes == sizeof(uint64_t) &&
                  (1 << nx::kWsSpec[(int)nx::WsKind::LzfEnc].lg) == nx::lzf::HSIZE,
              "LZF table geometry");

extern "C" int32_t nx_lzf_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                       const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    const size_t per = (size_t)nx::lzf::HSIZE * sizeof(uint64_t);
    nx::WsLease lease(nx::WsKind::LzfEnc, dev, st);
    NX_HIP_CHECK(lease.acquire(nx::ws_want(nx::WsKind::LzfEnc, n, cus)));
    nx::SharedWs& W = lease.ws();
    const nx::LaneGrid g = nx::ws_grid(nx::WsKind::LzfEnc, n, cus, W.slots);
    uint64_t* ws = static_cast<uint64_t*>(W.p);
    const uint32_t iters = (uint32_t)((n + g.slots - 1) / g.slots);
    if ((uint64_t)W.stamp + iters >= 65535u) {
        NX_HIP_CHECK(hipMemsetAsync(ws, 0, W.slots * per, st));
        W.stamp = 0;
    }
    if (g.spread)
        hipLaunchKernelGGL(nx::lzf::k_encode<true>, dim3(g.grid), dim3(g.block), 0, st, in, in_off, in_len, out, out_off, out_len, status,
                           n, ws, W.stamp);
    else
        hipLaunchKernelGGL(nx::lzf::k_encode<false>, dim3(g.grid), dim3(g.block), 0, st, in, in_off, in_len, out, out_off, out_len,
                           status, n, ws, W.stamp);
    NX_HIP_CHECK(hipGetLastError());
    W.stamp += iters;
    return NX_OK;
}

namespace {
struct LzfDecCtx {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    uint8_t* out;
    const uint64_t* out_off;
    const uint32_t* out_len;
    int32_t* status;
};
hipError_t lzf_dec_after(uint32_t base, uint32_t m, const uint32_t*, void* ctx, hipStream_t st) {
    const LzfDecCtx& x = *static_cast<const LzfDecCtx*>(ctx);
    hipLaunchKernelGGL(nx::lzf::k_decode_finish, dim3((m + 255) / 256), dim3(256), 0, st, x.in, x.in_off + base, x.in_len + base, x.out,
                       x.out_off + base, x.out_len + base, x.status + base, m);
    return hipGetLastError();
}
}  // namespace

// Blocks go through the record expander (snappy_decode.hip k_parse_lzf + k_expand); corrupt ones
// through the lane-serial decode_chunk(), which reports them.
extern "C" int32_t nx_lzf_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                       const uint64_t* out_off, const uint32_t* out_len, int32_t* status, uint32_t n,
                                       void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    LzfDecCtx ctx{in, in_off, in_len, out, out_off, out_len, status};
    return nx::dec::decode_records(nx::dec::RecCodec::Lzf, in, in_off, in_len, nullptr, out_len, out, out_off, status, n,
                                   (hipStream_t)stream, lzf_dec_after, &ctx);
}
