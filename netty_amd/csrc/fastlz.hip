// fastlz.hip — FastLZ level 1/2 compress + decompress (FastLz.java:96-557) and Adler32, batched.
//
// FastLZ is a serial byte-oriented LZ77 whose match search depends on an evolving 8192-entry
// hash table (FastLz.java:112,139-142), so each chunk runs as one lane's serial state machine;
// a batch of thousands of 4–64 KiB chunks fills the chip.  The hash table lives in a per-lane
// device workspace with a stamp as the Snappy encoder (64-bit entries: stamp | position | the 4 bytes
// at the position, compress() below).  Java's `htab` is initialised to 0 (= position 0) on every
// call; a stamp mismatch reads as position 0.
//
// The readU16 quirk (FastLz.java:552-557: an ABSOLUTE index compared against readableBytes())
// is reproduced through the per-chunk u16_limit = readableBytes() - inOffset of the Java call.
#include "nx_common.hpp"
#include "records.hpp"

namespace nx {
namespace flz {

constexpr int32_t MAX_DISTANCE = 8191;
constexpr int32_t MAX_FARDISTANCE = 65535 + MAX_DISTANCE - 1;
constexpr int32_t HASH_LOG = 13;
constexpr int32_t HASH_SIZE = 1 << HASH_LOG;
constexpr int32_t HASH_MASK = HASH_SIZE - 1;
constexpr int32_t MAX_COPY = 32;
constexpr int32_t MAX_LEN = 256 + 8;

__device__ __forceinline__ int32_t read_u16(const uint8_t* in, int32_t o, int32_t lim) {
    if (o + 1 >= lim) return in[o];
    return ((int32_t)in[o + 1] << 8) | in[o];
}

__device__ __forceinline__ int32_t hashf(const uint8_t* in, int32_t o, int32_t lim) {
    int32_t v = read_u16(in, o, lim);
    v ^= read_u16(in, o + 1, lim) ^ (v >> (16 - HASH_LOG));
    return v & HASH_MASK;
}

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }

// hashFunction at o from the dword w = bytes o..o+3 (readU16's limit applied per half)
__device__ __forceinline__ int32_t hash_w(uint32_t w, int32_t o, int32_t lim) {
    const int32_t b0 = (int32_t)(w & 0xFFu), b1 = (int32_t)((w >> 8) & 0xFFu), b2 = (int32_t)((w >> 16) & 0xFFu);
    int32_t v = o + 1 >= lim ? b0 : (b1 << 8) | b0;
    const int32_t u = o + 2 >= lim ? b1 : (b2 << 8) | b1;
    v ^= u ^ (v >> (16 - HASH_LOG));
    return v & HASH_MASK;
}

// The serial matcher of FastLz.compress (FastLz.java:96-399) with its reads batched: the hash and
// the literal byte come from one dword load, the first 3 (level-2 far: 5) bytes of a candidate are
// compared as one word, matches extend 8 bytes per compare (first mismatch by count-trailing-zeros,
// stopping where Java's byte loop stops: at ipBound, or one past the mismatch), and the table probe
// (read the slot, store the anchor) is one atomic exchange.  Positions near the chunk end, where a
// word load could pass it, take Java's byte reads.
// Table entries are 64-bit: stamp[63:48] | position[47:32] | the 4 bytes at the position[31:0], so
// the 3-byte candidate check reads no input (a level-2 far candidate loads its 5th byte).
template <class O>
__device__ int32_t compress(const uint8_t* __restrict__ in, int32_t inLength, O& out, int32_t proposedLevel,
                            int32_t lim, uint64_t* __restrict__ htab, uint32_t stamp) {
    const int32_t level = proposedLevel == 0 ? (inLength < 65536 ? 1 : 2) : proposedLevel;
    int32_t ip = 0;
    int32_t ipBound = ip + inLength - 2;
    const int32_t ipLimit = ip + inLength - 12;
    int32_t op = 0;
    int32_t copy;
    const uint64_t stag = (uint64_t)stamp << 48;
#define HENT(pos, w) (stag | ((uint64_t)(uint32_t)(pos) << 32) | (uint64_t)(w))
#define HSET(h, pos, w) __hip_atomic_store(htab + (h), HENT(pos, w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
    if (inLength < 4) {
        if (inLength != 0) {
            out.set(op++, (uint8_t)(inLength - 1));
            ipBound++;
            while (ip <= ipBound) out.set(op++, in[ip++]);
            out.finish(op);
            return inLength + 1;
        }
        return 0;
    }
    copy = 2;
    out.set(op++, MAX_COPY - 1);
    out.set(op++, in[ip++]);
    out.set(op++, in[ip++]);
    // Java's fresh table reads position 0 everywhere: a stale entry is position 0 and its bytes
    const uint32_t w_zero = ld32(in);  // inLength >= 4 here
    while (ip < ipLimit) {  // ip + 12 < inLength: word loads at ip - 1 .. ip + 8 stay in the chunk
        int32_t ref;
        int64_t distance;
        int32_t len = 3;
        const int32_t anchor = ip;
        const uint32_t w = ld32(in + ip);
        bool matchLabel = false;
        if (level == 2) {
            const uint32_t wm = ld32(in + ip - 1);  // bytes ip-1 .. ip+2
            const uint32_t c0 = wm & 0xFFu, c1 = (wm >> 8) & 0xFFu, c2 = (wm >> 16) & 0xFFu, c3 = wm >> 24;
            const uint32_t ua = ip >= lim ? c0 : (c1 << 8) | c0;       // readU16(ip - 1)
            const uint32_t ub = ip + 2 >= lim ? c2 : (c3 << 8) | c2;   // readU16(ip + 1)
            if (c1 == c0 && ua == ub) {
                distance = 1;
                ip += 3;
                ref = anchor + (3 - 1);
                matchLabel = true;
            }
        }
        if (!matchLabel) {
            const int32_t hval = hash_w(w, ip, lim);
            const uint64_t e = __hip_atomic_exchange(htab + hval, HENT(anchor, w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool fresh = (e & 0xFFFF000000000000ull) == stag;
            ref = fresh ? (int32_t)((e >> 32) & 0xFFFFu) : 0;
            const uint32_t rw = fresh ? (uint32_t)e : w_zero;  // the bytes at ref
            distance = anchor - ref;
            bool lit = distance == 0 || (level == 1 ? distance >= MAX_DISTANCE : distance >= MAX_FARDISTANCE);
            if (!lit) {
                lit = ((rw ^ w) & 0xFFFFFFu) != 0u;
                if (!lit && level == 2 && distance >= MAX_DISTANCE) {  // far: 5 bytes must match
                    lit = (rw >> 24) != (w >> 24) || in[ref + 4] != in[anchor + 4];
                    len += 2;
                }
            }
            if (lit) {
                out.set(op++, w & 0xFFu);  // in[anchor]
                ip = anchor + 1;
                copy++;
                if (copy == MAX_COPY) {
                    copy = 0;
                    out.set(op++, MAX_COPY - 1);
                }
                continue;
            }
            ref += len;
        }
        ip = anchor + len;
        distance--;
        if (distance == 0) {
            // a run of x = in[ip - 1]: Java compares in[ip - 1] and steps ip while it equals x and
            // ip < ipBound, so ip ends at (first position >= ip - 1 holding another byte) + 1, or ipBound
            const uint32_t x = in[ip - 1];
            const uint64_t x8 = (uint64_t)x * 0x0101010101010101ull;
            for (;;) {
                if (ip >= ipBound) break;
                const int32_t p = ip - 1;
                if (p + 8 > inLength) {
                    while (ip < ipBound && in[ip - 1] == x) ip++;
                    break;
                }
                const uint64_t d = ld64(in + p) ^ x8;
                const int32_t k = d ? (int32_t)(__builtin_ctzll(d) >> 3) : 8;
                const int32_t room = ipBound - ip;
                if (k < 8 || room <= 8) {
                    ip += k < room ? k : room;
                    break;
                }
                ip += 8;
            }
        } else {
            // the first 8 bytes unconditionally (ip + 8 <= inLength here), then until ipBound; ip ends
            // one past the first mismatch, or at ipBound (or at ip + 8 when that is already past it)
            const uint64_t x0 = ld64(in + ref) ^ ld64(in + ip);
            if (x0) {
                ip += (int32_t)(__builtin_ctzll(x0) >> 3) + 1;
            } else {
                ip += 8;
                ref += 8;
                for (;;) {
                    if (ip >= ipBound) break;
                    if (ip + 8 > inLength) {
                        while (ip < ipBound) {
                            if (in[ref++] != in[ip++]) break;
                        }
                        break;
                    }
                    const uint64_t x = ld64(in + ref) ^ ld64(in + ip);
                    const int32_t k = x ? (int32_t)(__builtin_ctzll(x) >> 3) : 8;
                    const int32_t room = ipBound - ip;
                    if (k < 8 && k < room) {
                        ip += k + 1;
                        break;
                    }
                    if (room <= 8) {
                        ip = ipBound;
                        break;
                    }
                    ip += 8;
                    ref += 8;
                }
            }
        }
        if (copy != 0) {
            out.set(op - copy - 1, (uint32_t)(copy - 1));
        } else {
            op--;
        }
        copy = 0;
        ip -= 3;
        len = ip - anchor;
        if (level == 2) {
            if (distance < MAX_DISTANCE) {
                if (len < 7) {
                    out.set(op++, (uint8_t)((len << 5) + (int32_t)(distance >> 8)));
                    out.set(op++, (uint8_t)(distance & 255));
                } else {
                    out.set(op++, (uint8_t)((7 << 5) + (int32_t)(distance >> 8)));
                    for (len -= 7; len >= 255; len -= 255) out.set(op++, 255);
                    out.set(op++, (uint8_t)len);
                    out.set(op++, (uint8_t)(distance & 255));
                }
            } else {
                distance -= MAX_DISTANCE;
                if (len < 7) {
                    out.set(op++, (uint8_t)((len << 5) + 31));
                    out.set(op++, 255);
                    out.set(op++, (uint8_t)(distance >> 8));
                    out.set(op++, (uint8_t)(distance & 255));
                } else {
                    out.set(op++, (uint8_t)((7 << 5) + 31));
                    for (len -= 7; len >= 255; len -= 255) out.set(op++, 255);
                    out.set(op++, (uint8_t)len);
                    out.set(op++, 255);
                    out.set(op++, (uint8_t)(distance >> 8));
                    out.set(op++, (uint8_t)(distance & 255));
                }
            }
        } else {
            if (len > MAX_LEN - 2) {
                while (len > MAX_LEN - 2) {
                    out.set(op++, (uint8_t)((7 << 5) + (int32_t)(distance >> 8)));
                    out.set(op++, (uint8_t)(MAX_LEN - 2 - 7 - 2));
                    out.set(op++, (uint8_t)(distance & 255));
                    len -= MAX_LEN - 2;
                }
            }
            if (len < 7) {
                out.set(op++, (uint8_t)((len << 5) + (int32_t)(distance >> 8)));
                out.set(op++, (uint8_t)(distance & 255));
            } else {
                out.set(op++, (uint8_t)((7 << 5) + (int32_t)(distance >> 8)));
                out.set(op++, (uint8_t)(len - 7));
                out.set(op++, (uint8_t)(distance & 255));
            }
        }
        // the two positions after the match (readU16 may reach past the chunk end here: bytes)
        // (an entry there is never probed again in this chunk, so its bytes may stay 0)
        for (int t = 0; t < 2; ++t) {
            const bool inside = ip + 4 <= inLength;
            const uint32_t wi = inside ? ld32(in + ip) : 0u;
            const int32_t hv = inside ? hash_w(wi, ip, lim) : hashf(in, ip, lim);
            HSET(hv, ip, wi);
            ip++;
        }
        out.set(op++, MAX_COPY - 1);
    }
    ipBound++;
    while (ip <= ipBound) {
        out.set(op++, in[ip++]);
        copy++;
        if (copy == MAX_COPY) {
            copy = 0;
            out.set(op++, MAX_COPY - 1);
        }
    }
    if (copy != 0) {
        out.set(op - copy - 1, (uint32_t)(copy - 1));
    } else {
        op--;
    }
    if (level == 2) out.set(0, out.get(0) | (1u << 5));
#undef HENT
#undef HSET
    out.finish(op);
    return op;
}

template <class O>
__device__ int32_t decompress(const uint8_t* __restrict__ in, int32_t inLength, int32_t in_avail, O& out, int32_t outLength) {
    bool oob = false;
#define FIN(i) ((i) < in_avail ? (int32_t)in[(i)] : (oob = true, 0))
    if (in_avail < 1) return NX_ERR_FASTLZ_INPUT_OOB;
    const int32_t level = ((int32_t)(int8_t)in[0] >> 5) + 1;
    if (level != 1 && level != 2) return NX_ERR_FASTLZ_BAD_LEVEL;
    int32_t ip = 0, op = 0;
    int64_t ctrl = in[ip++] & 31;
    int loop = 1;
    do {
        int64_t ref = op;
        int64_t len = ctrl >> 5;
        int64_t ofs = (ctrl & 31) << 8;
        if (ctrl >= 32) {
            len--;
            ref -= ofs;
            int32_t code;
            if (len == 6) {
                if (level == 1) {
                    len += FIN(ip);
                    ip++;
                } else {
                    do {
                        code = FIN(ip);
                        ip++;
                        if (oob) return NX_ERR_FASTLZ_INPUT_OOB;
                        len += code;
                    } while (code == 255);
                }
            }
            if (level == 1) {
                ref -= FIN(ip);
                ip++;
            } else {
                code = FIN(ip);
                ip++;
                ref -= code;
                if (code == 255 && ofs == (31 << 8)) {
                    ofs = (int64_t)FIN(ip) << 8;
                    ip++;
                    ofs += FIN(ip);
                    ip++;
                    ref = (int32_t)(op - ofs - MAX_DISTANCE);
                }
            }
            if (oob) return NX_ERR_FASTLZ_INPUT_OOB;
            if (op + len + 3 > outLength) return 0;
            if (ref - 1 < 0) return 0;
            if (ip < inLength) {
                ctrl = FIN(ip);
                ip++;
                if (oob) return NX_ERR_FASTLZ_INPUT_OOB;
            } else {
                loop = 0;
            }
            if (ref == op) {
                const uint32_t b = out.get((int32_t)ref - 1);
                out.set(op++, b);
                out.set(op++, b);
                out.set(op++, b);
                while (len != 0) {
                    out.set(op++, b);
                    --len;
                }
            } else {
                ref--;
                out.set(op++, out.get((int32_t)ref++));
                out.set(op++, out.get((int32_t)ref++));
                out.set(op++, out.get((int32_t)ref++));
                while (len != 0) {
                    out.set(op++, out.get((int32_t)ref++));
                    --len;
                }
            }
        } else {
            ctrl++;
            if (op + ctrl > outLength) return 0;
            if (ip + ctrl > inLength) return 0;
            out.set(op++, in[ip++]);
            for (--ctrl; ctrl != 0; ctrl--) out.set(op++, in[ip++]);
            loop = ip < inLength ? 1 : 0;
            if (loop) ctrl = in[ip++];
        }
    } while (loop != 0);
#undef FIN
    out.finish(op);
    return op;
}

template <bool SPREAD>
__global__ void __launch_bounds__(256) k_compress(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                  const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                  const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                  const int32_t* __restrict__ level, const int32_t* __restrict__ lim,
                                                  int32_t* __restrict__ status, uint32_t n, uint64_t* __restrict__ ws,
                                                  uint32_t stamp_base) {
    uint32_t tid, nthreads;
    if (!chunk_slot<SPREAD>(tid, nthreads)) return;
    uint64_t* htab = ws + (size_t)tid * HASH_SIZE;
    uint8_t* slot = nullptr;
    if constexpr (!SPREAD) {
        __shared__ __attribute__((aligned(16))) uint8_t stages[256 * kStageStride];
        slot = &stages[threadIdx.x * kStageStride];
    }
    uint32_t iter = 0;
    for (uint32_t c = tid; c < n; c += nthreads, ++iter) {
        const uint32_t len = in_len[c];
        const int32_t lv = level ? level[c] : 0;
        if (len > 65535u || (lv != 0 && lv != 1 && lv != 2)) {
            status[c] = NX_ERR_INVALID_ARG;
            out_len[c] = 0;
            continue;
        }
        const int32_t l16 = lim ? lim[c] : (int32_t)len;
        const uint32_t stamp = ((stamp_base + iter) % 65535u) + 1u;
        if (SPREAD) {
            GOut o{out + out_off[c]};
            out_len[c] = (uint32_t)compress(in + in_off[c], (int32_t)len, o, lv, l16, htab, stamp);
        } else {
            ByteStage o(slot, out + out_off[c]);  // dense form: whole 128-byte units (nx_common.hpp)
            out_len[c] = (uint32_t)compress(in + in_off[c], (int32_t)len, o, lv, l16, htab, stamp);
        }
        status[c] = NX_OK;
    }
}

// After the record path (records.hpp): blocks it left with kNeedSerial run the lane-serial decoder
// (Java's return value or status); the others return the length the parse produced.
__global__ void __launch_bounds__(256) k_decompress_finish(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                           const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ in_avail,
                                                           uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                           const uint32_t* __restrict__ out_lim, int32_t* __restrict__ result,
                                                           const uint32_t* __restrict__ olen, uint32_t n) {
    // output through 64-byte LDS units (nx_common.hpp ByteStageT; 17 KiB per block keeps 8 blocks/CU)
    __shared__ __attribute__((aligned(16))) uint8_t stages[256 * 68];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    if (result[c] != nx::dec::kNeedSerial) {
        result[c] = (int32_t)olen[c];
        return;
    }
    const uint32_t il = in_len[c];
    const uint32_t av = in_avail ? in_avail[c] : il;
    ByteStageT<64> o(&stages[threadIdx.x * 68], out + out_off[c]);
    result[c] = decompress(in + in_off[c], (int32_t)il, (int32_t)av, o, (int32_t)out_lim[c]);
}

// Adler32 (java.util.zip.Adler32): one wave per chunk, lanes take 16-byte slots of 1 KiB blocks.
// a = 1 + Σ b_i, b = n + Σ (n - i) b_i (mod 65521), computed with 64-bit partial sums.
__global__ void __launch_bounds__(256) k_adler32(const uint8_t* __restrict__ in, const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ len, uint32_t* __restrict__ out, uint32_t n) {
    const int lane = threadIdx.x & 63;
    const uint32_t wpb = blockDim.x / 64;
    for (uint32_t c = blockIdx.x * wpb + (threadIdx.x >> 6); c < n; c += gridDim.x * wpb) {
        const uint8_t* p = in + off[c];
        const uint32_t L = len[c];
        uint64_t sa = 0, sb = 0;  // Σ b_i, Σ (L - i) b_i
        const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
        const uint32_t* p4 = reinterpret_cast<const uint32_t*>(p - sh);
        for (uint32_t base = 0; base < L; base += 1024) {
            const uint32_t i0 = base + 16u * lane;
            if (i0 + 16u <= L) {
                // a full slot: aligned dword loads (alignbyte for a misaligned chunk), byte sums
                // with dot4: S = Σ b_k, T = Σ k b_k, so Σ (L - i0 - k) b_k = (L - i0) S - T
                const uint32_t* q = p4 + (i0 >> 2);
                uint32_t w[4];
                if (sh == 0u) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) w[k] = q[k];
                } else {
                    uint32_t d[5];
#pragma unroll
                    for (int k = 0; k < 5; ++k) d[k] = q[k];
#pragma unroll
                    for (int k = 0; k < 4; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
                }
                uint32_t S = 0, T = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    S = __builtin_amdgcn_udot4(w[k], 0x01010101u, S, false);
                    T = __builtin_amdgcn_udot4(w[k], 0x03020100u + 0x04040404u * (uint32_t)k, T, false);
                }
                sa += S;
                sb += (uint64_t)(L - i0) * S - T;
                continue;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t i = i0 + k;
                if (i < L) {
                    const uint32_t b = p[i];
                    sa += b;
                    sb += (uint64_t)(L - i) * b;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            sa += __shfl_xor(sa, 1 << j);
            sb += __shfl_xor(sb, 1 << j);
        }
        if (lane == 0) {
            const uint32_t a = (uint32_t)((1u + sa) % 65521u);
            const uint32_t b = (uint32_t)(((uint64_t)L + sb) % 65521u);
            out[c] = (b << 16) | a;
        }
    }
}

}  // namespace flz
}  // namespace nx

#include "workspace.hpp"
static_assert(nx::kWsSpec[(int)nx::WsKind::FastLzEnc].entry_bytes == sizeof(uint64_t) &&
                  (int)nx::kWsSpec[(int)nx::WsKind::FastLzEnc].lg == nx::flz::HASH_LOG,
              "FastLZ table geometry");

extern "C" int32_t nx_fastlz_compress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                            const uint64_t* out_off, uint32_t* out_len, const int32_t* level,
                                            const int32_t* u16_limit, int32_t* status, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    const size_t per = (size_t)nx::flz::HASH_SIZE * sizeof(uint64_t);
    nx::WsLease lease(nx::WsKind::FastLzEnc, dev, st);
    NX_HIP_CHECK(lease.acquire(nx::ws_want(nx::WsKind::FastLzEnc, n, cus)));
    nx::SharedWs& W = lease.ws();
    const nx::LaneGrid g = nx::ws_grid(nx::WsKind::FastLzEnc, n, cus, W.slots);
    uint64_t* ws = static_cast<uint64_t*>(W.p);
    const uint32_t iters = (uint32_t)((n + g.slots - 1) / g.slots);
    if ((uint64_t)W.stamp + iters >= 65535u) {
        NX_HIP_CHECK(hipMemsetAsync(ws, 0, W.slots * per, st));
        W.stamp = 0;
    }
    if (g.spread)
        hipLaunchKernelGGL(nx::flz::k_compress<true>, dim3(g.grid), dim3(g.block), 0, st, in, in_off, in_len, out, out_off, out_len, level,
                           u16_limit, status, n, ws, W.stamp);
    else
        hipLaunchKernelGGL(nx::flz::k_compress<false>, dim3(g.grid), dim3(g.block), 0, st, in, in_off, in_len, out, out_off, out_len,
                           level, u16_limit, status, n, ws, W.stamp);
    NX_HIP_CHECK(hipGetLastError());
    W.stamp += iters;
    return NX_OK;
}

namespace {
struct FlzDecCtx {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    const uint32_t* in_avail;
    uint8_t* out;
    const uint64_t* out_off;
    const uint32_t* lim;
    int32_t* result;
};
hipError_t flz_dec_after(uint32_t base, uint32_t m, const uint32_t* olen, void* ctx, hipStream_t st) {
    const FlzDecCtx& x = *static_cast<const FlzDecCtx*>(ctx);
    hipLaunchKernelGGL(nx::flz::k_decompress_finish, dim3((m + 255) / 256), dim3(256), 0, st, x.in, x.in_off + base, x.in_len + base,
                       x.in_avail ? x.in_avail + base : nullptr, x.out, x.out_off + base, x.lim + base, x.result + base, olen, m);
    return hipGetLastError();
}
}  // namespace

// Blocks go through the record expander (snappy_decode.hip k_parse_fastlz + k_expand); the few it
// does not take (malformed, reads past the block) through the lane-serial decompress().
extern "C" int32_t nx_fastlz_decompress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                              const uint32_t* in_avail, uint8_t* out, const uint64_t* out_off,
                                              const uint32_t* out_len_limit, int32_t* result, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len_limit || !result) return NX_ERR_INVALID_ARG;
    FlzDecCtx ctx{in, in_off, in_len, in_avail, out, out_off, out_len_limit, result};
    return nx::dec::decode_records(nx::dec::RecCodec::FastLz, in, in_off, in_len, in_avail, out_len_limit, out, out_off, result, n,
                                   (hipStream_t)stream, flz_dec_after, &ctx);
}

extern "C" int32_t nx_adler32_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t* out, uint32_t n,
                                    void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !off || !len || !out) return NX_ERR_INVALID_ARG;
    unsigned grid = n / 4 + 1;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(nx::flz::k_adler32, dim3(grid), dim3(256), 0, (hipStream_t)stream, in, off, len, out, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
