// snappy_encode.hip — Snappy block encoder, bit-exact with Netty's Snappy.encode (Snappy.java:82-313).
//
// One wave encodes one chunk; its 16384-entry u16 hash table (Java's short[], :97-100) lives in
// LDS (32 KiB; 4 waves = 4 chunks per workgroup, one workgroup per CU).
//
// Java's greedy matcher is a serial state machine: the probe order (`skip++ >> 5`, :107-115) and
// the evolving table decide the output.  The wave runs it over WINDOWS of 64 positions, lane l =
// position f + l, in three steps per window:
//
//  1. Speculate, lane-parallel.  Each lane hashes the big-endian word at its position (:177-179),
//     reads T[h] (the latest position inserted before the window with that hash; a fresh table
//     reads as position 0, :97-99) and finds the nearest earlier lane of the window with the same
//     hash (lanes write their id into T[h] and read it back: a different id marks a duplicate;
//     each duplicate group is resolved with one ballot).  Its speculative candidate is that lane's
//     position, else T[h].  Every lane loads 16 bytes at its candidate (duplicate lanes also at
//     T[h]) and computes getInt(p) == getInt(candidate) (:130,:154) and the match length
//     4 + findMatchingLength (:137, :224-239) up to 16 bytes.
//  2. Walk, uniform (scalar registers).  The walk replays Java's control flow over the window with
//     the per-lane results: a run of step-1 probes (:111-130) is one mask operation (first lane
//     that matches), a match jumps to its end (:135-146), inserts end-1 and tests end (:148-154).
//     Inserted positions are a 64-bit mask.  A lookup's speculative candidate is Java's T[h] when
//     its nearest same-hash lane was inserted; when no earlier lane of its group was inserted,
//     Java's T[h] is the pre-window value (the alternative computed in step 1).  Any other lookup
//     ends the window there and the next window starts at that position, where the committed table
//     is exact again.  The window also ends where the walk leaves it.
//  3. Emit + commit, lane-parallel.  Each match lane writes its literal header and copy tags
//     (encodeLiteral :268-281, encodeCopy :283-313) at offsets from a wave prefix sum; literal
//     bytes inside the window are stored by the lane of their position, older literal bytes by a
//     wave copy; the last inserted lane of each hash group writes its position into T, and the
//     lanes of groups with no insertion restore the value they read.
//
// Per 64 KiB text chunk this takes ~1000 windows for Java's ~16 500 probes and ~7 700 copies.
// The output is byte-identical to Snappy.encode (tests/test_gpu_snappy.py vs the oracle, which the
// SnappyTest.java:151-248 vectors pin).
#include <stdint.h>
#include <algorithm>
#include "../../netty_amd/csrc/nx_common.hpp"

namespace nx {
namespace enc {

constexpr int kWaves = 4;             // chunks (waves) per workgroup
constexpr int kTable = 16384;         // MAX_HT_SIZE (Snappy.java:33)
constexpr int kMinCompressible = 15;  // MIN_COMPRESSIBLE_BYTES (:34)

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u __attribute__((aligned(1))) v4uu;  // 16 bytes at any address (gfx950 unaligned global access)

__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return ((uint64_t)(uint32_t)rl((int)(v >> 32), l) << 32) | (uint32_t)rl((int)(uint32_t)v, l);
}
__device__ __forceinline__ int ffs64(uint64_t m) { return __builtin_ctzll(m); }       // m != 0
__device__ __forceinline__ int fls64(uint64_t m) { return 63 - __builtin_clzll(m); }  // m != 0
__device__ __forceinline__ uint64_t below(int l) { return l >= 64 ? ~0ull : ((1ull << l) - 1ull); }
__device__ __forceinline__ uint64_t range_mask(int a, int b) { return below(b + 1) & ~below(a); }  // lanes a..b
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }

// 16 bytes at p; bytes at or past `avail` read as 0 and are not touched in memory.
__device__ __forceinline__ uint4 load16(const uint8_t* p, int avail) {
    if (avail >= 16) {
        const v4u v = *reinterpret_cast<const v4uu*>(p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint32_t v[4] = {0, 0, 0, 0};
    for (int i = 0; i < avail; ++i) v[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// common-prefix length of two 16-byte groups whose first 4 bytes are equal: 4..16
__device__ __forceinline__ int prefix16(uint4 a, uint4 b) {
    uint32_t x = a.y ^ b.y;
    if (x) return 4 + (__builtin_ctz(x) >> 3);
    x = a.z ^ b.z;
    if (x) return 8 + (__builtin_ctz(x) >> 3);
    x = a.w ^ b.w;
    if (x) return 12 + (__builtin_ctz(x) >> 3);
    return 16;
}

// 4 + findMatchingLength(c + 4, p + 4, L) (:224-239) for a match known to extend past 16 bytes:
// the common-prefix length of in[c..] and in[p..] bounded by L - p, 256 bytes per wave step.
__device__ int extend_match(const uint8_t* __restrict__ in, int c, int p, int L, int lane) {
    const int lim = L - p;
    for (int m = 16; m < 70000; m += 256) {
        const int o = m + 4 * lane;
        int mis = 0;  // first differing byte of this lane's 4 (4 = none); a lane at or past the end stops
        if (o < lim) {
            if (o + 4 <= lim) {
                const uint32_t x = ld32(in + c + o) ^ ld32(in + p + o);
                mis = x ? (__builtin_ctz(x) >> 3) : 4;
            } else {
                mis = lim - o;
                for (int i = 0; i < lim - o; ++i)
                    if (in[c + o + i] != in[p + o + i]) {
                        mis = i;
                        break;
                    }
            }
        }
        const uint64_t stop = ballot(mis < 4);
        if (stop) {
            const int t = ffs64(stop);
            return m + 4 * t + rl(mis, t);
        }
    }
    return -1;
}

// dst[0..n) = src[0..n) with the whole wave (16 bytes per lane per step).
__device__ void copy_wave(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int n, int lane) {
    for (int o = lane * 16; o < n; o += 64 * 16) {
        if (o + 16 <= n) {
            *reinterpret_cast<v4uu*>(dst + o) = *reinterpret_cast<const v4uu*>(src + o);
        } else {
            for (int i = o; i < n; ++i) dst[i] = src[i];
        }
    }
}

// bytes of encodeCopy(offset, len) (:301-313 splitting into encodeCopyWithOffset :283-292 pieces)
__device__ __forceinline__ int copy_bytes(int off, int len) {
    int n = 0;
    if (len >= 68) {
        const int k = (len - 68) / 64 + 1;
        n = 3 * k;
        len -= 64 * k;
    }
    if (len > 64) {
        n += 3;
        len -= 60;
    }
    return n + ((len < 12 && off < 2048) ? 2 : 3);
}
__device__ __forceinline__ int lit_hdr_bytes(int len) {  // encodeLiteral's header (:269-279), len >= 1
    return len < 61 ? 1 : 2 + ((31 - __builtin_clz((uint32_t)(len - 1))) >> 3);
}
__device__ __forceinline__ void put_lit_hdr(uint8_t* o, int len) {
    if (len < 61) {
        o[0] = (uint8_t)((len - 1) << 2);
    } else {
        const int v = len - 1;
        const int nb = 1 + ((31 - __builtin_clz((uint32_t)v)) >> 3);
        o[0] = (uint8_t)((59 + nb) << 2);
        for (int i = 0; i < nb; ++i) o[1 + i] = (uint8_t)(v >> (8 * i));
    }
}
__device__ __forceinline__ uint8_t* put_copy1(uint8_t* o, int off, int len) {
    if (len < 12 && off < 2048) {
        o[0] = (uint8_t)(1 | ((len - 4) << 2) | ((off >> 8) << 5));
        o[1] = (uint8_t)off;
        return o + 2;
    }
    o[0] = (uint8_t)(2 | ((len - 1) << 2));
    o[1] = (uint8_t)off;
    o[2] = (uint8_t)(off >> 8);
    return o + 3;
}
__device__ __forceinline__ void put_copy(uint8_t* o, int off, int len) {
    while (len >= 68) {
        o = put_copy1(o, off, 64);
        len -= 64;
    }
    if (len > 64) {
        o = put_copy1(o, off, 60);
        len -= 60;
    }
    put_copy1(o, off, len);
}

enum { kProbe = 0, kMatch = 1, kChain = 2 };

#ifdef NX_ENC_TIMING  // experiment builds only (scripts/enc_bench.cpp): s_memtime per phase, summed per wave
__device__ unsigned long long* g_tim;
#define TSTAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define TACC(slot, a, b) do { tacc[slot] += (b) - (a); } while (0)
#define TIM_PARAM , unsigned long long* tacc
#define TIM_ARG , tacc
#else
#define TSTAMP(var) do { } while (0)
#define TACC(slot, a, b) do { } while (0)
#define TIM_PARAM
#define TIM_ARG
#endif

#ifdef NX_ENC_TRACE  // debug builds only (scripts/enc_trace.cpp): progress markers in host-visible memory
__device__ uint32_t* g_trace;
#define TRACE(slot, v) \
    do { if (lane == 0) __hip_atomic_store(g_trace + (slot), (uint32_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#else
#define TRACE(slot, v) do { } while (0)
#endif

// Encode one chunk with the calling wave.  Returns the compressed length, or -1 if the window
// loop's guard tripped (cannot happen: every window advances; the guard keeps a bug from spinning).
__device__ int encode_chunk(const uint8_t* __restrict__ in, const int L, uint8_t* __restrict__ out, uint16_t* T, const int lane TIM_PARAM) {
    int op = 0;  // output position (uniform)
    {            // preamble (:84-92)
        uint32_t b = (uint32_t)L;
        while (b & 0xFFFFFF80u) {
            if (lane == 0) out[op] = (uint8_t)((b & 0x7f) | 0x80);
            ++op;
            b >>= 7;
        }
        if (lane == 0) out[op] = (uint8_t)b;
        ++op;
    }
    int nextEmit = 0;
    if (L >= kMinCompressible) {
        uint32_t hts = 1u << (32 - __builtin_clz((uint32_t)(L - 1)));  // findNextPositivePowerOfTwo (MathUtil.java:34-37)
        if (hts > (uint32_t)kTable) hts = kTable;
        const int shift = __builtin_clz(hts) + 1;  // (:100)
        for (uint32_t i = lane * 8; i < hts; i += 64 * 8) *reinterpret_cast<v4u*>(T + i) = v4u{0, 0, 0, 0};
        int mode = kProbe;  // window entry: kProbe at q with `skip`, or kChain: a match ended at q
        int q = 1, skip = 32;
        for (int guard = 0;; ++guard) {
            if (guard > 2 * L + 64) return -1;
            TRACE(1, guard);
            TRACE(2, q);
            const int f = mode == kProbe ? q : q - 1;
            const int p = f + lane;
            const bool valid = p <= L - 4;
            // ---- 1. speculate
            TSTAMP(t0);
            const uint4 a = valid ? load16(in + p, L - p) : make_uint4(0, 0, 0, 0);
            const uint32_t h = valid ? (__builtin_bswap32(a.x) * 0x1e35a7bdu) >> shift : 0u;
            uint32_t tv = 0, rb = (uint32_t)lane;
            if (valid) {
                tv = T[h];
                T[h] = (uint16_t)lane;
                asm volatile("" ::: "memory");  // other lanes wrote T too: read it back from LDS
                rb = T[h];
            }
            uint64_t dupm = ballot(rb != (uint32_t)lane);
            uint64_t same = 1ull << lane;
            for (int dg = 0; dupm; ++dg) {
                if (dg > 64) return -3;
                const uint32_t hj = (uint32_t)rl((int)h, ffs64(dupm));
                const uint64_t g = ballot(valid && h == hj);
                if (valid && h == hj) same = g;
                dupm &= ~g;
            }
            const uint64_t lower = same & below(lane);
            const int ps = lower ? fls64(lower) : -1;  // nearest earlier lane with the same hash
            const int cs = ps >= 0 ? f + ps : (int)tv;
            TSTAMP(t1);
            bool eqs = false, eqt = false;
            int lens = 0, lent = 0;
            if (valid) {
                const uint4 b = load16(in + cs, L - cs);
                uint4 bt = b;
                if (ps >= 0) bt = load16(in + tv, L - (int)tv);
                const int lim = L - p;
                eqs = b.x == a.x;
                if (eqs) lens = min(prefix16(a, b), lim);
                eqt = bt.x == a.x;
                if (eqt) lent = min(prefix16(a, bt), lim);
            }
            const uint64_t EQ = ballot(eqs), EQT = ballot(eqt);
            TSTAMP(t2);
            // ---- 2. walk (uniform)
            uint64_t I = 0, M = 0, UT = 0;  // inserted lanes, match lanes, lanes whose candidate is T[h]
            int fin_len = 0;                // per match lane: its final length
            bool ended = false;
            const int nextEmit0 = nextEmit;
            int st = kProbe, l = 0, k = 0, wguard = 0;
            if (mode == kChain) {
                I = 1;  // lane 0 = q - 1 (:148-149)
                k = 1;
                st = kChain;
            }
            for (;;) {
                if (++wguard > 4096) return -2;
                TRACE(3, wguard);
                TRACE(4, st * 1000 + l);
                if (st == kProbe) {
                    if (f + l + (skip >> 5) > L - 4) {  // (:118-120)
                        ended = true;
                        break;
                    }
                    if (l >= 64) {
                        mode = kProbe;
                        q = f + l;
                        break;
                    }
                    if (skip < 64) {  // step-1 probes at lanes l .. last as one mask
                        const int last = min(min(l + 63 - skip, 63), L - 5 - f);
                        const uint64_t rng = range_mask(l, last);
                        const uint64_t V = ballot(ps >= 0 && ps < l && !((I >> ps) & 1ull));
                        const uint64_t cand = (EQ | V) & rng;
                        if (!cand) {
                            I |= rng;
                            skip += last - l + 1;
                            l = last + 1;
                            continue;
                        }
                        const int j = ffs64(cand);
                        if (j > l) I |= range_mask(l, j - 1);
                        skip += j - l;
                        l = j;
                        I |= 1ull << j;
                        if ((V >> j) & 1ull) {
                            if (rl64(same, j) & I & below(j)) {  // an older lane of its group was inserted
                                I &= ~(1ull << j);
                                mode = kProbe;
                                q = f + j;
                                break;
                            }
                            UT |= 1ull << j;
                            if (!((EQT >> j) & 1ull)) {
                                ++skip;
                                l = j + 1;
                                continue;
                            }
                        }
                        st = kMatch;
                        continue;
                    }
                    // one probe with a step of 2 or more
                    const int psl = rl(ps, l);
                    bool ut = false;
                    if (psl >= 0 && !((I >> psl) & 1ull)) {
                        if (rl64(same, l) & I & below(l)) {
                            mode = kProbe;
                            q = f + l;
                            break;
                        }
                        ut = true;
                        UT |= 1ull << l;
                    }
                    I |= 1ull << l;
                    if (((ut ? EQT : EQ) >> l) & 1ull) {
                        st = kMatch;
                        continue;
                    }
                    l += skip >> 5;
                    ++skip;
                } else if (st == kMatch) {  // a copy at lane l (:135-147)
                    M |= 1ull << l;
                    const bool ut = (UT >> l) & 1ull;
                    int len = ut ? rl(lent, l) : rl(lens, l);
                    if (len == 16 && L - (f + l) > 16) len = extend_match(in, ut ? rl((int)tv, l) : rl(cs, l), f + l, L, lane);
                    if (len < 4 || len > L - (f + l)) return -4;
                    if (lane == l) fin_len = len;
                    const int qq = f + l + len;
                    nextEmit = qq;
                    if (qq >= L - 4) {  // (:144-146)
                        ended = true;
                        break;
                    }
                    k = l + len;
                    if (k >= 64) {
                        mode = kChain;
                        q = qq;
                        break;
                    }
                    I |= 1ull << (k - 1);  // (:148-149)
                    st = kChain;
                } else {  // kChain: test the position after a copy (:150-154)
                    const int psk = rl(ps, k);
                    bool ut = false;
                    if (psk >= 0 && !((I >> psk) & 1ull)) {
                        if (rl64(same, k) & I & below(k)) {
                            mode = kChain;
                            q = f + k;
                            break;
                        }
                        ut = true;
                        UT |= 1ull << k;
                    }
                    I |= 1ull << k;
                    if (((ut ? EQT : EQ) >> k) & 1ull) {
                        l = k;
                        st = kMatch;
                    } else {
                        l = k + 1;  // (:156-157)
                        skip = 32;
                        st = kProbe;
                    }
                }
            }
            TRACE(5, 100 + guard);
            TSTAMP(t3);
            // ---- 3. emit the window's copies and the literals before them
            if (M) {
                const bool isM = (M >> lane) & 1ull;
                const int cand = ((UT >> lane) & 1ull) ? (int)tv : cs;
                const int mlen = isM ? fin_len : 0;
                const uint64_t pm = M & below(lane);
                const int pe = __shfl(p + mlen, pm ? fls64(pm) : 0);
                const int prevEnd = pm ? pe : nextEmit0;
                const int lit = isM ? p - prevEnd : 0;  // 0 for a copy that follows a copy
                const int hdr = lit ? lit_hdr_bytes(lit) : 0;
                const int sz = isM ? hdr + lit + copy_bytes(p - cand, mlen) : 0;
                if (ballot(isM && (lit < 0 || lit > L || p - cand <= 0 || p - cand > 65535 || mlen < 4))) return -5;
                int incl = sz;  // inclusive prefix sum over the wave
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int t = __shfl_up(incl, d);
                    if (lane >= d) incl += t;
                }
                const int o = op + incl - sz;
#ifndef NX_ENC_NO_EMIT
                if (isM) {
                    if (lit) put_lit_hdr(out + o, lit);
                    put_copy(out + o + hdr + lit, p - cand, mlen);
                }
                // literal bytes at the window's own positions: the first copy above a position owns it
                const uint64_t am = M & ~below(lane + 1);
                const int nm = am ? ffs64(am) : 0;
                const int dbase = __shfl(o + hdr - prevEnd, nm);  // output index of position x = dbase + x
                const int nprev = __shfl(prevEnd, nm);
                if (am && p >= nprev) out[dbase + p] = (uint8_t)a.x;
                // literal bytes older than the window (only the first copy's literal can start earlier)
                const int fm = ffs64(M);
                const int fprev = rl(prevEnd, fm);
                if (fprev < f) copy_wave(out + rl(o + hdr, fm), in + fprev, f - fprev, lane);
#endif
                op += rl(incl, 63);
            }
            // ---- commit this window's insertions to T (and restore the ids written in step 1)
            if (valid) {
                const uint64_t ins = same & I;
                if (ins) {
                    if (fls64(ins) == lane) T[h] = (uint16_t)p;
                } else {
                    T[h] = (uint16_t)tv;
                }
            }
            TRACE(6, 100 + guard);
            TSTAMP(t4);
            TACC(0, t0, t1);
            TACC(1, t1, t2);
            TACC(2, t2, t3);
            TACC(3, t3, t4);
            TACC(4, 0ull, 1ull);
            if (ended) break;
        }
    }
    TRACE(7, 1);
    if (nextEmit < L) {  // trailing literal (:162-164)
        const int n = L - nextEmit;
        TRACE(9, n);
        if (lane == 0) put_lit_hdr(out + op, n);
        TRACE(10, op);
        const int hb = lit_hdr_bytes(n);
        TRACE(11, hb);
        copy_wave(out + op + hb, in + nextEmit, n, lane);
        TRACE(12, 1);
        op += hb + n;
    }
    TRACE(13, op);
    return __builtin_amdgcn_readfirstlane(op);
}

__global__ void __launch_bounds__(64 * kWaves) k_snappy_encode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                              const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                              const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                              int32_t* __restrict__ status, uint32_t n) {
    __shared__ uint16_t tables[kWaves][kTable];
    const int lane = lane_id();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint16_t* T = tables[wave];
#ifdef NX_ENC_TIMING
    unsigned long long tacc[5] = {0, 0, 0, 0, 0};
#endif
    for (uint32_t c = blockIdx.x * kWaves + wave; c < n; c += gridDim.x * kWaves) {
        TRACE(0, 1000 + c);
        const uint32_t len = in_len[c];
        int32_t stv = NX_OK;
        int olen = 0;
        if (len > 65536u) {
            stv = NX_ERR_INVALID_ARG;
        } else {
            olen = encode_chunk(in + in_off[c], (int)len, out + out_off[c], T, lane TIM_ARG);
            TRACE(14, olen);
            if (olen < 0) {
                stv = NX_ERR_INTERNAL;
                olen = -olen;  // which guard tripped (debug aid)
            }
        }
        if (lane == 0) {
            out_len[c] = (uint32_t)olen;
            status[c] = stv;
        }
        TRACE(8, 1);
    }
#ifdef NX_ENC_TIMING
    if (lane == 0)
        for (int i = 0; i < 5; ++i) atomicAdd(g_tim + i, tacc[i]);
#endif
}

}  // namespace enc
}  // namespace nx

extern "C" int32_t nx_snappy_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                          const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream) {
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    // one workgroup (4 chunk waves, 128 KiB of tables) per CU; wave w of group g takes chunks
    // g * 4 + w, then + groups * 4, ...
    const uint32_t groups = std::min<uint32_t>((uint32_t)cus, (n + nx::enc::kWaves - 1) / nx::enc::kWaves);
    hipLaunchKernelGGL(nx::enc::k_snappy_encode, dim3(groups), dim3(64 * nx::enc::kWaves), 0, st, in, in_off, in_len, out, out_off,
                       out_len, status, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
