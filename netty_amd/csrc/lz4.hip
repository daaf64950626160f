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

// ---------------------------------------------------------------------------------------------
// LZ4 HC (Lz4FrameEncoder(highCompressor = true): lz4-java's highCompressor() = liblz4's
// LZ4_compress_HC at level 9, Lz4FrameEncoder.java:123-125,161-163).  Bit-exact with the oracle's
// restatement (oracle/netty_oracle.c orc_lz4hc_compress, pinned against pyarrow's liblz4 at level 9):
// the hash-chain match finder (256 candidates, pattern analysis) and the lazy three-match parse.
// One lane per block; its tables live in the Lz4HcEnc workspace (256 KiB per lane: u32 hash[2^15],
// u16 chain[2^16]).  liblz4 indexes positions from 64 KiB on a fresh context; a lane here gives its
// j-th block of a launch the base B = 64 KiB + (stamp + j) * kHcStride, so every entry an earlier
// block left lies below the new block's lowLimit (= B) and reads exactly as a fresh table does (an
// empty slot and an old index both end the chain; old chain deltas are only reached through old
// indices).  The host zeroes the tables before the bases would pass 2^32.
constexpr uint32_t kHcLog = 15, kHcDmax = 65535, kHcOptMl = 18, kHcAttempts = 256;
constexpr uint32_t kHcStride = (1u << 25) + (1u << 16);  // > a maximum block plus 64 KiB
constexpr uint32_t kHcTableWords = (1u << kHcLog) + (1u << 15);  // hash (u32) + chain (2^16 u16)

__device__ __forceinline__ uint32_t ld16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t hc_hash(const uint8_t* p) { return (ld32(p) * 2654435761u) >> (32 - kHcLog); }

struct Hc {
    const uint8_t* in;  // index i is in[i - B]
    uint32_t B;         // index of the block's byte 0 (dictLimit = lowLimit)
    uint32_t next;      // nextToUpdate
    uint32_t* hash;
    uint16_t* chain;
    __device__ __forceinline__ const uint8_t* P(uint32_t i) const { return in + (i - B); }
    __device__ __forceinline__ void insert(uint32_t target) {  // LZ4HC_Insert
        for (uint32_t idx = next; idx < target; ++idx) {
            const uint32_t h = hc_hash(P(idx));
            uint32_t delta = idx - hash[h];
            if (delta > kHcDmax) delta = kHcDmax;
            chain[(uint16_t)idx] = (uint16_t)delta;
            hash[h] = idx;
        }
        next = target;
    }
    __device__ __forceinline__ bool protect(uint32_t idx) const { return (uint32_t)((B - 1u) - idx) >= 3u; }
};
// LZ4HC_countPattern / LZ4HC_reverseCountPattern (the 4-byte pattern repeated)
__device__ __forceinline__ int32_t hc_count_pattern(const uint8_t* p, const uint8_t* end, uint32_t pat) {
    int32_t k = 0;
    while (p + 4 <= end && ld32(p) == pat) {
        p += 4;
        k += 4;
    }
    while (p < end && *p == (uint8_t)(pat >> (8 * (k & 3)))) {
        ++p;
        ++k;
    }
    return k;
}
__device__ __forceinline__ int32_t hc_rcount_pattern(const uint8_t* p, const uint8_t* low, uint32_t pat) {
    int32_t k = 0;
    while (p - 4 >= low && ld32(p - 4) == pat) {
        p -= 4;
        k += 4;
    }
    while (p > low && p[-1] == (uint8_t)(pat >> (8 * (3 - (k & 3))))) {
        --p;
        ++k;
    }
    return k;
}
__device__ __forceinline__ int32_t hc_count(const uint8_t* a, const uint8_t* b, const uint8_t* alim) {  // LZ4_count
    const uint8_t* s = a;
    while (a + 4 <= alim) {
        const uint32_t x = ld32(a) ^ ld32(b);
        if (x) return (int32_t)(a - s) + (int32_t)(__builtin_ctz(x) >> 3);
        a += 4;
        b += 4;
    }
    while (a < alim && *a == *b) {
        ++a;
        ++b;
    }
    return (int32_t)(a - s);
}

// LZ4HC_InsertAndGetWiderMatch (prefix only; chainSwap off, as LZ4HC_compress_hashChain calls it)
__device__ int32_t hc_wider(Hc& c, const uint8_t* ip, const uint8_t* ilow, const uint8_t* ihigh, int32_t longest,
                            const uint8_t** matchpos, const uint8_t** startpos) {
    const uint32_t ip_idx = (uint32_t)(ip - c.in) + c.B;
    const uint32_t lowest = (c.B + kHcDmax + 1u > ip_idx) ? c.B : ip_idx - kHcDmax;
    const int32_t look_back = (int32_t)(ip - ilow);
    int32_t attempts = (int32_t)kHcAttempts;
    const uint32_t pattern = ld32(ip);
    int repeat = 0;  // 0 untested, 1 confirmed, 2 not
    int32_t src_pattern_len = 0;
    c.insert(ip_idx);
    uint32_t mi = c.hash[hc_hash(ip)];
    while (mi >= lowest && attempts > 0) {
        --attempts;
        const uint8_t* mp = c.P(mi);
        if (ld16(ilow + longest - 1) == ld16(mp - look_back + longest - 1) && ld32(mp) == pattern) {
            int32_t back = 0;
            if (look_back) {
                const int32_t a = (int32_t)(ilow - ip), b = (int32_t)(c.in - mp);
                const int32_t mn = a > b ? a : b;
                while (back > mn && ip[back - 1] == mp[back - 1]) --back;
            }
            const int32_t ml = 4 + hc_count(ip + 4, mp + 4, ihigh) - back;
            if (ml > longest) {
                longest = ml;
                *matchpos = mp + back;
                *startpos = ip + back;
            }
        }
        if (c.chain[(uint16_t)mi] == 1u) {  // pattern analysis (levels 9+)
            const uint32_t cand = mi - 1u;
            if (repeat == 0) {
                if (((pattern & 0xFFFFu) == (pattern >> 16)) && ((pattern & 0xFFu) == (pattern >> 24))) {
                    repeat = 1;
                    src_pattern_len = hc_count_pattern(ip + 4, ihigh, pattern) + 4;
                } else {
                    repeat = 2;
                }
            }
            if (repeat == 1 && cand >= lowest && c.protect(cand)) {
                const uint8_t* cp = c.P(cand);
                if (ld32(cp) == pattern) {
                    const int32_t fwd = hc_count_pattern(cp + 4, ihigh, pattern) + 4;
                    int32_t bk = hc_rcount_pattern(cp, c.in, pattern);
                    {
                        const uint32_t lo = cand - (uint32_t)bk > lowest ? cand - (uint32_t)bk : lowest;
                        bk = (int32_t)(cand - lo);
                    }
                    const int32_t seg = bk + fwd;
                    if (seg >= src_pattern_len && fwd <= src_pattern_len) {
                        const uint32_t nmi = cand + (uint32_t)fwd - (uint32_t)src_pattern_len;
                        mi = c.protect(nmi) ? nmi : c.B;
                    } else {
                        const uint32_t nmi = cand - (uint32_t)bk;
                        if (!c.protect(nmi)) {
                            mi = c.B;
                        } else {
                            mi = nmi;
                            if (look_back == 0) {
                                const int32_t max_ml = seg < src_pattern_len ? seg : src_pattern_len;
                                if (longest < max_ml) {
                                    if (ip_idx - mi > kHcDmax) break;
                                    longest = max_ml;
                                    *matchpos = c.P(mi);
                                    *startpos = ip;
                                }
                                const uint32_t dp = c.chain[(uint16_t)mi];
                                if (dp > mi) break;
                                mi -= dp;
                            }
                        }
                    }
                    continue;
                }
            }
        }
        mi -= c.chain[(uint16_t)mi];
    }
    return longest;
}

// LZ4HC_encodeSequence
template <class O>
__device__ __forceinline__ uint32_t hc_sequence(O& out, uint32_t op, const uint8_t* in, const uint8_t*& ip, const uint8_t*& anchor,
                                                int32_t ml, const uint8_t* match) {
    const uint32_t token = op++;
    const uint32_t lit = (uint32_t)(ip - anchor);
    if (lit >= 15u) {
        out.set(token, 15u << 4);
        op = put_len(out, op, lit - 15u);
    } else {
        out.set(token, lit << 4);
    }
    for (uint32_t k = 0; k < lit; ++k) out.set(op + k, anchor[k]);
    op += lit;
    const uint32_t off = (uint32_t)(ip - match);
    out.set(op++, off & 0xFFu);
    out.set(op++, (off >> 8) & 0xFFu);
    uint32_t len = (uint32_t)ml - 4u;
    if (len >= 15u) {
        out.set(token, out.get(token) + 15u);
        op = put_len(out, op, len - 15u);  // (liblz4 writes 510-runs as pairs of 255: the same bytes)
    } else {
        out.set(token, out.get(token) + len);
    }
    ip += ml;
    anchor = ip;
    return op;
}

template <class O>
__device__ uint32_t encode_block_hc(const uint8_t* __restrict__ in, int32_t n, O& out, uint32_t* __restrict__ tabs, uint32_t B) {
    Hc c{in, B, B, tabs, reinterpret_cast<uint16_t*>(tabs + (1u << kHcLog))};
    const uint8_t* ip = in;
    const uint8_t* anchor = ip;
    const uint8_t* const iend = in + n;
    const uint8_t* const mflimit = iend - kMfLimit;
    const uint8_t* const matchlimit = iend - kLastLiterals;
    uint32_t op = 0;
    int32_t ml0, ml, ml2, ml3;
    const uint8_t *start0, *ref0, *ref = nullptr, *start2 = nullptr, *ref2 = nullptr, *start3 = nullptr, *ref3 = nullptr;
    if (n >= kMinLength) {
        while (ip <= mflimit) {
            {
                const uint8_t* useless = ip;
                ml = hc_wider(c, ip, ip, matchlimit, 3, &ref, &useless);  // LZ4HC_InsertAndFindBestMatch
            }
            if (ml < 4) {
                ++ip;
                continue;
            }
            start0 = ip;
            ref0 = ref;
            ml0 = ml;
        search2:
            if (ip + ml <= mflimit)
                ml2 = hc_wider(c, ip + ml - 2, ip, matchlimit, ml, &ref2, &start2);
            else
                ml2 = ml;
            if (ml2 == ml) {  // no better match: encode ML1
                op = hc_sequence(out, op, in, ip, anchor, ml, ref);
                continue;
            }
            if (start0 < ip && start2 < ip + ml0) {  // restore the initial ML1
                ip = start0;
                ref = ref0;
                ml = ml0;
            }
            if (start2 - ip < 3) {  // first match too small: removed
                ml = ml2;
                ip = start2;
                ref = ref2;
                goto search2;
            }
        search3:
            if (start2 - ip < (int32_t)kHcOptMl) {
                int32_t new_ml = ml;
                if (new_ml > (int32_t)kHcOptMl) new_ml = (int32_t)kHcOptMl;
                if (ip + new_ml > start2 + ml2 - 4) new_ml = (int32_t)(start2 - ip) + ml2 - 4;
                const int32_t corr = new_ml - (int32_t)(start2 - ip);
                if (corr > 0) {
                    start2 += corr;
                    ref2 += corr;
                    ml2 -= corr;
                }
            }
            if (start2 + ml2 <= mflimit)
                ml3 = hc_wider(c, start2 + ml2 - 3, start2, matchlimit, ml2, &ref3, &start3);
            else
                ml3 = ml2;
            if (ml3 == ml2) {  // no better match: encode ML1 and ML2
                if (start2 < ip + ml) ml = (int32_t)(start2 - ip);
                op = hc_sequence(out, op, in, ip, anchor, ml, ref);
                ip = start2;
                op = hc_sequence(out, op, in, ip, anchor, ml2, ref2);
                continue;
            }
            if (start3 < ip + ml + 3) {  // not enough space for match 2: remove it
                if (start3 >= ip + ml) {  // Seq1 goes now; Seq3 becomes Seq1
                    if (start2 < ip + ml) {
                        const int32_t corr = (int32_t)(ip + ml - start2);
                        start2 += corr;
                        ref2 += corr;
                        ml2 -= corr;
                        if (ml2 < 4) {
                            start2 = start3;
                            ref2 = ref3;
                            ml2 = ml3;
                        }
                    }
                    op = hc_sequence(out, op, in, ip, anchor, ml, ref);
                    ip = start3;
                    ref = ref3;
                    ml = ml3;
                    start0 = start2;
                    ref0 = ref2;
                    ml0 = ml2;
                    goto search2;
                }
                start2 = start3;
                ref2 = ref3;
                ml2 = ml3;
                goto search3;
            }
            // three ascending matches: write ML1
            if (start2 < ip + ml) {
                if (start2 - ip < (int32_t)kHcOptMl) {
                    if (ml > (int32_t)kHcOptMl) ml = (int32_t)kHcOptMl;
                    if (ip + ml > start2 + ml2 - 4) ml = (int32_t)(start2 - ip) + ml2 - 4;
                    const int32_t corr = ml - (int32_t)(start2 - ip);
                    if (corr > 0) {
                        start2 += corr;
                        ref2 += corr;
                        ml2 -= corr;
                    }
                } else {
                    ml = (int32_t)(start2 - ip);
                }
            }
            op = hc_sequence(out, op, in, ip, anchor, ml, ref);
            ip = start2;
            ref = ref2;
            ml = ml2;
            start2 = start3;
            ref2 = ref3;
            ml2 = ml3;
            goto search3;
        }
    }
    const uint32_t lit = (uint32_t)(iend - anchor);  // last literals
    if (lit >= 15u) {
        out.set(op++, 15u << 4);
        op = put_len(out, op, lit - 15u);
    } else {
        out.set(op++, lit << 4);
    }
    for (uint32_t k = 0; k < lit; ++k) out.set(op + k, anchor[k]);
    out.finish((int32_t)(op + lit));
    return op + lit;
}

template <bool SPREAD>
__global__ void __launch_bounds__(256) k_lz4hc_encode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                      const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                      const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                      int32_t* __restrict__ status, uint32_t n, uint32_t* __restrict__ workspace,
                                                      uint32_t stamp_base) {
    uint32_t tid, nthreads;
    if (!chunk_slot<SPREAD>(tid, nthreads)) return;
    uint32_t* tabs = workspace + (size_t)tid * kHcTableWords;
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
        const uint32_t B = 65536u + (stamp_base + iter) * kHcStride;
        if (SPREAD) {
            GOut o{out + out_off[c]};
            out_len[c] = encode_block_hc(in + in_off[c], (int32_t)len, o, tabs, B);
        } else {
            ByteStage o(slot, out + out_off[c]);
            out_len[c] = encode_block_hc(in + in_off[c], (int32_t)len, o, tabs, B);
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

namespace {
static_assert(nx::kWsSpec[(int)nx::WsKind::Lz4HcEnc].entry_bytes * (1u << nx::kWsSpec[(int)nx::WsKind::Lz4HcEnc].lg) ==
                  nx::lz4::kHcTableWords * sizeof(uint32_t),
              "LZ4 HC table geometry");
// block bases per lane between two zeroings: 65536 + (stamp + j) * kHcStride stays below 2^32 - 2^26
constexpr uint32_t kHcMaxStamp = (uint32_t)((0xFFFFFFFFull - (1ull << 26) - 65536ull) / nx::lz4::kHcStride);
}  // namespace

// Replaces LZ4Compressor.compress for lz4-java's highCompressor() (LZ4_compress_HC level 9) as
// Lz4FrameEncoder(highCompressor = true).flushBufferedData calls it (Lz4FrameEncoder.java:123-125,
// 161-163, 259-275); same contract as nx_lz4_encode_batch.
extern "C" int32_t nx_lz4hc_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                         const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    const size_t per = nx::lz4::kHcTableWords * sizeof(uint32_t);
    nx::WsLease lease(nx::WsKind::Lz4HcEnc, dev, st);
    NX_HIP_CHECK(lease.acquire(nx::ws_want(nx::WsKind::Lz4HcEnc, n, cus)));
    nx::SharedWs& W = lease.ws();
    const nx::LaneGrid g = nx::ws_grid(nx::WsKind::Lz4HcEnc, n, cus, W.slots);
    uint32_t* ws = static_cast<uint32_t*>(W.p);
    const size_t per_launch = g.slots * (kHcMaxStamp - 1);
    for (size_t base = 0; base < n; base += per_launch) {
        const uint32_t m = (uint32_t)std::min<size_t>(per_launch, n - base);
        const uint32_t iters = (uint32_t)((m + g.slots - 1) / g.slots);
        if (W.stamp + iters >= kHcMaxStamp) {
            NX_HIP_CHECK(hipMemsetAsync(ws, 0, W.slots * per, st));
            W.stamp = 0;
        }
        if (g.spread)
            hipLaunchKernelGGL(nx::lz4::k_lz4hc_encode<true>, dim3(g.grid), dim3(g.block), 0, st, in, in_off + base, in_len + base, out,
                               out_off + base, out_len + base, status + base, m, ws, W.stamp);
        else
            hipLaunchKernelGGL(nx::lz4::k_lz4hc_encode<false>, dim3(g.grid), dim3(g.block), 0, st, in, in_off + base, in_len + base,
                               out, out_off + base, out_len + base, status + base, m, ws, W.stamp);
        NX_HIP_CHECK(hipGetLastError());
        W.stamp += iters;
    }
    return NX_OK;
}

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
