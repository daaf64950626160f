// snappy_decode.hip — wave-cooperative Snappy decoder + fused CRC32C verify (gfx950).
//
// Replaces Snappy.decode (Snappy.java:315-650) as SnappyFrameDecoder drives it for one complete
// COMPRESSED_DATA chunk (SnappyFrameDecoder.java:194-224), fused with Snappy.validateChecksum
// (Snappy.java:700-707) over the produced bytes.  Bit-exact, including the reference's silent
// partial output on truncated input and its error precedence (offset 0 / negative / beyond,
// output overflow, invalid literal length, preamble > 4 bytes).
//
// One 64-lane wave decodes one frame; 24 waves (two 12-wave workgroups) are resident per CU.
// Per wave, in LDS:
//   stage  — 1 KiB ring of the compressed stream, refilled 512 B at a time by one 8-byte load per
//            lane that is issued a full half-ring ahead (register prefetch), so tag parsing and
//            literal reads never wait on HBM;
//   ring   — 4 KiB history of the decoded output (copies whose source lies within it are served
//            from LDS);
//   tags   — the current window's tag list.
// Steps per window (64 bytes of compressed stream that start at a tag):
//   parse   — lane l speculatively decodes "a tag at W+l" (2 ds_read_b32 + funnel shift); the real
//             tag chain is found by pointer doubling over ds_bpermute, which also compacts it
//             (lane m = m-th tag);
//   order   — the Java checks (NOT_ENOUGH_INPUT → silent stop, validateOffset, buffer capacity) run
//             per tag with bytes-written-so-far from a wave prefix sum; the first failing tag in
//             stream order decides, exactly as the serial state machine;
//   expand  — output is produced 64 bytes at a time, one byte per lane; the covering tag comes from a
//             tag-start bitmask + popcount; the byte from the stage (literal), the ring (near copy),
//             HBM (far copy: older output of this frame, already flushed and drained) or another lane
//             (overlapping copy, resolved by pointer jumping with ds_bpermute);
//   flush   — each completed 512 B block leaves the ring with one 8-byte store per lane; each lane
//             folds its 8 bytes into a per-lane CRC accumulator (slicing-by-4, then "shift by 512 B"),
//             and the 64 accumulators are combined once per frame (GF(2) shift tree), so the verify
//             costs neither an HBM pass nor a per-block reduction.
// HBM traffic per frame = compressed bytes read once + output written once (+ far-copy re-reads,
// mostly served from L2/MALL).
#include <stdlib.h>
#include <mutex>
#include "nx_common.hpp"

namespace nx {
namespace dec {

constexpr int kWaves = 12;        // waves per workgroup (2 workgroups per CU → 24 waves/CU at <= 80 VGPRs)
constexpr int kRing = 4096;       // decoded-output history per wave
constexpr int kStage = 1024;      // compressed-input ring per wave
constexpr int kFB = 512;          // flush block (64 lanes x 8 B)
constexpr int32_t kGuardTrip = -99;

// CRC tables staged in LDS per workgroup: slicing-by-4 (4 KiB), shift-by-512 B (4 KiB),
// nibble shift-by-8*2^j tables for the per-frame fold (3 KiB)
constexpr int kTabWords = 4 * 256 + 4 * 256 + 6 * 8 * 16;
constexpr int kTabBytes = kTabWords * 4;

struct Tag {  // 8 bytes in LDS
    uint32_t start;  // absolute output position
    uint32_t x;      // bit31 = copy; low 31 bits = literal source position (input) or copy offset
};

struct WaveLds {
    uint8_t ring[kRing];
    uint8_t stage[kStage];
    Tag tags[64];
    unsigned long long bmask;
    unsigned long long pad;
};
static_assert(sizeof(WaveLds) % 16 == 0, "keep per-wave LDS 16-byte aligned");

__device__ __forceinline__ uint32_t shift_byte_tab(const uint32_t* __restrict__ S, uint32_t c) {
    return S[c & 0xFF] ^ S[256 + ((c >> 8) & 0xFF)] ^ S[512 + ((c >> 16) & 0xFF)] ^ S[768 + (c >> 24)];
}

__device__ __forceinline__ uint32_t shift_nib_tab(const uint32_t* __restrict__ N, uint32_t c) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= N[k * 16 + ((c >> (4 * k)) & 15u)];
    return r;
}

// raw CRC (state 0) of 8 bytes (two LE dwords), slicing-by-4 twice
__device__ __forceinline__ uint32_t raw8(const uint32_t* __restrict__ T, uint32_t w0, uint32_t w1) {
    uint32_t c = w0;
    c = T[3 * 256 + (c & 0xFF)] ^ T[2 * 256 + ((c >> 8) & 0xFF)] ^ T[1 * 256 + ((c >> 16) & 0xFF)] ^ T[c >> 24];
    c ^= w1;
    c = T[3 * 256 + (c & 0xFF)] ^ T[2 * 256 + ((c >> 8) & 0xFF)] ^ T[1 * 256 + ((c >> 16) & 0xFF)] ^ T[c >> 24];
    return c;
}

// Wave-uniform value → SGPR (values loaded by vector memory ops or shuffles are otherwise VGPRs and
// every branch on them becomes exec-masked divergent code).
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ __forceinline__ uint64_t lanemask_le(int lane) { return lane == 63 ? ~0ull : ((2ull << lane) - 1ull); }

__device__ __forceinline__ uint32_t excl_scan(uint32_t x, int lane) {
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d);
        if (lane >= d) v += y;
    }
    return v - x;
}

struct Frame {
    const uint8_t* src;
    uint32_t in_len;
    uint8_t* dst;
    uint32_t cap;
};

__device__ void decode_frame(WaveLds& L, const Frame& f, const uint32_t* __restrict__ sT, const uint32_t* __restrict__ sSH,
                             const uint32_t* __restrict__ sNS, bool do_crc, uint32_t expect, bool check, uint32_t* out_len_p,
                             uint32_t* consumed_p, int32_t* status_p, uint32_t* crc_p, int lane) {
    const uint8_t* __restrict__ src = f.src;
    uint8_t* __restrict__ dst = f.dst;
    const uint32_t in_len = uni(f.in_len);
    const uint32_t cap = uni(f.cap < (1u << 24) ? f.cap : (1u << 24));
    int32_t st = NX_OK;
    uint32_t consumed = 0;
    uint32_t O = 0;        // output frontier (bytes final)
    uint32_t flushed = 0;  // bytes stored to HBM
    uint32_t acc = 0;      // this lane's CRC accumulator over its 8-byte slot of every flushed block
    const bool dst8 = (((uintptr_t)dst) & 7u) == 0;

    // ---- compressed-input stage (aligned coordinates: position p of the chunk is byte p + a)
    const uint32_t a = (uint32_t)((uintptr_t)src & 7u);
    const uint8_t* __restrict__ asrc = src - a;
    const uint32_t aend = a + in_len;
    uint32_t sbase = 0;
    uint2 pf = make_uint2(0, 0);
    auto load8 = [&](uint32_t apos) -> uint2 {
        return apos < aend ? *reinterpret_cast<const uint2*>(asrc + apos) : make_uint2(0, 0);
    };
    auto put8 = [&](uint32_t apos, uint2 v) { *reinterpret_cast<uint2*>(&L.stage[apos & (kStage - 1)]) = v; };
    auto prime = [&](uint32_t wa) {
        sbase = wa & ~511u;
        put8(sbase + 8u * lane, load8(sbase + 8u * lane));
        put8(sbase + 512u + 8u * lane, load8(sbase + 512u + 8u * lane));
        pf = load8(sbase + 1024u + 8u * lane);
    };
    auto advance = [&](uint32_t wa) {
        while (wa >= sbase + 512u) {
            if (wa >= sbase + 1536u) {
                prime(wa);
                break;
            }
            put8(sbase + 1024u + 8u * lane, pf);
            sbase += 512u;
            pf = load8(sbase + 1024u + 8u * lane);
        }
    };

    // ---- preamble (Snappy.readPreamble, :404-420) — uniform
    uint32_t W = 0;
    bool go = false;
    if (in_len > 0) {
        uint32_t ulen = 0;
        int bi = 0;
        bool complete = false;
        while (W < in_len) {
            const uint32_t cur = uni(src[W++]);
            ulen |= (cur & 0x7fu) << (bi++ * 7);
            if ((cur & 0x80u) == 0) {
                complete = true;
                break;
            }
            if (bi >= 4) {
                st = NX_ERR_SNAPPY_PREAMBLE_TOO_LONG;
                break;
            }
        }
        if (st == NX_OK && complete && ulen != 0) {
            if (ulen > cap) st = NX_ERR_SNAPPY_OUTPUT_OVERFLOW; else go = true;
        }
        consumed = W;
    }
    W = uni(W);
    if (go) prime(W + a);

    bool stop = !go;
    bool trip = false;
    uint32_t windows = 0;
    while (!stop && W < in_len) {
        if (++windows > in_len + 2) {
            st = kGuardTrip;
            break;
        }
        advance(W + a);
        // ---------------- parse: speculative tag decode at W + lane (bytes from the stage)
        const uint32_t p = W + lane;
        const uint32_t avail = p < in_len ? in_len - p : 0u;
        uint32_t b[5];
        {
            const uint32_t pa = p + a;
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(L.stage);
            const uint64_t d = (uint64_t)s32[(pa >> 2) & (kStage / 4 - 1)] |
                               ((uint64_t)s32[((pa >> 2) + 1) & (kStage / 4 - 1)] << 32);
            const uint64_t v = d >> (8 * (pa & 3u));
#pragma unroll
            for (int k = 0; k < 5; ++k) b[k] = ((uint32_t)k < avail) ? (uint32_t)((v >> (8 * k)) & 0xFFu) : 0u;
        }
        const uint32_t tag = b[0], type = tag & 3u;
        uint32_t size = 1;  // bytes of this tag in the stream (saturating)
        uint32_t olen = 0;  // output length (clamped to cap+1)
        uint32_t x = 0;     // literal source position
        bool nei = false;
        int32_t err = 0;
        const bool is_copy = type != 0;
        int64_t off64 = 0;
        if (type == 0) {  // decodeLiteral (:454-494)
            const uint32_t code = tag >> 2;
            uint32_t hdr = 1;
            int64_t jlen;
            if (code < 60) {
                jlen = (int64_t)code + 1;
            } else {
                const uint32_t nb = code - 59;
                hdr = 1 + nb;
                if (avail < hdr) {
                    nei = true;
                    jlen = 0;
                } else {
                    const uint32_t v = b[1] | (nb > 1 ? b[2] << 8 : 0u) | (nb > 2 ? b[3] << 16 : 0u) | (nb > 3 ? b[4] << 24 : 0u);
                    jlen = (nb == 4) ? (int64_t)(int32_t)(v + 1u) : (int64_t)v + 1;  // Java int `length += 1`
                }
            }
            if (!nei) {
                if (jlen >= 0 && (int64_t)(avail - hdr) < jlen) {
                    nei = true;
                } else if (jlen < 0) {
                    err = NX_ERR_SNAPPY_LITERAL_LEN_INVALID;
                }
            }
            const uint64_t sz = (uint64_t)hdr + (jlen > 0 ? (uint64_t)jlen : 0ull);
            size = sz > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)sz;
            olen = jlen > (int64_t)cap ? cap + 1 : (uint32_t)(jlen > 0 ? jlen : 0);
            x = (p + hdr) & 0x7FFFFFFFu;
        } else if (type == 1) {  // decodeCopyWith1ByteOffset (:509-538)
            size = 2;
            nei = avail < 2;
            olen = 4 + ((tag >> 2) & 7u);
            off64 = (int64_t)(((tag & 0xe0u) << 3) | b[1]);
        } else if (type == 2) {  // decodeCopyWith2ByteOffset (:553-582)
            size = 3;
            nei = avail < 3;
            olen = 1 + (tag >> 2);
            off64 = (int64_t)(b[1] | (b[2] << 8));
        } else {  // decodeCopyWith4ByteOffset (:597-626)
            size = 5;
            nei = avail < 5;
            olen = 1 + (tag >> 2);
            off64 = (int64_t)(int32_t)(b[1] | (b[2] << 8) | (b[3] << 16) | (b[4] << 24));
        }
        if (is_copy && !nei) {  // validateOffset (:637-650), part 1
            if (off64 == 0) err = NX_ERR_SNAPPY_OFFSET_ZERO;
            else if (off64 < 0) err = NX_ERR_SNAPPY_OFFSET_NEGATIVE;
        }
        const uint32_t nxt = (uint32_t)lane + size;  // relative position of the following tag

        // ---------------- tag chain by pointer doubling (no scalar walk)
        // J0[l] = next tag position if a tag starts at l (64 = leaves the window); positions at or
        // past the end of the input are fixed points.  Jk = J0^(2^k); lane m then composes the Jk
        // selected by the bits of m, so lane m ends on the position of the m-th tag: the chain comes
        // out compacted (lanes 0..T-1 = tags in stream order).
        const uint32_t lim = uni((in_len - W) < 64u ? (in_len - W) : 64u);
        uint32_t Jk[6];
        Jk[0] = (uint32_t)lane >= lim ? (uint32_t)lane : (nxt < 64u ? nxt : 64u);
#pragma unroll
        for (int k = 1; k < 6; ++k) {
            const uint32_t prev = Jk[k - 1];
            const uint32_t g = (uint32_t)__shfl((int)prev, (int)(prev & 63u));
            Jk[k] = prev >= 64u ? 64u : g;
        }
        uint32_t pos = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t g = (uint32_t)__shfl((int)Jk[k], (int)(pos & 63u));
            if (((uint32_t)lane >> k) & 1u) pos = pos >= 64u ? 64u : g;
        }
        const bool tv = pos < lim;  // lane m holds tag m
        const uint32_t T = (uint32_t)__popcll(__ballot(tv));
        // gather tag m's fields from lane pos
        const uint32_t src_l = (uint32_t)(pos & 63u);
        const uint32_t flags = (is_copy ? 1u : 0u) | (nei ? 2u : 0u) | ((uint32_t)(-err) << 8);
        const uint32_t xv = is_copy ? (off64 > 0x7FFFFFFFll ? 0x7FFFFFFFu : (uint32_t)(off64 < 0 ? 0 : off64)) : x;
        const uint32_t m_olen = (uint32_t)__shfl((int)olen, (int)src_l);
        const uint32_t m_flags = (uint32_t)__shfl((int)flags, (int)src_l);
        const uint32_t m_x = (uint32_t)__shfl((int)xv, (int)src_l);
        const bool m_copy = (m_flags & 1u) != 0;
        const bool m_nei = (m_flags & 2u) != 0;
        int32_t m_err = -(int32_t)(m_flags >> 8);
        // the window's exit: the position after the last tag
        const uint32_t lastpos = uni((uint32_t)__builtin_amdgcn_readlane((int)pos, (int)(T - 1)));
        const uint32_t exitrel = uni((uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)lastpos));

        // ---------------- ordering: bytes written before each tag, per-tag checks (stream order = lane order)
        const uint32_t mylen = tv ? m_olen : 0u;
        const uint32_t ostart = O + excl_scan(mylen, lane);
        if (tv && m_copy && !m_nei && m_err == 0 && m_x > ostart) m_err = NX_ERR_SNAPPY_OFFSET_BEYOND;
        if (tv && !m_nei && m_err == 0 && (uint64_t)ostart + m_olen > cap) m_err = NX_ERR_SNAPPY_OUTPUT_OVERFLOW;
        const uint64_t badm = __ballot(tv && (m_nei || m_err != 0));
        uint32_t nv = T;  // tags that execute
        const uint32_t Wnext = uni(W + exitrel);
        if (badm) {
            const uint32_t fb = (uint32_t)(__ffsll((long long)badm) - 1);
            nv = fb;
            const int32_t e = __builtin_amdgcn_readlane(m_err, (int)fb);
            const uint32_t fpos = uni((uint32_t)__builtin_amdgcn_readlane((int)pos, (int)fb));
            if (e != 0) {
                st = e;
                consumed = W + uni((uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)fpos));
            } else {
                consumed = W + fpos + 1;  // NOT_ENOUGH_INPUT: tag byte consumed, operands left unread
            }
            stop = true;
        } else {
            consumed = Wnext < in_len ? Wnext : in_len;
        }
        const bool mine = (uint32_t)lane < nv && m_olen > 0;  // an output-producing tag
        const uint64_t outm = __ballot(mine);
        const uint32_t ntags = (uint32_t)__popcll(outm);
        uint32_t E = O;
        if (ntags) {
            E = uni((uint32_t)__builtin_amdgcn_readlane((int)(ostart + mylen), (int)(nv - 1)));
            if (mine) {
                const uint32_t idx = (uint32_t)__popcll(outm & ((1ull << lane) - 1ull));
                Tag tg;
                tg.start = ostart;
                tg.x = m_copy ? (0x80000000u | m_x) : m_x;
                L.tags[idx] = tg;
            }
        }
        // ---------------- expand [O, E) 64 bytes at a time
        if (ntags) {
            int32_t jcur = -1;
            const uint32_t s_lo = sbase;  // stage window [sbase, sbase + kStage) in aligned coordinates
            const uint8_t* lds_bytes = L.ring;  // ring at [0, kRing), stage at [kRing, kRing + kStage)
            for (uint32_t S = O & ~63u; S < E && !trip; S += 64) {
                if (lane == 0) L.bmask = 0ull;
                if (mine && ostart >= S && ostart < S + 64u) atomicOr(&L.bmask, 1ull << (ostart - S));
                const uint64_t B = L.bmask;
                const uint32_t Blo = uni((uint32_t)B), Bhi = uni((uint32_t)(B >> 32));
                const uint32_t pp = S + lane;
                const bool act = pp >= O && pp < E;
                // tag covering byte pp = (number of tag starts <= pp) - 1
                const uint32_t below = __builtin_amdgcn_mbcnt_hi(Bhi, __builtin_amdgcn_mbcnt_lo(Blo, 0u));
                const uint32_t own = (uint32_t)((lane < 32 ? (Blo >> lane) : (Bhi >> (lane - 32))) & 1u);
                const int32_t idx = jcur + (int32_t)(below + own);
                jcur += (int32_t)(__builtin_popcount(Blo) + __builtin_popcount(Bhi));
                const uint32_t Oeff = S > O ? S : O;
                uint32_t v = 0;
                bool res = true;
                uint32_t sl = 0;
                if (act) {
                    const Tag tg = L.tags[idx];
                    const bool lit = (tg.x & 0x80000000u) == 0u;
                    const uint32_t xo = tg.x & 0x7FFFFFFFu;
                    const uint32_t pos = xo + (pp - tg.start);  // literal: input position
                    const uint32_t pa = pos + a;
                    const uint32_t q = pp - xo;                   // copy: source output position
                    const bool lit_stage = (pa - s_lo) < (uint32_t)kStage;
                    const bool intra = !lit && q >= Oeff;
                    const bool near = !lit && !intra && q + (uint32_t)kRing >= Oeff;
                    // one LDS byte read serves literals in the stage and copies in the history ring
                    const uint32_t loff = lit ? ((uint32_t)kRing + (pa & (kStage - 1))) : (q & (kRing - 1));
                    v = lds_bytes[loff];
                    const bool needg = lit ? !lit_stage : (!intra && !near);
                    if (needg) {  // rare: literal beyond the stage / far copy (global, not flat)
                        const uint8_t* gp = lit ? src + pos : dst + q;
                        v = *(const __attribute__((address_space(1))) uint8_t*)(gp);
                    }
                    res = !intra;
                    sl = q - S;
                }
                // overlapping copies inside this 64-byte group: pointer jumping, one ds_bpermute per
                // step carrying (value | resolved << 8 | source lane << 16)
                if (__any(!res)) {
                    uint32_t word = (v & 0xFFu) | (res ? 0x100u : 0u) | ((sl & 63u) << 16);
                    for (int guard = 0; __any(!res); ++guard) {
                        if (guard > 8) {
                            st = kGuardTrip + 2;
                            stop = trip = true;
                            break;
                        }
                        const uint32_t g = (uint32_t)__shfl((int)word, (int)sl);
                        if (!res) {
                            if (g & 0x100u) {
                                v = g & 0xFFu;
                                res = true;
                            } else {
                                sl = (g >> 16) & 63u;
                            }
                            word = (v & 0xFFu) | (res ? 0x100u : 0u) | (sl << 16);
                        }
                    }
                }
                if (act) L.ring[pp & (kRing - 1)] = (uint8_t)v;
                const uint32_t front = (S + 64u < E) ? S + 64u : E;
                while (front >= flushed + (uint32_t)kFB) {
                    // Far reads target q < Oeff - 4096, i.e. blocks at least two flushes older than the
                    // newest; vmcnt counts in issue order, so vmcnt(1) retires every store but (at most)
                    // the newest vector-memory op (the previous flush or the input prefetch).
                    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                    const uint2 d = *reinterpret_cast<const uint2*>(&L.ring[(flushed + 8u * lane) & (kRing - 1)]);
                    uint8_t* o = dst + flushed + 8u * lane;
                    if (dst8) {
                        *reinterpret_cast<uint2*>(o) = d;
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) o[i] = (uint8_t)((i < 4 ? d.x : d.y) >> (8 * (i & 3)));
                    }
                    if (do_crc) acc = shift_byte_tab(sSH, acc) ^ raw8(sT, d.x, d.y);
                    flushed += (uint32_t)kFB;
                }
            }
        }
        O = E;
        W = Wnext;
    }

    // ---- tail: store the last partial block, finish the CRC
    uint32_t crc = 0;
    const uint32_t rem = O - flushed;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    {
        const uint32_t b0 = 8u * lane;
        const uint32_t end = b0 + 8u < rem ? b0 + 8u : rem;
        uint32_t c = 0;
        for (uint32_t i = b0; i < end; ++i) {
            const uint8_t by = L.ring[(flushed + i) & (kRing - 1)];
            dst[flushed + i] = by;
            c = (c >> 8) ^ sT[(c ^ by) & 0xFFu];
        }
        if (do_crc) {
            // full blocks: total = XOR_l acc_l * x^(8*8*(63-l)) — 6-level tree with the nibble tables
            uint32_t fa = acc;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const uint32_t other = __shfl_xor(fa, 1 << j);
                const bool is_lo = ((lane >> j) & 1) == 0;
                fa = shift_nib_tab(sNS + j * 128, is_lo ? fa : other) ^ (is_lo ? other : fa);
            }
            // tail bytes: per-lane raw CRC shifted by the bytes after its slot
            const uint32_t after = end > b0 ? rem - end : 0u;
            c = end > b0 ? gf_multmodp(gf_x8n(after), c) : 0u;
#pragma unroll
            for (int j = 0; j < 6; ++j) c ^= __shfl_xor(c, 1 << j);
            // raw(M) = fold(full) * x^(8*rem) ^ raw(tail); crc = ~(~0 * x^(8|M|) ^ raw(M))
            const uint32_t raw = gf_multmodp(gf_x8n(rem), fa) ^ c;
            crc = ~(gf_multmodp(gf_x8n(O), 0xFFFFFFFFu) ^ raw);
        }
    }
    if (lane == 0) {
        const uint32_t m = mask_checksum(crc);
        if (st == NX_OK && check && m != expect) st = NX_ERR_SNAPPY_CRC_MISMATCH;
        *out_len_p = O;
        if (consumed_p) *consumed_p = consumed;
        *status_p = st;
        if (crc_p) *crc_p = m;
    }
}

__global__ void __launch_bounds__(kWaves * 64, 6) k_snappy_decode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                               const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                               const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                                                               uint32_t* __restrict__ out_len, uint32_t* __restrict__ consumed,
                                                               int32_t* __restrict__ status, const uint32_t* __restrict__ expect,
                                                               uint32_t* __restrict__ crc_out, uint32_t n,
                                                               const CrcTables* __restrict__ tabs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* sT = reinterpret_cast<uint32_t*>(smem);  // T8[0..3]
    uint32_t* sSH = sT + 4 * 256;                      // SH[5] = shift by 512 B
    uint32_t* sNS = sSH + 4 * 256;                     // NS[0..5]
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    if (do_crc) {
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) sSH[i] = (&tabs->SH[5][0][0])[i];
        for (int i = threadIdx.x; i < 6 * 128; i += blockDim.x) sNS[i] = (&tabs->NS[0][0][0])[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    WaveLds& L = *reinterpret_cast<WaveLds*>(smem + kTabBytes + wave * sizeof(WaveLds));
    // static wave -> frame assignment, neighbouring waves on neighbouring frames
    const uint32_t nw = gridDim.x * kWaves;
    for (uint32_t c = blockIdx.x * kWaves + (uint32_t)wave; c < n; c += nw) {
        Frame f{in + in_off[c], in_len[c], out + out_off[c], out_cap ? out_cap[c] : 65536u};
        decode_frame(L, f, sT, sSH, sNS, do_crc, expect ? expect[c] : 0u, expect != nullptr, &out_len[c],
                     consumed ? &consumed[c] : nullptr, &status[c], crc_out ? &crc_out[c] : nullptr, lane);
    }
}

}  // namespace dec
}  // namespace nx

extern "C" int32_t nx_snappy_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                          const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                                          uint32_t* consumed, int32_t* status, const uint32_t* expected_masked_crc,
                                          uint32_t* crc_out, uint32_t n, void* stream) {
    using namespace nx::dec;
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    if (nx::crc_tables_init() != NX_OK) return NX_ERR_HIP;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t lds = kTabBytes + kWaves * sizeof(WaveLds);
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [&] {
        attr_err = hipFuncSetAttribute((const void*)k_snappy_decode, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    NX_HIP_CHECK(attr_err);
    unsigned blocks_per_cu = (unsigned)(160 * 1024 / lds);
    if (blocks_per_cu < 1) blocks_per_cu = 1;
    const uint64_t want = (uint64_t)cus * blocks_per_cu;
    const uint64_t need = (n + kWaves - 1) / kWaves;
    const unsigned grid = (unsigned)(need < want ? need : want);
    hipLaunchKernelGGL(k_snappy_decode, dim3(grid), dim3(kWaves * 64), lds, (hipStream_t)stream, in, in_off, in_len, out, out_off,
                       out_cap, out_len, consumed, status, expected_masked_crc, crc_out, n, nx::crc_tables_dev());
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
