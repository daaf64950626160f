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
//   ring   — 4 KiB history of the decoded output (copies whose source lies within it are served
//            from LDS);
//   stage  — 1 KiB ring of the compressed stream, refilled 512 B at a time by one 8-byte load per
//            lane that is issued a full half-ring ahead (register prefetch);
//   tags   — the current window's tag records (start, source, length).
// Steps per window (64 bytes of compressed stream that start at a tag):
//   parse   — lane l decodes "a tag at W+l" branch-free from the stage; the real tag chain is a
//             scalar walk (one v_readlane per tag) that yields the tag-start lane mask; lanes keep
//             their tags in place (lane = stream position, so lane order = stream order);
//   order   — output starts by a DPP prefix sum; the Java checks (NOT_ENOUGH_INPUT → silent stop,
//             validateOffset, buffer capacity) run per tag and the first failing tag in stream
//             order decides, exactly as the serial state machine;
//   expand  — the window's output is cut into PIECES: the intersection of a tag with an aligned
//             output dword.  A pass gives one piece to each lane (64 pieces ≈ 200 output bytes):
//             the piece's tag comes from a piece-start bitmask (mbcnt + ffbh), its 1-4 bytes from
//             one unaligned 4-byte read of the stage (literal), the ring (copy ≤ 4 KiB back) or
//             HBM (older output of this frame, already flushed and drained), and it is written
//             with one ds_write_b32 (whole dword) or byte writes (tag boundary inside the dword).
//             Copies that read bytes produced in the same pass wait for a later round: round r
//             runs every piece whose source lies below the first unfinished piece, so the first
//             unfinished piece always runs and most passes finish in one round.  Overlapping
//             copies (offset < length) replicate their period byte-wise;
//   flush   — each completed 512 B block leaves the ring with one 8-byte store per lane; each lane
//             folds its 8 bytes into a per-lane CRC accumulator (slicing-by-4, then "shift by 512 B"),
//             and the 64 accumulators are combined once per frame (GF(2) shift tree), so the verify
//             costs neither an HBM pass nor a per-block reduction.
// HBM traffic per frame = compressed bytes read once + output written once (+ far-copy re-reads,
// mostly served from L2/MALL).
#include <stddef.h>
#include <stdlib.h>
#include <mutex>
#include "nx_common.hpp"

namespace nx {
namespace dec {

constexpr int kWaves = 12;        // waves per workgroup (2 workgroups per CU → 24 waves/CU)
constexpr int kRing = 4096;       // decoded-output history per wave
constexpr int kStage = 1024;      // compressed-input ring per wave
constexpr int kFB = 512;          // flush block (64 lanes x 8 B)
constexpr int32_t kGuardTrip = -99;

// CRC tables staged in LDS per workgroup: slicing-by-4 (4 KiB) and shift-by-512 B (4 KiB).  The
// nibble tables of the once-per-frame fold are read from global memory.
constexpr int kTabWords = 4 * 256 + 4 * 256;
constexpr int kTabBytes = kTabWords * 4;

struct WaveLds {
    uint32_t ring[kRing / 4];    // dword 0 .. 1023
    uint32_t stage[kStage / 4];  // dword 1024 .. 1279
    // tag records {start (absolute output position), x (bit31 = copy; low 31 bits = literal source
    // position or copy offset)}; the start of record r+1 is the end of record r (sentinel after the last)
    uint32_t tagw[2 * 64 + 2];
    uint32_t scratch[64];        // parse: tag-start marks; expand: first-piece marks
    uint32_t pad[2];
};
static_assert(sizeof(WaveLds) % 16 == 0, "keep per-wave LDS 16-byte aligned");
static_assert(2 * (kTabBytes + kWaves * sizeof(WaveLds)) <= 160 * 1024, "two workgroups per CU");

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1))) const u32u gu32u;

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

// Cross-lane hand-off through LDS inside one wave: without it the compiler may forward a lane's
// own earlier store to its later load (single-thread semantics) instead of reading what other
// lanes wrote.  Same pattern as rocPRIM's wave_barrier().
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t lanemask_le(int lane) { return lane == 63 ? ~0ull : ((2ull << lane) - 1ull); }

// Inclusive prefix sum over the 64 lanes (DPP row shifts + row broadcasts; all lanes active).
__device__ __forceinline__ uint32_t incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// Inclusive max-scan over the 64 lanes (same DPP pattern as incl_scan).
__device__ __forceinline__ uint32_t incl_max_scan(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}

__device__ __forceinline__ uint32_t g_ld32u(const uint8_t* p) { return *(gu32u*)(p); }  // unaligned global dword
__device__ __forceinline__ uint32_t g_ld8(const uint8_t* p) { return *(gu8*)(p); }

struct Frame {
    const uint8_t* src;
    uint32_t in_len;
    uint8_t* dst;
    uint32_t cap;
};

template <int MODE>  // experiment bits: 1 = skip expand, 2 = skip rounds, 4 = scalar-walk parse
__device__ void decode_frame(WaveLds& L, uint32_t lds_base, const Frame& f, const uint32_t* __restrict__ sT, const uint32_t* __restrict__ sSH,
                             const uint32_t* __restrict__ gNS, bool do_crc, uint32_t expect, bool check, uint32_t* out_len_p,
                             uint32_t* consumed_p, int32_t* status_p, uint32_t* crc_p, int lane) {
    const uint8_t* __restrict__ src = f.src;
    uint8_t* __restrict__ dst = f.dst;
    const uint32_t in_len = uni(f.in_len);
    const uint32_t cap = uni(f.cap < (1u << 24) ? f.cap : (1u << 24));
    uint8_t* const ring8 = reinterpret_cast<uint8_t*>(L.ring);
    uint32_t* const lds32 = L.ring;  // ring at dwords [0, 1024), stage at [1024, 1280)
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
    uint8_t* const stage8 = reinterpret_cast<uint8_t*>(L.stage);
    auto load8 = [&](uint32_t apos) -> uint2 {
        return apos < aend ? *reinterpret_cast<const uint2*>(asrc + apos) : make_uint2(0, 0);
    };
    auto put8 = [&](uint32_t apos, uint2 v) { *reinterpret_cast<uint2*>(&stage8[apos & (kStage - 1)]) = v; };
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
    // flush every complete 512 B block that ends at or below `limit`
    auto flush_to = [&](uint32_t limit) {
        while (flushed + (uint32_t)kFB <= limit) {
            wave_sync();
            // Far reads (below) target q + 4 <= flushed - 1024, i.e. blocks at least two flushes
            // older than the newest; vmcnt counts in issue order, so vmcnt(1) retires every store
            // but (at most) the newest vector-memory op.
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            const uint2 d = *reinterpret_cast<const uint2*>(&ring8[(flushed + 8u * lane) & (kRing - 1)]);
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
        wave_sync();  // stage bytes written by other lanes
        // ---------------- parse: branch-free speculative tag decode at W + lane (bytes from the stage)
        const uint32_t p = W + lane;
        const uint32_t avail = p < in_len ? in_len - p : 0u;
        uint64_t v;
        {
            const uint32_t pa = p + a;
            const uint32_t w0 = L.stage[(pa >> 2) & (kStage / 4 - 1)];
            const uint32_t w1 = L.stage[((pa >> 2) + 1) & (kStage / 4 - 1)];
            v = (((uint64_t)w1 << 32) | w0) >> (8 * (pa & 3u));
            if (avail < 5) v &= (1ull << (8 * avail)) - 1ull;  // bytes past the input read as 0
        }
        const uint32_t b0 = (uint32_t)v & 0xFFu;
        const uint32_t type = b0 & 3u;
        const uint32_t ops = (uint32_t)(v >> 8);  // operand bytes b1..b4, little-endian
        // literal (decodeLiteral, :454-494)
        const uint32_t code = b0 >> 2;
        const uint32_t nb = code >= 60u ? code - 59u : 0u;
        const uint32_t hdr = 1u + nb;
        const uint32_t field = nb == 0 ? 0u : (nb == 4 ? ops : (ops & ((1u << (8 * nb)) - 1u)));
        const uint32_t lj = nb == 0 ? code + 1u : field + 1u;  // Java int `length + 1` (wraps for nb == 4)
        const bool lneg = nb == 4 && (int32_t)lj < 0;          // IllegalArgumentException (:480-492)
        const bool lhdr_nei = avail < hdr;
        const bool l_nei = lhdr_nei || (!lneg && (avail - hdr) < lj);
        // copies (decodeCopyWith{1,2,4}ByteOffset, :509-626)
        const uint32_t csize = type == 1u ? 2u : (type == 2u ? 3u : 5u);
        const uint32_t colen = type == 1u ? 4u + ((b0 >> 2) & 7u) : 1u + (b0 >> 2);
        const uint32_t coff = type == 1u ? (((b0 & 0xe0u) << 3) | (ops & 0xFFu)) : (type == 2u ? (ops & 0xFFFFu) : ops);
        const bool c_nei = avail < csize;
        const bool is_copy = type != 0u;
        const bool nei = is_copy ? c_nei : l_nei;
        int32_t err = 0;
        if (is_copy) {
            if (!c_nei && coff == 0u) err = NX_ERR_SNAPPY_OFFSET_ZERO;                    // validateOffset (:637-650)
            else if (!c_nei && type == 3u && (int32_t)coff < 0) err = NX_ERR_SNAPPY_OFFSET_NEGATIVE;
        } else if (!lhdr_nei && lneg) {
            err = NX_ERR_SNAPPY_LITERAL_LEN_INVALID;
        }
        uint32_t size;  // bytes of this tag in the stream (saturating)
        uint32_t olen;  // output length (clamped to cap+1)
        if (is_copy) {
            size = csize;
            olen = colen;
        } else {
            const uint64_t sz = (uint64_t)hdr + (lneg ? 0ull : (uint64_t)lj);
            size = sz > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)sz;
            olen = lneg ? 0u : (lj > cap ? cap + 1u : lj);
        }
        const uint32_t xv = is_copy ? (0x80000000u | (coff & 0x7FFFFFFFu)) : ((p + hdr) & 0x7FFFFFFFu);
        const uint32_t nxt = (uint32_t)lane + size;  // relative position of the following tag

        bool tv;
        uint32_t exitrel;
        if (MODE & 4) {
            const uint32_t lim = uni((in_len - W) < 64u ? (in_len - W) : 64u);
            uint64_t tmask = 0;
            uint32_t pos = 0;
            while (pos < lim) {
                tmask |= 1ull << pos;
                pos = uni((uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)pos));
            }
            exitrel = pos;
            tv = ((tmask >> lane) & 1ull) != 0;
        } else {
        // ---------------- tag chain by pointer doubling (no scalar walk)
        // J0[l] = next tag position if a tag starts at l (64 = leaves the window); positions at or
        // past the end of the input are fixed points.  Jk = J0^(2^k); lane m then composes the Jk
        // selected by the bits of m, so lane m ends on the position of the m-th tag.  Those lanes
        // mark their positions in LDS, and every lane reads back whether a tag starts at it: tags
        // stay on their own lanes (lane = stream position).
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
        const bool tvm = pos < lim;  // lane m holds the position of tag m
        const uint32_t T = (uint32_t)__popcll(__ballot(tvm));
        const uint32_t lastpos = uni((uint32_t)__builtin_amdgcn_readlane((int)pos, (int)(T - 1)));
        exitrel = uni((uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)lastpos));
        L.scratch[lane] = 0;
        wave_sync();
        if (tvm) L.scratch[pos] = 1u;
        wave_sync();
        tv = L.scratch[lane] != 0u;
        }

        // ---------------- ordering: bytes written before each tag, per-tag checks (stream order = lane order)
        const uint32_t mylen = tv ? olen : 0u;
        const uint32_t incl = incl_scan(mylen);
        const uint32_t ostart = O + incl - mylen;
        if (tv && is_copy && !nei && err == 0 && (coff & 0x7FFFFFFFu) > ostart) err = NX_ERR_SNAPPY_OFFSET_BEYOND;
        if (tv && !nei && err == 0 && (uint64_t)ostart + olen > cap) err = NX_ERR_SNAPPY_OUTPUT_OVERFLOW;
        const uint64_t badm = __ballot(tv && (nei || err != 0));
        const uint32_t Wnext = uni(W + exitrel);
        uint32_t fb = 64;  // first failing tag (lane); tags on lanes below it execute
        uint32_t E;
        if (badm) {
            fb = (uint32_t)(__ffsll((long long)badm) - 1);
            const int32_t e = __builtin_amdgcn_readlane(err, (int)fb);
            if (e != 0) {
                st = e;
                consumed = W + uni((uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)fb));
            } else {
                consumed = W + fb + 1;  // NOT_ENOUGH_INPUT: tag byte consumed, operands left unread
            }
            stop = true;
            E = uni((uint32_t)__builtin_amdgcn_readlane((int)ostart, (int)fb));
        } else {
            consumed = Wnext < in_len ? Wnext : in_len;
            E = O + uni((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
        }
        const bool prod = tv && (uint32_t)lane < fb && olen > 0;  // an output-producing tag
        const uint64_t prodm = __ballot(prod);

        // ---------------- expand [O, E) in passes of 64 pieces
        if (prodm && !(MODE & 1)) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(prodm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)prodm, 0u));
            if (prod) *reinterpret_cast<uint2*>(&L.tagw[2 * rank]) = make_uint2(ostart, xv);
            if (lane == 0) L.tagw[2 * (uint32_t)__popcll(prodm)] = E;  // sentinel: end of the last tag
            // first piece of each tag: pieces before it = dwords from floor(O/4) to floor(start/4),
            // plus one for every producing tag after the first that starts inside a dword
            const uint64_t unal = __ballot(prod && (ostart & 3u) != 0u);
            const uint64_t first_bit = prodm & (~prodm + 1ull);
            const uint32_t pbase = (ostart >> 2) - (O >> 2) + (uint32_t)__popcll(unal & lanemask_le(lane) & ~first_bit);
            const uint32_t Ptot = ((E + 3u) >> 2) - (O >> 2) + (uint32_t)__popcll(unal & ~first_bit);
            uint32_t rc = 0;   // rank of the last tag started in an earlier pass
            uint32_t pbc = 0;  // its first piece
            for (uint32_t P0 = 0; P0 < Ptot && !trip; P0 += 64u) {
                // piece -> tag: each tag marks its first piece, then a max-scan over the lanes
                L.scratch[lane] = 0u;
                wave_sync();
                if (prod && pbase >= P0 && pbase < P0 + 64u) L.scratch[pbase - P0] = ((rank + 1u) << 6) | (pbase - P0);
                wave_sync();
                const uint32_t mk = incl_max_scan(L.scratch[lane]);
                const uint32_t P = P0 + lane;
                const bool valid = P < Ptot;
                uint32_t r = mk ? (mk >> 6) - 1u : rc;
                const uint32_t k = mk ? (uint32_t)lane - (mk & 63u) : P - pbc;
                r = valid ? r : 0u;
                {
                    const uint32_t mlast = uni((uint32_t)__builtin_amdgcn_readlane((int)mk, 63));
                    if (mlast) {
                        rc = (mlast >> 6) - 1u;
                        pbc = P0 + (mlast & 63u);
                    }
                }
                // record r and the start of record r+1 (= its end)
                const uint32_t tstart = L.tagw[2 * r], tx = L.tagw[2 * r + 1], tend = L.tagw[2 * r + 2];
                const uint32_t A = ((tstart >> 2) + k) << 2;
                const uint32_t x0 = A > tstart ? A : tstart;
                const uint32_t x1 = (A + 4u) < tend ? A + 4u : tend;
                const uint32_t last = (Ptot - P0) < 64u ? (Ptot - P0 - 1u) : 63u;
                const uint32_t ps = uni((uint32_t)__builtin_amdgcn_readlane((int)x0, 0));
                const uint32_t pe = uni((uint32_t)__builtin_amdgcn_readlane((int)x1, (int)last));
                flush_to(ps);
                // source of the piece's first byte x0
                const bool lit = (tx & 0x80000000u) == 0u;
                const uint32_t xo = tx & 0x7FFFFFFFu;
                const uint32_t tlen = tend - tstart;
                const bool overlap = !lit && xo < tlen;  // copy reads bytes it produces
                const uint32_t pin = xo + (x0 - tstart);  // literal: input position
                uint32_t sp, lbase, lmask;  // LDS read: dwords lbase + ((sp >> 2) [+1] & lmask)
                bool gl;
                if (lit) {
                    sp = pin + a;
                    gl = (sp - sbase) > (uint32_t)(kStage - 8);  // beyond the stage: read the input from HBM
                    lbase = kRing / 4;
                    lmask = kStage / 4 - 1;
                } else {
                    sp = x0 - xo;
                    gl = !overlap && pe > (uint32_t)kRing && sp < pe - (uint32_t)kRing;  // far copy
                    lbase = 0;
                    lmask = kRing / 4 - 1;
                }
                const uint32_t nbytes = x1 - x0;
                const uint32_t sh = 8u * (x0 & 3u);
                const uint32_t bmask = (nbytes >= 4u ? 0xFFFFFFFFu : ((1u << (8u * nbytes)) - 1u)) << sh;
                const uint32_t waddr = lds_base + 4u * ((x0 >> 2) & (kRing / 4 - 1));
                uint64_t pending = (MODE & 2) ? 0ull : __ballot(valid);
                for (int round = 0; pending; ++round) {
                    if (round > 64) {
                        st = kGuardTrip + 2;
                        stop = trip = true;
                        break;
                    }
                    const uint32_t j0 = (uint32_t)(__ffsll((long long)pending) - 1);
                    const uint32_t F = uni((uint32_t)__builtin_amdgcn_readlane((int)x0, (int)j0));
                    const bool ready = ((pending >> lane) & 1ull) != 0 &&
                                       (lit || gl || (overlap ? tstart <= F : sp + nbytes <= F));
                    // stage (literal) or ring (near copy): one unaligned 4-byte read, all lanes
                    const uint32_t w = sp >> 2;
                    const uint32_t lo = lds32[lbase + (w & lmask)];
                    const uint32_t hi = lds32[lbase + ((w + 1u) & lmask)];
                    uint32_t val = __builtin_amdgcn_alignbyte(hi, lo, sp & 3u);
                    if (__ballot(ready && gl)) {
                        if (ready && gl) {
                            if (!lit) {
                                val = g_ld32u(dst + sp);  // flushed and drained output of this frame
                            } else if (pin + 4u <= in_len) {
                                val = g_ld32u(src + pin);
                            } else {
                                val = 0;
#pragma unroll
                                for (uint32_t i = 0; i < 4; ++i)
                                    if (pin + i < in_len) val |= g_ld8(src + pin + i) << (8 * i);
                            }
                        }
                    }
                    if (__ballot(ready && overlap)) {
                        if (ready && overlap) {
                            // out[x] = out[tstart - xo + ((x - tstart) mod xo)]; xo < tlen <= 64
                            const uint32_t n0 = x0 - tstart;
                            const uint32_t inv = (uint32_t)(65536.0f / (float)xo) + 1u;
                            const uint32_t m0 = n0 - xo * ((n0 * inv) >> 16);
                            const uint32_t q = tstart - xo;
                            val = 0;
#pragma unroll
                            for (uint32_t i = 0; i < 4; ++i) {
                                uint32_t mi = m0 + i;
                                mi -= mi >= xo ? xo : 0u;
                                mi -= mi >= xo ? xo : 0u;
                                mi -= mi >= xo ? xo : 0u;
                                val |= (uint32_t)ring8[(q + mi) & (kRing - 1)] << (8 * i);
                            }
                        }
                    }
                    // one masked atomic write per lane: the piece's bytes, or nothing (mask 0)
                    const uint32_t m = ready ? bmask : 0u;
                    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(waddr), "v"(m), "v"((val << sh) & m) : "memory");
                    pending &= ~__ballot(ready);
                }
            }
        }
        O = E;
        W = Wnext;
    }

    // ---- tail: store what is left in the ring, finish the CRC
    flush_to(O);
    wave_sync();
    uint32_t crc = 0;
    const uint32_t rem = O - flushed;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    {
        const uint32_t b0 = 8u * lane;
        const uint32_t end = b0 + 8u < rem ? b0 + 8u : rem;
        uint32_t c = 0;
        for (uint32_t i = b0; i < end; ++i) {
            const uint8_t by = ring8[(flushed + i) & (kRing - 1)];
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
                fa = shift_nib_tab(gNS + j * 128, is_lo ? fa : other) ^ (is_lo ? other : fa);
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

template <int MODE>
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
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    if (do_crc) {
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) sSH[i] = (&tabs->SH[5][0][0])[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // wave index as an SGPR: divergence analysis cannot see that threadIdx.x >> 6 is wave-uniform,
    // and everything derived from it (the frame, its pointers, sizes, positions) would otherwise
    // live in VGPRs with exec-masked control flow
    const int wave = (int)uni(threadIdx.x >> 6);
    WaveLds& L = *reinterpret_cast<WaveLds*>(smem + kTabBytes + wave * sizeof(WaveLds));
    // LDS byte address of L for the inline-asm atomics: the low 32 bits of a flat pointer into the
    // LDS aperture are the LDS offset
    const uint32_t lds_base = (uint32_t)(uintptr_t)&L;
    // static wave -> frame assignment, neighbouring waves on neighbouring frames
    const uint32_t nw = gridDim.x * kWaves;
    for (uint32_t c = blockIdx.x * kWaves + (uint32_t)wave; c < n; c += nw) {
        Frame f{in + in_off[c], in_len[c], out + out_off[c], out_cap ? out_cap[c] : 65536u};
        decode_frame<MODE>(L, lds_base, f, sT, sSH, &tabs->NS[0][0][0], do_crc, expect ? expect[c] : 0u, expect != nullptr, &out_len[c],
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
        for (const void* k : {(const void*)k_snappy_decode<0>, (const void*)k_snappy_decode<1>, (const void*)k_snappy_decode<2>,
                              (const void*)k_snappy_decode<4>})
            if (attr_err == hipSuccess) attr_err = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    NX_HIP_CHECK(attr_err);
    unsigned blocks_per_cu = (unsigned)(160 * 1024 / lds);
    if (blocks_per_cu < 1) blocks_per_cu = 1;
    const uint64_t want = (uint64_t)cus * blocks_per_cu;
    const uint64_t need = (n + kWaves - 1) / kWaves;
    const unsigned grid = (unsigned)(need < want ? need : want);
    static const int mode = getenv("NX_DEC_MODE") ? atoi(getenv("NX_DEC_MODE")) : 0;
    auto kern = mode == 1 ? k_snappy_decode<1> : mode == 2 ? k_snappy_decode<2> : mode == 4 ? k_snappy_decode<4> : k_snappy_decode<0>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWaves * 64), lds, (hipStream_t)stream, in, in_off, in_len, out, out_off,
                       out_cap, out_len, consumed, status, expected_masked_crc, crc_out, n, nx::crc_tables_dev());
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
