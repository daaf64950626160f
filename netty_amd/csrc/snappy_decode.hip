// snappy_decode.hip — Snappy block decoder + fused CRC32C verify (gfx950).
//
// Replaces Snappy.decode (Snappy.java:315-650) as SnappyFrameDecoder drives it for one complete
// COMPRESSED_DATA chunk (SnappyFrameDecoder.java:194-224), fused with Snappy.validateChecksum
// (Snappy.java:700-707) over the produced bytes.  Bit-exact, including the reference's silent
// partial output on truncated input and its error precedence (offset 0 / negative / beyond,
// output overflow, invalid literal length, preamble > 4 bytes).
//
// Two kernels per sub-batch of frames:
//
//   k_parse  — one LANE per frame runs Snappy.decode's tag state machine (all of Java's checks,
//              in stream order) without touching output bytes.  It emits one 32-bit RECORD per
//              output-producing tag (literals longer than 64 bytes are split into 64-byte records):
//                  bit 31 copy | bits 30..25 length-1 | bits 24..0 input position (literal) or offset (copy)
//              into a per-frame slot of kRecCap records, and the frame's out_len / consumed /
//              status.  A tag costs ~30 lane instructions, i.e. half a wave instruction per tag
//              with 64 frames per wave — the serial part of decoding is paid once per frame, not
//              once per lane of a cooperating wave.
//   k_expand — one WAVE per frame executes the records, 64 at a time, with the output history in
//              LDS and coalesced HBM stores:
//     pieces — the batch's output is cut into PIECES: the intersection of a record with an aligned
//              output dword.  A pass gives one piece to each lane; the piece's record comes from a
//              piece-start bitmask (mbcnt + max-scan), its 1-4 bytes from one unaligned 4-byte read
//              of the input stage (literal), the ring (copy <= 4 KiB back) or HBM (older output of
//              this frame, already flushed and drained), and it is written with one ds_mskor.
//     rounds — a copy whose source bytes are produced in the same pass waits until the pieces
//              producing them (found through a per-pass byte -> piece map) are done; overlapping
//              copies (offset < length) replicate their period.
//     flush  — each completed 512 B block leaves the ring with one 8-byte store per lane; each
//              lane folds its 8 bytes into a per-lane CRC accumulator (slicing-by-4, then "shift by
//              512 B"), and the 64 accumulators are combined once per frame (GF(2) shift tree), so
//              the verify costs neither an HBM pass nor a per-block reduction.
//
// Frames whose records do not fit the slot (or whose input is >= 32 MiB) are marked by k_parse and
// decoded by k_decode_fused, the single-kernel form in which the wave also parses: lane l decodes
// "a tag at W+l" of a 64-byte window speculatively, pointer doubling finds the real tag chain,
// and the same piece expansion runs on the window's tags.
//
// HBM traffic per frame = compressed bytes read twice (parse, literal stage) + records written and
// read once (4 B per tag) + output written once (+ far-copy re-reads, mostly served from MALL).
#include <stddef.h>
#include <stdlib.h>
#include <type_traits>
#include <string.h>
#include <algorithm>
#include <map>
#include <mutex>
#include "nx_common.hpp"
#include "workspace.hpp"
#include "records.hpp"

namespace nx {
namespace dec {

constexpr int kWaves = 12;        // waves per workgroup (2 workgroups per CU → 24 waves/CU)
#ifndef NX_RING  // decoded-output history per wave, bytes (a power of two, >= 2048: far reads stay two flushes back)
#define NX_RING 2048  // (round 6: 4096 -> 2048 makes room for 32 k_expand waves per CU, below)
#endif
constexpr int kRing = NX_RING;     // decoded-output history per wave
static_assert((kRing & (kRing - 1)) == 0 && kRing >= 2048, "ring");
constexpr int kStage = 1024;      // compressed-input ring per wave
constexpr int kFB = 512;          // flush block (64 lanes x 8 B)
constexpr int32_t kGuardTrip = -99;
constexpr uint32_t kRecCap = 16384;      // records per frame slot (64 KiB)
constexpr int32_t kNeedFused = -1000;    // internal status: the frame goes to k_decode_fused
constexpr uint32_t kSubBatch = NX_DEC_MAX_FRAMES;  // frames per parse/expand launch pair (262 144: 16 GiB of record slots)
constexpr uint32_t kFusedMaxFrames = 32768;  // batches up to this size decode on k_decode_fused alone
constexpr int kDecodeAuto = 0, kDecodeFused = 1, kDecodePair = 2;  // decode_batch modes

// CRC tables staged in LDS per workgroup: slicing-by-4 (4 KiB) and shift-by-512 B (4 KiB).  The
// nibble tables of the once-per-frame fold are read from global memory.
constexpr int kTabWords = 4 * 256 + 4 * 256;
constexpr int kTabBytes = kTabWords * 4;

struct WaveLds {
    uint32_t ring[kRing / 4];    // dword 0 .. 1023
    // tag records {start (absolute output position), x (bit31 = copy; low 31 bits = literal source
    // position or copy offset)}; the start of record r+1 is the end of record r (sentinel after the last)
    uint32_t tagw[2 * 64 + 2];
    uint32_t scratch[65];        // parse: tag-start marks; expand: first-piece marks (+ a spare slot), then byte -> piece map
    uint32_t pad[1];
    uint32_t stage[kStage / 4];  // last: a kernel without the stage allocates offsetof(WaveLds, stage) per wave
};
constexpr uint32_t kStageDw = offsetof(WaveLds, stage) / 4;
static_assert(sizeof(WaveLds) % 16 == 0 && offsetof(WaveLds, stage) % 16 == 0, "keep per-wave LDS 16-byte aligned");
static_assert(2 * (kTabBytes + kWaves * sizeof(WaveLds)) <= 160 * 1024, "two workgroups per CU");

// k_expand's shape (round 4, `scripts/ab_dec.sh`, one box, ms per 262 144 frames incl. k_parse):
// * no compressed-input stage: literal pieces read the chunk from HBM like far copies (they are
//   issued with them, before the producer map); the stage's block loads and their waits cost more
//   than they saved: 12 waves/WG x 2, staged 53.8 -> unstaged 50.5;
// * 8 waves per workgroup, three workgroups per CU (24 waves, 6 per SIMD): 49.8.  Time follows the
//   busiest SIMD: 6+6+6+6 waves beat 8+8+4+4 (6-wave WGs x 4: 60.8), 4+4+3+3 x 2 (14-wave WGs:
//   59.2), 8 per SIMD (16-wave WGs without CRC tables: 59.1) and 4 per SIMD (8 x 2: 55.9);
// * the CRC32C stays fused: a separate verify pass over the output was slower (56.5 vs 50.5);
// * one piece per lane: 128-piece passes with two pieces per lane (halving the passes and their
//   scalar control) were bit-exact but slower, 56.7 vs 49.9: the kernel is issue-bound (PMC: each
//   wave issues 36 % of its cycles, stalls on issue 27 %), and the longer dependency chains of
//   128-piece passes cost more rounds than the shared control saved.
// Round 6 (`profiles/r06/s16`, three alternations on one box, ms of k_expand per 262 144 frames): more
// waves per SIMD pay once the round loop is short.  Residency was capped at 6 per SIMD twice over: by
// SGPRs (106 per wave: floor(800 / (112 + 16)) = 6) and by LDS (4 KiB ring per wave).  A 2 KiB ring
// alone (more far copies, same waves) 35.69 -> 35.97; with 4-wave workgroups, 7 per CU (94 SGPRs, 28
// waves) 35.28; 8 per CU (the launch bounds hold SGPRs to 78, the rest spilled to VGPR lanes; 32
// waves, 8 per SIMD) **34.79**, and the FastLZ / LZ4 decoders 5-6.5 % faster.  Shipped: 2 KiB ring,
// 4-wave workgroups, 8 per CU.
// NX_EXPAND_STAGE=1 / NX_EXPAND_WAVES=n / NX_EXPAND_MINB=n / NX_EXPAND_NUM_SGPR=n rebuild the alternatives for A/B runs.
#ifndef NX_EXPAND_STAGE
#define NX_EXPAND_STAGE 0
#endif
constexpr bool kExpandStaged = NX_EXPAND_STAGE != 0;
constexpr size_t kExpandWaveLds = kExpandStaged ? sizeof(WaveLds) : offsetof(WaveLds, stage);
#ifndef NX_EXPAND_WAVES
#define NX_EXPAND_WAVES (NX_EXPAND_STAGE ? 12 : 4)
#endif
constexpr int kExpandWaves = NX_EXPAND_WAVES;
#ifndef NX_EXPAND_MINB  // launch bounds: workgroups per CU the register budget must allow (8 x 4 waves: 78 SGPRs)
#define NX_EXPAND_MINB (NX_EXPAND_STAGE ? 3 : 8)
#endif
static_assert(kTabBytes + kExpandWaves * kExpandWaveLds <= 160 * 1024 / NX_EXPAND_MINB, "k_expand workgroups per CU");

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1))) const u32u gu32u;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gv4u;

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

// Per-frame state of a decoding wave: the compressed-input stage, the output ring and its flush
// to HBM with the per-lane CRC accumulators.
struct FrameIO {
    WaveLds& L;
    const uint8_t* __restrict__ src;
    uint8_t* __restrict__ dst;
    const uint32_t* __restrict__ sT;
    const uint32_t* __restrict__ sSH;
    uint32_t in_len;
    uint32_t a;        // src & 7: position p of the chunk is stage coordinate p + a
    uint32_t aend;
    uint32_t sbase;    // stage holds stage coordinates [sbase, sbase + kStage)
    uint2 pf;          // register prefetch of the next 512 B stage block
    uint32_t flushed;  // output bytes stored to HBM
    uint32_t acc;      // this lane's CRC accumulator over its 8-byte slot of every flushed block
    bool dst8, do_crc;
    int lane;

    __device__ __forceinline__ FrameIO(WaveLds& L_, const Frame& f, const uint32_t* T, const uint32_t* SH, bool crc, int ln)
        : L(L_), src(f.src), dst(f.dst), sT(T), sSH(SH), in_len(uni(f.in_len)), sbase(0), pf(make_uint2(0, 0)), flushed(0),
          acc(0), do_crc(crc), lane(ln) {
        a = (uint32_t)((uintptr_t)src & 7u);
        aend = a + in_len;
        dst8 = (((uintptr_t)dst) & 7u) == 0;
    }
    __device__ __forceinline__ uint2 load8(uint32_t apos) const {
        return apos < aend ? *reinterpret_cast<const uint2*>(src - a + apos) : make_uint2(0, 0);
    }
    __device__ __forceinline__ void put8(uint32_t apos, uint2 v) {
        *reinterpret_cast<uint2*>(&reinterpret_cast<uint8_t*>(L.stage)[apos & (kStage - 1)]) = v;
    }
    __device__ __forceinline__ void prime(uint32_t wa) {
        sbase = wa & ~511u;
        put8(sbase + 8u * lane, load8(sbase + 8u * lane));
        put8(sbase + 512u + 8u * lane, load8(sbase + 512u + 8u * lane));
        pf = load8(sbase + 1024u + 8u * lane);
    }
    // make stage coordinate wa (monotone over calls) the start of the staged range
    __device__ __forceinline__ void advance(uint32_t wa) {
        while (wa >= sbase + 512u) {
            if (wa >= sbase + 1536u) {
                prime(wa);
                break;
            }
            put8(sbase + 1024u + 8u * lane, pf);
            sbase += 512u;
            pf = load8(sbase + 1024u + 8u * lane);
        }
    }
    // flush every complete 512 B block that ends at or below `limit`
    __device__ __forceinline__ void flush_to(uint32_t limit) {
        const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);
        while (flushed + (uint32_t)kFB <= limit) {
            wave_sync();
            // Far reads target q + 4 <= flushed - 1024, i.e. blocks at least two flushes older than
            // the newest; vmcnt counts in issue order, so vmcnt(1) retires every store but (at
            // most) the newest vector-memory op.
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            const uint2 d = *reinterpret_cast<const uint2*>(&ring8[(flushed + 8u * lane) & (kRing - 1)]);
            uint8_t* o = dst + flushed + 8u * lane;
            if (dst8) {
                *reinterpret_cast<uint2*>(o) = d;
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) o[i] = (uint8_t)((i < 4 ? d.x : d.y) >> (8 * (i & 3)));
            }
            // output bytes 0..3 enter the CRC XORed with 0xFF: the ~0 initial state folded into the data
            if (do_crc) acc = shift_byte_tab(sSH, acc) ^ raw8(sT, (flushed == 0u && lane == 0) ? ~d.x : d.x, d.y);
            flushed += (uint32_t)kFB;
        }
    }
    // Store what is left in the ring and return the CRC32C of output bytes [0, O).  The ~0 initial
    // state is folded into the data (output bytes 0..3 enter the CRC XORed with 0xFF), so the CRC is
    // ~raw(M) with raw the state-0 CRC, and no x^(8n) product is needed: raw(M) = shift(raw(flushed
    // blocks), tail) ^ raw(tail), the flushed blocks folded from the 64 lane accumulators (XOR_l acc_l *
    // x^(8*8*(63-l))), the tail's whole 8-byte slots right-aligned in lanes 64-k..63 (leading zero
    // slots add nothing to a state-0 CRC) and folded the same way, its last partial slot byte by byte.
    // A frame shorter than 8 bytes is CRCed byte by byte from ~0.
    __device__ uint32_t finish(uint32_t O, const uint32_t* __restrict__ gNS) {
        const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);
        flush_to(O);
        wave_sync();
        const uint32_t rem = O - flushed;  // < kFB
        const uint32_t k = rem >> 3;       // whole 8-byte tail slots
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        {
            const uint32_t b0 = 8u * lane, b1 = b0 + 8u < rem ? b0 + 8u : rem;
            for (uint32_t i = b0; i < b1; ++i) dst[flushed + i] = ring8[(flushed + i) & (kRing - 1)];
        }
        uint32_t crc = 0;
        if (do_crc) {
            auto fold = [&](uint32_t v) {
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const uint32_t other = __shfl_xor(v, 1 << j);
                    const bool is_lo = ((lane >> j) & 1) == 0;
                    v = shift_nib_tab(gNS + j * 128, is_lo ? v : other) ^ (is_lo ? other : v);
                }
                return v;
            };
            uint32_t R = fold(acc);  // raw CRC of the flushed blocks
            uint32_t c2 = 0;
            if ((uint32_t)lane >= 64u - k) {  // tail slot j = lane - (64 - k), right-aligned
                const uint32_t pos = flushed + 8u * ((uint32_t)lane - (64u - k));
                const uint2 d = *reinterpret_cast<const uint2*>(&ring8[pos & (kRing - 1)]);
                c2 = raw8(sT, pos == 0u ? ~d.x : d.x, d.y);
            }
            c2 = fold(c2);
#pragma unroll
            for (int j = 0; j < 6; ++j)  // R * x^(8 * 8k)
                if ((k >> j) & 1u) R = shift_nib_tab(gNS + j * 128, R);
            R ^= c2;
            if (O < 8u) R = 0xFFFFFFFFu;  // short frame: the plain CRC from ~0 (no fold)
            for (uint32_t i = flushed + 8u * k; i < O; ++i) R = (R >> 8) ^ sT[(R ^ ring8[i & (kRing - 1)]) & 0xFFu];
            crc = ~R;
        }
        return crc;
    }
};

// Where k_expand's next record window starts: its first record (relative to this window), the
// pieces of that record already produced, and the record's output start.
struct Window {
    uint32_t rec, pdone, O;
};

// Expand output [O, E) from the producing tags on lanes `prodm` (lane order = stream order):
// tag on lane l starts at output position ostart, xv = bit31 copy | offset, or the literal's input
// position.  Returns false if the round guard tripped (never on valid input: the lowest pending
// piece always has its producers done).
// Pieces [0, P0s) are already produced.  `last`: run to the end, the final pass partial; otherwise
// run only full 64-piece passes and report in *nw where the next window starts (k_expand slides its
// 64-record window there, so no pass is cut short at a window's end; prodm must be a lane prefix).
// `rn` (k_expand): the next window's records, loaded at the window's start; every pass takes delivery
// of them once its rounds are done (see the passes loop).
__device__ bool expand_tags(FrameIO& io, uint32_t lds_base, uint32_t O, uint32_t E, bool prod, uint64_t prodm, uint32_t ostart,
                            uint32_t xv, int lane, uint32_t P0s = 0u, bool last = true, Window* nw = nullptr, uint32_t* rn = nullptr,
                            bool staged = true) {
    WaveLds& L = io.L;
    const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);
    const uint32_t* lds32 = L.ring;  // ring at dwords [0, 1024), stage at [kStageDw, kStageDw + 256)
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(prodm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)prodm, 0u));
    if (prod) *reinterpret_cast<uint2*>(&L.tagw[2 * rank]) = make_uint2(ostart, xv);
    if (lane == 0) L.tagw[2 * (uint32_t)__popcll(prodm)] = E;  // sentinel: end of the last tag
    // first piece of each tag: pieces before it = dwords from floor(O/4) to floor(start/4), plus
    // one for every producing tag after the first that starts inside a dword
    const uint64_t unal = __ballot(prod && (ostart & 3u) != 0u);
    const uint64_t first_bit = prodm & (~prodm + 1ull);
    const uint32_t pbase = (ostart >> 2) - (O >> 2) + (uint32_t)__popcll(unal & lanemask_le(lane) & ~first_bit);
    const uint32_t Ptot = ((E + 3u) >> 2) - (O >> 2) + (uint32_t)__popcll(unal & ~first_bit);
    uint32_t rc = 0;   // rank of the last tag started in an earlier pass
    uint32_t pbc = 0;  // its first piece
    // (a non-last window holds >= 64 unproduced pieces: its first record has one, every other one)
    const uint32_t Pend = last ? Ptot : P0s + ((Ptot - P0s) & ~63u);
    // marks go to scratch[pbase - P0]; a tag whose first piece lies outside the pass writes the spare
    // slot scratch[64] instead, so the store needs no divergent branch
    uint32_t* const marks = L.scratch;
    // The next window's records (*rn) are waited for after the first pass's rounds, where the wait for
    // that pass's far loads (issued after them) has already retired them.  Waited for at the slide
    // instead, they cost a wait for the last pass's flush stores in every window: gfx950's vmcnt
    // retires loads and stores in issue order and the compiler, unable to count the variable number
    // of stores in between, waits for all of them.  The do-while gives every path one such wait, so
    // the compiler sees the value delivered at the slide on all of them.
    uint32_t P0 = P0s;
    if (P0 >= Pend) {
        if (rn) asm volatile("" : "+v"(*rn));
    } else do {
        // piece -> tag: each tag marks its first piece, then a max-scan over the lanes
        L.scratch[lane] = 0u;
        wave_sync();
        {
            const uint32_t rel = pbase - P0;  // wraps for pbase < P0
            const bool in_pass = prod && rel < 64u;
            marks[in_pass ? rel : 64u] = ((rank + 1u) << 6) | (rel & 63u);
        }
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

        // source of the piece's first byte x0
        const bool lit = (tx & 0x80000000u) == 0u;
        const uint32_t xo = tx & 0x7FFFFFFFu;
        const uint32_t tlen = tend - tstart;
        const bool overlap = !lit && xo < tlen;  // copy reads bytes it produces
        const uint32_t pin = xo + (x0 - tstart);  // literal: input position
        // LDS read: dwords lbase + ((sp >> 2) [+1] & lmask); selects, not a divergent branch
        const uint32_t sp = lit ? pin + io.a : x0 - xo;
        const bool gl = lit ? (!staged || (sp - io.sbase) > (uint32_t)(kStage - 8))          // outside the stage: HBM
                            : (!overlap && pe > (uint32_t)kRing && sp < pe - (uint32_t)kRing);  // far copy
        const uint32_t lbase = lit && staged ? kStageDw : 0u;
        const uint32_t lmask = lit && staged ? (uint32_t)(kStage / 4 - 1) : (uint32_t)(kRing / 4 - 1);
        const uint32_t nbytes = x1 - x0;
        const uint32_t sh = 8u * (x0 & 3u);
        const uint32_t bmask = (nbytes >= 4u ? 0xFFFFFFFFu : ((1u << (8u * nbytes)) - 1u)) << sh;
        const uint32_t waddr = lds_base + 4u * ((x0 >> 2) & (kRing / 4 - 1));
        // Sources that do not depend on this pass, loaded first so that their latency overlaps the
        // producer map and the first round: far copies (the frame's own flushed output) and literal
        // bytes outside the stage, from HBM.  A literal piece among the chunk's last 3 bytes reads
        // the chunk's last dword and shifts (chunks under 4 bytes take the byte loop).
        // (gval is used untouched until the first round: any operation on it here, a phi with
        // another path's value included, would make the compiler wait for the load at once.)
        uint32_t gval;       // read only by lanes with gl (a zero store here made the compiler wait for every in-flight load and store)
        uint32_t gsh = 0;    // right shift of gval (a read of the chunk's last dword)
        uint32_t gtiny = 0;  // chunks under 4 bytes: the bytes, read one by one
        const bool gld = valid && gl;
        const bool tiny = io.in_len < 4u;
        if (__ballot(gld)) {
            const bool tail = lit && pin + 4u > io.in_len;
            const uint8_t* ga = !lit ? io.dst + sp : io.src + (tail ? io.in_len - 4u : pin);
            if (gld && !tiny) gval = g_ld32u(ga);
            gsh = tail ? 8u * (pin + 4u - io.in_len) : 0u;
            if (tiny && __ballot(gld)) {
                if (gld) {
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i)
                        if (pin + i < io.in_len) gtiny |= g_ld8(io.src + pin + i) << (8 * i);
                }
            }
        }
        // Producer map: byte x of this pass holds the lane (piece) that writes it.  A copy whose
        // source bytes lie in this pass depends on the contiguous piece range that produces them,
        // and runs in the first round after all of those are done.  The map aliases `scratch`
        // (its piece marks were consumed above).
        // Only a near copy whose source reaches into this pass's output [ps, pe) can depend on it;
        // passes without one (all literals, far or older sources) skip the map and run one round.
        const uint32_t psal = ps & ~3u;
        const uint32_t dhi = overlap ? tstart : sp + nbytes;  // end of the source bytes this piece reads
        const bool dep = valid && !lit && !gl && dhi > ps;
        uint64_t need = 0;
        const uint64_t depm = __ballot(dep);
        if (depm) {
            wave_sync();
            {
                const uint32_t mm = valid ? bmask : 0u;
                const uint32_t maddr = lds_base + (uint32_t)offsetof(WaveLds, scratch) + (valid ? 4u * ((x0 >> 2) - (psal >> 2)) : 0u);
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(maddr), "v"(mm), "v"(((uint32_t)lane * 0x01010101u) & mm) : "memory");
            }
            wave_sync();
            // every lane reads (non-dependent lanes at byte 0) and keeps the result only if dependent
            const uint32_t lo0 = overlap ? tstart - xo : sp;
            const uint8_t* M8 = reinterpret_cast<const uint8_t*>(L.scratch);
            const uint32_t lo = lo0 > ps ? lo0 : ps;
            const uint32_t pa = M8[dep ? lo - psal : 0u], pb = M8[dep ? dhi - 1u - psal : 0u];
            const uint64_t nm = (pb >= 63u ? ~0ull : ((2ull << pb) - 1ull)) & ~((1ull << (pa & 63u)) - 1ull);
            need = dep ? nm : 0ull;
        }
        // Overlapping copies (offset < length): out[x] = out[tstart - xo + ((x - tstart) mod xo)],
        // xo < tlen <= 64; the four ring byte addresses, packed 4 x 12 bits into two dwords
        // (computed by every lane, used by overlapping pieces only).
        const bool has_ov = __ballot(valid && overlap) != 0ull;
        uint32_t ova = 0, ovb = 0;
        if (has_ov) {
            const uint32_t n0 = x0 - tstart;
            const uint32_t inv = (uint32_t)(__builtin_amdgcn_rcpf((float)xo) * 65536.0f) + 1u;  // floor(n0/xo) exact for n0, xo < 64
            const uint32_t m0 = n0 - xo * ((n0 * inv) >> 16);
            const uint32_t q = tstart - xo;
            uint32_t ad[4];
            uint32_t mi = m0;  // (n0 + i) mod xo, stepped: m0 < xo, so one wrap test per byte
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                if (i) mi = mi + 1u == xo ? 0u : mi + 1u;
                ad[i] = (q + mi) & (kRing - 1);
            }
            ova = ad[0] | (ad[1] << 16);
            ovb = ad[2] | (ad[3] << 16);
        }
        // Rounds.  Round 0 writes every piece with no producer in this pass; then a pending piece is
        // ready once none of its producers is pending (every valid piece not pending is written).
        // Round 6 (profiles/r06/s12): from round 1 on, every valid piece whose producers are all written
        // writes again, pending or not (its sources are final, so a piece written in an earlier round
        // writes the same bytes), so the update needs no test of the lane's own pending bit; and the
        // lanes that write are a lane mask in an SGPR pair selecting the write mask (inline v_cndmask)
        // instead of a per-lane bool rebuilt from exec-masked pieces every round.  14 -> 8 VALU and
        // 5 fewer SALU per round; k_expand 36.9 -> 35.1 ms per 262 144 frames.
        const uint32_t w = sp >> 2;
        const uint32_t ra0 = lbase + (w & lmask), ra1 = lbase + ((w + 1u) & lmask);
        uint64_t pending = depm;
        const uint64_t validm = last >= 63u ? ~0ull : ((2ull << last) - 1ull);  // the valid pieces: lanes 0..last
        uint64_t readym = validm & ~depm;  // round 0: every valid piece without a producer in the pass
        for (int round = 0;; ++round) {
            // stage (literal) or ring (near copy): one unaligned 4-byte read, all lanes
            uint32_t lo = lds32[ra0];
            uint32_t hi = lds32[ra1];
            asm volatile("" : "+v"(lo), "+v"(hi));  // read on every lane: no exec-mask branch around the reads
            uint32_t val = gl ? (tiny ? gtiny : gval >> gsh) : __builtin_amdgcn_alignbyte(hi, lo, sp & 3u);
            if (has_ov) {
                const uint32_t ov = (uint32_t)ring8[ova & 0xFFFFu] | ((uint32_t)ring8[ova >> 16] << 8) |
                                    ((uint32_t)ring8[ovb & 0xFFFFu] << 16) | ((uint32_t)ring8[ovb >> 16] << 24);
                val = overlap ? ov : val;
            }
            // one masked atomic write per lane: the piece's bytes, or nothing (mask 0)
            uint32_t m;
            asm volatile("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m) : "v"(bmask), "s"(readym));
            asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(waddr), "v"(m), "v"((val << sh) & m) : "memory");
            if (!pending || round >= 64) break;
            readym = __ballot((need & pending) == 0ull) & validm;  // every producer written (a ballot of the compare itself)
            pending &= ~readym;
        }
        if (pending) return false;  // the round guard tripped
        if (rn) asm volatile("" : "+v"(*rn));
        // Flush at the END of the pass, its bytes final (round 3; was at the start, flush_to(ps)): the
        // flush's stores then precede the next pass's far-copy loads by a pass of work, so the wait
        // for those loads (gfx950's vmcnt also counts older stores) rarely waits on a fresh store.
        // Same blocks, one pass earlier; 58.8 -> 57.9 ms per 262 144 frames with the gval change below.
        io.flush_to(pe);
    } while ((P0 += 64u) < Pend);
    if (!last) {
        if (Pend == Ptot) {  // the window is done: the next starts at its successor
            nw->rec = (uint32_t)__popcll(prodm);
            nw->pdone = 0u;
            nw->O = E;
        } else {  // the record holding piece Pend (the last one starting at or before it)
            const uint32_t idx = (uint32_t)__popcll(__ballot(prod && pbase <= Pend)) - 1u;
            nw->rec = idx;
            nw->pdone = Pend - uni((uint32_t)__builtin_amdgcn_readlane((int)pbase, (int)idx));
            nw->O = uni((uint32_t)__builtin_amdgcn_readlane((int)ostart, (int)idx));
        }
    }
    return true;
}

__device__ __forceinline__ void write_result(int lane, uint32_t crc, int32_t st, bool check, uint32_t expect, uint32_t O,
                                             uint32_t consumed, uint32_t* out_len_p, uint32_t* consumed_p, int32_t* status_p,
                                             uint32_t* crc_p) {
    if (lane == 0) {
        const uint32_t m = mask_checksum(crc);
        if (st == NX_OK && check && m != expect) st = NX_ERR_SNAPPY_CRC_MISMATCH;
        *out_len_p = O;
        if (consumed_p) *consumed_p = consumed;
        *status_p = st;
        if (crc_p) *crc_p = m;
    }
}

// =====================================================================================
// Fused single-kernel form: the wave parses 64-byte windows of the compressed stream itself.
// =====================================================================================
__device__ void decode_frame_fused(WaveLds& L, uint32_t lds_base, const Frame& f, const uint32_t* __restrict__ sT,
                                   const uint32_t* __restrict__ sSH, const uint32_t* __restrict__ gNS, bool do_crc, uint32_t expect,
                                   bool check, uint32_t* out_len_p, uint32_t* consumed_p, int32_t* status_p, uint32_t* crc_p,
                                   int lane) {
    FrameIO io(L, f, sT, sSH, do_crc, lane);
    const uint8_t* __restrict__ src = f.src;
    const uint32_t in_len = io.in_len;
    const uint32_t cap = uni(f.cap < (1u << 24) ? f.cap : (1u << 24));
    int32_t st = NX_OK;
    uint32_t consumed = 0;
    uint32_t O = 0;  // output frontier (bytes final)

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
    if (go) io.prime(W + io.a);

    bool stop = !go;
    uint32_t windows = 0;
    while (!stop && W < in_len) {
        if (++windows > in_len + 2) {
            st = kGuardTrip;
            break;
        }
        io.advance(W + io.a);
        wave_sync();  // stage bytes written by other lanes
        // ---------------- parse: branch-free speculative tag decode at W + lane (bytes from the stage)
        const uint32_t p = W + lane;
        const uint32_t avail = p < in_len ? in_len - p : 0u;
        uint64_t v;
        {
            const uint32_t pa = p + io.a;
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

        // ---------------- tag chain by pointer doubling
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
        const uint32_t exitrel = uni((uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)lastpos));
        L.scratch[lane] = 0;
        wave_sync();
        if (tvm) L.scratch[pos] = 1u;
        wave_sync();
        const bool tv = L.scratch[lane] != 0u;

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
        if (prodm && !expand_tags(io, lds_base, O, E, prod, prodm, ostart, xv, lane)) {
            st = kGuardTrip + 2;
            break;
        }
        O = E;
        W = Wnext;
    }
    const uint32_t crc = io.finish(O, gNS);
    write_result(lane, crc, st, check, expect, O, consumed, out_len_p, consumed_p, status_p, crc_p);
}

// Loads the workgroup's CRC tables into LDS and yields (wave's LDS block, its LDS byte address, wave index).
struct WaveSetup {
    uint32_t* sT;
    uint32_t* sSH;
    WaveLds* L;
    uint32_t lds_base;
    uint32_t wave;
};
__device__ __forceinline__ WaveSetup wave_setup(uint8_t* smem, const CrcTables* __restrict__ tabs, bool do_crc,
                                                size_t wave_lds = sizeof(WaveLds)) {
    WaveSetup s;
    s.sT = reinterpret_cast<uint32_t*>(smem);  // T8[0..3]
    s.sSH = s.sT + 4 * 256;                    // SH[5] = shift by 512 B
    if (do_crc) {
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) s.sT[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) s.sSH[i] = (&tabs->SH[5][0][0])[i];
    }
    __syncthreads();
    // wave index as an SGPR: divergence analysis cannot see that threadIdx.x >> 6 is wave-uniform,
    // and everything derived from it (the frame, its pointers, sizes, positions) would otherwise
    // live in VGPRs with exec-masked control flow
    s.wave = uni(threadIdx.x >> 6);
    s.L = reinterpret_cast<WaveLds*>(smem + kTabBytes + s.wave * wave_lds);
    // LDS byte address of L for the inline-asm atomics: the low 32 bits of a flat pointer into the
    // LDS aperture are the LDS offset
    s.lds_base = (uint32_t)(uintptr_t)s.L;
    return s;
}

// filter: decode only frames whose status holds kNeedFused (the fallback after k_parse)
__global__ void __launch_bounds__(kWaves * 64, 6)
    k_decode_fused(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
                   uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                   uint32_t* __restrict__ out_len, uint32_t* __restrict__ consumed, int32_t* __restrict__ status,
                   const uint32_t* __restrict__ expect, uint32_t* __restrict__ crc_out, uint32_t n, const CrcTables* __restrict__ tabs,
                   int filter, const uint32_t* __restrict__ need) {
    // the fallback launch of a batch in which no frame was handed over returns at once (need: the
    // batch's flag, set by whichever kernel marked a frame kNeedFused)
    if (filter && need && __builtin_nontemporal_load(need) == 0u) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    const WaveSetup s = wave_setup(smem, tabs, do_crc);
    const int lane = threadIdx.x & 63;
    // static wave -> frame assignment, neighbouring waves on neighbouring frames
    const uint32_t nw = gridDim.x * kWaves;
    for (uint32_t c = blockIdx.x * kWaves + s.wave; c < n; c += nw) {
        if (filter && uni((uint32_t)status[c]) != (uint32_t)kNeedFused) continue;
        Frame f{in + in_off[c], in_len[c], out + out_off[c], out_cap ? out_cap[c] : 65536u};
        decode_frame_fused(*s.L, s.lds_base, f, s.sT, s.sSH, &tabs->NS[0][0][0], do_crc, expect ? expect[c] : 0u, expect != nullptr,
                           &out_len[c], consumed ? &consumed[c] : nullptr, &status[c], crc_out ? &crc_out[c] : nullptr, lane);
    }
}

// =====================================================================================
// k_parse: one lane per frame — Snappy.decode's state machine (Snappy.java:315-393) emitting records
// =====================================================================================

// Burst window: 64 bytes of the lane's compressed stream staged in LDS (17-dword lane stride:
// conflict-free across the wave).  The parse runs in bursts: every lane whose next tag header is
// not in its window reloads it (four 16-byte aligned loads; a 16-byte block holding at least one
// byte of the chunk never crosses a page, blocks wholly past the end are not loaded), the wave
// waits once, then each lane parses tags until its window runs out.  One memory latency per ~20
// tags instead of one per tag for whichever lane happens to cross a block.
#ifndef NX_PARSE_BLOCK  // lanes per k_parse workgroup (build option: 128 fits a block beside three k_expand workgroups)
#define NX_PARSE_BLOCK 256
#endif
constexpr int kParseBlock = NX_PARSE_BLOCK;
constexpr int kWinDw = 17;
// (Round 4: a register prefetch of the following window at each reload measured 1.5 % slower end to
// end, 54.7 vs 53.9 ms per 262 144 frames on one box, and was removed.)
template <uint32_t NB>  // window of NB 16-byte blocks; LDS stride 4 * NB + 1 dwords (conflict-free)
struct BurstWinT {
    static constexpr uint32_t kBytes = 16u * NB;
    static constexpr int kStride = 4 * (int)NB + 1;
    const uint8_t* origin;  // chunk start rounded down to 16 bytes
    uint32_t pad, end;      // chunk start - origin; chunk end, origin-relative
    uint32_t base;          // window = origin-relative [base, base + kBytes)
    uint32_t* w;            // this lane's LDS window
    __device__ __forceinline__ void init(const uint8_t* in, uint32_t length, uint32_t* lds) {
        origin = reinterpret_cast<const uint8_t*>((uintptr_t)in & ~(uintptr_t)15);
        pad = (uint32_t)((uintptr_t)in & 15u);
        end = pad + length;
        base = 0xFFFFFF00u;
        w = lds;
    }
    // are the (up to) 5 header bytes at chunk position p in the window?
    __device__ __forceinline__ bool has(uint32_t p) const {
        const uint32_t q = p + pad;
        // bitwise, not short-circuit: one compare chain instead of nested exec-mask regions
        return (q >= base) & ((q + 5u <= base + kBytes) | (base + kBytes >= end));
    }
    // (called with p inside the chunk, so end >= 1).  Every block is loaded, those wholly past the
    // end from the last block that holds a chunk byte instead (their bytes are unspecified), so the
    // NB loads issue back to back and the lane waits once; a guarded load per block made the
    // compiler wait after each one (NB memory latencies per burst).
    __device__ __forceinline__ void load(uint32_t p) {
        base = (p + pad) & ~15u;
        const uint32_t last = (end - 1u) & ~15u;
        v4u x[NB];
#pragma unroll
        for (uint32_t k = 0; k < NB; ++k) {
            const uint32_t o = base + 16u * k;
            x[k] = *(const gv4u*)(origin + (o <= last ? o : last));
        }
#pragma unroll
        for (uint32_t k = 0; k < NB; ++k) {
            w[4 * k] = x[k].x;
            w[4 * k + 1] = x[k].y;
            w[4 * k + 2] = x[k].z;
            w[4 * k + 3] = x[k].w;
        }
    }
    // 8 bytes at chunk position p, has(p) (bytes at or past the chunk end are unspecified)
    __device__ __forceinline__ uint64_t get8(uint32_t p) const {
        const uint32_t off = p + pad - base;
        const uint32_t i = off >> 2, s = off & 3u;
        const uint32_t d0 = w[i], d1 = w[i + 1], d2 = w[i + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
    }
};
using BurstWin = BurstWinT<4>;
static_assert(BurstWin::kStride == kWinDw, "k_parse window stride");

// Line window (NX_PARSE_LINE): the 128-byte line holding the lane's next tag header plus the 16 bytes
// before it, [B - 16, B + 128) with B a multiple of 128 (origin-relative).  Streaming forward, a reload
// keeps the previous window's last 16 bytes (an LDS move, not a load) and reads exactly one new line,
// so each line of the chunk is fetched once; the 64-byte burst window above re-reads the line it sits
// in at every reload (3.1x read amplification in round 4's PMC).  Twice the bytes per reload, half
// the reloads.
struct BurstWinLine {
    static constexpr int kStride = 37;
    const uint8_t* origin;
    uint32_t pad, end;
    uint32_t lb;  // B: the window is origin-relative [B - 16, B + 128), w[0..3] holding [B - 16, B)
    uint32_t* w;
    __device__ __forceinline__ void init(const uint8_t* in, uint32_t length, uint32_t* lds) {
        origin = reinterpret_cast<const uint8_t*>((uintptr_t)in & ~(uintptr_t)15);
        pad = (uint32_t)((uintptr_t)in & 15u);
        end = pad + length;
        lb = 0xFFFFFF00u;
        w = lds;
    }
    __device__ __forceinline__ bool has(uint32_t p) const {
        const uint32_t q = p + pad;
        return q + 16u >= lb && (q + 5u <= lb + 128u || lb + 128u >= end);
    }
    __device__ __forceinline__ void load(uint32_t p) {
        const uint32_t B = (p + pad + 16u) & ~127u;
        const uint32_t last = (end - 1u) & ~15u;
        const bool carry = B != 0u && lb + 128u == B;  // streaming on: the carry block is in LDS
        v4u x[9];
#pragma unroll
        for (uint32_t k = 1; k < 9; ++k) {
            const uint32_t o = B + 16u * (k - 1u);
            x[k] = *(const gv4u*)(origin + (o <= last ? o : last));
        }
        if (carry) {
            x[0].x = w[32];
            x[0].y = w[33];
            x[0].z = w[34];
            x[0].w = w[35];
        } else if (B != 0u) {
            x[0] = *(const gv4u*)(origin + (B - 16u <= last ? B - 16u : last));
        } else {  // B = 0: nothing precedes the chunk (p >= 0 = B, so these bytes are never read)
            x[0] = v4u{0u, 0u, 0u, 0u};
        }
        lb = B;
#pragma unroll
        for (uint32_t k = 0; k < 9; ++k) {
            w[4 * k] = x[k].x;
            w[4 * k + 1] = x[k].y;
            w[4 * k + 2] = x[k].z;
            w[4 * k + 3] = x[k].w;
        }
    }
    __device__ __forceinline__ uint64_t get8(uint32_t p) const {
        const uint32_t off = p + pad + 16u - lb;
        const uint32_t i = off >> 2, s = off & 3u;
        const uint32_t d0 = w[i], d1 = w[i + 1], d2 = w[i + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
    }
};
#ifndef NX_PARSE_LINE
#define NX_PARSE_LINE 0
#endif
#ifndef NX_PARSE_DEFER
#define NX_PARSE_DEFER 0
#endif
#ifndef NX_PARSE_RELOAD_K  // 0: reload when every running lane is out of window (rounds 2-5)
#define NX_PARSE_RELOAD_K 16
#endif


// Record writer: a lane's records gather QR at a time in its LDS queue row and leave as one run of
// QR/4 back-to-back 16-byte stores (QR = 16: a 64-byte half-line the L2 merges) instead of scattered
// partial-line writes.  The row is LDS, not registers: a register queue needs a 16-way select per
// record (32 VALU: v_cmp + v_cndmask per entry), an LDS row one ds_write.  Rows of QR = 16 are
// 16-byte aligned (stride 20 dwords); smaller rows take an odd stride (QR + 1: conflict-free writes)
// and are read back dword by dword.  DEFER: the full row is read into registers at its last record
// and stored at the next put (or at finish), so the lane does not wait on those LDS reads alone: the
// next window read's wait covers them (LDS returns in order).
template <uint32_t QR, bool DEFER = false>
struct RecWriterT {
    static_assert(QR == 4 || QR == 8 || QR == 16, "record row");
    static constexpr uint32_t kStride = QR == 16 ? 20u : QR + 1u;
    static constexpr uint32_t kV = QR / 4;  // 16-byte stores per row
    uint4* slot;
    uint32_t* q;  // this lane's LDS row
    uint32_t n;   // records emitted
    v4u p0, p1, p2, p3;  // DEFER: the row being flushed (native vectors: uint4 members went to scratch)
    uint32_t pend_at;    // DEFER: its first record index, all ones when none
    __device__ __forceinline__ RecWriterT(uint4* s, uint32_t* row) : slot(s), q(row), n(0), pend_at(0xFFFFFFFFu) {}
    __device__ __forceinline__ v4u row(uint32_t k) const {
        if constexpr (QR == 16) {
            return reinterpret_cast<const v4u*>(q)[k];
        } else {
            return v4u{q[4 * k], q[4 * k + 1], q[4 * k + 2], q[4 * k + 3]};
        }
    }
    __device__ __forceinline__ void drain() {
        if constexpr (DEFER) {
            if (pend_at != 0xFFFFFFFFu) {
                v4u* d = reinterpret_cast<v4u*>(slot + (pend_at >> 2));
                d[0] = p0;
                if constexpr (kV > 1) d[1] = p1;
                if constexpr (kV > 2) {
                    d[2] = p2;
                    d[3] = p3;
                }
                pend_at = 0xFFFFFFFFu;
            }
        }
    }
    __device__ __forceinline__ bool put(uint32_t r) {
        if constexpr (!DEFER) {  // the row write needs no exec region: a lane at capacity writes its own row
            const bool ok = n < kRecCap;
            q[n & (QR - 1u)] = r;
            if (ok & ((n & (QR - 1u)) == QR - 1u)) {
                v4u* d = reinterpret_cast<v4u*>(slot + ((n - (QR - 1u)) >> 2));
#pragma unroll
                for (uint32_t k = 0; k < kV; ++k) d[k] = row(k);
            }
            n += ok ? 1u : 0u;
            return ok;
        }
        if (n >= kRecCap) return false;
        drain();
        q[n & (QR - 1u)] = r;
        if ((n & (QR - 1u)) == QR - 1u) {
            if constexpr (DEFER) {
                p0 = row(0);
                if constexpr (kV > 1) p1 = row(1);
                if constexpr (kV > 2) {
                    p2 = row(2);
                    p3 = row(3);
                }
                pend_at = n - (QR - 1u);
            } else {
                v4u* d = reinterpret_cast<v4u*>(slot + ((n - (QR - 1u)) >> 2));
#pragma unroll
                for (uint32_t k = 0; k < kV; ++k) d[k] = row(k);
            }
        }
        ++n;
        return true;
    }
    __device__ __forceinline__ void finish() {
        drain();
        const uint32_t k = n & (QR - 1u);
        if (k) {
            v4u* d = reinterpret_cast<v4u*>(slot + ((n - k) >> 2));
#pragma unroll
            for (uint32_t j = 0; j < kV; ++j)
                if (4u * j < k) d[j] = row(j);
        }
    }
};
using RecWriter = RecWriterT<16>;
constexpr int kQDw = (int)RecWriter::kStride;
#ifndef NX_PARSE_QR
#define NX_PARSE_QR 16
#endif
#ifndef NX_PARSE_NB
#define NX_PARSE_NB 4
#endif
// k_parse's window and record row (build options; the alt-codec parses keep BurstWin and RecWriter)
using ParseRec = RecWriterT<NX_PARSE_QR, NX_PARSE_DEFER != 0>;
using ParseBurst = BurstWinT<NX_PARSE_NB>;
using ParseWin = std::conditional_t<NX_PARSE_LINE != 0, BurstWinLine, ParseBurst>;

// The wave's steps between burst reloads: every lane whose window holds its next header takes a step,
// until no lane's does, or (K > 0) as soon as K running lanes wait for a reload, so that lanes idle
// less between reloads (those whose window still holds their next header keep it and go on after the
// reload).  `step` clears `run` when its lane stops.
template <int K, class Has, class Step>
__device__ __forceinline__ void burst_steps(const bool& run, Has has, Step step) {
    if constexpr (K > 0) {
        for (;;) {
            const bool act = run & has();
            if (!__any(act) || __popcll(__ballot(run & !act)) >= K) break;
            if (act) step();
        }
    } else {
        while (run & has()) step();
    }
}
#ifndef NX_ALT_RELOAD_K  // the FastLZ / LZF parses: the all-lanes rule measured best (round 5 s27)
#define NX_ALT_RELOAD_K 0
#endif

__global__ void __launch_bounds__(kParseBlock) k_parse(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                       const uint32_t* __restrict__ in_len_a, const uint32_t* __restrict__ out_cap,
                                                       uint32_t* __restrict__ rec, uint32_t* __restrict__ nrec,
                                                       uint32_t* __restrict__ out_len, uint32_t* __restrict__ consumed_a,
                                                       int32_t* __restrict__ status, uint32_t n, uint32_t* __restrict__ need_fused) {
    __shared__ uint32_t wins[kParseBlock * ParseWin::kStride + 4];
    __shared__ __attribute__((aligned(16))) uint32_t recq[kParseBlock * ParseRec::kStride];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t in_len = in_len_a[c];
    uint32_t cap = out_cap ? out_cap[c] : 65536u;
    cap = cap < (1u << 24) ? cap : (1u << 24);
    if (in_len >= (1u << 25)) {  // literal positions need 25 bits
        status[c] = kNeedFused;
        if (need_fused) *need_fused = 1u;
        return;
    }
    ParseWin win;
    win.init(in + in_off[c], in_len, &wins[threadIdx.x * ParseWin::kStride]);
    ParseRec rw(reinterpret_cast<uint4*>(rec + (size_t)c * kRecCap), &recq[threadIdx.x * ParseRec::kStride]);
    uint32_t ip = 0, op = 0;
    int32_t st = NX_OK;
    bool run = false;
    // ---- preamble (readPreamble, :404-420): at most 4 bytes
    if (in_len > 0) {
        win.load(0);
        const uint64_t v = win.get8(0);
        uint32_t ulen = 0;
        int bi = 0;
        bool complete = false;
        while (ip < in_len) {
            const uint32_t cur = (uint32_t)(v >> (8 * ip)) & 0xFFu;
            ++ip;
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
            if (ulen > cap) st = NX_ERR_SNAPPY_OUTPUT_OVERFLOW; else run = true;
        }
    }
    // ---- tags (:328-392, decodeLiteral :454-494, decodeCopyWith*ByteOffset :509-626, validateOffset :637-650)
    // one tag at ip (in the window), branch-free: both interpretations are computed and selected by the type
    auto step = [&]() {
        const uint64_t v = win.get8(ip);
        const uint32_t tag = (uint32_t)v & 0xFFu;
        const uint32_t ops = (uint32_t)(v >> 8);  // operand bytes (valid where < in_len)
        const uint32_t after_tag = ip + 1u;
        const uint32_t avail = in_len - after_tag;
        const uint32_t type = tag & 3u;
        const bool isl = type == 0u;
        const uint32_t code = tag >> 2;
        // literal (decodeLiteral): nb length bytes after the tag, Java int length + 1
        const uint32_t nb = (isl && code >= 60u) ? code - 59u : 0u;
        const uint32_t fmask = nb >= 4u ? 0xFFFFFFFFu : ((1u << (8u * nb)) - 1u);
        const uint32_t lj = nb == 0u ? code + 1u : (ops & fmask) + 1u;
        // copy (decodeCopyWith{1,2,4}ByteOffset)
        const uint32_t csize = type == 1u ? 1u : (type == 2u ? 2u : 4u);
        const uint32_t clen = type == 1u ? 4u + (code & 7u) : 1u + code;
        const uint32_t coff = type == 1u ? (((tag & 0xe0u) << 3) | (ops & 0xFFu)) : (type == 2u ? (ops & 0xFFFFu) : ops);
        const uint32_t hdr = isl ? nb : csize;
        const uint32_t dpos = after_tag + hdr;
        const bool lneg = isl && (int32_t)lj < 0;
        // NOT_ENOUGH_INPUT (silent stop, the tag byte consumed): operands, or the literal's bytes
        const bool nei = avail < hdr || (isl && !lneg && in_len - dpos < lj);
        const uint32_t len = isl ? lj : clen;
        // any error: a negative literal length; an offset of zero, negative or beyond the output
        // (coff - 1 >= op covers all three: op <= cap < 2^31); the output limit (op <= cap: no wrap)
        const bool bad = (uint32_t)(isl ? lneg : coff - 1u >= op) | (uint32_t)(len > cap - op);  // (no short circuit: selects)
        if (nei | bad) {  // rare: the frame stops here, with Java's check order for the error code
            const int32_t cerr = coff == 0u ? NX_ERR_SNAPPY_OFFSET_ZERO
                                            : ((int32_t)coff < 0 ? NX_ERR_SNAPPY_OFFSET_NEGATIVE : (coff > op ? NX_ERR_SNAPPY_OFFSET_BEYOND : 0));
            const int32_t terr = isl ? (lneg ? NX_ERR_SNAPPY_LITERAL_LEN_INVALID : 0) : cerr;
            ip = nei ? after_tag : dpos;
            st = nei ? NX_OK : (terr != 0 ? terr : NX_ERR_SNAPPY_OUTPUT_OVERFLOW);
            run = false;
            return;
        }
        const uint32_t m0 = lj < 64u ? lj : 64u;
        const uint32_t r = isl ? (((m0 - 1u) << 25) | dpos) : (0x80000000u | ((clen - 1u) << 25) | coff);
        bool fit = (isl && lj == 0u) || rw.put(r);  // a zero-length literal (field 0xFFFFFFFF) emits nothing
        if (isl && lj > 64u) {  // literals longer than 64 bytes: one record per 64 bytes
            for (uint32_t k = 64u; k < lj && fit; k += 64u) {
                const uint32_t m = lj - k < 64u ? lj - k : 64u;
                fit = rw.put(((m - 1u) << 25) | (dpos + k));
            }
        }
        if (!fit) {
            st = kNeedFused;
            run = false;
            return;
        }
        ip = dpos + (isl ? lj : 0u);
        op += len;
        run = ip < in_len;
    };
    for (;;) {
        run = run && ip < in_len;
        if (!__any(run)) break;
        if (run && !win.has(ip)) win.load(ip);  // burst reload: one wait for the whole wave
        burst_steps<NX_PARSE_RELOAD_K>(run, [&] { return win.has(ip); }, step);
    }
    if (st == kNeedFused) {
        status[c] = kNeedFused;
        if (need_fused) *need_fused = 1u;
        return;
    }
    rw.finish();
    nrec[c] = rw.n;
    out_len[c] = op;
    if (consumed_a) consumed_a[c] = ip;
    status[c] = st;
}

// =====================================================================================
// k_expand: one wave per frame executes the frame's records
// =====================================================================================
#ifdef NX_EXPAND_NUM_SGPR  // an explicit SGPR budget (residency: floor(800 / (ceil(sgprs / 16) * 16 + 16)) waves per SIMD)
#define NX_EXPAND_SGPR_ATTR __attribute__((amdgpu_num_sgpr(NX_EXPAND_NUM_SGPR)))
#else
#define NX_EXPAND_SGPR_ATTR
#endif
__global__ void __launch_bounds__(kExpandWaves * 64, NX_EXPAND_MINB) NX_EXPAND_SGPR_ATTR
    k_expand(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
             uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ rec,
             const uint32_t* __restrict__ nrec, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
             const uint32_t* __restrict__ expect, uint32_t* __restrict__ crc_out, uint32_t n, const CrcTables* __restrict__ tabs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    const WaveSetup s = wave_setup(smem, tabs, do_crc, kExpandWaveLds);
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * kExpandWaves;
    for (uint32_t c = blockIdx.x * kExpandWaves + s.wave; c < n; c += nw) {
        int32_t st = (int32_t)uni((uint32_t)status[c]);
        if (st == kNeedFused) continue;
        const uint32_t N = uni(nrec[c]);
        const uint32_t Ofin = uni(out_len[c]);
        Frame f{in + in_off[c], in_len[c], out + out_off[c], 0u};
        FrameIO io(*s.L, f, s.sT, s.sSH, do_crc, lane);
        const uint32_t* __restrict__ R = rec + (size_t)c * kRecCap;
        // A window of 64 records [b, b + 64) whose first `pdone` pieces are produced; it runs full
        // 64-piece passes only, then slides to the record holding the first piece left (round 3: the
        // window's last pass was ~85 % full on average; 456 -> ~370 passes per text frame).
        uint32_t O = 0;  // output start of record b
        uint32_t pdone = 0;
        bool primed = false;
        uint32_t r = (uint32_t)lane < N ? R[lane] : 0u;
        asm volatile("" : "+v"(r));  // delivered here: at the window loop's head r then never waits on vmcnt (see expand_tags)
        for (uint32_t b = 0; b < N;) {
            const bool valid = b + (uint32_t)lane < N;
            const bool isc = (r >> 31) != 0u;
            const uint32_t len = valid ? ((r >> 25) & 63u) + 1u : 0u;
            // Issue the next window's prefetch only after this window's records are in use: vmcnt counts
            // in order, so a wait for `r` placed after the new load also waited for the new load
            // (a memory latency per window; 57.8 -> 57.0 ms per 262 144 frames).
            asm volatile("" ::"v"(len) : "memory");
            uint32_t rnext = b + 64u + (uint32_t)lane < N ? R[b + 64u + lane] : 0u;  // records [b + 64, b + 128)
            const uint32_t x = r & 0x1FFFFFFu;
            const uint32_t incl = incl_scan(len);
            const uint32_t ostart = O + incl - len;
            const uint32_t E = O + uni((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
            // the stage follows the first literal of the batch (literal positions are monotone)
            const uint64_t litm = kExpandStaged ? __ballot(valid && !isc) : 0ull;
            if (litm) {
                const uint32_t w = uni((uint32_t)__builtin_amdgcn_readlane((int)x, __ffsll((long long)litm) - 1));
                if (!primed) {
                    io.prime(w + io.a);
                    primed = true;
                } else {
                    io.advance(w + io.a);
                }
                wave_sync();  // stage bytes written by other lanes
            }
            const uint32_t xv = isc ? (0x80000000u | x) : x;
            const bool last = b + 64u >= N;
            Window nw{0u, 0u, 0u};
            if (!expand_tags(io, s.lds_base, O, E, valid, __ballot(valid), ostart, xv, lane, pdone, last, &nw, &rnext, kExpandStaged)) {
                st = kGuardTrip + 2;
                break;
            }
            if (last) {
                O = E;
                break;
            }
            // slide: the new window's lane l takes record b + nw.rec + l, from this window or the prefetch
            const uint32_t src = (uint32_t)lane + nw.rec;
            const uint32_t from_r = (uint32_t)__shfl((int)r, (int)(src & 63u));
            const uint32_t from_n = (uint32_t)__shfl((int)rnext, (int)(src & 63u));
            r = src < 64u ? from_r : from_n;
            b += nw.rec;
            pdone = nw.pdone;
            O = nw.O;
        }
        if (st == kGuardTrip + 2) O = Ofin;  // unreachable on a consistent record stream
        const uint32_t crc = io.finish(O, &tabs->NS[0][0][0]);
        write_result(lane, crc, st, expect != nullptr, expect ? expect[c] : 0u, O, 0u, &out_len[c], nullptr, &status[c],
                     crc_out ? &crc_out[c] : nullptr);
    }
}




// =====================================================================================
// LZ4 blocks through the same record expander
// =====================================================================================
// The LZ4 block format (lz4-java 1.8.0 as Lz4FrameDecoder.java:203-208 drives it: the decompressor
// must produce exactly decompressedLength bytes): sequences of token | literal-length extension |
// literals | 2-byte LE offset | match-length extension (+4); the last sequence is literals only.
// k_parse_lz4 walks a block per lane and emits the same 32-bit records as k_parse (literal runs and
// matches split at 64 bytes: a match's bytes repeat at its distance, so the split is exact); k_expand
// produces the bytes.  Checks (each NX_ERR_LZ4_MALFORMED, oracle/netty_oracle.c orc_lz4_decompress):
// reading past the block, an offset of 0 or beyond the bytes produced, output past want, and a block
// that ends with the output short of want.

// A copy of `len` bytes at distance `dist` splits into 64-byte records exactly (its bytes repeat at
// the distance); a literal run of FastLZ / LZF is at most 32 bytes, one record.
__device__ __forceinline__ bool put_copy(RecWriter& rw, uint32_t len, uint32_t dist) {
    bool fit = true;
    for (uint32_t k = 0; k < len && fit; k += 64u) {
        const uint32_t m = len - k < 64u ? len - k : 64u;
        fit = rw.put(0x80000000u | ((m - 1u) << 25) | dist);
    }
    return fit;
}

template <class Win>
__device__ __forceinline__ uint32_t win_byte(Win& win, uint32_t p) {
    if (!win.has(p)) win.load(p);
    return (uint32_t)win.get8(p) & 0xFFu;
}

// One lane per block, byte at a time through the lane's LDS window (win_byte).  A burst form (one
// header per step from an 8-byte view, wave-wide reloads, as k_parse) measured slower on configs[3]'s
// mixed blocks: 35.5 vs 21.1 ms per 262 144 blocks (half of them random: one 64 KiB literal run).
__global__ void __launch_bounds__(kParseBlock) k_parse_lz4(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                           const uint32_t* __restrict__ in_len_a, const uint32_t* __restrict__ want_a,
                                                           uint32_t* __restrict__ rec, uint32_t* __restrict__ nrec,
                                                           uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t n) {
    __shared__ uint32_t wins[kParseBlock * kWinDw + 4];
    __shared__ __attribute__((aligned(16))) uint32_t recq[kParseBlock * kQDw];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t in_len = in_len_a[c];
    const uint32_t want = want_a[c];
    // literal positions need 25 bits; blocks of more than 64 KiB output (Lz4FrameEncoder block sizes
    // above the default, :158-166) go to the lane-serial kernel, which has no window limit
    if (in_len >= (1u << 25) || want > 65536u) {
        status[c] = kNeedFused;
        return;
    }
    BurstWin win;
    win.init(in + in_off[c], in_len, &wins[threadIdx.x * kWinDw]);
    RecWriter rw(reinterpret_cast<uint4*>(rec + (size_t)c * kRecCap), &recq[threadIdx.x * kQDw]);
    uint32_t ip = 0, op = 0;
    int32_t st = NX_OK;
    bool fit = true;
    for (;;) {
        if (ip >= in_len) {  // a block ends after a literal run, never before a token
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        const uint32_t token = win_byte(win, ip++);
        uint32_t lit = token >> 4;
        if (lit == 15u) {
            uint32_t b = 255u;
            while (b == 255u && ip < in_len) {
                b = win_byte(win, ip++);
                lit += b;  // < 15 + 255 * 2^25: no wrap
            }
            if (b == 255u) {
                st = NX_ERR_LZ4_MALFORMED;
                break;
            }
        }
        if (lit > in_len - ip || lit > want - op) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        for (uint32_t k = 0; k < lit && fit; k += 64u) {
            const uint32_t m = lit - k < 64u ? lit - k : 64u;
            fit = rw.put(((m - 1u) << 25) | (ip + k));
        }
        if (!fit) break;
        ip += lit;
        op += lit;
        if (ip == in_len) break;  // the last sequence
        if (in_len - ip < 2u) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        const uint32_t off = win_byte(win, ip) | (win_byte(win, ip + 1u) << 8);
        ip += 2u;
        if (off == 0u || off > op) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        uint32_t ml = token & 15u;
        if (ml == 15u) {
            uint32_t b = 255u;
            while (b == 255u && ip < in_len) {
                b = win_byte(win, ip++);
                ml += b;
            }
            if (b == 255u) {
                st = NX_ERR_LZ4_MALFORMED;
                break;
            }
        }
        ml += 4u;
        if (ml > want - op) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        for (uint32_t k = 0; k < ml && fit; k += 64u) {
            const uint32_t m = ml - k < 64u ? ml - k : 64u;
            fit = rw.put(0x80000000u | ((m - 1u) << 25) | off);
        }
        if (!fit) break;
        op += ml;
    }
    if (!fit) {
        status[c] = kNeedFused;
        return;
    }
    if (st == NX_OK && op != want) st = NX_ERR_LZ4_MALFORMED;
    rw.finish();
    nrec[c] = rw.n;
    out_len[c] = op;
    status[c] = st;
}

// Blocks k_parse_lz4 could not slot (more than kRecCap records, or >= 32 MiB): one lane decodes the
// block byte by byte, same checks.
__global__ void __launch_bounds__(256) k_lz4_serial(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint32_t* __restrict__ in_len_a, const uint32_t* __restrict__ want_a,
                                                    uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                    int32_t* __restrict__ status, uint32_t n) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n || status[c] != kNeedFused) return;
    const uint8_t* s = in + in_off[c];
    uint8_t* d = out + out_off[c];
    const uint64_t in_len = in_len_a[c], want = want_a[c];
    uint64_t ip = 0, op = 0;
    int32_t st = NX_OK;
    for (;;) {
        if (ip >= in_len) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        const uint32_t token = s[ip++];
        uint64_t lit = token >> 4;
        if (lit == 15u) {
            uint32_t b = 255u;
            while (b == 255u && ip < in_len) {
                b = s[ip++];
                lit += b;
            }
            if (b == 255u) {
                st = NX_ERR_LZ4_MALFORMED;
                break;
            }
        }
        if (lit > in_len - ip || lit > want - op) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        for (uint64_t k = 0; k < lit; ++k) d[op + k] = s[ip + k];
        ip += lit;
        op += lit;
        if (ip == in_len) break;
        if (in_len - ip < 2u) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        const uint64_t off = (uint64_t)s[ip] | ((uint64_t)s[ip + 1] << 8);
        ip += 2;
        if (off == 0u || off > op) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        uint64_t ml = token & 15u;
        if (ml == 15u) {
            uint32_t b = 255u;
            while (b == 255u && ip < in_len) {
                b = s[ip++];
                ml += b;
            }
            if (b == 255u) {
                st = NX_ERR_LZ4_MALFORMED;
                break;
            }
        }
        ml += 4u;
        if (ml > want - op) {
            st = NX_ERR_LZ4_MALFORMED;
            break;
        }
        for (uint64_t k = 0; k < ml; ++k) d[op + k] = d[op + k - off];
        op += ml;
    }
    if (st == NX_OK && op != want) st = NX_ERR_LZ4_MALFORMED;
    status[c] = st;
}

// =====================================================================================
// FastLZ and LZF blocks through the same record expander (configs[3]; records.hpp)
// =====================================================================================

#ifndef FLZ_WIN_BLOCKS
#define FLZ_WIN_BLOCKS 4
#endif
// FastLz.decompress (FastLz.java:409-543; the lane-serial form is fastlz.hip decompress()).  Block
// byte 0 carries the level (bits 7..5) and the first literal-run control (bits 4..0); then runs of
// ctrl+1 literal bytes (ctrl < 32) and back-references of (ctrl >> 5) + 2 (+ extension bytes) bytes
// at distance ((ctrl & 31) << 8) + code + 1, level 2 with a 16-bit far distance (+ MAX_DISTANCE)
// after a 255 code.  Every check of the Java method that can fail sends the block to the serial path
// (kNeedSerial), as does any read at or past in_len (Java reads those through the array's readable
// bytes, fastlz.hip FIN).
//
// Burst form, as k_parse: the lanes whose next control byte is not in their LDS window reload it
// together (one wait for the wave), then each lane decodes tokens from an 8-byte register view of
// its window until it runs out.  A token's header is at most 5 bytes (control, length extension,
// code, two far-distance bytes), inside what BurstWin::has guarantees; only a level-2 length
// extension that continues past a 255 byte takes the byte-at-a-time slow path.
__global__ void __launch_bounds__(kParseBlock) k_parse_fastlz(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                              const uint32_t* __restrict__ in_len_a, const uint32_t* __restrict__ avail_a,
                                                              const uint32_t* __restrict__ lim_a, uint32_t* __restrict__ rec,
                                                              uint32_t* __restrict__ nrec, uint32_t* __restrict__ out_len,
                                                              int32_t* __restrict__ status, uint32_t n) {
    using Win = BurstWinT<FLZ_WIN_BLOCKS>;
    __shared__ uint32_t wins[kParseBlock * Win::kStride + 4];
    __shared__ __attribute__((aligned(16))) uint32_t recq[kParseBlock * kQDw];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t in_len = in_len_a[c];
    const uint32_t lim = lim_a[c];
    // record fields, and a block whose readable bytes end inside it (in_avail): the serial path decides
    if (in_len < 1u || in_len >= (1u << 24) || lim >= (1u << 24) || (avail_a && avail_a[c] < in_len)) {
        status[c] = kNeedSerial;
        return;
    }
    Win win;
    win.init(in + in_off[c], in_len, &wins[threadIdx.x * Win::kStride]);
    RecWriter rw(reinterpret_cast<uint4*>(rec + (size_t)c * kRecCap), &recq[threadIdx.x * kQDw]);
    win.load(0);
    const uint32_t b0 = (uint32_t)win.get8(0) & 0xFFu;
    const uint32_t level = (b0 >> 5) + 1u;  // (in[0] >> 5) + 1 on the signed byte: 5..8 for b0 >= 0x80
    const uint32_t k0 = (b0 & 31u) + 1u;    // the first literal run
    bool ok = (level == 1u || level == 2u) && k0 <= lim && 1u + k0 <= in_len && rw.put(((k0 - 1u) << 25) | 1u);
    uint32_t ip = 1u + k0, op = k0;  // ip: the next control byte
    bool run = ok && ip < in_len;
    for (;;) {
        if (!__any(run)) break;
        if (run && !win.has(ip)) win.load(ip);  // burst reload: one wait for the whole wave
        burst_steps<NX_ALT_RELOAD_K>(run, [&] { return win.has(ip); }, [&] {
            const uint64_t v = win.get8(ip);
            const uint32_t ctrl = (uint32_t)v & 0xFFu;
            uint32_t adv, len, dist;
            bool put_ok;
            if (ctrl < 32u) {  // literal run
                const uint32_t k = ctrl + 1u;
                if (op + k > lim || ip + 1u + k > in_len) {
                    ok = false;
                    run = false;
                    return;
                }
                put_ok = rw.put(((k - 1u) << 25) | (ip + 1u));
                adv = 1u + k;
                len = k;
            } else {
                len = (ctrl >> 5) - 1u;
                const uint32_t ofs = (ctrl & 31u) << 8;
                uint32_t p = 1u;  // header bytes used so far
                if (len == 6u && level == 2u && ((uint32_t)(v >> 8) & 0xFFu) == 255u) {
                    // slow path: a level-2 extension run of 255s (matches of 264+ bytes)
                    uint32_t code = 255u;
                    while (code == 255u) {
                        if (ip + p >= in_len) break;
                        code = win_byte(win, ip + p);
                        ++p;
                        len += code;
                    }
                    if (code == 255u || ip + p + 2u >= in_len + 0u) {
                        // ran off the block (or too close to its end for the code/far bytes): serial
                        ok = false;
                        run = false;
                        return;
                    }
                    const uint32_t cd = win_byte(win, ip + p);
                    ++p;
                    dist = ofs + cd + 1u;
                    if (cd == 255u && ofs == (31u << 8)) {
                        dist = ((win_byte(win, ip + p) << 8) | win_byte(win, ip + p + 1u)) + 8192u;  // + MAX_DISTANCE + 1
                        p += 2u;
                    }
                } else {
                    if (len == 6u) {
                        len += (uint32_t)(v >> 8) & 0xFFu;
                        p = 2u;
                    }
                    const uint32_t code = (uint32_t)(v >> (8u * p)) & 0xFFu;
                    ++p;
                    dist = ofs + code + 1u;
                    if (level == 2u && code == 255u && ofs == (31u << 8)) {
                        const uint32_t hi = (uint32_t)(v >> (8u * p)) & 0xFFu, lo = (uint32_t)(v >> (8u * p + 8u)) & 0xFFu;
                        dist = ((hi << 8) | lo) + 8192u;  // + MAX_DISTANCE + 1
                        p += 2u;
                    }
                }
                // every header byte inside the block; Java: op + len + 3 > outLength -> 0, ref - 1 < 0 -> 0
                if (ip + p > in_len || op + len + 3u > lim || dist > op) {
                    ok = false;
                    run = false;
                    return;
                }
                len += 3u;
                put_ok = put_copy(rw, len, dist);
                adv = p;
            }
            if (!put_ok) {
                ok = false;
                run = false;
                return;
            }
            ip += adv;
            op += len;
            run = ip < in_len;  // Java: a control byte follows while ip < inLength
        });
        if (!ok) run = false;
    }
    if (!ok) {
        status[c] = kNeedSerial;
        return;
    }
    rw.finish();
    nrec[c] = rw.n;
    out_len[c] = op;
    status[c] = NX_OK;
}

#ifndef LZF_WIN_BLOCKS
#define LZF_WIN_BLOCKS 8  // 128-byte windows: 13.3 -> 12.3 ms per 131072 text blocks (literal runs of up to 33 bytes)
#endif
// ChunkDecoder.decodeChunk (compress-lzf 1.0.3, as LzfDecoder.java:205 calls it; lane-serial form:
// lzf.hip decode_chunk): runs of ctrl+1 literal bytes (ctrl < 32) and back-references of
// (ctrl >> 5) + 2 (+ an extension byte when the length field is 7) bytes at distance
// ((ctrl & 31) << 8) + next byte + 1, until exactly lim bytes are produced.  Any corrupt block goes to
// the serial path (kNeedSerial), which reports it.  Burst form as k_parse_fastlz (headers <= 3 bytes).
__global__ void __launch_bounds__(kParseBlock) k_parse_lzf(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                           const uint32_t* __restrict__ in_len_a, const uint32_t* __restrict__ lim_a,
                                                           uint32_t* __restrict__ rec, uint32_t* __restrict__ nrec,
                                                           uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t n) {
    using Win = BurstWinT<LZF_WIN_BLOCKS>;
    __shared__ uint32_t wins[kParseBlock * Win::kStride + 4];
    __shared__ __attribute__((aligned(16))) uint32_t recq[kParseBlock * kQDw];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t in_len = in_len_a[c];
    const uint32_t lim = lim_a[c];
    if (in_len == 0u || lim == 0u || in_len >= (1u << 24) || lim >= (1u << 24)) {  // (lim 0 or no input: always corrupt)
        status[c] = kNeedSerial;
        return;
    }
    Win win;
    win.init(in + in_off[c], in_len, &wins[threadIdx.x * Win::kStride]);
    RecWriter rw(reinterpret_cast<uint4*>(rec + (size_t)c * kRecCap), &recq[threadIdx.x * kQDw]);
    uint32_t ip = 0, op = 0;
    bool ok = true, run = true;  // run: op < lim, and the next control byte at ip < in_len
    for (;;) {
        if (!__any(run)) break;
        if (run && !win.has(ip)) win.load(ip);
        burst_steps<NX_ALT_RELOAD_K>(run, [&] { return win.has(ip); }, [&] {
            const uint64_t v = win.get8(ip);
            const uint32_t ctrl = (uint32_t)v & 0xFFu, b1 = (uint32_t)(v >> 8) & 0xFFu, b2 = (uint32_t)(v >> 16) & 0xFFu;
            const bool lit = ctrl < 32u;
            const bool ext = (ctrl >> 5) == 7u;
            const uint32_t k = ctrl + 1u;
            const uint32_t hdr = lit ? 1u : (ext ? 3u : 2u);
            const uint32_t len = lit ? k : (ctrl >> 5) + (ext ? b1 : 0u) + 2u;
            const uint32_t dist = ((ctrl & 31u) << 8) + (ext ? b2 : b1) + 1u;
            const bool bad = lit ? (ip + 1u + k > in_len || op + k > lim) : (ip + hdr > in_len || dist > op || op + len > lim);
            if (bad || !(lit ? rw.put(((k - 1u) << 25) | (ip + 1u)) : put_copy(rw, len, dist))) {
                ok = false;
                run = false;
                return;
            }
            ip += lit ? 1u + k : hdr;
            op += len;
            run = op < lim;
            if (run && ip >= in_len) ok = false;  // more output wanted, no control byte left
            run = run && ok;
        });
        if (!ok) run = false;
    }
    if (!ok) {
        status[c] = kNeedSerial;
        return;
    }
    rw.finish();
    nrec[c] = rw.n;
    out_len[c] = op;
    status[c] = NX_OK;
}

}  // namespace dec
}  // namespace nx

static_assert(nx::kDecSlotBytes == nx::dec::kRecCap * sizeof(uint32_t) + 2 * sizeof(uint32_t) &&
                  nx::kDecMaxFrames == nx::dec::kSubBatch,
              "record workspace geometry");

// The record slots of the device's shared workspace (workspace.hpp): rec[frames][kRecCap], then the
// record counts and (LZ4) the block lengths produced.
struct DecSlots {
    uint32_t* rec;
    uint32_t* nrec;
    uint32_t* olen;
    uint32_t frames;
};
// slots [first, first + count) of the record workspace (a part lease)
static DecSlots dec_slots(nx::SharedWs& W, size_t first, size_t count) {
    uint32_t* p = static_cast<uint32_t*>(W.p);
    const size_t f = W.slots;
    return {p + first * nx::dec::kRecCap, p + f * nx::dec::kRecCap + first, p + f * nx::dec::kRecCap + f + first, (uint32_t)count};
}

constexpr size_t kExpandLds = nx::dec::kTabBytes + nx::dec::kExpandWaves * nx::dec::kExpandWaveLds;

// Dynamic-LDS limit of the wave kernels, set once per process (`lds`: k_decode_fused's).
static hipError_t wave_kernel_attrs(size_t lds) {
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [&] {
        attr_err = hipFuncSetAttribute((const void*)nx::dec::k_decode_fused, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (attr_err == hipSuccess)
            attr_err = hipFuncSetAttribute((const void*)nx::dec::k_expand, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kExpandLds);
    });
    return attr_err;
}

// one launch of the record expander over m frames
static hipError_t launch_expand(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out, const uint64_t* out_off,
                                const uint32_t* rec, const uint32_t* nrec, uint32_t* out_len, int32_t* status, const uint32_t* expect,
                                uint32_t* crc_out, uint32_t m, int cus, hipStream_t st) {
    using namespace nx::dec;
#ifdef NX_EXPAND_BLOCKS_PER_CU
    const uint64_t per_cu = NX_EXPAND_BLOCKS_PER_CU;
#else
    const uint64_t per_cu = 160 * 1024 / kExpandLds;
#endif
    const uint64_t want = (uint64_t)cus * per_cu, need = (m + kExpandWaves - 1) / kExpandWaves;
    hipLaunchKernelGGL(k_expand, dim3((unsigned)(need < want ? need : want)), dim3(kExpandWaves * 64), kExpandLds, st, in, in_off, in_len,
                       out, out_off, rec, nrec, out_len, status, expect, crc_out, m, nx::crc_tables_dev());
    return hipGetLastError();
}

static int32_t decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out, const uint64_t* out_off,
                            const uint32_t* out_cap, uint32_t* out_len, uint32_t* consumed, int32_t* status,
                            const uint32_t* expected_masked_crc, uint32_t* crc_out, uint32_t n, void* stream, int mode) {
    NX_CLEAR_STALE_ERROR();
    using namespace nx::dec;
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    if (nx::crc_tables_init() != NX_OK) return NX_ERR_HIP;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t lds = kTabBytes + kWaves * sizeof(WaveLds);
    NX_HIP_CHECK(wave_kernel_attrs(lds));
    unsigned blocks_per_cu = (unsigned)(160 * 1024 / lds);
    if (blocks_per_cu < 1) blocks_per_cu = 1;
    const hipStream_t st = (hipStream_t)stream;
    const uint64_t want = (uint64_t)cus * blocks_per_cu;
    auto wave_grid = [&](uint32_t m) {
        const uint64_t need = (m + kWaves - 1) / kWaves;
        return (unsigned)(need < want ? need : want);
    };
    // Batch-size policy (round 5, profiles/r05/s1/dec_latency.log): k_parse walks a frame's tags on
    // one lane, ~4-7 ms for any batch that does not fill the chip, while k_decode_fused parses each
    // frame wave-parallel (0.85 ms for one frame, 1.9 ms for 4 096, 5.6 ms for 16 384, against 4.3 /
    // 7.4 / 9.1 for the pair).  The pair wins from ~34 K frames on (65 536: 16.4 vs 20.5 ms).
    const bool fused_only = mode == kDecodeFused || (mode == kDecodeAuto && n <= kFusedMaxFrames);
    if (fused_only) {
        hipLaunchKernelGGL(k_decode_fused, dim3(wave_grid(n)), dim3(kWaves * 64), lds, st, in, in_off, in_len, out, out_off, out_cap,
                           out_len, consumed, status, expected_masked_crc, crc_out, n, nx::crc_tables_dev(), 0, nullptr);
        NX_HIP_CHECK(hipGetLastError());
        return NX_OK;
    }
    nx::WsLease lease(nx::WsKind::DecRecords, dev, st);
    size_t first = 0, count = 0;
    NX_HIP_CHECK(lease.acquire_part(nx::ws_want(nx::WsKind::DecRecords, n, cus), &first, &count));
    const DecSlots W = dec_slots(lease.ws(), first, count);
    const uint32_t sb = n < W.frames ? n : W.frames;  // a held workspace caps the sub-batch
    for (uint32_t base = 0; base < n; base += sb) {
        const uint32_t m = n - base < sb ? n - base : sb;
        // W.olen[0] (unused by this path): set when any frame of the sub-batch is handed to the fallback
        NX_HIP_CHECK(hipMemsetAsync(W.olen, 0, sizeof(uint32_t), st));
        hipLaunchKernelGGL(k_parse, dim3((m + kParseBlock - 1) / kParseBlock), dim3(kParseBlock), 0, st, in, in_off + base, in_len + base,
                           out_cap ? out_cap + base : nullptr, W.rec, W.nrec, out_len + base, consumed ? consumed + base : nullptr,
                           status + base, m, W.olen);
        NX_HIP_CHECK(hipGetLastError());
        NX_HIP_CHECK(launch_expand(in, in_off + base, in_len + base, out, out_off + base, W.rec, W.nrec, out_len + base, status + base,
                                   expected_masked_crc ? expected_masked_crc + base : nullptr, crc_out ? crc_out + base : nullptr, m,
                                   cus, st));
        // frames k_parse could not slot (more than kRecCap records, or input >= 32 MiB)
        hipLaunchKernelGGL(k_decode_fused, dim3(wave_grid(m)), dim3(kWaves * 64), lds, st, in, in_off + base, in_len + base, out,
                           out_off + base, out_cap ? out_cap + base : nullptr, out_len + base, consumed ? consumed + base : nullptr,
                           status + base, expected_masked_crc ? expected_masked_crc + base : nullptr,
                           crc_out ? crc_out + base : nullptr, m, nx::crc_tables_dev(), 1, W.olen);
        NX_HIP_CHECK(hipGetLastError());
    }
    return NX_OK;
}

extern "C" int32_t nx_snappy_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                          const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                                          uint32_t* consumed, int32_t* status, const uint32_t* expected_masked_crc,
                                          uint32_t* crc_out, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    return decode_batch(in, in_off, in_len, out, out_off, out_cap, out_len, consumed, status, expected_masked_crc, crc_out, n, stream,
                        nx::dec::kDecodeAuto);
}

extern "C" int32_t nx_snappy_decode_batch_fused(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                                const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                                                uint32_t* consumed, int32_t* status, const uint32_t* expected_masked_crc,
                                                uint32_t* crc_out, uint32_t n, void* stream) {
    return decode_batch(in, in_off, in_len, out, out_off, out_cap, out_len, consumed, status, expected_masked_crc, crc_out, n, stream,
                        nx::dec::kDecodeFused);
}

extern "C" int32_t nx_snappy_decode_batch_pair(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                               const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                                               uint32_t* consumed, int32_t* status, const uint32_t* expected_masked_crc,
                                               uint32_t* crc_out, uint32_t n, void* stream) {
    return decode_batch(in, in_off, in_len, out, out_off, out_cap, out_len, consumed, status, expected_masked_crc, crc_out, n, stream,
                        nx::dec::kDecodePair);
}

// Replaces LZ4FastDecompressor.decompress as Lz4FrameDecoder.decode calls it for one
// BLOCK_TYPE_COMPRESSED block (Lz4FrameDecoder.java:199-208): block i = in[in_off[i] .. +in_len[i])
// must decode to exactly out_len[i] bytes at out + out_off[i].
extern "C" int32_t nx_lz4_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                       const uint64_t* out_off, const uint32_t* out_len, int32_t* status, uint32_t n,
                                       void* stream) {
    NX_CLEAR_STALE_ERROR();
    using namespace nx::dec;
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    if (nx::crc_tables_init() != NX_OK) return NX_ERR_HIP;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t lds = kTabBytes + kWaves * sizeof(WaveLds);
    NX_HIP_CHECK(wave_kernel_attrs(lds));
    unsigned blocks_per_cu = (unsigned)(160 * 1024 / lds);
    if (blocks_per_cu < 1) blocks_per_cu = 1;
    const hipStream_t st = (hipStream_t)stream;
    const uint64_t want = (uint64_t)cus * blocks_per_cu;
    nx::WsLease lease(nx::WsKind::DecRecords, dev, st);
    size_t first = 0, count = 0;
    NX_HIP_CHECK(lease.acquire_part(nx::ws_want(nx::WsKind::DecRecords, n, cus), &first, &count));
    const DecSlots Ws = dec_slots(lease.ws(), first, count);
    const DecSlots* W = &Ws;
    const uint32_t sb = n < W->frames ? n : W->frames;
    for (uint32_t base = 0; base < n; base += sb) {
        const uint32_t m = n - base < sb ? n - base : sb;
        const uint64_t need = (m + kWaves - 1) / kWaves;
        hipLaunchKernelGGL(k_parse_lz4, dim3((m + kParseBlock - 1) / kParseBlock), dim3(kParseBlock), 0, st, in, in_off + base,
                           in_len + base, out_len + base, W->rec, W->nrec, W->olen, status + base, m);
        NX_HIP_CHECK(hipGetLastError());
        (void)need;
        (void)want;
        NX_HIP_CHECK(launch_expand(in, in_off + base, in_len + base, out, out_off + base, W->rec, W->nrec, W->olen, status + base, nullptr,
                                   nullptr, m, cus, st));
        hipLaunchKernelGGL(k_lz4_serial, dim3((m + 255) / 256), dim3(256), 0, st, in, in_off + base, in_len + base, out_len + base,
                           out, out_off + base, status + base, m);
        NX_HIP_CHECK(hipGetLastError());
    }
    return NX_OK;
}

// FastLZ / LZF blocks: codec parse -> k_expand -> the codec's finish kernel (records.hpp).
int32_t nx::dec::decode_records(RecCodec codec, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* avail,
                                const uint32_t* lim,
                                uint8_t* out, const uint64_t* out_off, int32_t* status, uint32_t n, hipStream_t st, RecAfter after,
                                void* ctx) {
    NX_CLEAR_STALE_ERROR();
    static_assert(kNeedSerial == kNeedFused, "one marker for the serial fallback");
    if (n == 0) return NX_OK;
    if (nx::crc_tables_init() != NX_OK) return NX_ERR_HIP;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t lds = kTabBytes + kWaves * sizeof(WaveLds);
    NX_HIP_CHECK(wave_kernel_attrs(lds));
    unsigned blocks_per_cu = (unsigned)(160 * 1024 / lds);
    if (blocks_per_cu < 1) blocks_per_cu = 1;
    nx::WsLease lease(nx::WsKind::DecRecords, dev, st);
    size_t first = 0, count = 0;
    NX_HIP_CHECK(lease.acquire_part(nx::ws_want(nx::WsKind::DecRecords, n, cus), &first, &count));
    const DecSlots W = dec_slots(lease.ws(), first, count);
    const uint32_t sb = n < W.frames ? n : W.frames;
    for (uint32_t base = 0; base < n; base += sb) {
        const uint32_t m = n - base < sb ? n - base : sb;
        const dim3 pg((m + kParseBlock - 1) / kParseBlock), pb(kParseBlock);
        if (codec == RecCodec::FastLz)
            hipLaunchKernelGGL(k_parse_fastlz, pg, pb, 0, st, in, in_off + base, in_len + base, avail ? avail + base : nullptr,
                               lim + base, W.rec, W.nrec, W.olen, status + base, m);
        else
            hipLaunchKernelGGL(k_parse_lzf, pg, pb, 0, st, in, in_off + base, in_len + base, lim + base, W.rec, W.nrec, W.olen,
                               status + base, m);
        NX_HIP_CHECK(hipGetLastError());
        NX_HIP_CHECK(launch_expand(in, in_off + base, in_len + base, out, out_off + base, W.rec, W.nrec, W.olen, status + base, nullptr,
                                   nullptr, m, cus, st));
        NX_HIP_CHECK(after(base, m, W.olen, ctx, st));
    }
    return NX_OK;
}
