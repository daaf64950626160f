// expand_units.hpp — k_expand_u, the unit-lane record expander (round 5; included by snappy_decode.hip
// inside namespace nx::dec, after k_expand and its helpers).
//
// Same contract as k_expand (records of k_parse / k_parse_{lz4,fastlz,lzf} → output bytes + fused
// CRC32C), different work mapping.  k_expand cuts the output into ~2.8-byte pieces (record ∩ output
// dword) and places every byte with a ds_mskor after a piece → record map and a producer map, ~370
// instructions per 64-piece pass.  Here a LANE owns an aligned 16-byte output UNIT and
// assembles it in four registers from its SEGMENTS (record ∩ unit, 1-16 per unit, ~3.4 on text):
//   * a segment's 16 source bytes are read ALIGNED TO THE UNIT (source of unit byte j = source of the
//     segment start + j - b0), so a segment costs one 16-byte read and four v_bfi_b32 merges under a
//     byte-range mask, whatever its length;
//   * a copy's source lies in the LDS history ring (one 5-dword read + alignbyte) or, older than the
//     ring, in the frame's flushed output in HBM; a literal's in the compressed chunk in HBM.  HBM
//     sources are one unaligned 16-byte load issued in one round and merged in the next, so the wave
//     never waits on memory inside a round;
//   * readiness is per BYTE: every unit publishes its applied-byte mask (16 bits) beside its bytes at
//     the end of each round; a copy segment runs once the bytes it reads are applied (units below the
//     lowest pending one are final), so chains resolve as soon as their source bytes exist rather
//     than a pass at a time;
//   * the window SLIDES: a lane whose unit is complete takes the next unassigned unit (up to kUxAhead
//     units past the lowest pending one), so no lane idles at a pass boundary.  Each round a lane
//     attempts its kUxK lowest pending segments.
// Model on the bench corpus (scripts/experiments/unit_model.py and the round-5 slide model): ~390
// rounds and ~790 segment attempts per 64 KiB text frame, against k_expand's ~1 030 rounds in 370
// passes.
// Flush: each 1 KiB block below the lowest pending unit leaves the ring as one 16-byte store per lane;
// the lane folds its 16 bytes into a per-lane CRC accumulator (slicing-by-4 x4, then "shift by
// 1 KiB"), the 64 accumulators are combined once per frame (GF(2) shift tree, NS tables).
//
// Bounds: every HBM read lies inside the chunk (literals: the 16 bytes from the unit-aligned source
// start must lie inside in_len, else the segment's bytes are read one by one) or inside the frame's
// flushed output (far copies); no read precedes a chunk's or a frame's first byte.

#ifndef NX_UX_RING
#define NX_UX_RING 4096
#endif
#ifndef NX_UX_WAVES
#define NX_UX_WAVES 6
#endif
#ifndef NX_UX_AHEAD
#define NX_UX_AHEAD 128
#endif
#ifndef NX_UX_K
#define NX_UX_K 2
#endif
constexpr uint32_t kUxRing = NX_UX_RING;     // output history per wave (bytes, power of two)
constexpr uint32_t kUxSlots = kUxRing / 16;  // unit slots in the ring
constexpr uint32_t kUxRR = 256;              // record ring entries (output start, record)
constexpr uint32_t kUxUF = 256;              // unit -> first record ring entries
constexpr uint32_t kUxIn = 32;               // records per intake (<= 2 KiB of output: 16 * kUxUF >= 2 * kUxIn * 64)
static_assert(16u * kUxUF >= 2u * kUxIn * 64u, "an intake fits the unit-first ring beside the unit being assigned");
constexpr uint32_t kUxAhead = NX_UX_AHEAD;   // units assigned past the lowest pending one
constexpr int kUxWaves = NX_UX_WAVES;        // waves (frames in flight) per workgroup
constexpr int kUxK = NX_UX_K;                // segment attempts per lane per round
constexpr uint32_t kUxFB = 1024;             // flush block: 64 lanes x 16 bytes
constexpr uint32_t kUxNone = 0xFFFFFFFFu;
static_assert(kUxSlots >= kUxAhead + kUxFB / 16, "the ring holds the window and a flush block of history");
static_assert(kRecCap <= 65536, "record indices are kept as 16 bits");

struct UxLds {
    uint32_t ring[kUxRing / 4 + 4];  // output history; dwords [kUxRing/4, +4) mirror dwords [0, 4)
    uint2 rr[kUxRR];                 // record ring: (output start, record)
    uint16_t umask[kUxSlots];        // applied-byte mask of the unit in each ring slot
    uint16_t uf[kUxUF];              // first record (the one holding byte 16v) of unit v
    uint32_t litb[kUxRR / 32];       // bit r % 32 of word (r / 32) % 8: record r is a literal
    uint32_t pad2[(16 - (kUxRR / 32) % 16) % 4];
};
static_assert(sizeof(UxLds) % 16 == 0, "keep per-wave LDS 16-byte aligned");
// per workgroup: slicing-by-4 (4 KiB), shift by 1 KiB (4 KiB), byte-range masks lowm[b] (17 x 16 B)
constexpr uint32_t kUxTabBytes = 2 * 4096 + 17 * 16;
constexpr size_t kUxLds = kUxTabBytes + (size_t)kUxWaves * sizeof(UxLds);

typedef v4u __attribute__((aligned(1))) v4uu;  // unaligned 16 bytes (gfx950: one dwordx4 access)
typedef __attribute__((address_space(1))) const v4uu gv4uu;
typedef __attribute__((address_space(1))) v4uu gv4uw;
__device__ __forceinline__ uint4 g_ld16u(const uint8_t* p) {
    const v4u v = *(const gv4uu*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void g_st16u(uint8_t* p, uint4 d) {
    v4u v;
    v.x = d.x;
    v.y = d.y;
    v.z = d.z;
    v.w = d.w;
    *(gv4uw*)p = v;
}

__device__ __forceinline__ uint32_t t4(const uint32_t* __restrict__ T, uint32_t c) {
    return T[3 * 256 + (c & 0xFF)] ^ T[2 * 256 + ((c >> 8) & 0xFF)] ^ T[1 * 256 + ((c >> 16) & 0xFF)] ^ T[c >> 24];
}
// raw CRC (state 0) of 16 bytes (four LE dwords)
__device__ __forceinline__ uint32_t raw16(const uint32_t* __restrict__ T, uint4 d) {
    uint32_t c = t4(T, d.x);
    c = t4(T, c ^ d.y);
    c = t4(T, c ^ d.z);
    return t4(T, c ^ d.w);
}
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
__device__ __forceinline__ uint32_t bits16(uint32_t b0, uint32_t b1) { return ((1u << b1) - 1u) & ~((1u << b0) - 1u); }

// Inclusive min-scan over the 64 lanes (DPP; all lanes active); lane 63 holds the minimum.
__device__ __forceinline__ uint32_t incl_min_scan(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xa, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) { return uni((uint32_t)__builtin_amdgcn_readlane((int)incl_min_scan(v), 63)); }

__global__ void __launch_bounds__(kUxWaves * 64)
    k_expand_u(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
               uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ rec,
               const uint32_t* __restrict__ nrec, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
               const uint32_t* __restrict__ expect, uint32_t* __restrict__ crc_out, uint32_t n, const CrcTables* __restrict__ tabs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    uint32_t* const sT = reinterpret_cast<uint32_t*>(smem);  // T8[0..3]
    uint32_t* const sSH = sT + 1024;                         // SH[6] = shift by 1 KiB
    uint4* const lowm = reinterpret_cast<uint4*>(sT + 2048);  // bytes [0, b) set
    if (do_crc) {
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) sSH[i] = (&tabs->SH[6][0][0])[i];
    }
    for (int i = threadIdx.x; i < 17 * 4; i += blockDim.x) {
        const uint32_t b = (uint32_t)i >> 2, k = (uint32_t)i & 3u;
        reinterpret_cast<uint32_t*>(lowm)[i] = b >= 4u * k + 4u ? 0xFFFFFFFFu : (b <= 4u * k ? 0u : (1u << (8u * (b - 4u * k))) - 1u);
    }
    __syncthreads();
    const uint32_t wave = uni(threadIdx.x >> 6);
    UxLds& L = *reinterpret_cast<UxLds*>(smem + kUxTabBytes + wave * sizeof(UxLds));
    uint8_t* const ring8 = reinterpret_cast<uint8_t*>(L.ring);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t* __restrict__ gNS = &tabs->NS[0][0][0];
    const uint32_t nw = gridDim.x * kUxWaves;
    for (uint32_t c = blockIdx.x * kUxWaves + wave; c < n; c += nw) {
        int32_t st = (int32_t)uni((uint32_t)status[c]);
        if (st == kNeedFused) continue;
        const uint32_t N = uni(nrec[c]);
        const uint32_t Ofin = uni(out_len[c]);
        const uint32_t ilen = uni(in_len[c]);
        const uint8_t* __restrict__ src = in + in_off[c];
        uint8_t* __restrict__ dst = out + out_off[c];
        const uint32_t* __restrict__ R = rec + (size_t)c * kRecCap;
        const uint32_t NU = (Ofin + 15u) >> 4;
        // wave state
        uint32_t nxt = 0, lowpend = 0, flushed = 0, rin = 0, Oin = 0, rlow = 0, rounds = 0;
        // lane state: unit, its first record, pending segments (bit k = record rf + k), applied bytes,
        // the unit's bytes, and the HBM load in flight (its bytes, its byte range b0 | b1 << 8)
        uint32_t u = kUxNone, rf = 0, pend = 0, am = 0, ldb = 0, hbm = 0;
        bool infl = false;
        uint4 dat = make_uint4(0, 0, 0, 0), ldv = make_uint4(0, 0, 0, 0);
        uint32_t acc = 0;
        uint32_t rpre = lane < kUxIn && lane < N ? R[lane] : 0u;
        bool guard = false;
        for (;;) {
            // ---- intake: 32 records at a time (at most 2 KiB of output, so the unit-first ring of 256
            // units always has room for them beside the unit being assigned) into the record ring, output
            // starts by a prefix sum, and each unit whose first byte lies in a record marks that record
            for (int t = 0; t < 2; ++t) {
                if (!(rin < N && rin + kUxIn <= rlow + kUxRR)) break;
                const bool valid = lane < kUxIn && rin + lane < N;
                const uint32_t r = rpre;
                const uint32_t len = valid ? ((r >> 25) & 63u) + 1u : 0u;
                const uint32_t incl = incl_scan(len);
                if (Oin + uni((uint32_t)__builtin_amdgcn_readlane((int)incl, 63)) > 16u * (nxt + kUxUF)) break;
                const uint32_t os = Oin + incl - len;
                {
                    const uint64_t lm = __ballot(valid && (r >> 31) == 0u);  // rin is a multiple of kUxIn
                    if (lane == 0) L.litb[(rin >> 5) & (kUxRR / 32 - 1)] = (uint32_t)lm;
                }
                if (valid) {
                    L.rr[(rin + lane) & (kUxRR - 1)] = make_uint2(os, r);
                    const uint32_t c0 = (os + 15u) >> 4;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        if (16u * (c0 + k) < os + len) L.uf[(c0 + k) & (kUxUF - 1)] = (uint16_t)(rin + lane);
                }
                Oin += uni((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
                rin = rin + kUxIn < N ? rin + kUxIn : N;
                rpre = lane < kUxIn && rin + lane < N ? R[rin + lane] : 0u;
            }
            wave_sync();
            // ---- refill: free lanes take the next units, in unit order by lane rank
            {
                const bool freel = u == kUxNone;
                const uint64_t fm = __ballot(freel);
                uint32_t take = (uint32_t)__popcll(fm);
                const uint32_t lim_cov = rin == N ? NU : ((Oin >> 4) > 0u ? (Oin - 1u) >> 4 : 0u);  // 16(v+1) < Oin
                const uint32_t lims[4] = {NU, lowpend + kUxAhead, (flushed >> 4) + kUxSlots, lim_cov};
#pragma unroll
                for (int i = 0; i < 4; ++i) take = min(take, lims[i] > nxt ? lims[i] - nxt : 0u);
                if (take) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                    if (freel && rank < take) {
                        const uint32_t v = nxt + rank;
                        const uint32_t f = L.uf[v & (kUxUF - 1)];
                        const uint32_t e = 16u * (v + 1u);
                        const uint32_t nx = e < Ofin ? (uint32_t)L.uf[(v + 1u) & (kUxUF - 1)] : N;
                        const uint32_t rl = (nx < N && L.rr[nx & (kUxRR - 1)].x < e) ? nx : nx - 1u;
                        u = v;
                        rf = f;
                        pend = (2u << (rl - f)) - 1u;
                        {   // literal segments read the compressed chunk in HBM: the load step's
                            const uint64_t lw = (uint64_t)L.litb[(f >> 5) & (kUxRR / 32 - 1)] |
                                                ((uint64_t)L.litb[((f >> 5) + 1u) & (kUxRR / 32 - 1)] << 32);
                            hbm = (uint32_t)(lw >> (f & 31u)) & ((2u << (rl - f)) - 1u);
                        }
                        am = 0;
                        dat = make_uint4(0, 0, 0, 0);
                        L.umask[v & (kUxSlots - 1)] = 0;
                    }
                    nxt += take;
                }
            }
            wave_sync();
            // ---- attempts: the kUxK lowest pending segments that read LDS (ring copies); a segment found
            // to read HBM (literal, or a copy older than the ring) is marked and left to the load step
            const uint32_t farU = nxt > kUxSlots ? nxt - kUxSlots : 0u;  // units below this are not in the ring
            uint32_t tried = hbm;
            for (int a = 0; a < kUxK; ++a) {
                const uint32_t cand = pend & ~tried;
                if (!__ballot(cand != 0u)) break;
                if (cand) {
                    const uint32_t k = (uint32_t)__builtin_ctz(cand);
                    tried |= 1u << k;
                    const uint2 e = L.rr[(rf + k) & (kUxRR - 1)];
                    const uint32_t os = e.x, r = e.y;
                    const uint32_t len = ((r >> 25) & 63u) + 1u, x = r & 0x1FFFFFFu;
                    const uint32_t U0 = u << 4;
                    const uint32_t q0 = max(os, U0), q1 = min(os + len, U0 + 16u);
                    const uint32_t b0 = q0 - U0, b1 = q1 - U0;
                    // A copy with offset x < 16 repeats its first x bytes: once a segment byte lies dm - x or
                    // more into the copy (dm = the least multiple of x >= 16), every byte of the segment is
                    // the byte dm back, an ordinary unit-aligned ring read; only the first bytes of such a
                    // copy (per) read its period [os - x, os) byte by byte.
                    uint32_t xs = x;
                    if (x < 16u) {
                        const uint32_t m = (uint32_t)((float)(15u + x) * __builtin_amdgcn_rcpf((float)x) + 1e-3f);
                        if (q0 + x >= os + m * x) xs = m * x;
                    }
                    const bool per = xs < 16u;
                    const uint32_t s0 = per ? os - x : q0 - xs, s1 = per ? os : q1 - xs;
                    const uint32_t v0 = s0 >> 4, v1 = (s1 - 1u) >> 4;
                    if (!per && v1 < farU) {  // older than the ring: the load step reads it from HBM
                        hbm |= 1u << k;
                    } else {
                        // bytes applied? (own unit: the lane's mask; below lowpend: final).  v0 < farU <= v1
                        // (a copy straddling the ring's end): v0 is flushed, so below lowpend and final;
                        // its bytes are read one by one, from HBM and the ring.
                        const uint32_t n0 = bits16(s0 & 15u, v1 == v0 ? ((s1 - 1u) & 15u) + 1u : 16u);
                        const uint32_t n1 = v1 == v0 ? 0u : bits16(0u, ((s1 - 1u) & 15u) + 1u);
                        const uint32_t m0 = v0 == u ? am : (v0 < lowpend ? 0xFFFFu : (uint32_t)L.umask[v0 & (kUxSlots - 1)]);
                        const uint32_t m1 = v1 == u ? am : (v1 < lowpend ? 0xFFFFu : (uint32_t)L.umask[v1 & (kUxSlots - 1)]);
                        if ((m0 & n0) == n0 && (m1 & n1) == n1) {
                            uint4 v;
                            if (per) {  // the period, byte by byte from the ring (own bytes stored first)
                                *reinterpret_cast<uint4*>(&L.ring[(U0 & (kUxRing - 1)) >> 2]) = dat;
                                uint32_t w[4] = {0u, 0u, 0u, 0u};
                                const uint32_t n = U0 + b0 - os;  // < 80
                                uint32_t t = n - x * (uint32_t)((float)n * __builtin_amdgcn_rcpf((float)x) + 1e-3f);
                                for (uint32_t j = b0; j < b1; ++j) {
                                    w[j >> 2] |= (uint32_t)ring8[(os - x + t) & (kUxRing - 1)] << (8u * (j & 3u));
                                    t = t + 1u == x ? 0u : t + 1u;
                                }
                                v = make_uint4(w[0], w[1], w[2], w[3]);
                            } else if (v0 < farU) {  // straddling the ring's end (rare): HBM and ring bytes
                                uint32_t w[4] = {0u, 0u, 0u, 0u};
                                for (uint32_t j = b0; j < b1; ++j) {
                                    const uint32_t p = U0 + j - xs;
                                    w[j >> 2] |= (uint32_t)((p >> 4) < farU ? dst[p] : ring8[p & (kUxRing - 1)]) << (8u * (j & 3u));
                                }
                                v = make_uint4(w[0], w[1], w[2], w[3]);
                            } else {  // ring: 5 dwords from the unit-aligned source start
                                const uint32_t sa = (U0 - xs) & (kUxRing - 1);
                                const uint32_t* q = &L.ring[sa >> 2];
                                const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
                                const uint32_t sh = sa & 3u;
                                v = make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                                               __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
                            }
                            const uint4 m0 = lowm[b0], m1 = lowm[b1];
                            dat.x = bfi32(m0.x ^ m1.x, v.x, dat.x);
                            dat.y = bfi32(m0.y ^ m1.y, v.y, dat.y);
                            dat.z = bfi32(m0.z ^ m1.z, v.z, dat.z);
                            dat.w = bfi32(m0.w ^ m1.w, v.w, dat.w);
                            am |= bits16(b0, b1);
                            pend &= ~(1u << k);
                        }
                    }
                }
            }
            // ---- merge the HBM bytes loaded last round (a round of LDS work after their issue).  The wait
            // also retires last round's flush stores, so a far copy issued below never reads a line
            // before its bytes reach the L2.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (infl) {
                const uint4 m0 = lowm[ldb & 31u], m1 = lowm[ldb >> 8];
                dat.x = bfi32(m0.x ^ m1.x, ldv.x, dat.x);
                dat.y = bfi32(m0.y ^ m1.y, ldv.y, dat.y);
                dat.z = bfi32(m0.z ^ m1.z, ldv.z, dat.z);
                dat.w = bfi32(m0.w ^ m1.w, ldv.w, dat.w);
                am |= bits16(ldb & 31u, ldb >> 8);
                infl = false;
            }
            // ---- load step: each lane's lowest pending HBM segment, one 16-byte load aligned to the unit,
            // merged next round (at a chunk's edges: its bytes one by one now)
            if (__ballot((pend & hbm) != 0u)) {
                const uint32_t hm = pend & hbm;
                if (hm) {
                    const uint32_t k = (uint32_t)__builtin_ctz(hm);
                    const uint2 e = L.rr[(rf + k) & (kUxRR - 1)];
                    const uint32_t os = e.x, r = e.y;
                    const uint32_t len = ((r >> 25) & 63u) + 1u, x = r & 0x1FFFFFFu;
                    const bool isc = (r >> 31) != 0u;
                    const uint32_t U0 = u << 4;
                    const uint32_t q0 = max(os, U0), q1 = min(os + len, U0 + 16u);
                    const uint32_t b0 = q0 - U0, b1 = q1 - U0;
                    // literal: input position of unit byte 0; far copy: output position of unit byte 0
                    const uint32_t ga = isc ? U0 - x : x + U0 - os;
                    const bool gfast = isc ? (U0 >= x) : (x + U0 >= os && ga + 16u <= ilen);
                    if (gfast) {
                        ldv = g_ld16u(isc ? dst + ga : src + ga);
                        ldb = b0 | (b1 << 8);
                        infl = true;
                    } else {
                        uint32_t w[4] = {0u, 0u, 0u, 0u};
                        for (uint32_t j = b0; j < b1; ++j)
                            w[j >> 2] |= (uint32_t)(isc ? dst[U0 + j - x] : src[x + U0 + j - os]) << (8u * (j & 3u));
                        const uint4 m0 = lowm[b0], m1 = lowm[b1];
                        dat.x = bfi32(m0.x ^ m1.x, w[0], dat.x);
                        dat.y = bfi32(m0.y ^ m1.y, w[1], dat.y);
                        dat.z = bfi32(m0.z ^ m1.z, w[2], dat.z);
                        dat.w = bfi32(m0.w ^ m1.w, w[3], dat.w);
                        am |= bits16(b0, b1);
                    }
                    pend &= ~(1u << k);
                }
            }
            // ---- publish the units' bytes and applied masks; completed units free their lanes
            const bool busy = u != kUxNone;
            if (busy) {
                const uint32_t sl = u & (kUxSlots - 1);
                *reinterpret_cast<uint4*>(&L.ring[4u * sl]) = dat;
                if (sl == 0u) *reinterpret_cast<uint4*>(&L.ring[kUxRing / 4]) = dat;
                L.umask[sl] = (uint16_t)am;
            }
            if (busy && pend == 0u && !infl) u = kUxNone;
            lowpend = wave_min(u != kUxNone ? u : kUxNone);
            if (lowpend == kUxNone) lowpend = nxt;
            rlow = wave_min(u != kUxNone ? rf : kUxNone);
            if (rlow == kUxNone) rlow = (nxt < NU && 16u * nxt < Oin) ? (uint32_t)L.uf[nxt & (kUxUF - 1)] : rin;
            wave_sync();
            // ---- flush the 1 KiB blocks below the lowest pending unit
            const uint32_t fl = min(lowpend << 4, Ofin);
            while (flushed + kUxFB <= fl) {
                const uint4 d = *reinterpret_cast<const uint4*>(&L.ring[((flushed + 16u * lane) & (kUxRing - 1)) >> 2]);
                g_st16u(dst + flushed + 16u * lane, d);
                if (do_crc) {
                    const uint4 dc = make_uint4(flushed == 0u && lane == 0u ? ~d.x : d.x, d.y, d.z, d.w);
                    acc = shift_byte_tab(sSH, acc) ^ raw16(sT, dc);
                }
                flushed += kUxFB;
            }
            if (nxt >= NU && lowpend >= NU) break;
            if (++rounds > 64u * NU + 4096u) {  // unreachable on a consistent record stream
                guard = true;
                break;
            }
        }
        if (guard) st = kGuardTrip + 3;
        // ---- tail [flushed, Ofin) and the frame's CRC (the folded-init form of k_expand's FrameIO::finish
        // with 16-byte lane slots)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t rem = Ofin - flushed;  // < kUxFB (the whole frame when the guard tripped early)
        {
            const uint32_t b0 = 16u * lane, b1 = min(b0 + 16u, rem);
            if (b0 + 16u <= rem) {
                g_st16u(dst + flushed + b0, *reinterpret_cast<const uint4*>(&L.ring[((flushed + b0) & (kUxRing - 1)) >> 2]));
            } else {
                for (uint32_t i = b0; i < b1; ++i) dst[flushed + i] = ring8[(flushed + i) & (kUxRing - 1)];
            }
        }
        uint32_t crc = 0;
        if (do_crc && !guard) {
            auto fold = [&](uint32_t v) {
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const uint32_t other = __shfl_xor(v, 1 << j);
                    const bool is_lo = ((lane >> j) & 1u) == 0u;
                    v = shift_nib_tab(gNS + (j + 1) * 128, is_lo ? v : other) ^ (is_lo ? other : v);
                }
                return v;
            };
            const uint32_t k = rem >> 4;  // whole 16-byte tail slots
            uint32_t Rc = fold(acc);      // raw CRC of the flushed blocks
            uint32_t c2 = 0;
            if (lane >= 64u - k) {  // tail slot j = lane - (64 - k), right-aligned
                const uint32_t pos = flushed + 16u * (lane - (64u - k));
                const uint4 d = *reinterpret_cast<const uint4*>(&L.ring[(pos & (kUxRing - 1)) >> 2]);
                c2 = raw16(sT, make_uint4(pos == 0u ? ~d.x : d.x, d.y, d.z, d.w));
            }
            c2 = fold(c2);
#pragma unroll
            for (int j = 0; j < 6; ++j)  // Rc * x^(8 * 16k)
                if ((k >> j) & 1u) Rc = shift_nib_tab(gNS + (j + 1) * 128, Rc);
            Rc ^= c2;
            uint32_t i0 = flushed + 16u * k;
            if (Ofin < 16u) {  // short frame: the plain CRC from ~0 (no fold)
                Rc = 0xFFFFFFFFu;
                i0 = 0;
            }
            for (uint32_t i = i0; i < Ofin; ++i) Rc = (Rc >> 8) ^ sT[(Rc ^ ring8[i & (kUxRing - 1)]) & 0xFFu];
            crc = ~Rc;
        }
        write_result((int)lane, crc, st, expect != nullptr, expect ? expect[c] : 0u, Ofin, 0u, &out_len[c], nullptr, &status[c],
                     crc_out ? &crc_out[c] : nullptr);
        wave_sync();
    }
}
