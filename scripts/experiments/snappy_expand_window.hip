// snappy_expand_window.hip — EXPERIMENT (not built into libnetty_amd.so): the sliding-window record
// expander tried in round 2 as a replacement for nx::dec::k_expand.  To rebuild it, paste this section
// into netty_amd/csrc/snappy_decode.hip after k_expand and launch it from decode_batch in place of
// k_expand (lds = kTabBytes + kWavesW * sizeof(WinLds), kWavesW * 64 threads, 2 workgroups per CU).
// Bit-exact on all 69 decode/handler/batcher/LZ4 GPU tests, but slower: 55.1 ms (24 waves/CU) and
// 51.6 ms (32 waves/CU) per 262 144 frames against k_expand's 46.4 ms
// (profiles/r02/notes/decoder_experiments.md, "sliding-window expander").

// =====================================================================================
// k_expand_w: one WAVE per frame, a sliding window of pending records (round 2)
// =====================================================================================
// Each lane holds one pending RECORD (from k_parse) and, per pass, produces the part of it that
// falls in one aligned 16-byte output unit.  A pass:
//   refill  — free lanes take the next records in stream order (bpermute from a 3-batch register
//             prefetch, a prefix sum gives their output positions), while the window's output span
//             stays within the ring;
//   flush   — every 512 B block whose bytes are all written (a bitmap with one bit per ring byte)
//             leaves the ring with one 8-byte store per lane and is folded into the lane's CRC32C;
//   ready   — a literal is always ready; a copy when the bytes it reads are flushed or their bits
//             are set (true dataflow: copies of recently produced bytes wait only for those bytes);
//   execute — the unit's source bytes come from the compressed input (literal; HBM/L2), the ring
//             (copy at most ~3.5 KiB back) or the frame's flushed output (older copy), aligned to
//             the unit with alignbyte, and are written with up to four ds_mskor; overlapping copies
//             (offset < bytes produced) replicate their period in registers.
// No per-pass byte->piece map, no dependency rounds: a stalled copy just keeps its lane, and the
// lowest pending record is always ready, so every pass makes progress.  On the bench corpus a
// 64 KiB frame takes ~450 passes with ~29 ready lanes each (scripts/experiments/sim_window.py).
constexpr int kWR = 4096;                  // output history ring per wave (bytes)
constexpr int kWB = 512;                   // flush block (64 lanes x 8 B)
constexpr uint32_t kWLimit = kWR - kWB - 64;  // window span: Emax <= flushed + kWLimit

struct WinLds {
    uint32_t ring[kWR / 4];  // output positions p -> byte p % kWR
    uint32_t bits[kWR / 32]; // bit (p % kWR): byte p written (cleared when its block is flushed)
};
static_assert(sizeof(WinLds) % 16 == 0, "keep per-wave LDS 16-byte aligned");
constexpr int kWavesW = 16;  // waves per workgroup of k_expand_w (2 workgroups per CU -> 32 waves/CU)
static_assert(2 * (kTabBytes + kWavesW * sizeof(WinLds)) <= 160 * 1024, "two workgroups per CU");

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef v4u32 __attribute__((aligned(1))) v4u32u;
typedef __attribute__((address_space(1))) const v4u32u gv4u32u;
// 16 bytes from an unaligned global address (one global_load_dwordx4)
__device__ __forceinline__ uint4 g_ld128u(const uint8_t* p) {
    const v4u32 x = *(gv4u32u*)(p);
    return make_uint4(x.x, x.y, x.z, x.w);
}

// 16 bytes starting at byte address a of the ring (wrapping), as 4 dwords
__device__ __forceinline__ uint4 ring16(const uint32_t* __restrict__ ring, uint32_t a) {
    const uint32_t w = a >> 2, sh = a & 3u;
    const uint32_t d0 = ring[w & (kWR / 4 - 1)], d1 = ring[(w + 1u) & (kWR / 4 - 1)], d2 = ring[(w + 2u) & (kWR / 4 - 1)],
                   d3 = ring[(w + 3u) & (kWR / 4 - 1)], d4 = ring[(w + 4u) & (kWR / 4 - 1)];
    return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                      __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
}

// 128-bit value shifted towards higher byte addresses by k bytes (0 <= k < 16), zeros shifted in
__device__ __forceinline__ uint4 shl_bytes(uint4 v, uint32_t k) {
    const uint32_t q = k >> 2, r = k & 3u;
    uint32_t a[4] = {v.x, v.y, v.z, v.w}, o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i0 = j - (int)q, i1 = j - (int)q - 1;
        const uint32_t hi = i0 >= 0 ? (i0 == 0 ? a[0] : i0 == 1 ? a[1] : i0 == 2 ? a[2] : a[3]) : 0u;
        const uint32_t lo = i1 >= 0 ? (i1 == 0 ? a[0] : i1 == 1 ? a[1] : i1 == 2 ? a[2] : a[3]) : 0u;
        o[j] = r ? __builtin_amdgcn_alignbyte(hi, lo, 4u - r) : hi;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Bytes [0, L) of v repeated with period L up to 16 bytes (1 <= L < 16)
__device__ __forceinline__ uint4 replicate(uint4 v, uint32_t L) {
    for (uint32_t len = L; len < 16u; len += len) {
        const uint4 t = shl_bytes(v, len);
        // keep bytes [0, len) of v, take bytes [len, 2len) from the shifted copy
        const uint32_t m0 = len >= 4u ? 0xFFFFFFFFu : ((1u << (8u * len)) - 1u);
        const uint32_t m1 = len >= 8u ? 0xFFFFFFFFu : (len <= 4u ? 0u : ((1u << (8u * (len - 4u))) - 1u));
        const uint32_t m2 = len >= 12u ? 0xFFFFFFFFu : (len <= 8u ? 0u : ((1u << (8u * (len - 8u))) - 1u));
        const uint32_t m3 = len <= 12u ? 0u : ((1u << (8u * (len - 12u))) - 1u);
        v = make_uint4((v.x & m0) | (t.x & ~m0), (v.y & m1) | (t.y & ~m1), (v.z & m2) | (t.z & ~m2), (v.w & m3) | (t.w & ~m3));
    }
    return v;
}

__device__ __forceinline__ uint32_t nib_to_bytes(uint32_t nib) { return ((nib * 0x00204081u) & 0x01010101u) * 0xFFu; }

__global__ void __launch_bounds__(kWavesW * 64, 8)
    k_expand_w(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
               uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ rec,
               const uint32_t* __restrict__ nrec, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
               const uint32_t* __restrict__ expect, uint32_t* __restrict__ crc_out, uint32_t n, const CrcTables* __restrict__ tabs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    const uint32_t* sT = reinterpret_cast<uint32_t*>(smem);
    const uint32_t* sSH = sT + 4 * 256;
    if (do_crc) {
        uint32_t* t = reinterpret_cast<uint32_t*>(smem);
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) t[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) t[4 * 256 + i] = (&tabs->SH[5][0][0])[i];
    }
    __syncthreads();
    const uint32_t wave = uni(threadIdx.x >> 6);
    WinLds& L = *reinterpret_cast<WinLds*>(smem + kTabBytes + wave * sizeof(WinLds));
    const uint32_t lds_ring = (uint32_t)(uintptr_t)L.ring;
    const uint32_t lds_bits = (uint32_t)(uintptr_t)L.bits;
    const int lane = threadIdx.x & 63;
    const uint32_t* gNS = &tabs->NS[0][0][0];
    const uint32_t nw = gridDim.x * kWavesW;
    for (uint32_t c = blockIdx.x * kWavesW + wave; c < n; c += nw) {
        int32_t st = (int32_t)uni((uint32_t)status[c]);
        if (st == kNeedFused) continue;
        const uint32_t N = uni(nrec[c]);
        const uint32_t Ofin = uni(out_len[c]);
        const uint32_t ilen = uni(in_len[c]);
        const uint8_t* __restrict__ src = in + in_off[c];
        uint8_t* __restrict__ dst = out + out_off[c];
        const bool dst8 = (((uintptr_t)dst) & 7u) == 0;
        const uint32_t* __restrict__ R = rec + (size_t)c * kRecCap;
        L.bits[lane] = 0u;
        L.bits[lane + 64] = 0u;
        wave_sync();
        uint32_t rb0 = (uint32_t)lane < N ? R[lane] : 0u;
        uint32_t rb1 = 64u + (uint32_t)lane < N ? R[64u + lane] : 0u;
        uint32_t rb2 = 128u + (uint32_t)lane < N ? R[128u + lane] : 0u;
        uint32_t k = 0, bb = 0, Emax = 0, flushed = 0, safe = 0;  // records taken, prefetch base, window end, flushed, stores waited
        bool pend = false, pc = false;
        uint32_t pd = 0, prem = 0, px = 0;  // pending piece: output position, bytes left, literal input position / copy offset
        uint32_t acc = 0;                   // this lane's CRC accumulator over its 8-byte slot of every flushed block
        uint32_t guard = 0;
        const uint32_t guard_max = 5u * N + Ofin / 8u + 64u;
        for (;;) {
            // ---------------- refill: free lanes take the next records (stream order = lane order among them)
            const uint64_t fm = __ballot(!pend);
            if (k < N && fm) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                const uint32_t j = k - bb + rank;  // < 128 for free lanes: k - bb < 64
                const uint32_t r0 = (uint32_t)__shfl((int)rb0, (int)(j & 63u)), r1 = (uint32_t)__shfl((int)rb1, (int)(j & 63u));
                const uint32_t r = j < 64u ? r0 : r1;
                const bool nv = !pend && k + rank < N;
                const uint32_t len = nv ? ((r >> 25) & 63u) + 1u : 0u;
                const uint32_t incl = incl_scan(len);
                const uint32_t end = Emax + incl;
                const bool take = nv && end <= flushed + kWLimit;  // monotone in rank: a prefix of the free lanes
                const uint64_t tm = __ballot(take);
                if (tm) {
                    const int last = 63 - __builtin_clzll(tm);
                    Emax = uni((uint32_t)__builtin_amdgcn_readlane((int)end, last));
                    k += (uint32_t)__popcll(tm);
                    if (take) {
                        pend = true;
                        pd = end - len;
                        prem = len;
                        pc = (r >> 31) != 0u;
                        px = r & 0x1FFFFFFu;
                    }
                    while (k - bb >= 64u) {
                        rb0 = rb1;
                        rb1 = rb2;
                        bb += 64u;
                        rb2 = bb + 128u + (uint32_t)lane < N ? R[bb + 128u + lane] : 0u;
                    }
                }
            }
            // ---------------- flush every complete 512 B block
            for (;;) {
                if (flushed + (uint32_t)kWB > Emax) break;
                const uint32_t bw = ((flushed & (kWR - 1)) >> 5) + ((uint32_t)lane & 15u);
                const uint32_t w = L.bits[bw];
                if (__ballot(lane < 16 && w != 0xFFFFFFFFu)) break;
                // stores of earlier flushes are complete before far reads may target them
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                safe = flushed;
                const uint2 d = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(L.ring) + ((flushed + 8u * lane) & (kWR - 1)));
                uint8_t* o = dst + flushed + 8u * lane;
                if (dst8) {
                    *reinterpret_cast<uint2*>(o) = d;
                } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i) o[i] = (uint8_t)((i < 4 ? d.x : d.y) >> (8 * (i & 3)));
                }
                if (do_crc) acc = shift_byte_tab(sSH, acc) ^ raw8(sT, d.x, d.y);
                wave_sync();
                if (lane < 16) L.bits[bw] = 0u;
                wave_sync();
                flushed += (uint32_t)kWB;
            }
            const uint64_t pm = __ballot(pend);
            if (!pm && k >= N) break;
            if (++guard > guard_max) {
                st = kGuardTrip + 3;
                break;
            }
            if (!pm) continue;  // the window limit held the refill back; the flush above moved it
            // ---------------- readiness (branch-free: every lane evaluates every form)
            const uint32_t sh = pd & 15u;
            uint32_t nb = 16u - sh;
            nb = prem < nb ? prem : nb;      // bytes of this pass
            const uint32_t s0 = pd - px;     // copy source of the first byte
            const bool ovl = pc && px < nb;  // the source overlaps the bytes produced
            const bool far = pc && s0 + (uint32_t)kWR < Emax;
            bool ready;
            {
                const uint32_t hi = ovl ? pd : s0 + nb;  // bytes [s0, hi) must exist; below `flushed` they do
                const uint32_t lo = s0 > flushed ? s0 : flushed;
                const uint32_t q = lo & (kWR - 1);
                const uint32_t w0 = L.bits[q >> 5], w1 = L.bits[((q >> 5) + 1u) & (kWR / 32 - 1)];
                const uint64_t ww = (((uint64_t)w1 << 32) | w0) >> (q & 31u);
                uint32_t cnt = hi > lo ? hi - lo : 0u;
                cnt = cnt < 32u ? cnt : 32u;
                const uint64_t need = (1ull << cnt) - 1ull;
                ready = pend && (!pc || far || (ww & need) == need);
            }
            const bool gl = ready && (!pc || far);  // source bytes from global memory (input, or flushed output)
            if (__ballot(far && ready && s0 + 16u > safe)) {  // rare: a far source in a block whose store may be in flight
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                safe = flushed;
            }
            // ---------------- the unit's source bytes, aligned to the unit
            uint4 v = ring16(L.ring, (ovl ? s0 : s0 - sh) & (kWR - 1));  // near copies (all lanes read; cheap)
            const uint32_t gpos = pc ? s0 : px;                          // first source byte in global memory
            const bool gfast = gpos >= sh && (pc || gpos - sh + 16u <= ilen);
            if (__ballot(gl)) {
                const uint8_t* gp = (pc ? dst : src) + (gl && gfast ? gpos - sh : 0u);
                const uint4 g = g_ld128u(gp);
                if (gl) v = g;
                if (__ballot(gl && !gfast)) {  // rare: the unit starts before the buffer or ends past the input
                    if (gl && !gfast) {
                        const uint8_t* b8 = pc ? dst : src;
                        uint32_t b[4] = {0, 0, 0, 0};
                        for (uint32_t i = 0; i < nb; ++i) b[(sh + i) >> 2] |= (uint32_t)b8[gpos + i] << (8u * ((sh + i) & 3u));
                        v = make_uint4(b[0], b[1], b[2], b[3]);
                    }
                }
            }
            if (__ballot(ready && ovl)) {  // overlapping copies: the period [s0, pd) repeated
                if (ready && ovl) v = shl_bytes(replicate(v, px), sh);
            }
            // ---------------- write the unit's bytes [sh, sh + nb) with masked ORs, mark them written
            {
                const uint32_t m16 = ready ? (((1u << nb) - 1u) << sh) : 0u;
                const uint32_t ua = lds_ring + ((pd & ~15u) & (kWR - 1));
                const uint32_t m0 = nib_to_bytes(m16 & 15u), m1 = nib_to_bytes((m16 >> 4) & 15u), m2 = nib_to_bytes((m16 >> 8) & 15u),
                               m3 = nib_to_bytes(m16 >> 12);
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(ua), "v"(m0), "v"(v.x & m0) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2 offset:4" ::"v"(ua), "v"(m1), "v"(v.y & m1) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2 offset:8" ::"v"(ua), "v"(m2), "v"(v.z & m2) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2 offset:12" ::"v"(ua), "v"(m3), "v"(v.w & m3) : "memory");
                const uint32_t q = pd & (kWR - 1);
                const uint32_t bm = ready ? (((1u << nb) - 1u) << (q & 31u)) : 0u;
                asm volatile("ds_or_b32 %0, %1" ::"v"(lds_bits + 4u * (q >> 5)), "v"(bm) : "memory");
            }
            wave_sync();
            const uint32_t adv = ready ? nb : 0u;
            pd += adv;
            prem -= adv;
            px += pc ? 0u : adv;
            pend = pend && prem != 0u;
        }
        // ---------------- the tail block, and the frame's CRC32C
        uint32_t O = Ofin;
        if (st == kGuardTrip + 3) O = flushed;  // unreachable on a consistent record stream
        uint32_t crc = 0;
        {
            wave_sync();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);
            const uint32_t rem = O - flushed;  // < 512
            const uint32_t b0 = 8u * lane;
            const uint32_t e = b0 + 8u < rem ? b0 + 8u : rem;
            uint32_t cc = 0;
            for (uint32_t i = b0; i < e; ++i) {
                const uint8_t by = ring8[(flushed + i) & (kWR - 1)];
                dst[flushed + i] = by;
                cc = (cc >> 8) ^ sT[(cc ^ by) & 0xFFu];
            }
            if (do_crc) {
                uint32_t fa = acc;
#pragma unroll
                for (int jj = 0; jj < 6; ++jj) {
                    const uint32_t other = __shfl_xor(fa, 1 << jj);
                    const bool is_lo = ((lane >> jj) & 1) == 0;
                    fa = shift_nib_tab(gNS + jj * 128, is_lo ? fa : other) ^ (is_lo ? other : fa);
                }
                const uint32_t after = e > b0 ? rem - e : 0u;
                cc = e > b0 ? gf_multmodp(gf_x8n(after), cc) : 0u;
#pragma unroll
                for (int jj = 0; jj < 6; ++jj) cc ^= __shfl_xor(cc, 1 << jj);
                const uint32_t raw = gf_multmodp(gf_x8n(rem), fa) ^ cc;
                crc = ~(gf_multmodp(gf_x8n(O), 0xFFFFFFFFu) ^ raw);
            }
        }
        write_result(lane, crc, st, expect != nullptr, expect ? expect[c] : 0u, O, 0u, &out_len[c], nullptr, &status[c],
                     crc_out ? &crc_out[c] : nullptr);
    }
}

