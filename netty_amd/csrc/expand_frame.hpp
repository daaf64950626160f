// expand_frame.hpp — k_expand_f, the frame-window record expander (round 5 experiment; included by
// snappy_decode.hip inside namespace nx::dec after expand_units.hpp; selected by NX_EXPANDER=frame).
//
// VERDICT r4 item 1 / SURVEY §7: hold a whole 64 KiB frame's output in LDS, so no copy ever reads HBM
// and no ring has to be managed; copies run as 16-byte LDS moves as soon as their source bytes exist.
// Same contract as k_expand (records of k_parse → output bytes + fused CRC32C).
//
// A workgroup holds TWO frames (2 x 74 KiB window + the CRC tables: one workgroup per CU) and four
// waves, two per frame:
//   * the LOADER wave walks the frame's records 512 at a time: output starts by prefix sums, literal
//     bytes loaded from the compressed chunk (all loads of the 512 records in flight at once) and
//     written into the window, their bytes marked in a written-byte bitmap; then the copy records
//     go, compacted, into a 256-entry FIFO (dst, length, offset).  A copy enters the FIFO only after
//     every literal before it is written, so the oldest pending copy can always run;
//   * the COPY wave: each lane takes one copy from the FIFO and moves it in chunks of up to 16 bytes
//     (ds_read_b128 / ds_write_b128 at any byte address), each chunk once the bitmap shows its source
//     bytes written, then sets its own bits (ds_or).  A copy with offset x < 16 moves x bytes, then
//     2x, 4x, ... (the copy's own output extends its period) until 16 per chunk.
// When both are done, the copy wave stores the window to HBM with the folded CRC (16-byte lane slots
// of 1 KiB blocks, as k_expand_u's flush).  Frames whose output exceeds 64 KiB are handed to the
// k_decode_fused fallback (status kNeedFused) before anything is written.
//
// The bound this design faces: two frames per CU in flight, each needing ~depth
// (≈ 300 dependent levels) rounds of a few LDS round trips.

constexpr uint32_t kFxOut = 65536;    // frame window (bytes)
constexpr uint32_t kFxFifo = 256;     // copy FIFO entries per frame
constexpr uint32_t kFxGroup = 8;      // loader: record groups of 64 per step
struct FxLds {
    uint8_t out[kFxOut + 16];         // the frame's output; +16 for 16-byte reads near the end
    uint32_t bm[kFxOut / 32 + 4];     // written-byte bitmap
    uint2 fifo[kFxFifo];              // copies: (dst | (len - 1) << 16, offset)
    uint32_t tail, done, abort, pad;  // FIFO tail, loader finished, copy wave gave up
    uint32_t head, pad2[3];           // FIFO head (copy wave)
};
static_assert(sizeof(FxLds) % 16 == 0, "keep per-frame LDS 16-byte aligned");
constexpr size_t kFxLds = kUxTabBytes + 2 * sizeof(FxLds);
static_assert(kFxLds <= 160 * 1024, "two frame windows per workgroup");

typedef uint64_t __attribute__((aligned(1))) u64u_;
typedef uint32_t __attribute__((aligned(1))) u32u_;
typedef uint16_t __attribute__((aligned(1))) u16u_;

// n (< 16 or == 16) bytes of v at p (LDS, any byte address)
__device__ __forceinline__ void lds_put(uint8_t* p, uint4 v, uint32_t n) {
    if (n == 16u) {
        *reinterpret_cast<v4uu*>(p) = v4u{v.x, v.y, v.z, v.w};
        return;
    }
    if (n & 8u) {
        *reinterpret_cast<u64u_*>(p) = (uint64_t)v.x | ((uint64_t)v.y << 32);
        p += 8;
        v.x = v.z;
        v.y = v.w;
    }
    if (n & 4u) {
        *reinterpret_cast<u32u_*>(p) = v.x;
        p += 4;
        v.x = v.y;
    }
    if (n & 2u) {
        *reinterpret_cast<u16u_*>(p) = (uint16_t)v.x;
        p += 2;
        v.x >>= 16;
    }
    if (n & 1u) *p = (uint8_t)v.x;
}
__device__ __forceinline__ uint4 lds_get16(const uint8_t* p) {
    const v4u v = *reinterpret_cast<const v4uu*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
// mark bytes [a, a + n) written (n <= 64)
__device__ __forceinline__ void bm_set(uint32_t* bm, uint32_t a, uint32_t n) {
    const uint32_t e = a + n;
    while (a < e) {
        const uint32_t b = a & 31u, cnt = min(32u - b, e - a);
        const uint32_t m = (cnt == 32u ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << b;
        __hip_atomic_fetch_or(&bm[a >> 5], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        a += cnt;
    }
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

__global__ void __launch_bounds__(256)
    k_expand_f(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
               uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ rec,
               const uint32_t* __restrict__ nrec, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
               const uint32_t* __restrict__ expect, uint32_t* __restrict__ crc_out, uint32_t n, const CrcTables* __restrict__ tabs,
               uint32_t* __restrict__ need_fused) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    uint32_t* const sT = reinterpret_cast<uint32_t*>(smem);
    uint32_t* const sSH = sT + 1024;
    if (do_crc) {
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) sSH[i] = (&tabs->SH[6][0][0])[i];
    }
    const uint32_t wave = uni(threadIdx.x >> 6);
    const uint32_t slot = wave & 1u;
    const bool loader = wave >= 2u;
    FxLds& L = *reinterpret_cast<FxLds*>(smem + kUxTabBytes + slot * sizeof(FxLds));
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t* __restrict__ gNS = &tabs->NS[0][0][0];
    const uint32_t pairs = (n + 1u) / 2u;
    if (loader && lane == 0) {  // FIFO control words start (and are reset after each frame) at 0
        lds_st(&L.tail, 0);
        lds_st(&L.head, 0);
        lds_st(&L.done, 0);
        lds_st(&L.abort, 0);
    }
    for (uint32_t p = blockIdx.x; p < pairs; p += gridDim.x) {
        __syncthreads();  // the windows are free (and the tables loaded)
        const uint32_t c = 2u * p + slot;
        bool skip = c >= n;
        int32_t st = 0;
        uint32_t N = 0, Ofin = 0, ilen = 0;
        if (!skip) {
            st = (int32_t)uni((uint32_t)status[c]);
            N = uni(nrec[c]);
            Ofin = uni(out_len[c]);
            ilen = uni(in_len[c]);
            if (st == kNeedFused) skip = true;
        }
        if (!skip && Ofin > kFxOut) {  // larger than the window: the fused fallback decodes it
            if (loader && lane == 0) {
                status[c] = kNeedFused;
                if (need_fused) *need_fused = 1u;
            }
            skip = true;
        }
        if (!skip && loader) {
            const uint8_t* __restrict__ src = in + in_off[c];
            const uint32_t* __restrict__ R = rec + (size_t)c * kRecCap;
            uint4* bm4 = reinterpret_cast<uint4*>(L.bm);
            for (uint32_t i = lane; i < (Ofin + 127u) / 128u + 1u; i += 64u) bm4[i] = make_uint4(0, 0, 0, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            uint32_t D = 0, tail = 0;
            for (uint32_t base = 0; base < N; base += 64u * kFxGroup) {
                uint32_t r[kFxGroup], os[kFxGroup];
#pragma unroll
                for (uint32_t j = 0; j < kFxGroup; ++j) r[j] = base + 64u * j + lane < N ? R[base + 64u * j + lane] : 0u;
#pragma unroll
                for (uint32_t j = 0; j < kFxGroup; ++j) {
                    const uint32_t len = base + 64u * j + lane < N ? ((r[j] >> 25) & 63u) + 1u : 0u;
                    const uint32_t incl = incl_scan(len);
                    os[j] = D + incl - len;
                    D += uni((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
                }
                // literal bytes: every 16-byte piece of the group's literals in flight at once
                uint4 v[kFxGroup][4];
#pragma unroll
                for (uint32_t j = 0; j < kFxGroup; ++j) {
                    const bool lit = base + 64u * j + lane < N && (r[j] >> 31) == 0u;
                    const uint32_t len = ((r[j] >> 25) & 63u) + 1u, x = r[j] & 0x1FFFFFFu;
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q) {
                        v[j][q] = make_uint4(0, 0, 0, 0);
                        if (lit && 16u * q < len) {
                            if (x + 16u * q + 16u <= ilen) {
                                v[j][q] = g_ld16u(src + x + 16u * q);
                            } else {  // the chunk's last bytes: one by one
                                uint32_t w[4] = {0u, 0u, 0u, 0u};
                                for (uint32_t b = 0; b < min(16u, len - 16u * q); ++b)
                                    w[b >> 2] |= (uint32_t)src[x + 16u * q + b] << (8u * (b & 3u));
                                v[j][q] = make_uint4(w[0], w[1], w[2], w[3]);
                            }
                        }
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (uint32_t j = 0; j < kFxGroup; ++j) {
                    const bool lit = base + 64u * j + lane < N && (r[j] >> 31) == 0u;
                    const uint32_t len = ((r[j] >> 25) & 63u) + 1u;
                    if (lit) {
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q)
                            if (16u * q < len) lds_put(L.out + os[j] + 16u * q, v[j][q], min(16u, len - 16u * q));
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (uint32_t j = 0; j < kFxGroup; ++j) {
                    const bool lit = base + 64u * j + lane < N && (r[j] >> 31) == 0u;
                    if (lit) bm_set(L.bm, os[j], ((r[j] >> 25) & 63u) + 1u);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                // the group's copies, in record order, into the FIFO
                bool aborted = false;
#pragma unroll
                for (uint32_t j = 0; j < kFxGroup; ++j) {
                    const bool cp = base + 64u * j + lane < N && (r[j] >> 31) != 0u;
                    const uint64_t cm = __ballot(cp);
                    const uint32_t cnt = (uint32_t)__popcll(cm);
                    if (cnt == 0u) continue;
                    for (;;) {  // room for cnt entries
                        if (tail + cnt - uni(lds_ld(&L.head)) <= kFxFifo) break;
                        if (uni(lds_ld(&L.abort))) {
                            aborted = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    if (aborted) break;
                    if (cp) {
                        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
                        L.fifo[(tail + rank) & (kFxFifo - 1u)] = make_uint2(os[j] | (((r[j] >> 25) & 63u) << 16), r[j] & 0x1FFFFFFu);
                    }
                    tail += cnt;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) lds_st(&L.tail, tail);
                }
                if (aborted) break;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) lds_st(&L.done, 1u + tail);  // done: the final tail + 1
        }
        bool guard = false;
        if (!skip && !loader) {
            // ---- copy wave
            uint32_t head = 0, rounds = 0;
            bool act = false;
            uint32_t d = 0, len = 0, x = 0, k = 0, Dx = 0;
            for (;;) {
                if (++rounds > 2u * kFxOut + 4096u) {  // unreachable: the oldest copy always runs (>= 1 byte a round)
                    guard = true;
                    lds_st(&L.abort, 1u);
                    break;
                }
                const uint32_t dn = uni(lds_ld(&L.done));
                const uint32_t tl = dn ? dn - 1u : uni(lds_ld(&L.tail));
                const uint64_t fm = __ballot(!act);
                const uint32_t take = min((uint32_t)__popcll(fm), tl - head);
                if (take) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                    if (!act && rank < take) {
                        const uint2 e = L.fifo[(head + rank) & (kFxFifo - 1u)];
                        d = e.x & 0xFFFFu;
                        len = (e.x >> 16) + 1u;
                        x = e.y;
                        k = 0;
                        Dx = x;
                        act = true;
                    }
                    head += take;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) lds_st(&L.head, head);
                }
                if (!__ballot(act)) {
                    if (dn && head == tl) break;
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                if (act) {
                    const uint32_t nb = min(len - k, Dx < 16u ? Dx : 16u);
                    const uint32_t s = d + k - Dx;
                    const uint32_t w = s >> 5, b = s & 31u;
                    const uint64_t bits = ((uint64_t)lds_ld(&L.bm[w + 1u]) << 32) | lds_ld(&L.bm[w]);
                    const uint64_t need = ((1ull << nb) - 1ull) << b;
                    if ((bits & need) == need) {
                        const uint4 v = lds_get16(L.out + s);
                        lds_put(L.out + d + k, v, nb);
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        bm_set(L.bm, d + k, nb);
                        k += nb;
                        if (Dx < 16u) Dx *= 2u;
                        if (k == len) act = false;
                    }
                }
            }
        }
        __syncthreads();  // both frames' windows complete
        if (!skip && !loader) {
            if (guard) st = kGuardTrip + 4;
            uint8_t* __restrict__ dst = out + out_off[c];
            const uint8_t* const w8 = L.out;
            uint32_t acc = 0, flushed = 0;
            for (; flushed + kUxFB <= Ofin; flushed += kUxFB) {
                const uint4 dd = lds_get16(w8 + flushed + 16u * lane);
                g_st16u(dst + flushed + 16u * lane, dd);
                if (do_crc) acc = shift_byte_tab(sSH, acc) ^ raw16(sT, make_uint4(flushed == 0u && lane == 0u ? ~dd.x : dd.x, dd.y, dd.z, dd.w));
            }
            const uint32_t rem = Ofin - flushed;
            {
                const uint32_t b0 = 16u * lane, b1 = min(b0 + 16u, rem);
                if (b0 + 16u <= rem) {
                    g_st16u(dst + flushed + b0, lds_get16(w8 + flushed + b0));
                } else {
                    for (uint32_t i = b0; i < b1; ++i) dst[flushed + i] = w8[flushed + i];
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
                const uint32_t kk = rem >> 4;
                uint32_t Rc = fold(acc);
                uint32_t c2 = 0;
                if (lane >= 64u - kk) {
                    const uint32_t pos = flushed + 16u * (lane - (64u - kk));
                    const uint4 dd = lds_get16(w8 + pos);
                    c2 = raw16(sT, make_uint4(pos == 0u ? ~dd.x : dd.x, dd.y, dd.z, dd.w));
                }
                c2 = fold(c2);
#pragma unroll
                for (int j = 0; j < 6; ++j)
                    if ((kk >> j) & 1u) Rc = shift_nib_tab(gNS + (j + 1) * 128, Rc);
                Rc ^= c2;
                uint32_t i0 = flushed + 16u * kk;
                if (Ofin < 16u) {
                    Rc = 0xFFFFFFFFu;
                    i0 = 0;
                }
                for (uint32_t i = i0; i < Ofin; ++i) Rc = (Rc >> 8) ^ sT[(Rc ^ w8[i]) & 0xFFu];
                crc = ~Rc;
            }
            write_result((int)lane, crc, st, expect != nullptr, expect ? expect[c] : 0u, Ofin, 0u, &out_len[c], nullptr, &status[c],
                         crc_out ? &crc_out[c] : nullptr);
        }
        if (loader && lane == 0) {
            lds_st(&L.tail, 0);
            lds_st(&L.head, 0);
            lds_st(&L.done, 0);
            lds_st(&L.abort, 0);
        }
    }
}
