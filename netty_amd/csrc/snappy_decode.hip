// snappy_decode.hip — wave-cooperative Snappy decoder + fused CRC32C verify (gfx950).
//
// Replaces Snappy.decode (Snappy.java:315-650) as SnappyFrameDecoder drives it for one complete
// COMPRESSED_DATA chunk (SnappyFrameDecoder.java:194-224), fused with Snappy.validateChecksum
// (Snappy.java:700-707) over the produced bytes.  Bit-exact, including the reference's silent
// partial output on truncated input and its error precedence (offset 0 / negative / beyond,
// output overflow, invalid literal length, preamble > 4 bytes).
//
// Design (one 64-lane wave per frame, many frames per CU):
//   parse   — the compressed stream is read in windows that always start at a tag.  Lane l
//             speculatively decodes "a tag starting at W+l" (type, operand bytes, length,
//             offset) from 5 bytes; the true tag chain is then walked from lane 0 with
//             v_readlane (scalar unit), giving a 64-bit tag mask for the window.
//   order   — per-tag Java checks (NOT_ENOUGH_INPUT → silent stop, validateOffset, capacity)
//             with the bytes-written-so-far from a wave prefix sum of tag lengths; the first
//             failing tag in stream order decides, exactly as the serial state machine would.
//   expand  — surviving tags are compacted into a per-wave LDS list; the window's output is
//             produced 64 bytes at a time, one byte per lane: the covering tag comes from a
//             tag-start bitmask + popcount, the byte from (a) the compressed input (literal),
//             (b) the per-wave LDS history ring (copies within RING bytes), (c) HBM (older
//             output of this frame, already flushed and drained), or (d) another lane of the same
//             64-byte group (overlapping copies), resolved by pointer jumping over ds_bpermute.
//   flush   — every completed 1 KiB of output leaves the ring with one 16-byte store per lane
//             and is folded into the running CRC32C (slicing-by-8 per lane + a 6-level GF(2)
//             shift tree from LDS tables), so the verify costs no extra HBM pass.
// HBM traffic per frame = compressed bytes read once + output written once (+ far-copy re-reads,
// mostly served from L2/MALL).
#include "nx_common.hpp"

namespace nx {

namespace dec {

constexpr int kWaves = 8;                 // waves per workgroup
constexpr int32_t kGuardTrip = -99;       // an internal loop bound tripped (never expected)
constexpr int kTabBytes = (8 * 256 + 7 * 1024) * 4;  // CRC tables in LDS (36 KiB)

__device__ __forceinline__ uint32_t shift_tab(const uint32_t* __restrict__ S, uint32_t c) {
    return S[c & 0xFF] ^ S[256 + ((c >> 8) & 0xFF)] ^ S[512 + ((c >> 16) & 0xFF)] ^ S[768 + (c >> 24)];
}

__device__ __forceinline__ uint32_t raw16_l(const uint32_t* __restrict__ T, uint32_t w0, uint32_t w1, uint32_t w2,
                                            uint32_t w3) {
    uint32_t c = w0;
    c = T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^ T[4 * 256 + (c >> 24)] ^
        T[3 * 256 + (w1 & 0xFF)] ^ T[2 * 256 + ((w1 >> 8) & 0xFF)] ^ T[1 * 256 + ((w1 >> 16) & 0xFF)] ^ T[0 * 256 + (w1 >> 24)];
    c ^= w2;
    c = T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^ T[4 * 256 + (c >> 24)] ^
        T[3 * 256 + (w3 & 0xFF)] ^ T[2 * 256 + ((w3 >> 8) & 0xFF)] ^ T[1 * 256 + ((w3 >> 16) & 0xFF)] ^ T[0 * 256 + (w3 >> 24)];
    return c;
}

__device__ __forceinline__ uint32_t fold64(const uint32_t* __restrict__ SH, uint32_t c, int lane) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        uint32_t other = __shfl_xor(c, 1 << j);
        bool is_lo = ((lane >> j) & 1) == 0;
        uint32_t lo = is_lo ? c : other;
        uint32_t hi = is_lo ? other : c;
        c = shift_tab(SH + j * 1024, lo) ^ hi;
    }
    return c;
}

__device__ __forceinline__ uint64_t lanemask_le(int lane) {
    return lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
}

__device__ __forceinline__ uint32_t excl_scan(uint32_t x, int lane) {
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(v, d);
        if (lane >= d) v += y;
    }
    return v - x;
}

struct Tag {  // 8 bytes in LDS
    uint32_t start;  // absolute output position
    uint32_t x;      // bit31 = copy; low 31 bits = literal source position (input) or copy offset
};

template <int RING>
struct WaveLds {
    uint8_t ring[RING];
    Tag tags[64];
    unsigned long long bmask;
    unsigned long long pad;
};

// Flush output block [from, from+1024) from the ring to HBM and fold it into the CRC state.
template <int RING>
__device__ __forceinline__ uint32_t flush_block(WaveLds<RING>& L, uint8_t* __restrict__ dst, uint32_t from, bool dst16,
                                                const uint32_t* __restrict__ sT, const uint32_t* __restrict__ sSH,
                                                uint32_t crc, bool do_crc, int lane) {
    // previous flushes must have reached L2 before any far read targets them (see header)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint4 d = *reinterpret_cast<const uint4*>(&L.ring[(from + 16u * lane) & (RING - 1)]);
    uint8_t* o = dst + from + 16u * lane;
    if (dst16) {
        *reinterpret_cast<uint4*>(o) = d;
    } else {
        const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
    if (do_crc) {
        uint32_t c = raw16_l(sT, d.x, d.y, d.z, d.w);
        c = fold64(sSH, c, lane);
        crc = shift_tab(sSH + 6 * 1024, crc) ^ c;
    }
    return crc;
}

template <int RING>
__device__ void decode_frame(WaveLds<RING>& L, const uint8_t* __restrict__ src, uint32_t in_len, uint8_t* __restrict__ dst,
                             uint32_t cap, const uint32_t* __restrict__ sT, const uint32_t* __restrict__ sSH, bool do_crc,
                             uint32_t expect, bool check, uint32_t* out_len_p, uint32_t* consumed_p, int32_t* status_p,
                             uint32_t* crc_p, int lane) {
    int32_t st = NX_OK;
    uint32_t consumed = 0;
    uint32_t O = 0;  // output frontier (bytes final)
    uint32_t flushed = 0;
    uint32_t crc = 0xFFFFFFFFu;
    const bool dst16 = (((uintptr_t)dst) & 15u) == 0;

    // ---- preamble (Snappy.readPreamble, :404-420) — uniform
    uint32_t W = 0;
    bool go = false;
    if (in_len > 0) {
        uint32_t ulen = 0;
        int bi = 0;
        bool complete = false;
        while (W < in_len) {
            uint32_t cur = src[W++];
            ulen |= (cur & 0x7fu) << (bi++ * 7);
            if ((cur & 0x80u) == 0) { complete = true; break; }
            if (bi >= 4) { st = NX_ERR_SNAPPY_PREAMBLE_TOO_LONG; break; }
        }
        if (st == NX_OK) {
            if (!complete || ulen == 0) {
                consumed = W;
            } else if (ulen > cap) {
                st = NX_ERR_SNAPPY_OUTPUT_OVERFLOW;
            } else {
                go = true;
            }
        }
        consumed = W;
    }

    bool stop = !go;
    uint32_t windows = 0;
    bool trip = false;
    while (!stop && W < in_len) {
        if (++windows > in_len + 2) { st = kGuardTrip; break; }  // -99
        // ---------------- parse: speculative tag decode at W + lane
        const uint32_t p = W + lane;
        const uint32_t avail = p < in_len ? in_len - p : 0u;
        uint32_t b[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) b[k] = ((uint32_t)k < avail) ? (uint32_t)src[p + k] : 0u;
        const uint32_t tag = b[0], type = tag & 3u;
        uint32_t size = 1;        // bytes of this tag in the stream (saturating)
        uint32_t olen = 0;        // output length (clamped to cap+1)
        uint32_t x = 0;           // literal source / copy offset
        bool nei = false;
        int32_t err = 0;
        bool is_copy = type != 0;
        int64_t off64 = 0;
        if (type == 0) {
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
                    uint32_t v = b[1] | (nb > 1 ? b[2] << 8 : 0u) | (nb > 2 ? b[3] << 16 : 0u) | (nb > 3 ? b[4] << 24 : 0u);
                    jlen = (nb == 4) ? (int64_t)(int32_t)(v + 1u) : (int64_t)v + 1;
                }
            }
            if (!nei) {
                if (jlen >= 0 && (int64_t)(avail - hdr) < jlen) {
                    nei = true;
                } else if (jlen < 0) {
                    err = NX_ERR_SNAPPY_LITERAL_LEN_INVALID;
                }
            }
            uint64_t sz = (uint64_t)hdr + (jlen > 0 ? (uint64_t)jlen : 0ull);
            size = sz > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)sz;
            olen = jlen > (int64_t)cap ? cap + 1 : (uint32_t)(jlen > 0 ? jlen : 0);
            x = (p + hdr) & 0x7FFFFFFFu;
        } else if (type == 1) {
            size = 2;
            nei = avail < 2;
            olen = 4 + ((tag >> 2) & 7u);
            off64 = (int64_t)(((tag & 0xe0u) << 3) | b[1]);
        } else if (type == 2) {
            size = 3;
            nei = avail < 3;
            olen = 1 + (tag >> 2);
            off64 = (int64_t)(b[1] | (b[2] << 8));
        } else {
            size = 5;
            nei = avail < 5;
            olen = 1 + (tag >> 2);
            off64 = (int64_t)(int32_t)(b[1] | (b[2] << 8) | (b[3] << 16) | (b[4] << 24));
        }
        if (is_copy && !nei) {
            if (off64 == 0) err = NX_ERR_SNAPPY_OFFSET_ZERO;
            else if (off64 < 0) err = NX_ERR_SNAPPY_OFFSET_NEGATIVE;
        }
        const uint32_t nxt = (uint32_t)lane + size;  // relative next tag (saturating: size < 2^31)

        // ---------------- chain walk from lane 0 (scalar)
        uint64_t chain = 0;
        uint32_t t = 0, exitrel = 0;
        for (int guard = 0;; ++guard) {
            if (guard > 64) { st = kGuardTrip + 1; stop = true; exitrel = 1; break; }
            if (W + t >= in_len) { exitrel = t; break; }
            chain |= 1ull << t;
            uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)t);
            if (n2 >= 64u) { exitrel = n2; break; }
            t = n2;
        }
        const bool is_tag = (chain >> lane) & 1ull;

        // ---------------- ordering: bytes written before each tag, per-tag checks
        const uint32_t mylen = is_tag ? olen : 0u;
        const uint32_t ostart = O + excl_scan(mylen, lane);
        if (is_tag && is_copy && !nei && err == 0) {
            if ((uint64_t)off64 > ostart) err = NX_ERR_SNAPPY_OFFSET_BEYOND;
        }
        if (is_tag && !nei && err == 0 && (uint64_t)ostart + olen > cap) err = NX_ERR_SNAPPY_OUTPUT_OVERFLOW;
        const uint64_t badm = __ballot(is_tag && (nei || err != 0));
        uint64_t valid = chain;
        uint32_t Wnext = W + exitrel;
        if (badm) {
            const int fb = __ffsll((long long)badm) - 1;
            valid = chain & ((1ull << fb) - 1ull);
            const int32_t e = __shfl(err, fb);
            const uint32_t pf = W + (uint32_t)fb;
            if (e != 0) {
                st = e;
                consumed = pf + (uint32_t)__shfl((int)size, fb);
            } else {
                consumed = pf + 1;  // NOT_ENOUGH_INPUT: tag byte consumed, operands left
            }
            stop = true;
        } else {
            consumed = Wnext < in_len ? Wnext : in_len;
        }
        const bool vt = (valid >> lane) & 1ull;
        const uint64_t outm = __ballot(vt && olen > 0);
        const uint32_t ntags = (uint32_t)__popcll(outm);
        const uint32_t total = (uint32_t)__shfl((int)(ostart + mylen), 63) - O;  // includes cut tags
        uint32_t E = O;
        if (ntags) {
            // end = start + len of the last output tag
            const int lastl = 63 - __clzll((long long)outm);
            E = (uint32_t)__shfl((int)(ostart + olen), lastl);
        }
        (void)total;
        if ((outm >> lane) & 1ull) {
            const uint32_t idx = (uint32_t)__popcll(outm & ((1ull << lane) - 1ull));
            Tag tg;
            tg.start = ostart;
            tg.x = is_copy ? (0x80000000u | (uint32_t)off64) : x;
            L.tags[idx] = tg;
        }
        // ---------------- expand [O, E) 64 bytes at a time
        if (ntags) {
            int32_t jcur = -1;
            uint32_t S = O & ~63u;
            for (; S < E && !trip; S += 64) {
                if (lane == 0) L.bmask = 0ull;
                const int32_t jj = jcur + 1 + lane;
                if (jj < (int32_t)ntags) {
                    const uint32_t s = L.tags[jj].start;
                    if (s < S + 64u) atomicOr(&L.bmask, 1ull << (s - S));
                }
                const uint64_t B = L.bmask;
                const uint32_t pp = S + lane;
                const bool act = pp >= O && pp < E;
                const int32_t idx = jcur + (int32_t)__popcll(B & lanemask_le(lane));
                jcur += (int32_t)__popcll(B);
                const uint32_t Oeff = S > O ? S : O;
                uint32_t v = 0;
                bool res = true;
                uint32_t sl = 0;
                if (act) {
                    const Tag tg = L.tags[idx];
                    if ((tg.x & 0x80000000u) == 0u) {
                        v = src[(tg.x & 0x7FFFFFFFu) + (pp - tg.start)];
                    } else {
                        const uint32_t q = pp - (tg.x & 0x7FFFFFFFu);
                        if (q >= Oeff) {
                            res = false;
                            sl = q - S;
                        } else if (q + (uint32_t)RING >= Oeff) {
                            v = L.ring[q & (RING - 1)];
                        } else {
                            v = dst[q];
                        }
                    }
                }
                for (int guard = 0; __any(!res); ++guard) {
                    if (guard > 64) { st = kGuardTrip + 2; stop = trip = true; break; }
                    const uint32_t v2 = (uint32_t)__shfl((int)v, (int)sl);
                    const int r2 = __shfl((int)res, (int)sl);
                    const uint32_t sl2 = (uint32_t)__shfl((int)sl, (int)sl);
                    if (!res) {
                        if (r2) {
                            v = v2;
                            res = true;
                        } else {
                            sl = sl2;
                        }
                    }
                }
                if (act) L.ring[pp & (RING - 1)] = (uint8_t)v;
                const uint32_t front = (S + 64u < E) ? S + 64u : E;
                for (int guard = 0; front >= flushed + 1024u; ++guard) {
                    if (guard > 64) { st = kGuardTrip + 3; stop = trip = true; break; }
                    crc = flush_block<RING>(L, dst, flushed, dst16, sT, sSH, crc, do_crc, lane);
                    flushed += 1024u;
                }
            }
        }
        O = E;
        W = Wnext;
    }

    // ---- tail flush (partial block) + CRC finish
    if (O > flushed) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t rem = O - flushed;
        const uint32_t b0 = 16u * lane;
        const uint32_t end = b0 + 16u < rem ? b0 + 16u : rem;
        uint32_t c = 0;
        for (uint32_t i = b0; i < end; ++i) {
            const uint8_t by = L.ring[(flushed + i) & (RING - 1)];
            dst[flushed + i] = by;
            c = (c >> 8) ^ sT[(c ^ by) & 0xFFu];
        }
        if (do_crc) {
            const uint32_t after = end > b0 ? rem - end : 0u;
            c = end > b0 ? gf_multmodp(gf_x8n(after), c) : 0u;
#pragma unroll
            for (int j = 0; j < 6; ++j) c ^= __shfl_xor(c, 1 << j);
            crc = gf_multmodp(gf_x8n(rem), crc) ^ c;
        }
        flushed = O;
    }
    if (lane == 0) {
        const uint32_t m = mask_checksum(~crc);
        if (st == NX_OK && check && m != expect) st = NX_ERR_SNAPPY_CRC_MISMATCH;
        *out_len_p = O;
        if (consumed_p) *consumed_p = consumed;
        *status_p = st;
        if (crc_p) *crc_p = m;
    }
}

template <int RING>
__global__ void __launch_bounds__(kWaves * 64) k_snappy_decode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                               const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                               const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                                                               uint32_t* __restrict__ out_len, uint32_t* __restrict__ consumed,
                                                               int32_t* __restrict__ status, const uint32_t* __restrict__ expect,
                                                               uint32_t* __restrict__ crc_out, uint32_t n, uint32_t* __restrict__ ticket,
                                                               const CrcTables* __restrict__ tabs, int dbg_mode) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* sT = reinterpret_cast<uint32_t*>(smem);
    uint32_t* sSH = sT + 8 * 256;
    const uint32_t* gT = &tabs->T8[0][0];
    const uint32_t* gS = &tabs->SH[0][0][0];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    if (do_crc) {
        for (int i = threadIdx.x; i < 8 * 256; i += blockDim.x) sT[i] = gT[i];
        for (int i = threadIdx.x; i < 7 * 1024; i += blockDim.x) sSH[i] = gS[i];
    }
    __syncthreads();
    if (dbg_mode == 1) return;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    WaveLds<RING>& L = *reinterpret_cast<WaveLds<RING>*>(smem + kTabBytes + wave * sizeof(WaveLds<RING>));
    // static wave -> frame assignment (interleaved so that neighbouring waves take neighbouring frames)
    const uint32_t gw = blockIdx.x * kWaves + (uint32_t)wave;
    const uint32_t nw = gridDim.x * kWaves;
    (void)ticket;
    for (uint32_t c = gw; c < n; c += nw) {
        if (dbg_mode == 2) {
            if (lane == 0) status[c] = 7;
            continue;
        }
        const uint32_t cap = out_cap ? out_cap[c] : 65536u;
        decode_frame<RING>(L, in + in_off[c], in_len[c], out + out_off[c], cap, sT, sSH, do_crc, expect ? expect[c] : 0u,
                           expect != nullptr, &out_len[c], consumed ? &consumed[c] : nullptr, &status[c],
                           crc_out ? &crc_out[c] : nullptr, lane);
    }
}

}  // namespace dec
}  // namespace nx

#include <mutex>
#include <stdlib.h>
namespace {
std::mutex g_tk_mu;
uint32_t* g_ticket = nullptr;
int g_ticket_dev = -1;
constexpr int kRing = 4096;
template <int R>
int32_t launch_decode(int dbg, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                      const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len, uint32_t* consumed, int32_t* status,
                      const uint32_t* expected_masked_crc, uint32_t* crc_out, uint32_t n, hipStream_t stream, int cus) {
    using namespace nx::dec;
    const size_t lds = kTabBytes + kWaves * sizeof(WaveLds<R>);
    static bool attr_done = false;
    if (!attr_done) {
        NX_HIP_CHECK(hipFuncSetAttribute((const void*)k_snappy_decode<R>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_done = true;
    }
    NX_HIP_CHECK(hipMemsetAsync(g_ticket, 0, 16, stream));
    unsigned blocks_per_cu = (unsigned)(160 * 1024 / lds);
    if (blocks_per_cu < 1) blocks_per_cu = 1;
    uint64_t want = (uint64_t)cus * blocks_per_cu;
    uint64_t need = (n + kWaves - 1) / kWaves;
    unsigned grid = (unsigned)(need < want ? need : want);
    hipLaunchKernelGGL(k_snappy_decode<R>, dim3(grid), dim3(kWaves * 64), lds, stream, in, in_off, in_len, out, out_off, out_cap,
                       out_len, consumed, status, expected_masked_crc, crc_out, n, g_ticket, nx::crc_tables_dev(), dbg);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
}  // namespace

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
    {
        std::lock_guard<std::mutex> lk(g_tk_mu);
        if (!g_ticket || g_ticket_dev != dev) {
            NX_HIP_CHECK(hipMalloc(&g_ticket, 256 * sizeof(uint32_t)));
            g_ticket_dev = dev;
        }
    }
    static const int dbg = getenv("NX_DEC_DEBUG") ? atoi(getenv("NX_DEC_DEBUG")) : 0;
    if (dbg == 3)
        return launch_decode<1024>(0, in, in_off, in_len, out, out_off, out_cap, out_len, consumed, status, expected_masked_crc,
                                   crc_out, n, (hipStream_t)stream, cus);
    return launch_decode<kRing>(dbg, in, in_off, in_len, out, out_off, out_cap, out_len, consumed, status, expected_masked_crc,
                                crc_out, n, (hipStream_t)stream, cus);
}
