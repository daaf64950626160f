// expand_window_kernel.hip — k_window, the sliding-window record expander (two frames per wave,
// lanes hold records, exact readiness through a done-bitmap), built and measured in round 3 and NOT
// shipped: bit-exact on every decode / LZ4 / handler / batcher GPU test as a drop-in for k_expand
// (same signature, records from k_parse), but slower — 51-56 ms per 262 144 frames against k_expand's
// 44 ms (profiles/r03/notes/decoder_window.md).  Its C model is expand_window_model.c.  To measure it,
// paste this block back into netty_amd/csrc/snappy_decode.hip (namespace nx::dec, after k_expand) and
// launch it from launch_expand() with kWaves * sizeof(WaveL) + kTabBytes bytes of dynamic LDS.
// =====================================================================================
// k_window: the record expander with a sliding window of records, two frames per wave
// =====================================================================================
// Each half-wave (32 lanes) owns one frame.  A lane holds one record (a literal of <= 64 bytes or a
// copy) and writes it into the frame's 4 KiB LDS ring, up to two aligned output qwords per round,
// with one masked 64-bit LDS write each.  Records enter free lanes in stream order (at most 32 in
// flight, and only while they end within kHz bytes of the frontier F, the first output byte not yet
// final); a lane leaves when its record is written.  A record is executed as soon as its sources
// are final, not in stream order:
//   - literals and FAR copies (source older than the ring keeps) load their bytes from HBM at
//     admission and after each step, 16 bytes aligned to the destination qwords, used one round later;
//   - NEAR copies read the ring and run when every source byte at or above F is done: a done-bitmap
//     (one bit per ring byte) is set as bytes are written and cleared when their block is flushed;
//   - a copy whose piece reads its own output (offset < piece length) replicates the period before
//     its start.
// Every 512-byte block below F leaves the ring as one 16-byte store per lane and is folded into the
// lane's CRC32C accumulator (slicing-by-4, shift by 512 B); the 32 accumulators are combined once per
// frame.  scripts/experiments/expand_window_model.c is the C model this follows (bit-exact on the
// bench corpus and on periodic / random / zero data): ~310 rounds per frame-equivalent on the bench
// corpus against k_expand's ~1 090 (456 passes x 2.39 rounds) at 64 lanes per frame.
namespace win {
constexpr int kWaves = 15;               // waves per workgroup, one workgroup per CU (LDS)
constexpr uint32_t kRing = 4096;         // output history per frame (bytes)
constexpr uint32_t kHz = 2048;           // admission horizon ahead of the frontier
constexpr uint32_t kW = kRing - kHz;     // history the ring always keeps below the frontier
constexpr uint32_t kBlk = 512;           // flush block: 32 lanes x 16 B
constexpr uint32_t kBitDw = kRing / 32;  // done-bitmap dwords
constexpr uint32_t kQ = 64;              // record queue entries (stream index i at i & 63)
// (Unaligned LDS reads would save the realignment below, but on gfx950 they run ~5x slower than
// aligned ones: scripts/micro/lds_unaligned.hip.)
struct Half {
    uint64_t ring[kRing / 8];
    uint32_t bits[kBitDw];
    uint2 q[kQ];  // (record, output start)
};
struct WaveL {
    Half h[2];
};
static_assert(kWaves * sizeof(WaveL) + kTabBytes <= 160 * 1024, "one workgroup per CU");

// inclusive prefix sum within each 32-lane half (rows of 16, then row 0 -> 1 and 2 -> 3)
__device__ __forceinline__ uint32_t half_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    return v;
}
// minimum of each half, broadcast to the half (inclusive min-scan; lanes 31 / 63 hold the minima)
__device__ __forceinline__ uint32_t half_min(uint32_t v, bool hi) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xa, 0xf, false));
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 31), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return hi ? b : a;
}
__device__ __forceinline__ uint32_t half_lane(uint32_t v, int k, bool hi) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, k), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 32 + k);
    return hi ? b : a;
}

__device__ __forceinline__ uint32_t crc_step4(const uint32_t* __restrict__ T, uint32_t c) {
    return T[3 * 256 + (c & 0xFF)] ^ T[2 * 256 + ((c >> 8) & 0xFF)] ^ T[1 * 256 + ((c >> 16) & 0xFF)] ^ T[c >> 24];
}

typedef uint32_t v4 __attribute__((ext_vector_type(4)));
typedef v4 __attribute__((aligned(1))) v4u;
typedef __attribute__((address_space(1))) const v4u gv4u;
// 16 bytes at base + a, bytes outside [0, lim) as 0 (slow path: byte loads)
__device__ __forceinline__ uint4 load16_slow(const uint8_t* base, int32_t a, int32_t lim) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j)
        if (a + j >= 0 && a + j < lim) w[j >> 2] |= (uint32_t)base[a + j] << (8 * (j & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void lds_mskor64(uint32_t addr, uint64_t mask, uint64_t data) {
    asm volatile("ds_mskor_b64 %0, %1, %2" ::"v"(addr), "v"(mask), "v"(data & mask) : "memory");
}
// bytes [lo, hi) of a qword, 0 <= lo < hi <= 8
__device__ __forceinline__ uint64_t byte_mask(uint32_t lo, uint32_t hi) { return (~0ull << (8u * lo)) & (~0ull >> (64u - 8u * hi)); }

struct Frame2 {
    const uint8_t* src;
    uint8_t* dst;
    const uint32_t* rec;
    uint32_t in_len, N, Ofin, c;
    int32_t st;
};

__global__ void __launch_bounds__(kWaves * 64, 1)
    k_window(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len_a,
             uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ rec,
             const uint32_t* __restrict__ nrec, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
             const uint32_t* __restrict__ expect, uint32_t* __restrict__ crc_out, uint32_t n, const CrcTables* __restrict__ tabs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool do_crc = (expect != nullptr) || (crc_out != nullptr);
    uint32_t* sT = reinterpret_cast<uint32_t*>(smem);
    uint32_t* sSH = sT + 4 * 256;
    if (do_crc) {
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) sSH[i] = (&tabs->SH[5][0][0])[i];
    }
    __syncthreads();
    const uint32_t wave = uni(threadIdx.x >> 6);
    WaveL* WL = reinterpret_cast<WaveL*>(smem + kTabBytes + wave * sizeof(WaveL));
    const int lane = threadIdx.x & 63;
    const bool hi = lane >= 32;
    const uint32_t t = (uint32_t)lane & 31u;
    const uint64_t hmask = hi ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
    Half& L = WL->h[hi ? 1 : 0];
    const uint32_t ring_base = (uint32_t)(uintptr_t)L.ring;  // LDS byte address
    const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);
    const uint32_t* gNS = &tabs->NS[0][0][0];

    const uint32_t stride = gridDim.x * kWaves * 2u;
    uint32_t c = (blockIdx.x * kWaves + wave) * 2u + (hi ? 1u : 0u);

    // ---- per-half frame state (half-uniform)
    Frame2 f{};
    bool active = false;
    uint32_t F = 0, flushed = 0, next = 0, qtail = 0, obase = 0, acc = 0, Bn = 0, rounds = 0, guard = 0;
    // ---- lane state: the record [s, e), its literal input position or copy offset x, the next
    // output byte cur; has = holds a record, copy / far / mid its kind, elig = may execute this round,
    // ldp = its 16 data bytes arrive this round
    bool has = false, elig = false, copy = false, far = false, mid = false, ldp = false;
    uint32_t s = 0, e = 0, x = 0, cur = 0;
    uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;  // this round's 16 data bytes (literal / far lanes)
    uint32_t n0_ = 0, n1_ = 0, n2_ = 0, n3_ = 0;  // the next 16, in flight

    // records [qtail, qtail + 32) (raw in Bn) -> queue with their output starts; prefetch the next 32
    auto refill = [&]() {
        const bool v = qtail + t < f.N;
        const uint32_t len = v ? ((Bn >> 25) & 63u) + 1u : 0u;
        const uint32_t inc = half_scan(len);
        L.q[(qtail + t) & (kQ - 1)] = make_uint2(Bn, obase + inc - len);
        obase += half_lane(inc, 31, hi);
        qtail += 32u;
        // always issued (clamped inside the frame's slot), so the load lands in Bn itself: a
        // conditional load would be merged through a copy that waits for it at once
        Bn = f.rec[min(qtail + t, kRecCap - 1u)];
    };
    auto start = [&]() {
        active = false;
        while (c < n) {
            if (status[c] != kNeedFused) {
                active = true;
                break;
            }
            c += stride;
        }
        if (!active) return;
        f.c = c;
        f.src = in + in_off[c];
        f.dst = out + out_off[c];
        f.in_len = in_len_a[c];
        f.N = nrec[c];
        f.Ofin = out_len[c];
        f.st = status[c];
        f.rec = rec + (size_t)c * kRecCap;
        F = flushed = next = qtail = obase = acc = rounds = 0;
        guard = 4u * (f.Ofin + f.N) + 256u;
        has = elig = ldp = false;
#pragma unroll
        for (uint32_t k = 0; k < kBitDw / 32; ++k) L.bits[k * 32 + t] = 0u;
        Bn = f.rec[t];
        refill();
        refill();
        c += stride;
    };
    // Store the tail (< kBlk bytes after the last flushed block) and finish the CRC.  The ~0 initial
    // state is folded into the data (output bytes 0..3 enter the CRC XORed with 0xFF, flush_block),
    // so the CRC is ~raw(M) with raw the state-0 CRC: no x^(8n) products per frame.  raw(M) =
    // shift(raw(full blocks), tail) ^ raw(tail): the full blocks fold from the 32 lane accumulators
    // (XOR_t acc_t * x^(8*16*(31-t))), the tail's whole 16-byte slots sit right-aligned in lanes
    // 32-k..31 (leading zero slots add nothing to a state-0 CRC) and fold the same way, and its last
    // partial slot continues byte by byte.  A frame shorter than 16 bytes is CRCed byte by byte from ~0.
    auto finish = [&]() {
        const uint32_t O = f.Ofin;
        const uint32_t rem = O - flushed;  // < kBlk
        const uint32_t k = rem >> 4;       // whole tail slots
        {
            const uint32_t b0 = 16u * t, b1 = min(b0 + 16u, rem);
            for (uint32_t i = b0; i < b1; ++i) f.dst[flushed + i] = ring8[(flushed + i) & (kRing - 1)];
        }
        uint32_t crc = 0;
        if (do_crc) {
            auto fold = [&](uint32_t v) {
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const uint32_t other = (uint32_t)__shfl_xor((int)v, 1 << j);
                    const bool is_lo = ((t >> j) & 1u) == 0u;
                    v = shift_nib_tab(gNS + (j + 1) * 128, is_lo ? v : other) ^ (is_lo ? other : v);
                }
                return v;
            };
            uint32_t R = fold(acc);  // raw CRC of the flushed blocks
            uint32_t c2 = 0;
            if (t >= 32u - k) {      // tail slot j = t - (32 - k), right-aligned
                const uint32_t pos = flushed + 16u * (t - (32u - k));
                const uint4 v = *reinterpret_cast<const uint4*>(&ring8[pos & (kRing - 1)]);
                const uint32_t v0 = pos == 0u ? ~v.x : v.x;  // output bytes 0..3: the folded initial state
                c2 = crc_step4(sT, v0);
                c2 = crc_step4(sT, c2 ^ v.y);
                c2 = crc_step4(sT, c2 ^ v.z);
                c2 = crc_step4(sT, c2 ^ v.w);
            }
            c2 = fold(c2);  // raw CRC of the tail's whole slots
#pragma unroll
            for (int j = 0; j < 5; ++j)  // R * x^(8 * 16k)
                if ((k >> j) & 1u) R = shift_nib_tab(gNS + (j + 1) * 128, R);
            R ^= c2;
            const uint32_t p0 = flushed + 16u * k;
            if (O < 16u) R = 0xFFFFFFFFu;  // short frame: the plain CRC from ~0 (no fold)
            for (uint32_t i = p0; i < O; ++i) R = (R >> 8) ^ sT[(R ^ ring8[i & (kRing - 1)]) & 0xFFu];
            crc = ~R;
        }
        if (t == 0) {
            int32_t st = f.st;
            const uint32_t m = mask_checksum(crc);
            if (st == NX_OK && expect && m != expect[f.c]) st = NX_ERR_SNAPPY_CRC_MISMATCH;
            out_len[f.c] = O;
            status[f.c] = st;
            if (crc_out) crc_out[f.c] = m;
        }
    };
    // one 512-byte block [flushed, +512) out of the ring: a 16-byte store and a CRC fold per lane, done
    // bits cleared for the ring's next lap
    auto flush_block = [&]() {
        const uint32_t pos = flushed + 16u * t;
        const uint4 v = *reinterpret_cast<const uint4*>(&ring8[pos & (kRing - 1)]);
        uint8_t* o = f.dst + pos;
        if ((((uintptr_t)o) & 15u) == 0u) {
            *reinterpret_cast<uint4*>(o) = v;
        } else {
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) o[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
        }
        if (do_crc) {
            uint32_t cc = crc_step4(sT, pos == 0u ? ~v.x : v.x);  // output bytes 0..3: the folded initial state
            cc = crc_step4(sT, cc ^ v.y);
            cc = crc_step4(sT, cc ^ v.z);
            cc = crc_step4(sT, cc ^ v.w);
            acc = shift_byte_tab(sSH, acc) ^ cc;
        }
        if (t < kBlk / 32u) L.bits[((flushed & (kRing - 1)) >> 5) + t] = 0u;
        flushed += kBlk;
    };

    start();
    for (;;) {
        if (!__ballot(active)) break;
        if (active) {
            // ============ 1. data loaded last round (the wave's one vmcnt wait per round: everything
            //              it waits for was issued a round ago)
            if (ldp) {
                d0 = n0_;
                d1 = n1_;
                d2 = n2_;
                d3 = n3_;
                elig = true;
                ldp = false;
            }
            // ============ 2. record queue: keep >= 32 records ahead of the admission cursor
            if (qtail - next <= 32u && qtail < f.N) refill();
            // ============ 3. flush every 512-byte block below F (the previous round's frontier)
            while (flushed + kBlk <= F) flush_block();
            // ============ 4. admission: free lanes take the next records in stream order, while they
            //              end within kHz of F
            bool fresh = false;
            if (__ballot(!has) & hmask) {
                const uint64_t fm = __ballot(!has) & hmask;
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                const uint32_t idx = next + rank;
                const uint2 ent = L.q[idx & (kQ - 1)];
                const uint32_t len = ((ent.x >> 25) & 63u) + 1u;
                const bool adm = !has && idx < min(qtail, f.N) && ent.y + len <= F + kHz;
                if (adm) {
                    s = ent.y;
                    e = ent.y + len;
                    cur = ent.y;
                    x = ent.x & 0x1FFFFFFu;
                    copy = (int32_t)ent.x < 0;
                    // a copy reads the ring when its offset is within kW (always kept); else HBM once its
                    // source is flushed; else the ring while holding F within kW of its source ("mid")
                    far = copy && x > kW && s - x + len <= flushed;
                    mid = copy && x > kW && !far;
                    has = true;
                    elig = copy && !far;
                    fresh = !elig;
                }
                next += (uint32_t)__popcll(__ballot(adm) & hmask);
            }
            // ============ 5. execute: up to two aligned output qwords per eligible lane
            uint32_t ncur = cur;
            {
                const bool near = copy && !far;
                const uint32_t q = cur >> 3, lo0 = cur & 7u;
                const uint32_t e0 = min(e, q * 8u + 8u), e1 = min(e, q * 8u + 16u);
                const uint32_t n0 = e0 - cur;
                bool two = e0 < e;
                bool go = has && elig;
                uint32_t w0 = d0, w1 = d1, w2 = d2, w3 = d3;
                // copies whose piece reads its own output (offset < piece length): rare, per byte
                const bool modl = go && near && x < n0;
                if (__ballot(modl)) {
                    if (modl) {
                        bool ok = true;
                        for (uint32_t b = s - x; b < s; ++b)
                            if (b >= F && ((L.bits[(b & (kRing - 1)) >> 5] >> (b & 31u)) & 1u) == 0u) ok = false;
                        uint32_t v0 = 0, v1 = 0;
                        const uint32_t inv = (uint32_t)(__builtin_amdgcn_rcpf((float)x) * 65536.0f) + 1u;  // floor(m/x), m, x < 64
                        for (uint32_t j = lo0; j < 8u && q * 8u + j < e0; ++j) {
                            const uint32_t m = q * 8u + j - s;
                            const uint32_t md = m - x * ((m * inv) >> 16);
                            const uint32_t by = (uint32_t)ring8[(s - x + md) & (kRing - 1)] << (8 * (j & 3));
                            if (j < 4) v0 |= by; else v1 |= by;
                        }
                        w0 = v0;
                        w1 = v1;
                        go = ok;
                        two = false;
                    }
                }
                const bool rd = go && near && !modl;
                if (__ballot(rd)) {
                    if (rd) {
                        // readiness: the bytes the pieces read at or above F must be done; a second piece
                        // only when it cannot read the first's bytes
                        two = two && x >= 16u;
                        const uint32_t a0 = cur - x, a1 = (two ? e1 : e0) - x;
                        uint32_t got = 0xFFFFFFFFu;
                        if (a1 > F) {
                            const uint32_t b = a0 & (kRing - 1);
                            const uint32_t i0 = b >> 5;
                            got = __builtin_amdgcn_alignbit(L.bits[(i0 + 1u) & (kBitDw - 1)], L.bits[i0], b & 31u);
                            if (F > a0) got |= (F - a0 >= 32u) ? 0xFFFFFFFFu : ((1u << (F - a0)) - 1u);
                        }
                        const uint32_t m0 = (1u << n0) - 1u, mall = (1u << (a1 - a0)) - 1u;
                        go = (got & m0) == m0;
                        two = two && (got & mall) == mall;
                        // ring bytes [q*8 - x, +16), aligned to the destination qwords
                        const uint32_t ra = q * 8u - x;
                        const uint32_t qa = (ra >> 3) & (kRing / 8 - 1), bs = ra & 3u;
                        const uint2 A = *reinterpret_cast<const uint2*>(&L.ring[qa]);
                        const uint2 B = *reinterpret_cast<const uint2*>(&L.ring[(qa + 1u) & (kRing / 8 - 1)]);
                        const uint2 C = *reinterpret_cast<const uint2*>(&L.ring[(qa + 2u) & (kRing / 8 - 1)]);
                        const bool ws = (ra & 4u) != 0u;
                        const uint32_t u0 = ws ? A.y : A.x, u1 = ws ? B.x : A.y, u2 = ws ? B.y : B.x, u3 = ws ? C.x : B.y, u4 = ws ? C.y : C.x;
                        w0 = __builtin_amdgcn_alignbyte(u1, u0, bs);
                        w1 = __builtin_amdgcn_alignbyte(u2, u1, bs);
                        w2 = __builtin_amdgcn_alignbyte(u3, u2, bs);
                        w3 = __builtin_amdgcn_alignbyte(u4, u3, bs);
                    }
                }
                if (go) {
                    const uint32_t q0 = q & (kRing / 8 - 1), q1 = (q + 1u) & (kRing / 8 - 1);
                    const uint64_t v0 = ((uint64_t)w1 << 32) | w0, v1 = ((uint64_t)w3 << 32) | w2;
                    const uint64_t m0 = byte_mask(lo0, e0 - q * 8u);
                    lds_mskor64(ring_base + 8u * q0, m0, v0);
                    if (two) lds_mskor64(ring_base + 8u * q1, byte_mask(0, e1 - q * 8u - 8u), v1);
                    ncur = two ? e1 : e0;
                    // done bits [cur, ncur): <= 16 bits
                    const uint32_t b = cur & (kRing - 1);
                    const uint64_t bm = (uint64_t)((1u << (ncur - cur)) - 1u) << (b & 31u);
                    const uint32_t i0 = b >> 5;
                    __hip_atomic_fetch_or(&L.bits[i0], (uint32_t)bm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    if ((uint32_t)(bm >> 32))
                        __hip_atomic_fetch_or(&L.bits[(i0 + 1u) & (kBitDw - 1)], (uint32_t)(bm >> 32), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
            }
            // ============ 6. post: finished lanes leave; literal / far lanes fetch their next 16 bytes
            {
                const bool moved = ncur != cur;
                cur = ncur;
                if (moved && cur >= e) has = false;
                const bool more = moved && has && !(copy && !far);  // literal / far with bytes left
                const bool ld = fresh || more;
                if (more) elig = false;
                if (__ballot(ld)) {
                    if (ld) {
                        const uint32_t d = cur & 7u;
                        const int32_t a = copy ? (int32_t)(cur - x) - (int32_t)d : (int32_t)(x + (cur - s)) - (int32_t)d;
                        const uint8_t* base = copy ? f.dst : f.src;
                        const int32_t lim = (int32_t)(copy ? f.Ofin : f.in_len);
                        if (a >= 0 && a + 16 <= lim) {
                            const v4 r = *(gv4u*)(base + a);
                            n0_ = r.x;
                            n1_ = r.y;
                            n2_ = r.z;
                            n3_ = r.w;
                        } else {
                            const uint4 r = load16_slow(base, a, lim);
                            n0_ = r.x;
                            n1_ = r.y;
                            n2_ = r.z;
                            n3_ = r.w;
                        }
                        ldp = true;
                    }
                }
            }
            wave_sync();
            // ============ 7. frontier: the first output byte not final (a "mid" copy holds it within kW of
            //              its source, so no admitted record reaches the source's ring slot first)
            {
                const uint32_t fr = next < qtail ? L.q[next & (kQ - 1)].y : (next < f.N ? obase : f.Ofin);
                const uint32_t mine = has ? (mid ? min(cur, cur - x + kW) : cur) : 0xFFFFFFFFu;
                F = min(half_min(mine, hi), fr);
            }
            if (++rounds > guard) {  // never on a consistent record stream
                f.st = kGuardTrip + 3;
                F = f.Ofin;
                has = false;
                next = f.N;
            }
            if (next >= f.N && F >= f.Ofin) {  // (half-uniform: F reaches the end only when no lane holds a record)
                while (flushed + kBlk <= F) flush_block();  // the last whole blocks, then the tail
                finish();
                start();
            }
        }
    }
}
}  // namespace win
