// crc32c.hip — CRC32C tables + the batched masked-CRC kernel.
//
// Replaces Crc32c.update/getValue (Crc32c.java:97-124) + Snappy.maskChecksum (Snappy.java:720-722)
// as called by Snappy.calculateChecksum (Snappy.java:668-676), one wave per chunk.
//
// Layout: the chunk is read as a virtual stream V = 0^z || M' || 0^k cut into 8 KiB blocks, lane l
// taking bytes [128l, 128l+128) of every block (a whole 128-byte line per lane, eight 16-byte loads
// in flight):
//   - k in [0, 16) trailing zeros make the end of V 16-byte aligned, z leading zeros make |V| a
//     multiple of 8 KiB, so every lane slot starts on a 16-byte boundary whatever the chunk's
//     address and length (bytes outside the chunk are masked to zero, never loaded from another
//     page);
//   - M' is the chunk with its first four bytes XORed with 0xFFFFFFFF, which folds the ~0 initial
//     state in (raw CRC with state 0 is linear; leading zeros add nothing to it);
//   - each lane keeps a raw-CRC accumulator over its slots (slicing-by-8, then "shift by 8 KiB" per
//     block), the 64 accumulators are combined once per chunk by a 6-level GF(2) shift tree, and the
//     k trailing zeros are taken out with one multiply by x^(-8k).
// Per byte this is one table lookup per lane; the previous form (16 bytes per lane, a tree fold
// per 1 KiB block) spent ~2.5x the VALU and kept only 1 KiB per wave in flight.
#include "nx_common.hpp"
#include <mutex>
#include <vector>


namespace nx {

static std::mutex g_crc_mu;
static CrcTables* g_crc_dev[64] = {nullptr};
static uint32_t h_T0[256];

static void build_tables(CrcTables* t) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : (c >> 1);
        t->T8[0][i] = c;
        h_T0[i] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = t->T8[k - 1][i];
            t->T8[k][i] = (c >> 8) ^ t->T8[0][c & 0xFF];
        }
    for (int j = 0; j < 10; ++j) {
        uint32_t K = gf_x8n(16ull << j);
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) t->SH[j][k][b] = gf_multmodp(K, b << (8 * k));
    }
    for (int j = 0; j < 7; ++j) {
        uint32_t K = gf_x8n(8ull << j);
        for (int k = 0; k < 8; ++k)
            for (uint32_t v = 0; v < 16; ++v) t->NS[j][k][v] = gf_multmodp(K, v << (4 * k));
    }
    // x^-8: solve gf_multmodp(x^8, y) = x^0 (GF(2) Gaussian elimination on the 32 columns)
    {
        const uint32_t a = gf_x8n(1), one = 0x80000000u;
        uint32_t col[32];
        for (int i = 0; i < 32; ++i) col[i] = gf_multmodp(a, 1u << i);
        // rows r: bit r of each column; augment with bit r of `one`
        uint64_t row[32];
        for (int r = 0; r < 32; ++r) {
            uint64_t v = 0;
            for (int i = 0; i < 32; ++i) v |= (uint64_t)((col[i] >> r) & 1u) << i;
            row[r] = v | ((uint64_t)((one >> r) & 1u) << 32);
        }
        for (int c = 0, r0 = 0; c < 32; ++c) {
            int piv = -1;
            for (int r = r0; r < 32; ++r)
                if ((row[r] >> c) & 1u) { piv = r; break; }
            if (piv < 0) continue;  // (x^8 is invertible modulo the CRC polynomial: never taken)
            const uint64_t t2 = row[piv]; row[piv] = row[r0]; row[r0] = t2;
            for (int r = 0; r < 32; ++r)
                if (r != r0 && ((row[r] >> c) & 1u)) row[r] ^= row[r0];
            ++r0;
        }
        uint32_t inv = 0;
        for (int r = 0; r < 32; ++r)
            for (int c = 0; c < 32; ++c)
                if ((row[r] >> c) & 1u) { inv |= (uint32_t)((row[r] >> 32) & 1u) << c; break; }
        t->XI[0] = one;
        for (int k = 1; k < 16; ++k) t->XI[k] = gf_multmodp(t->XI[k - 1], inv);
    }
}

int crc_tables_init() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return NX_ERR_HIP;
    std::lock_guard<std::mutex> lk(g_crc_mu);
    if (g_crc_dev[dev]) return NX_OK;
    std::vector<CrcTables> t(1);
    build_tables(t.data());
    CrcTables* d = nullptr;
    if (hipMalloc(&d, sizeof(CrcTables)) != hipSuccess) return NX_ERR_HIP;
    if (hipMemcpy(d, t.data(), sizeof(CrcTables), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return NX_ERR_HIP;
    }
    g_crc_dev[dev] = d;
    return NX_OK;
}

const CrcTables* crc_tables_dev() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_crc_mu);
    return g_crc_dev[dev];
}

uint32_t host_crc32c(const uint8_t* p, size_t n) {
    static std::once_flag once;
    std::call_once(once, [] {
        std::vector<CrcTables> t(1);
        build_tables(t.data());
    });
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) c = (c >> 8) ^ h_T0[(c ^ p[i]) & 0xFF];
    return ~c;
}

uint32_t host_mask(uint32_t c) { return mask_checksum(c); }

constexpr uint32_t kBlk = 8192;  // 64 lanes x 128 B

// slicing-by-8 step: state c (already XORed with the first word) and the second word w1
__device__ __forceinline__ uint32_t step8(const uint32_t* __restrict__ T, uint32_t c, uint32_t w1) {
    return T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^ T[4 * 256 + (c >> 24)] ^
           T[3 * 256 + (w1 & 0xFF)] ^ T[2 * 256 + ((w1 >> 8) & 0xFF)] ^ T[1 * 256 + ((w1 >> 16) & 0xFF)] ^ T[w1 >> 24];
}

__device__ __forceinline__ uint32_t shift_tab(const uint32_t* __restrict__ S, uint32_t c) {
    return S[c & 0xFF] ^ S[256 + ((c >> 8) & 0xFF)] ^ S[512 + ((c >> 16) & 0xFF)] ^ S[768 + (c >> 24)];
}

// Byte mask of the dword at real chunk position r0 (bytes r0..r0+3): bytes outside [0, L) cleared.
__device__ __forceinline__ uint32_t edge_mask(int64_t r0, uint32_t L) {
    uint32_t m = 0xFFFFFFFFu;
    if (r0 < 0) m = r0 <= -4 ? 0u : m << (8 * (uint32_t)(-r0));
    const int64_t over = r0 + 4 - (int64_t)L;
    if (over > 0) m &= over >= 4 ? 0u : (0xFFFFFFFFu >> (8 * (uint32_t)over));
    return m;
}
// Init fold: 0xFF on the bytes of this dword that are chunk bytes 0..3.
__device__ __forceinline__ uint32_t init_mask(int64_t r0) {
    if (r0 <= -4 || r0 >= 4) return 0u;
    return r0 >= 0 ? (0xFFFFFFFFu >> (8 * (uint32_t)r0)) : (0xFFFFFFFFu << (8 * (uint32_t)(-r0)));
}

// One lane slot of the virtual stream: 8 granules of 16 bytes at virtual position v (16-aligned);
// chunk byte i sits at virtual position i + z.  `edge`: the slot may hold bytes outside the chunk.
__device__ __forceinline__ void load_slot(const uint8_t* __restrict__ p, uint32_t L, uint32_t z, uint32_t v, bool edge, uint4 q[8]) {
    const int64_t r = (int64_t)v - (int64_t)z;  // real position of the slot's first byte
    if (!edge) {
#pragma unroll
        for (int g = 0; g < 8; ++g) q[g] = *reinterpret_cast<const uint4*>(p + r + 16 * g);
        return;
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const int64_t rg = r + 16 * g;
        // a granule holding at least one chunk byte is read whole (it cannot cross a page)
        q[g] = (rg + 16 > 0 && rg < (int64_t)L) ? *reinterpret_cast<const uint4*>(p + rg) : make_uint4(0, 0, 0, 0);
        q[g].x &= edge_mask(rg, L);
        q[g].y &= edge_mask(rg + 4, L);
        q[g].z &= edge_mask(rg + 8, L);
        q[g].w &= edge_mask(rg + 12, L);
        q[g].x ^= init_mask(rg);
        q[g].y ^= init_mask(rg + 4);
        q[g].z ^= init_mask(rg + 8);
        q[g].w ^= init_mask(rg + 12);
    }
}

__device__ __forceinline__ uint32_t raw128(const uint32_t* __restrict__ T, const uint4 q[8]) {
    uint32_t c = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        c = step8(T, c ^ q[g].x, q[g].y);
        c = step8(T, c ^ q[g].z, q[g].w);
    }
    return c;
}

// Masked CRC32C of chunk p[0..L) by one wave (result valid in every lane).  T = T8 (8 KiB), SH =
// SH[3..9] (shift by 128 B .. 8 KiB), both in LDS; XI from global memory.
__device__ uint32_t wave_crc32c(const uint32_t* __restrict__ T, const uint32_t* __restrict__ SH, const uint32_t* __restrict__ XI,
                                const uint8_t* __restrict__ p, uint32_t L, int lane) {
    if (L < 4) {  // the init fold needs four bytes: byte-serial (every lane computes the same)
        uint32_t c = 0xFFFFFFFFu;
        for (uint32_t i = 0; i < L; ++i) c = (c >> 8) ^ T[(c ^ p[i]) & 0xFF];
        return ~c;
    }
    const uint32_t k = (uint32_t)((16u - (((uintptr_t)p + L) & 15u)) & 15u);
    const uint32_t nb = (L + k + kBlk - 1) / kBlk;
    const uint32_t z = nb * kBlk - (L + k);
    // p - z is 16-byte aligned: virtual slot starts are multiples of 16
    uint32_t acc = 0;
    uint4 cur[8], nxt[8];
    const uint32_t v0 = 128u * (uint32_t)lane;
    // blocks that may hold bytes outside the chunk or chunk bytes 0..3 (which reach block 1 when z > 8188)
    auto edge = [&](uint32_t bb) { return bb == 0 || bb + 1 == nb || (bb == 1 && z + 4 > kBlk); };
    load_slot(p, L, z, v0, true, cur);
    for (uint32_t b = 0; b < nb; ++b) {
        if (b + 1 < nb) load_slot(p, L, z, (b + 1) * kBlk + v0, edge(b + 1), nxt);
        acc = shift_tab(SH + 6 * 1024, acc) ^ raw128(T, cur);
#pragma unroll
        for (int g = 0; g < 8; ++g) cur[g] = nxt[g];
    }
    // sum_l acc_l * x^(8*128*(63-l)): pair (lo, hi) at level j -> shift_{128*2^j}(lo) ^ hi
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t other = __shfl_xor(acc, 1 << j);
        const bool is_lo = ((lane >> j) & 1) == 0;
        acc = shift_tab(SH + j * 1024, is_lo ? acc : other) ^ (is_lo ? other : acc);
    }
    // raw(V) = raw(M') * x^(8k);  crc = ~raw(M')
    return ~(k ? gf_multmodp(XI[k], acc) : acc);
}

__global__ void __launch_bounds__(256) k_crc32c_masked(const uint8_t* __restrict__ in, const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, uint32_t* __restrict__ out,
                                                       uint32_t n, const CrcTables* __restrict__ tabs) {
    __shared__ uint32_t sT[8 * 256];
    __shared__ uint32_t sSH[7 * 1024];
    for (int i = threadIdx.x; i < 8 * 256; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
    for (int i = threadIdx.x; i < 7 * 1024; i += blockDim.x) sSH[i] = (&tabs->SH[3][0][0])[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t waves_per_block = blockDim.x / 64;
    for (uint32_t c = blockIdx.x * waves_per_block + (threadIdx.x >> 6); c < n; c += gridDim.x * waves_per_block) {
        const uint32_t crc = wave_crc32c(sT, sSH, tabs->XI, in + off[c], len[c], lane);
        if (lane == 0) out[c] = mask_checksum(crc);
    }
}

}  // namespace nx

using namespace nx;

extern "C" int32_t nx_crc32c_masked_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len,
                                          uint32_t* masked_out, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !off || !len || !masked_out) return NX_ERR_INVALID_ARG;
    if (crc_tables_init() != NX_OK) return NX_ERR_HIP;
    unsigned grid = n / 4 + 1;
    if (grid > 2048) grid = 2048;
    hipLaunchKernelGGL(k_crc32c_masked, dim3(grid), dim3(256), 0, (hipStream_t)stream, in, off, len, masked_out, n,
                       crc_tables_dev());
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
