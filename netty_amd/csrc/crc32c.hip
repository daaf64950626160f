// crc32c.hip — CRC32C tables + the batched masked-CRC kernel.
//
// Replaces Crc32c.update/getValue (Crc32c.java:97-124) + Snappy.maskChecksum (Snappy.java:720-722)
// as called by Snappy.calculateChecksum (Snappy.java:668-676), one wave per chunk.
//
// Layout: the chunk is swept in 1 KiB blocks; lane l takes bytes [16l, 16l+16) of a block with one
// coalesced 16-byte load, computes their raw CRC with slicing-by-8 (two steps), and the 64 lane
// values are folded pairwise in a 6-level tree with the "shift by 16*2^j bytes" tables (CRC is
// linear over GF(2): raw(A||B) = raw(A)*x^(8|B|) ^ raw(B)).  The running state is shifted by
// 1 KiB per block.  The tail (< 1 KiB) goes through the same tree with zero-padded lanes and a
// final un-shift by the pad length.
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
    for (int j = 0; j < 7; ++j) {
        uint32_t K = gf_x8n(16ull << j);
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) t->SH[j][k][b] = gf_multmodp(K, b << (8 * k));
    }
    for (int j = 0; j < 6; ++j) {
        uint32_t K = gf_x8n(8ull << j);
        for (int k = 0; k < 8; ++k)
            for (uint32_t v = 0; v < 16; ++v) t->NS[j][k][v] = gf_multmodp(K, v << (4 * k));
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

// raw CRC (state 0) of 16 bytes held as 4 LE dwords, slicing-by-8 twice.
__device__ inline uint32_t raw16(const uint32_t* __restrict__ T, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    // T = flattened T8[8][256]
    uint32_t c = w0;
    c = T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^ T[4 * 256 + (c >> 24)] ^
        T[3 * 256 + (w1 & 0xFF)] ^ T[2 * 256 + ((w1 >> 8) & 0xFF)] ^ T[1 * 256 + ((w1 >> 16) & 0xFF)] ^ T[0 * 256 + (w1 >> 24)];
    c ^= w2;
    c = T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^ T[4 * 256 + (c >> 24)] ^
        T[3 * 256 + (w3 & 0xFF)] ^ T[2 * 256 + ((w3 >> 8) & 0xFF)] ^ T[1 * 256 + ((w3 >> 16) & 0xFF)] ^ T[0 * 256 + (w3 >> 24)];
    return c;
}

__device__ inline uint32_t shift_tab(const uint32_t* __restrict__ S, uint32_t c) {
    return S[c & 0xFF] ^ S[256 + ((c >> 8) & 0xFF)] ^ S[512 + ((c >> 16) & 0xFF)] ^ S[768 + (c >> 24)];
}

// Fold the 64 per-lane raw CRCs (lane l covers bytes [16l,16l+16) of a 1 KiB block) into the
// block's raw CRC.  Result valid in every lane.
__device__ inline uint32_t fold_block(const uint32_t* __restrict__ SH, uint32_t c, int lane) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        uint32_t other = __shfl_xor(c, 1 << j);
        // pair (lo, hi): combined = shift_{16*2^j}(lo) ^ hi
        bool is_lo = ((lane >> j) & 1) == 0;
        uint32_t lo = is_lo ? c : other;
        uint32_t hi = is_lo ? other : c;
        c = shift_tab(SH + j * 1024, lo) ^ hi;
    }
    return c;
}

// Wave-cooperative raw-CRC update of state `st` over bytes p[0..len) (p may be unaligned).
__device__ uint32_t wave_crc_update(const uint32_t* __restrict__ T, const uint32_t* __restrict__ SH, uint32_t st,
                                    const uint8_t* __restrict__ p, uint32_t len, int lane) {
    uint32_t pos = 0;
    const bool aligned = (((uintptr_t)p) & 3) == 0;
    while (pos + 1024 <= len) {
        const uint8_t* q = p + pos + 16 * lane;
        uint32_t w0, w1, w2, w3;
        if (aligned) {
            const uint32_t* q4 = (const uint32_t*)q;
            w0 = q4[0]; w1 = q4[1]; w2 = q4[2]; w3 = q4[3];
        } else {
            // aligned dword loads, words cut out with alignbyte: the fifth dword holds byte q[15]
            // (sb >= 1), so no load leaves the chunk's last dword
            const uint32_t sb = (uint32_t)((uintptr_t)q & 3u);
            const uint32_t* q4 = (const uint32_t*)(q - sb);
            const uint32_t d0 = q4[0], d1 = q4[1], d2 = q4[2], d3 = q4[3], d4 = q4[4];
            w0 = __builtin_amdgcn_alignbyte(d1, d0, sb);
            w1 = __builtin_amdgcn_alignbyte(d2, d1, sb);
            w2 = __builtin_amdgcn_alignbyte(d3, d2, sb);
            w3 = __builtin_amdgcn_alignbyte(d4, d3, sb);
        }
        uint32_t c = raw16(T, w0, w1, w2, w3);
        c = fold_block(SH, c, lane);
        st = shift_tab(SH + 6 * 1024, st) ^ c;
        pos += 1024;
    }
    uint32_t rem = len - pos;
    if (rem) {
        // byte-serial per lane over its (possibly partial) 16-byte slot, then tree fold of the
        // zero-padded 1 KiB block, then "un-pad": raw(block_padded) = raw(tail) * x^(8*pad).
        // Instead of dividing, fold lanes with an explicit shift by the bytes that follow each
        // lane's slot inside the tail.
        uint32_t b0 = 16u * lane;
        uint32_t c = 0;
        uint32_t end = b0 + 16 < rem ? b0 + 16 : rem;
        for (uint32_t i = b0; i < end; ++i) c = (c >> 8) ^ T[(c ^ p[pos + i]) & 0xFF];
        uint32_t after = end > b0 ? rem - end : 0;
        c = end > b0 ? gf_multmodp(gf_x8n(after), c) : 0u;
        // XOR-reduce
#pragma unroll
        for (int j = 0; j < 6; ++j) c ^= __shfl_xor(c, 1 << j);
        st = gf_multmodp(gf_x8n(rem), st) ^ c;
    }
    return st;
}

__global__ void __launch_bounds__(256) k_crc32c_masked(const uint8_t* __restrict__ in, const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, uint32_t* __restrict__ out,
                                                       uint32_t n, const CrcTables* __restrict__ tabs) {
    __shared__ uint32_t sT[8 * 256];
    __shared__ uint32_t sSH[7 * 1024];
    for (int i = threadIdx.x; i < 8 * 256; i += blockDim.x) sT[i] = (&tabs->T8[0][0])[i];
    for (int i = threadIdx.x; i < 7 * 1024; i += blockDim.x) sSH[i] = (&tabs->SH[0][0][0])[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t waves_per_block = blockDim.x / 64;
    for (uint32_t c = blockIdx.x * waves_per_block + (threadIdx.x >> 6); c < n; c += gridDim.x * waves_per_block) {
        uint32_t st = wave_crc_update(sT, sSH, 0xFFFFFFFFu, in + off[c], len[c], lane);
        if (lane == 0) out[c] = mask_checksum(~st);
    }
}

}  // namespace nx

using namespace nx;

extern "C" int32_t nx_crc32c_masked_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len,
                                          uint32_t* masked_out, uint32_t n, void* stream) {
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
