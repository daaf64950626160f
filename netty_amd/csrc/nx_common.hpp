// nx_common.hpp — shared device/host helpers for the gfx950 codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/netty_amd_status.h"

#define NX_WAVE 64

#define NX_HIP_CHECK(x)                                  \
    do {                                                 \
        hipError_t _e = (x);                             \
        if (_e != hipSuccess) return NX_ERR_HIP;         \
    } while (0)

namespace nx {

// CRC32C (Castagnoli, reflected poly 0x82F63B78) — Crc32c.java:27-124.
constexpr uint32_t kCrcPoly = 0x82F63B78u;

// Device-side CRC tables (filled once by crc_tables_init() on the host):
//   T8[k][b]   : slicing-by-8 tables, T8[0] = byte table of Crc32c.java:27-92
//   SH[j][k][b]: "shift by 16*2^j bytes" linear maps, j = 0..9 (16 B .. 8 KiB), byte k of the state
//   NS[j][k][v]: nibble form of "shift by 8*2^j bytes", j = 0..5 (8 B .. 256 B), nibble k of the state
//   XI[k]      : x^(-8k) mod P, k = 0..15 ("un-shift" by k zero bytes)
struct CrcTables {
    uint32_t T8[8][256];
    uint32_t SH[10][4][256];
    uint32_t NS[6][8][16];
    uint32_t XI[16];
};
// Device copy of the tables, allocated once per device by crc_tables_init() (kernels take the
// pointer as an argument: no cross-TU device symbols, so no -fgpu-rdc).
int crc_tables_init();                 // host: build + upload (idempotent). Returns NX_OK / NX_ERR_HIP.
const CrcTables* crc_tables_dev();     // device pointer for the current device
// host helpers (also used by the host handler layer)
uint32_t host_crc32c(const uint8_t* p, size_t n);
uint32_t host_mask(uint32_t c);

__host__ __device__ inline uint32_t mask_checksum(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// GF(2) multiply modulo P in CRC (reflected) representation (zlib multmodp).
__host__ __device__ inline uint32_t gf_multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; ++i) {
        p ^= (a & 0x80000000u) ? b : 0u;
        a <<= 1;
        b = (b & 1u) ? ((b >> 1) ^ kCrcPoly) : (b >> 1);
    }
    return p;
}

// x^(8n) mod P (reflected), by square-and-multiply.
__host__ __device__ inline uint32_t gf_x8n(uint64_t n) {
    uint32_t result = 0x80000000u;  // x^0
    uint32_t sq = 0x00800000u;      // x^8
    while (n) {
        if (n & 1) result = gf_multmodp(sq, result);
        sq = gf_multmodp(sq, sq);
        n >>= 1;
    }
    return result;
}

// Lane-per-chunk encoders (LZ4, FastLZ, LZF; Snappy has its own three forms): the dense form gives
// every lane a chunk; for batches up to kSpreadMaxChunks the SPREAD form gives each wave one chunk
// on lane 0, so the serial matchers of different chunks never share a wave's divergent control
// flow (64 divergent matchers in one wave run ~6x longer than one).  Table slot = lane or wave.
constexpr uint32_t kSpreadMaxChunks = 16384;
template <bool SPREAD>
__device__ __forceinline__ bool chunk_slot(uint32_t& slot, uint32_t& slots) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, t = gridDim.x * blockDim.x;
    slot = SPREAD ? g >> 6 : g;
    slots = SPREAD ? t >> 6 : t;
    return !SPREAD || (g & 63u) == 0u;
}
struct LaneGrid {
    bool spread;
    size_t slots;  // table slots the launch uses (lanes or waves)
    unsigned grid, block;
};
inline LaneGrid lane_grid(uint32_t n, int cus, unsigned waves_per_cu) {
    LaneGrid g;
    g.spread = n <= kSpreadMaxChunks;
    const size_t want = (size_t)cus * waves_per_cu * (g.spread ? 1u : 64u);
    g.slots = n < want ? (g.spread ? (size_t)n : ((size_t)n + 255) / 256 * 256) : want;
    g.block = g.spread ? 64u : 256u;
    g.grid = (unsigned)(g.spread ? g.slots : g.slots / 256);
    return g;
}

// Output of the byte-writing lane-per-chunk encoders (LZ4, FastLZ, LZF).  A lane's scattered byte
// stores are partial-line writes the L2 has usually evicted before the lane's next byte comes, so
// every one costs a line merge / write-back; the dense forms therefore stage the 128-byte-aligned
// unit of the destination being written in the lane's own LDS slot and store it as eight 16-byte
// writes when the lane moves past it (Snappy's WriterL does the same with dwords).  Positions are
// relative to the chunk's output start; writes are sequential except for back-patches (token,
// literal-run count), which land in LDS while their unit is staged and in global memory after.
// GOut is the plain global form (small-batch forms, large LZ4 blocks).
constexpr uint32_t kStageUnit = 128;
constexpr uint32_t kStageStride = 132;  // bytes per lane slot: 33 dwords, lanes' dwords on distinct banks
struct GOut {
    uint8_t* p;
    __device__ __forceinline__ void set(int32_t pos, uint32_t v) { p[pos] = (uint8_t)v; }
    __device__ __forceinline__ uint32_t get(int32_t pos) const { return p[pos]; }
    __device__ __forceinline__ void finish(int32_t) {}
};
// UNIT-byte units (64 or 128) in a lane slot of UNIT + 4 bytes
template <uint32_t UNIT>
struct ByteStageT {
    uint8_t* st;   // the lane's LDS slot
    uint8_t* dst;  // output byte 0
    int32_t u0;    // position of the staged unit's byte 0 (negative for the first, partial unit)
    __device__ __forceinline__ ByteStageT(uint8_t* slot, uint8_t* out)
        : st(slot), dst(out), u0(-(int32_t)((uintptr_t)out & (UNIT - 1))) {}
    __device__ __forceinline__ void flush_unit() {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(st);
        if (u0 >= 0) {
            uint4* g = reinterpret_cast<uint4*>(dst + u0);
#pragma unroll
            for (int q = 0; q < (int)UNIT / 16; ++q) g[q] = make_uint4(s32[4 * q], s32[4 * q + 1], s32[4 * q + 2], s32[4 * q + 3]);
        } else {
            for (int32_t j = -u0; j < (int32_t)UNIT; ++j) dst[u0 + j] = st[j];
        }
        u0 += (int32_t)UNIT;
    }
    __device__ __forceinline__ void set(int32_t pos, uint32_t v) {
        while (pos >= u0 + (int32_t)UNIT) flush_unit();
        if (pos >= u0)
            st[pos - u0] = (uint8_t)v;
        else
            dst[pos] = (uint8_t)v;
    }
    __device__ __forceinline__ uint32_t get(int32_t pos) const { return pos >= u0 ? st[pos - u0] : dst[pos]; }
    // store the staged bytes [u0, end)
    __device__ __forceinline__ void finish(int32_t end) {
        int32_t j = u0 < 0 ? -u0 : 0;
        if (u0 >= 0) {
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(st);
            for (; j + 16 <= end - u0; j += 16)
                *reinterpret_cast<uint4*>(dst + u0 + j) = make_uint4(s32[j / 4], s32[j / 4 + 1], s32[j / 4 + 2], s32[j / 4 + 3]);
        }
        for (; j < end - u0; ++j) dst[u0 + j] = st[j];
    }
};
using ByteStage = ByteStageT<kStageUnit>;

// Kernel launch helper: grid-stride sizes.
inline unsigned grid_for(uint64_t threads, unsigned block) {
    uint64_t g = (threads + block - 1) / block;
    if (g > 65535u * 16u) g = 65535u * 16u;
    return (unsigned)(g ? g : 1);
}

}  // namespace nx
