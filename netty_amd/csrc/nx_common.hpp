// nx_common.hpp — shared device/host helpers for the gfx950 codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../include/netty_amd_status.h"

#define NX_WAVE 64

// A failing HIP call returns NX_ERR_HIP; with NX_HIP_DEBUG set in the environment the call site and
// HIP's error string go to stderr (diagnostics only).
#define NX_HIP_CHECK(x)                                                      \
    do {                                                                     \
        hipError_t _e = (x);                                                 \
        if (_e != hipSuccess) return nx_hip_fail(_e, __FILE__, __LINE__);    \
    } while (0)
// Launch checks read hipGetLastError(), which also returns an error any earlier HIP call of this
// thread left behind (an expected failure the caller already handled, a NotReady from a query):
// the kernel-launching entry points clear it first, so a check reports only their own launches.
#define NX_CLEAR_STALE_ERROR() ((void)hipGetLastError())
inline int32_t nx_hip_fail(hipError_t e, const char* file, int line) {
    static const bool dbg = getenv("NX_HIP_DEBUG") != nullptr;
    if (dbg) fprintf(stderr, "netty_amd: %s:%d: %s\n", file, line, hipGetErrorString(e));
    return NX_ERR_HIP;
}

namespace nx {

// CRC32C (Castagnoli, reflected poly 0x82F63B78) — Crc32c.java:27-124.
constexpr uint32_t kCrcPoly = 0x82F63B78u;

// Device-side CRC tables (filled once by crc_tables_init() on the host):
//   T8[k][b]   : slicing-by-8 tables, T8[0] = byte table of Crc32c.java:27-92
//   SH[j][k][b]: "shift by 16*2^j bytes" linear maps, j = 0..9 (16 B .. 8 KiB), byte k of the state
//   NS[j][k][v]: nibble form of "shift by 8*2^j bytes", j = 0..6 (8 B .. 512 B), nibble k of the state
//   XI[k]      : x^(-8k) mod P, k = 0..15 ("un-shift" by k zero bytes)
struct CrcTables {
    uint32_t T8[8][256];
    uint32_t SH[10][4][256];
    uint32_t NS[7][8][16];  // shift by 8 * 2^j bytes (j = 6: 512 B, the unit expander's 16-byte lane slots)
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
#ifndef NX_STAGE_UNIT  // build option for A/B runs (scripts/build_lib_variant.sh): 64 halves the LDS per block
#define NX_STAGE_UNIT 128
#endif
constexpr uint32_t kStageUnit = NX_STAGE_UNIT;
constexpr uint32_t kStageStride = kStageUnit + 4;  // bytes per lane slot: lanes' dwords on distinct banks
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

// Hash-table workspace placement (the lane-per-chunk encoders' per-lane tables).  How fast the memory
// system serves a lane's chain of random table exchanges depends on where the workspace landed: the
// Snappy encoder runs 260-274 or 330-345 ms per 262 144 chunks on the same box depending only on the
// placement of its 32 GiB workspace, and a 3-4 ms run of k_ws_probe — lane t: `steps` dependent
// exchanges at pseudo-random slots of its own table, the encoders' probe request without their
// compute — predicts which (profiles/r02/s3/placement_selection.log).
template <typename E>
__global__ void __launch_bounds__(256) k_ws_probe(E* __restrict__ ws, uint32_t per_lane, uint32_t lg, uint32_t steps) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    E* tab = ws + (size_t)t * per_lane;
    uint32_t h = t * 0x9E3779B9u + 1u;
    for (uint32_t i = 0; i < steps; ++i) {
        const E v = __hip_atomic_exchange(&tab[(h * 0x1e35a7bdu) >> (32u - lg)], (E)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h = h * 0x85EBCA77u + (uint32_t)v + i;
    }
}
constexpr size_t kPlaceMinBytes = (size_t)2 << 30;  // smaller workspaces (handler / batcher sizes): allocated directly
constexpr int kPlaceCandidates = 6;  // drawn at once (each while the others are held, so each lands elsewhere)
constexpr int kPlaceRounds = 4;      // draws; the best so far is held through the next draw
constexpr uint32_t kPlaceSteps = 256;
constexpr size_t kPlaceFreeReserve = (size_t)8 << 30;  // a candidate is drawn only while this much stays free

// Process-wide bound on the placement (nx_workspace_placement_config): the bytes the candidates of one
// workspace may hold at once (0: half of the device's memory; ~0: everything but kPlaceFreeReserve, the
// round-5 behaviour) and the candidates drawn in all (0: kPlaceCandidates * kPlaceRounds).  A server
// sharing its GPU keeps the default; a process that owns the device (bench.py) may lift it.
inline uint64_t& placement_peak_cap() {
    static uint64_t v = 0;
    return v;
}
inline int& placement_max_candidates() {
    static int v = 0;
    return v;
}

// Allocate a zeroed workspace of `lanes` tables of 2^lg entries each.  A large one is the fastest of
// kPlaceRounds draws of up to kPlaceCandidates allocations under k_ws_probe: within a draw the
// candidates stay allocated while the next is drawn, so each lands elsewhere; between draws all but
// the best so far are freed, and the next draw lands on other placements again (a box whose first six
// candidates were all slow, profiles/r03/s6, left the encoder ~4 % slower; scripts/experiments/
// placement_redraw.py shows later draws reaching the fast placements; round 4: a box whose twelve
// candidates in two draws held no fast one ran the encoder at 55.3 GiB/s against 57.0-57.8 elsewhere,
// profiles/r04/s5, so four draws of six).  A candidate is only drawn while kPlaceFreeReserve stays
// free and while the candidates held at once stay within placement_peak_cap() (round 6: by default
// half of the device, so reserving a workspace never takes all free HBM, even for a moment).
struct PlacementReport {
    int n = 0;      // candidates probed (0: allocated directly, below kPlaceMinBytes)
    int pick = -1;  // the one kept
    float ms[kPlaceCandidates * kPlaceRounds] = {};
    uint64_t peak = 0;  // most bytes the candidates held at once
};
template <typename E>
inline hipError_t alloc_placed_workspace(size_t lanes, uint32_t lg, hipStream_t st, E** out, PlacementReport* rep = nullptr) {
    const size_t bytes = lanes * ((size_t)sizeof(E) << lg);
    *out = nullptr;
    if (bytes < kPlaceMinBytes || lanes % 256 != 0) {
        hipError_t e = hipMalloc(out, bytes);
        if (e == hipSuccess) e = hipMemsetAsync(*out, 0, bytes, st);
        if (e == hipSuccess && rep) {
            *rep = PlacementReport{};
            rep->peak = bytes;
        }
        return e;
    }
    uint64_t peak_cap = placement_peak_cap();
    if (peak_cap == 0) {
        size_t free_b = 0, total_b = 0;
        peak_cap = hipMemGetInfo(&free_b, &total_b) == hipSuccess ? total_b / 2 : 4 * (uint64_t)bytes;
    }
    const int max_cand = placement_max_candidates() > 0 ? placement_max_candidates() : kPlaceCandidates * kPlaceRounds;
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e = hipEventCreate(&a);
    if (e == hipSuccess) e = hipEventCreate(&b);
    E* best_p = nullptr;
    float best_ms = 3.4e38f;
    int n_all = 0, pick = -1;
    uint64_t peak = 0;
    float all_ms[kPlaceCandidates * kPlaceRounds];
    for (int round = 0; round < kPlaceRounds && e == hipSuccess && n_all < max_cand; ++round) {
        E* cand[kPlaceCandidates];
        float ms[kPlaceCandidates];
        int nc = 0;
        uint64_t held = best_p ? (uint64_t)bytes : 0;
        while (nc < kPlaceCandidates && n_all + nc < max_cand && e == hipSuccess) {
            size_t free_b = 0, total_b = 0;
            if ((nc > 0 || best_p) &&
                (held + bytes > peak_cap || hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < bytes + kPlaceFreeReserve))
                break;
            E* p = nullptr;
            if (hipMalloc(&p, bytes) != hipSuccess) {
                (void)hipGetLastError();  // no memory for another candidate: choose among those drawn
                break;
            }
            held += bytes;
            if (held > peak) peak = held;
            cand[nc] = p;
            ms[nc] = 3.4e38f;
            ++nc;
            e = hipMemsetAsync(p, 0, bytes, st);  // first touch outside the timed probe
            if (e == hipSuccess) e = hipEventRecord(a, st);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_ws_probe<E>, dim3((unsigned)(lanes / 256)), dim3(256), 0, st, p, 1u << lg, lg, kPlaceSteps);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipEventRecord(b, st);
            if (e == hipSuccess) e = hipEventSynchronize(b);
            if (e == hipSuccess) e = hipEventElapsedTime(&ms[nc - 1], a, b);
        }
        for (int k = 0; k < nc; ++k) {
            all_ms[n_all] = ms[k];
            if (e == hipSuccess && ms[k] < best_ms) {
                if (best_p) (void)hipFree(best_p);
                best_p = cand[k];
                best_ms = ms[k];
                pick = n_all;
            } else {
                (void)hipFree(cand[k]);
            }
            ++n_all;
        }
        if (nc == 0) break;  // no memory for another draw
    }
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (e != hipSuccess) {
        if (best_p) (void)hipFree(best_p);
        return e;
    }
    if (!best_p) return hipErrorOutOfMemory;
    *out = best_p;
    if (rep) {
        rep->n = n_all;
        rep->pick = pick;
        for (int k = 0; k < n_all; ++k) rep->ms[k] = all_ms[k];
        rep->peak = peak;
    }
    return hipMemsetAsync(*out, 0, bytes, st);  // the probe wrote entries: back to a zeroed table
}

// Kernel launch helper: grid-stride sizes.
inline unsigned grid_for(uint64_t threads, unsigned block) {
    uint64_t g = (threads + block - 1) / block;
    if (g > 65535u * 16u) g = 65535u * 16u;
    return (unsigned)(g ? g : 1);
}

}  // namespace nx
