// batcher.cpp — asynchronous, cross-channel batching executor for the Snappy frame handlers.
//
// Netty runs one SnappyFrameEncoder / SnappyFrameDecoder per channel on that channel's event loop
// (ByteToMessageDecoder.java:194-196) and the event loop must not block (BlockHound,
// common/.../internal/Hidden.java:38).  One encode()/decode() call carries ~1-33 chunks, far too few
// to fill an MI355X, so the batcher turns those calls into jobs of one shared GPU launch:
//
//   submit  (event loop, non-blocking)  the handler's framing runs on the host at once — the stream
//           identifier and slice split of SnappyFrameEncoder.encode (SnappyFrameEncoder.java:79-117),
//           the chunk-header walk of SnappyFrameDecoder.decode (:85-231) — so the handle's state
//           advances in call order; the chunk payloads are copied into a pinned staging arena
//           (MessageToByteEncoder releases `in` when encode() returns, :109), or, for an encoder input
//           the caller registered with nx_host_register and keeps alive, DMA'd straight from it.
//   flush   the staging arena and registered inputs to the device (one gather launch reading the
//           mapped pages; a large staging arena by one DMA copy), then ONE launch per kernel for every
//           job of every channel: CRC32C + Snappy.encode of all encoder slices, Snappy.decode (+ CRC
//           verify) of all compressed chunks, CRC32C of uncompressed chunks, and a finish kernel that
//           writes each job's result — framed encoder output, or the decoder's messages — straight
//           into mapped pinned host memory, or into a device mirror moved by one DMA copy when the
//           decoded messages fill most of a large result arena (only result bytes cross PCIe).
//   poll    hipEventQuery: 1 when the job's batch is done (never blocks); wait() blocks (tests).
//   streams flushes go round-robin to kStreams HIP streams, so one batch's host gather / result
//           writes (PCIe) overlap the next batch's kernels; results are still APPLIED in flush order
//           (a later batch waits for the earlier ones), which keeps each decoder's corrupted state
//           exactly as a serial execution would leave it.  An optional auto-flush threshold
//           (nx_batcher_set_flush_bytes) launches the collecting batch once its input reaches it.
//   result  zero-copy views of the job's output in the pinned arena, valid until release().
//
// Results are applied in submission order per decoder: a failing chunk marks the decoder corrupted
// (:227-230) and the jobs submitted after it on that decoder deliver nothing (Java skips all later
// input, :86-89).  A validating decoder's compressed chunk that decodes fewer bytes than its length
// leaves the rest to be parsed again as a chunk header (:206-212); that is known only at apply().  So a
// validating decoder keeps the bytes its unapplied jobs walked (and any partial chunk after them, which
// it carries into the next submit instead of leaving it in the caller's cumulation), and apply() walks
// them again from the leftover: the job continues in the collecting batch (launched by the next
// poll/wait) with the messages it has so far, and the decoder's jobs walked before that deliver
// nothing (their bytes are in the continuation).  Messages and errors equal the synchronous
// nx_snappy_frame_decoder_decode's, in the same order; they may arrive on an earlier ticket.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>
#include "../../include/netty_amd.h"
#include "frame_parse.hpp"
#include "handles.hpp"
#include "alt_frames.hpp"
#include "nx_common.hpp"
#include "workspace.hpp"

namespace nx {
namespace bt {

struct EncSlice {  // one SnappyFrameEncoder slice (:99-112) or the small-message unencoded chunk (:114-124)
    uint64_t in_off;
    uint64_t slot_off;
    uint32_t len;
    uint32_t comp;
};
struct EncJob {
    uint64_t out_off;  // in the mapped output arena
    uint32_t s0, ns;   // slices
    uint32_t stream_start;
    uint32_t pad;
};
struct DecAct {  // one UNCOMPRESSED_DATA (kind 1) or COMPRESSED_DATA (kind 2) chunk, in stream order
    uint64_t in_off;  // payload in the device input arena
    uint32_t len;     // payload bytes
    uint32_t kind;
    uint32_t chunk;   // kind 2: index into the decode batch; kind 1: index into the uncompressed-CRC batch
    uint32_t crc;     // stored masked CRC32C
    uint32_t cap;     // bytes reserved for its message: kind 2 the preamble's length (capped by the bound)
    uint32_t pad;
};
constexpr uint64_t kSpilled = ~0ull;  // DecRes::off of a message longer than its chunk's preamble said that
                                      // did not fit the flush's spill area (apply copies it from the slot)
constexpr uint64_t kSpillBytes = 1ull << 20;  // a flush's spill area (bytes; at most 64 KiB per compressed chunk)
struct DecJob {
    uint64_t out_off;
    uint32_t a0, na;
    uint32_t validate;
    uint32_t pad;
};
struct DecRes {  // per action, written by k_dec_finish
    uint64_t off;    // message bytes in the output arena
    uint32_t len;
    int32_t status;  // NX_OK or the chunk's error
    uint32_t crc;    // computed masked CRC32C (uncompressed chunks; compressed: see decode crc_out)
    uint32_t cons;   // compressed: input bytes consumed
};

// Copy n bytes device -> mapped host with the whole wave: 16-byte stores at 16-byte-aligned
// destinations (one PCIe write per lane), bytes at the ragged ends.
//
// The kernels that move bytes across PCIe (k_gather_host reads mapped host pages, the finish kernels
// write the results into them) run on a capped grid, kPcieBlocks workgroups looping over the jobs:
// their speed is the link's, not the CUs', and a grid of one wave per job held every CU for the
// whole transfer, so the next batch's parse / expand / encode on another stream could not start
// (round 4 e2e trace: k_parse 5.9 ms alone, 17-23 ms beside a full-grid k_dec_finish).
#ifndef NX_PCIE_BLOCKS
#define NX_PCIE_BLOCKS 64
#endif
constexpr uint32_t kPcieBlocks = NX_PCIE_BLOCKS;
constexpr uint64_t kDmaOutMin = 64ull << 20;  // launch_inner: result arenas at least this large may go by DMA
constexpr uint64_t kGatherStageMax = 8ull << 20;  // launch_inner: staging arenas up to this size move by k_gather_host
constexpr uint64_t kGatherPiece = 64ull << 10;    // ... in ops of this many bytes
inline dim3 pcie_grid(uint32_t jobs) { return dim3(std::min((jobs + 3u) / 4u, kPcieBlocks)); }
__device__ void wave_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t n, int lane) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    typedef v4 __attribute__((aligned(1))) v4u;
    const uint32_t head = (uint32_t)((16u - ((uintptr_t)dst & 15u)) & 15u) < n ? (uint32_t)((16u - ((uintptr_t)dst & 15u)) & 15u) : n;
    if ((uint32_t)lane < head) dst[lane] = src[lane];
    const uint32_t nv = (n - head) >> 4;
    uint32_t i = lane;
    for (; i + 192u < nv; i += 256u) {  // 4 KiB per wave per step: four loads in flight, then four stores
        v4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const v4u*>(src + head + 16u * (i + 64u * u));
#pragma unroll
        for (int u = 0; u < 4; ++u) *reinterpret_cast<v4*>(dst + head + 16u * (i + 64u * u)) = x[u];
    }
    for (; i < nv; i += 64u) *reinterpret_cast<v4*>(dst + head + 16u * i) = *reinterpret_cast<const v4u*>(src + head + 16u * i);
    const uint32_t t = head + (nv << 4);
    if (t + (uint32_t)lane < n) dst[t + lane] = src[t + lane];
}

// Registered host inputs -> the device input arena: one wave per input range, 16-byte loads from the
// mapped host pages (one launch instead of one DMA command per pooled-buffer message).
struct GatherOp {
    const uint8_t* src;  // device address of registered host memory
    uint64_t dst;        // offset in the device input arena
    uint64_t len;
};
__global__ void __launch_bounds__(256) k_gather_host(const GatherOp* __restrict__ ops, uint32_t n, uint8_t* __restrict__ din) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    typedef v4 __attribute__((aligned(1))) v4u;
    const int lane = threadIdx.x & 63;
    for (uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += gridDim.x * 4) {
        const GatherOp g = ops[k];
        uint8_t* d = din + g.dst;  // 16-byte aligned
        const uint64_t nv = g.len >> 4;
        uint64_t i = lane;
        for (; i + 192u < nv; i += 256u) {  // four PCIe reads per lane in flight
            v4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const v4u*>(g.src + 16 * (i + 64u * u));
#pragma unroll
            for (int u = 0; u < 4; ++u) *reinterpret_cast<v4*>(d + 16 * (i + 64u * u)) = x[u];
        }
        for (; i < nv; i += 64) *reinterpret_cast<v4*>(d + 16 * i) = *reinterpret_cast<const v4u*>(g.src + 16 * i);
        for (uint64_t q = (nv << 4) + lane; q < g.len; q += 64) d[q] = g.src[q];
    }
}

// one wave per encoder job: [stream identifier] then [type][len+4: u24 LE][masked crc LE][payload] per slice
// res_len[j]: the job's framed bytes, or (negative) the Snappy.encode status of its first failing slice
__global__ void __launch_bounds__(256) k_enc_finish(const uint8_t* __restrict__ din, const uint8_t* __restrict__ slots,
                                                    const EncSlice* __restrict__ sl, const uint32_t* __restrict__ clen,
                                                    const int32_t* __restrict__ est, const uint32_t* __restrict__ crc,
                                                    const EncJob* __restrict__ jobs, uint32_t njobs, uint8_t* __restrict__ out,
                                                    int64_t* __restrict__ res_len) {
    const int lane = threadIdx.x & 63;
    for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < njobs; j += gridDim.x * 4) [&] {
        const EncJob J = jobs[j];
        for (uint32_t s = J.s0; s < J.s0 + J.ns; ++s) {
            if (sl[s].comp && est[s] != NX_OK) {
                if (lane == 0) res_len[j] = est[s];
                return;
            }
        }
        uint8_t* o = out + J.out_off;
        uint64_t pos = 0;
        if (J.stream_start) {  // ff 06 00 00 "sNaPpY" (SnappyFrameEncoder.java:52-54)
            const uint64_t v = lane < 8 ? (0x50614e73000006ffull >> (8 * lane)) : (0x5970ull >> (8 * (lane - 8)));  // LE bytes
            if (lane < 10) o[lane] = (uint8_t)v;
            pos = 10;
        }
        for (uint32_t s = J.s0; s < J.s0 + J.ns; ++s) {
            const EncSlice S = sl[s];
            const uint32_t L = S.comp ? clen[s] : S.len;
            const uint32_t cl = L + 4;  // setChunkLength (:126-132) / writeUnencodedChunk (:119-124)
            const uint32_t c = crc[s];
            if (lane < 8) {
                const uint32_t b = lane == 0 ? (S.comp ? 0u : 1u) : lane < 4 ? (cl >> (8 * (lane - 1))) & 0xFF : (c >> (8 * (lane - 4))) & 0xFF;
                o[pos + lane] = (uint8_t)b;
            }
            wave_copy(o + pos + 8, S.comp ? slots + S.slot_off : din + S.in_off, L, lane);
            pos += 8 + L;
        }
        if (lane == 0) res_len[j] = (int64_t)pos;
    }();
}

// Bytes a Snappy block of clen bytes can decode to: at most 64 per 3 input bytes (a copy-2 tag; a
// copy-1 gives 11 per 2, a copy-4 64 per 5, a literal its own length), and never more than the frame
// decoder's 65536-byte buffer (SnappyFrameDecoder.java:203).  Sizes the decode slots and the job's
// output reservation, so a flush of many small chunks does not take 64 KiB for each.
__host__ __device__ inline uint32_t snappy_decoded_bound(uint32_t clen) {
    const uint64_t b = 64ull * ((clen + 2ull) / 3ull);
    return b < 65536u ? (uint32_t)b : 65536u;
}
inline uint64_t dec_slot_bytes(uint32_t clen) { return ((uint64_t)snappy_decoded_bound(clen) + 64u + 15u) & ~15ull; }

// one wave per decoder job: the decoded messages back to back, stopping at the first failing chunk
__global__ void __launch_bounds__(256) k_dec_finish(const uint8_t* __restrict__ din, const uint8_t* __restrict__ slots,
                                                    const uint64_t* __restrict__ dslot,
                                                    const DecAct* __restrict__ acts, const DecJob* __restrict__ jobs, uint32_t njobs,
                                                    const uint32_t* __restrict__ dlen, const uint32_t* __restrict__ dcons,
                                                    const int32_t* __restrict__ dstat, const uint32_t* __restrict__ dcrc,
                                                    const uint32_t* __restrict__ ucrc, uint8_t* __restrict__ out,
                                                    DecRes* __restrict__ res, uint64_t spill_off, uint32_t spill_cap,
                                                    uint32_t* __restrict__ spill_cur) {
    const int lane = threadIdx.x & 63;
    for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < njobs; j += gridDim.x * 4) [&] {
        const DecJob J = jobs[j];
        uint64_t pos = J.out_off;
        for (uint32_t a = J.a0; a < J.a0 + J.na; ++a) {
            const DecAct A = acts[a];
            DecRes R{pos, 0, NX_OK, 0, 0};
            if (A.kind == 1) {
                R.crc = ucrc[A.chunk];
                R.len = A.len;
                if (J.validate && R.crc != A.crc) R.status = NX_ERR_SNAPPY_CRC_MISMATCH;  // (:171-175)
                else wave_copy(out + pos, din + A.in_off, A.len, lane);
            } else {
                R.status = dstat[A.chunk];
                // the decode launch verifies CRCs when any decoder of the batch validates; a decoder
                // built without validateChecksums ignores them (:205-216)
                if (R.status == NX_ERR_SNAPPY_CRC_MISMATCH && !J.validate) R.status = NX_OK;
                R.len = dlen[A.chunk];
                R.crc = dcrc[A.chunk];
                R.cons = dcons[A.chunk];
                if (R.status == NX_ERR_SNAPPY_LITERAL_LEN_INVALID && R.cons >= 4u) {  // the literal's length field, for the message
                    const uint8_t* f = din + A.in_off + R.cons - 4u;
                    R.crc = f[0] | (f[1] << 8) | (f[2] << 16) | ((uint32_t)f[3] << 24);
                }
                // a chunk that decodes past its preamble's length (Java allows it up to 65 536 bytes,
                // SnappyFrameDecoder.java:203) has no room here: it goes to the flush's spill area, or,
                // when that is full, apply() copies it from the slot
                if (R.status == NX_OK && R.len > A.cap) {
                    uint32_t at = 0;
                    if (lane == 0) at = atomicAdd(spill_cur, R.len);
                    at = (uint32_t)__shfl((int)at, 0);
                    if ((uint64_t)at + R.len <= spill_cap) {
                        R.off = spill_off + at;
                        wave_copy(out + R.off, slots + dslot[A.chunk], R.len, lane);
                    } else {
                        R.off = kSpilled;
                    }
                    if (lane == 0) res[a] = R;
                    continue;  // the message reservation holds nothing of it: pos stays
                } else if (R.status == NX_OK) {
                    wave_copy(out + pos, slots + dslot[A.chunk], R.len, lane);
                }
            }
            if (lane == 0) res[a] = R;
            if (R.status != NX_OK) break;
            pos += R.len;
        }
    }();
}

// ---------------------------------------------------------------- FastLZ / LZF / LZ4 jobs
// An alt-codec job's output is a list of PIECES in stream order: for an encoder one framed block each
// (written back to back into the job's output), for a decoder one block's message each.  The codec
// kernels of the flush leave their results in the alt slots and result arrays; k_alt_finish (one wave
// per job) writes each piece into mapped host memory and records where it went.
enum : uint32_t {
    AK_FLZ_ENC = 1,  // FastLzFrameEncoder block (:115-168): header, then compressed (slot) or raw (input) bytes
    AK_LZF_ENC,      // a complete "ZV" block from the LZF encoder (slot)
    AK_LZF_RAW,      // a non-compressed "ZV" block (encodeNonCompress, LzfEncoder.java:223-246)
    AK_LZ4_ENC,      // a framed block from the LZ4 frame encoder (slot; header included)
    AK_LZ4_END,      // Lz4FrameEncoder's end block (:326-335)
    AK_RAW,          // input bytes as they are (Lz4FrameEncoder after close(), :233-239)
    AK_DEC_FLZ,      // a FastLZ block decoded into its slot
    AK_DEC_LZF,      // an LZF block decoded into its slot
    AK_DEC_LZ4,      // an LZ4 block decoded into its slot
    AK_DEC_RAW,      // a non-compressed block: its payload (input)
};
struct AltPiece {
    uint64_t src;   // input arena offset of the raw bytes / payload
    uint64_t slot;  // alt slot offset of the codec's output
    uint32_t len;   // input bytes
    uint32_t olen;  // decoder: decoded bytes
    uint32_t kind;
    uint32_t res;   // index into the codec's result arrays
    uint32_t aux;   // AK_FLZ_ENC: bit 0 = with Adler32; AK_LZ4_END: compression level
    uint32_t pad;
};
struct AltJobD {
    uint64_t out_off;  // in the mapped output arena
    uint32_t p0, np;   // pieces
};
struct AltRes {  // per piece
    uint64_t off;    // bytes in the output arena
    uint32_t len;    // AK_DEC_FLZ failing: decompress()'s return value
    int32_t status;  // NX_OK, or the codec status
    uint32_t cks;    // decoder pieces with a checksum: Adler32 / XXH32 of the block's bytes
    uint32_t pad;
};
struct AltArrays {  // the flush's codec result arrays (device)
    const uint32_t* flz_clen;
    const int32_t* flz_st;
    const uint32_t* flz_adler;
    const uint32_t* lzf_olen;
    const int32_t* lzf_st;
    const uint32_t* lz4_olen;
    const int32_t* lz4_st;
    const int32_t* dflz_r;
    const int32_t* dlzf_st;
    const int32_t* dlz4_st;
    const uint32_t* dcks;  // decoder checksums, indexed by AltPiece::aux - 1
};

__global__ void __launch_bounds__(256) k_alt_finish(const uint8_t* __restrict__ din, const uint8_t* __restrict__ aslots,
                                                    const AltPiece* __restrict__ pcs, const AltJobD* __restrict__ jobs, uint32_t njobs,
                                                    AltArrays R, uint8_t* __restrict__ out, AltRes* __restrict__ res) {
    const int lane = threadIdx.x & 63;
    for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < njobs; j += gridDim.x * 4) [&] {
        const AltJobD J = jobs[j];
        uint64_t pos = J.out_off;
        for (uint32_t k = J.p0; k < J.p0 + J.np; ++k) {
            const AltPiece P = pcs[k];
            AltRes r{pos, 0, NX_OK, 0, 0};
            if (P.kind >= AK_DEC_FLZ && P.aux) r.cks = R.dcks[P.aux - 1];
            uint8_t* o = out + pos;
            switch (P.kind) {
                case AK_FLZ_ENC: {  // FastLzFrameEncoder.java:115-168
                    const bool cks = (P.aux & 1u) != 0;
                    const int32_t st = R.flz_st[P.res];
                    if (st != NX_OK) {
                        r.status = st;
                        break;
                    }
                    const uint32_t clen = R.flz_clen[P.res];
                    const bool comp = P.len >= 32u && clen < P.len;  // MIN_LENGTH_TO_COMPRESSION, :150-158
                    const uint32_t hdr = 4u + (cks ? 4u : 0u) + (comp ? 4u : 2u);
                    if (lane == 0) {
                        o[0] = 'F';
                        o[1] = 'L';
                        o[2] = 'Z';
                        o[3] = (uint8_t)((comp ? 1u : 0u) | (cks ? 0x10u : 0u));
                        uint32_t q = 4;
                        if (cks) {
                            const uint32_t a = R.flz_adler[P.res];
                            o[4] = (uint8_t)(a >> 24);
                            o[5] = (uint8_t)(a >> 16);
                            o[6] = (uint8_t)(a >> 8);
                            o[7] = (uint8_t)a;
                            q = 8;
                        }
                        if (comp) {
                            o[q] = (uint8_t)(clen >> 8);
                            o[q + 1] = (uint8_t)clen;
                            q += 2;
                        }
                        o[q] = (uint8_t)(P.len >> 8);
                        o[q + 1] = (uint8_t)P.len;
                    }
                    if (comp) wave_copy(o + hdr, aslots + P.slot, clen, lane);
                    else wave_copy(o + hdr, din + P.src, P.len, lane);
                    r.len = hdr + (comp ? clen : P.len);
                    break;
                }
                case AK_LZF_ENC:
                case AK_LZ4_ENC: {
                    const int32_t st = P.kind == AK_LZF_ENC ? R.lzf_st[P.res] : R.lz4_st[P.res];
                    if (st != NX_OK) {
                        r.status = st;
                        break;
                    }
                    r.len = P.kind == AK_LZF_ENC ? R.lzf_olen[P.res] : R.lz4_olen[P.res];
                    wave_copy(o, aslots + P.slot, r.len, lane);
                    break;
                }
                case AK_LZF_RAW:  // LZFChunk.appendNonCompressed: 'Z' 'V' 0 len(BE16) bytes
                    if (lane == 0) {
                        o[0] = 'Z';
                        o[1] = 'V';
                        o[2] = 0;
                        o[3] = (uint8_t)(P.len >> 8);
                        o[4] = (uint8_t)P.len;
                    }
                    wave_copy(o + 5, din + P.src, P.len, lane);
                    r.len = 5u + P.len;
                    break;
                case AK_LZ4_END:  // magic, token = BLOCK_TYPE_NON_COMPRESSED | level, then 12 zero bytes
                    if (lane < 21) o[lane] = lane < 8 ? (uint8_t)"LZ4Block"[lane] : (lane == 8 ? (uint8_t)(0x10u | P.aux) : 0);
                    r.len = 21;
                    break;
                case AK_RAW:
                case AK_DEC_RAW:
                    wave_copy(o, din + P.src, P.len, lane);
                    r.len = P.len;
                    break;
                case AK_DEC_FLZ: {  // FastLzFrameDecoder.java:154-165: decompress() must return originalLength
                    const int32_t v = R.dflz_r[P.res];
                    if (v < 0 || (uint32_t)v != P.olen) {
                        r.status = v < 0 ? v : NX_ERR_FASTLZ_LENGTH_MISMATCH;
                        r.len = (uint32_t)v;  // the value, for the message
                        break;
                    }
                    wave_copy(o, aslots + P.slot, P.olen, lane);
                    r.len = P.olen;
                    break;
                }
                case AK_DEC_LZF:
                case AK_DEC_LZ4: {
                    const int32_t st = P.kind == AK_DEC_LZF ? R.dlzf_st[P.res] : R.dlz4_st[P.res];
                    if (st != NX_OK) {
                        r.status = st;
                        break;
                    }
                    wave_copy(o, aslots + P.slot, P.olen, lane);
                    r.len = P.olen;
                    break;
                }
                default:
                    r.status = NX_ERR_INTERNAL;
            }
            if (lane == 0) res[k] = r;
            if (r.status != NX_OK) break;
            pos += r.len;
        }
    }();
}

}  // namespace bt
}  // namespace nx

using nx::bt::DecAct;
using nx::bt::DecJob;
using nx::bt::DecRes;
using nx::bt::EncJob;
using nx::bt::EncSlice;
using nx::fr::SAct;
using nx::fr::SnappyAction;

namespace {

struct ArenaCount {  // the batcher's pinned arenas: allocations made (growth included) and bytes held
    uint64_t allocs = 0, bytes = 0;
};

struct Pinned {  // hipHostMalloc'd, mapped into the device address space; grows keeping its bytes
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    ArenaCount* cnt = nullptr;
    bool ensure(size_t n, size_t keep) {
        if (n <= cap) return true;
        size_t c = cap ? cap : (1u << 20);
        while (c < n) c *= 2;
        uint8_t *nh = nullptr, *nd = nullptr;
        // coarse-grained (host-cached) pinned memory: the GPU's writes are visible once the batch's
        // event completes, and host reads of the results run at cache speed
        if (hipHostMalloc((void**)&nh, c, hipHostMallocMapped | hipHostMallocNonCoherent) != hipSuccess) return false;
        if (hipHostGetDevicePointer((void**)&nd, nh, 0) != hipSuccess) {
            (void)hipHostFree(nh);
            return false;
        }
        if (h && keep) memcpy(nh, h, keep < cap ? keep : cap);
        if (h) (void)hipHostFree(h);
        if (cnt) {
            cnt->allocs += 1;
            cnt->bytes += c - cap;
        }
        h = nh;
        d = nd;
        cap = c;
        return true;
    }
    ~Pinned() {
        if (h) (void)hipHostFree(h);
        if (cnt) cnt->bytes -= cap;
    }
};

struct Job {
    uint64_t ticket = 0;
    int kind = 0;  // 0 Snappy encode, 1 Snappy decode, 2 alt-codec encode, 3 alt-codec decode
    nx_snappy_frame_decoder* dec = nullptr;
    uint32_t index = 0;  // EncJob / DecJob index in its batch
    std::vector<SnappyAction> acts;  // decode: the parsed actions (host copy, stream order)
    std::string parse_err;           // decode: the header-level error after them, if any
    bool has_parse_err = false;
    bool applied = false;
    int32_t status = NX_OK;
    std::vector<nx_msg> msgs;
    std::string err;
    // decode, validating decoders: the walked bytes start at stream position s_base (acts[].data is
    // relative to it), under the decoder's re-walk epoch; `walked` = s_base is in dec->outstanding
    uint64_t s_base = 0, epoch = 0;
    bool walked = false;
    std::vector<std::vector<uint8_t>> owned;  // messages delivered before a re-walk moved the job (a moved
                                              // vector keeps its buffer; a deque would allocate per Job)
    // alt-codec jobs (FastLZ / LZF / LZ4)
    int codec = -1;                     // 0 FastLZ, 1 LZF, 2 LZ4
    nx_alt_decoder_base* adec = nullptr;  // decoder jobs hold a reference (alt_frames.hpp)
    bool validate = false;
    std::vector<nx::af::Blk> ablk;      // decoder: the walked blocks, in order
    nx::af::WalkErr awerr;              // decoder: the walk's header failure after them
    uint64_t astage = 0;                // decoder: staging offset of the walked bytes (block data are relative)
    Job() = default;
    Job(const Job&) = delete;
    Job& operator=(const Job&) = delete;
    ~Job() {  // a decoder job holds a reference to its handle (handles.hpp)
        nx_decoder_unref(dec);
        nx_alt_decoder_unref(adec);
    }
};

struct Batch {
    Pinned staging;  // chunk payloads, then the device arrays (one H2D copy at flush)
    size_t st_used = 0;
    struct Direct {
        const uint8_t* src;  // host address (adjacency test)
        const uint8_t* dsrc; // its device address (mapped registration)
        size_t len;
        uint64_t din_off;
    };
    std::vector<Direct> direct;  // registered inputs / cumulations, gathered at flush (din_off in the direct region)
    uint64_t direct_used = 0;
    std::vector<EncSlice> esl;
    std::vector<uint8_t> esl_direct;  // slice input lies in the direct region
    std::vector<EncJob> ejob;
    uint64_t eslots = 0;
    std::vector<DecAct> dact;
    std::vector<uint8_t> dact_direct;  // payload lies in the direct region (registered cumulation)
    std::vector<DecJob> djob;
    std::vector<uint64_t> dc_off;  // compressed chunks: payload offsets / lengths / expected CRC
    std::vector<uint32_t> dc_len, dc_crc;
    bool dc_validate = false;
    std::vector<uint8_t> dc_direct;
    std::vector<uint64_t> du_off;  // uncompressed chunks (CRC32C)
    std::vector<uint32_t> du_len;
    std::vector<uint8_t> du_direct;
    // alt-codec jobs: their pieces and the launch lists of the codec kernels (inputs all staged)
    std::vector<nx::bt::AltPiece> apc;
    std::vector<nx::bt::AltJobD> ajob;
    uint64_t aslots = 0;  // alt slot bytes
    struct AltList {
        std::vector<uint64_t> off, slot;
        std::vector<uint32_t> len, aux;  // aux: FastLZ encode level / decode in_avail; LZ4 encode level; decode olen
        std::vector<int32_t> lim;        // FastLZ encode: readU16 limit
        void clear() {
            off.clear();
            slot.clear();
            len.clear();
            aux.clear();
            lim.clear();
        }
        size_t size() const { return off.size(); }
    };
    AltList flz_e, lzf_e, lz4_e, flz_d, lzf_d, lz4_d;
    Pinned out;  // mapped result arena: job outputs, then the result records
    uint64_t out_used = 0, res_enc = 0, res_dec = 0, res_alt = 0;
    // Bytes the finish kernels are known to write into `out`: decoded messages (lengths from the
    // chunks' preambles).  Encoder outputs are not counted (they fill ~half of their bound-sized
    // reservation).  When the known bytes fill most of a large arena the finish kernels write a device
    // mirror instead and one DMA copy moves it (launch_inner).
    uint64_t est_out = 0;
    uint64_t res_spill = 0;  // the flush's spill area (decoded messages longer than their preamble said)
    std::vector<uint64_t> dslot_off;  // decode slot of each compressed chunk (device, from slots + eslots)
    std::vector<Job*> jobs;
    nx::h::DevBuf din, slots;
    Pinned gops;  // k_gather_host's op list, read by the kernel from pinned memory
    hipEvent_t ev = nullptr;
    uint64_t seq = 0;  // flush order
    bool inflight = false, done = false;
    size_t live = 0;  // jobs not yet released
    void reset() {
        st_used = 0;
        direct.clear();
        direct_used = 0;
        esl.clear();
        esl_direct.clear();
        ejob.clear();
        eslots = 0;
        dact.clear();
        dact_direct.clear();
        djob.clear();
        dc_off.clear();
        dc_len.clear();
        dc_crc.clear();
        dc_direct.clear();
        dc_validate = false;
        du_off.clear();
        du_len.clear();
        du_direct.clear();
        out_used = res_enc = res_dec = res_alt = res_spill = 0;
        est_out = 0;
        dslot_off.clear();
        apc.clear();
        ajob.clear();
        aslots = 0;
        flz_e.clear();
        lzf_e.clear();
        lz4_e.clear();
        flz_d.clear();
        lzf_d.clear();
        lz4_d.clear();
        for (Job* j : jobs) delete j;
        jobs.clear();
        inflight = done = false;
        live = 0;
    }
    uint8_t* stage(size_t n, uint64_t* din_off) {  // reserve n staging bytes (16-aligned)
        const size_t at = (st_used + 15) & ~(size_t)15;
        if (!staging.ensure(at + n + 16, st_used)) return nullptr;
        st_used = at + n;
        *din_off = at;
        return staging.h + at;
    }
    bool reserve_out(size_t n, uint64_t* off) {
        const uint64_t at = (out_used + 15) & ~15ull;
        if (!out.ensure(at + n + 16, out_used)) return false;
        out_used = at + n;
        *off = at;
        return true;
    }
    ~Batch() {
        for (Job* j : jobs) delete j;
        if (ev) (void)hipEventDestroy(ev);
    }
};

}  // namespace

namespace {
// nx_host_register'd ranges: host base -> (length, device address of the mapping)
std::mutex g_reg_mu;
std::map<uintptr_t, std::pair<size_t, uint8_t*>> g_reg;
const uint8_t* registered_device_ptr(const uint8_t* p, size_t n) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound((uintptr_t)p);
    if (it == g_reg.begin()) return nullptr;
    --it;
    const uintptr_t off = (uintptr_t)p - it->first;
    if (off + n > it->second.first) return nullptr;
    return it->second.second + off;
}
}  // namespace

#ifndef NX_BATCHER_STREAMS
#define NX_BATCHER_STREAMS 4
#endif
constexpr int kStreams = NX_BATCHER_STREAMS;
struct nx_batcher {
    std::mutex mu;
    hipStream_t s[kStreams] = {};
    // DMA result path: one device mirror per stream (flushes on one stream are ordered, so the next
    // flush on it reuses the mirror after the previous result copy), not one per batch object
    nx::h::DevBuf dmirror[kStreams];
    int dev = 0;
    uint32_t held = 0;  // bit per nx::WsKind whose shared workspace the batcher holds (workspace.hpp)
    std::deque<Batch*> all;  // every batch object (collecting, in flight, or done)
    Batch* cur = nullptr;    // the collecting batch
    std::unordered_map<uint64_t, std::pair<Batch*, Job*>> tickets;
    uint64_t next_ticket = 1;
    uint64_t launches = 0, chunks = 0, flushes = 0;
    uint64_t dma_flushes = 0, dma_bytes = 0;
    uint64_t applied = 0;     // batches applied, in flush order (Batch::seq < applied)
    size_t flush_bytes = 0;   // auto-flush threshold on a batch's input bytes (0 = only explicit flushes)
    ArenaCount arena;         // pinned staging / result arenas of all batches
    std::vector<std::pair<Job*, Batch*>> cont;  // re-walked jobs to queue again (found by apply())
    bool kick = false;        // the collecting batch holds a re-walked job: launch it at the next poll/wait
};

namespace {

bool advance(nx_batcher* b, uint64_t upto, bool block);

Batch* reuse_or_new_batch(nx_batcher* b) {
    for (Batch* x : b->all) {
        if (!x->inflight && x->live == 0 && x != b->cur) {
            x->reset();
            return x;
        }
    }
    Batch* x = new Batch();
    if (hipEventCreateWithFlags(&x->ev, hipEventDisableTiming) != hipSuccess) {
        delete x;
        return nullptr;
    }
    x->staging.cnt = x->out.cnt = x->gops.cnt = &b->arena;
    b->all.push_back(x);
    return x;
}

Batch* fresh_batch(nx_batcher* b) {
    advance(b, ~0ull, false);  // apply every completed batch (in flush order), even if its jobs were released unpolled
    return reuse_or_new_batch(b);
}

Batch* collecting(nx_batcher* b) {
    if (!b->cur) {
        Batch* x = fresh_batch(b);
        if (!b->cur) b->cur = x;  // advance() may have opened one for re-walked jobs
    }
    return b->cur;
}

// Drop the stream segments no unapplied job of a validating decoder can re-walk any more.
void trim_hist(nx_snappy_frame_decoder* d) {
    if (d->corrupted) {  // (:86-89): nothing is parsed again
        d->hist.clear(d->parse_pos);
        return;
    }
    d->hist.drop_before(d->outstanding.empty() ? d->parse_pos : *d->outstanding.begin());
}

void unwalk(Job* j) {  // the job no longer needs its walked bytes kept
    if (!j->walked) return;
    nx_snappy_frame_decoder* d = j->dec;
    auto it = d->outstanding.find(j->s_base);
    if (it != d->outstanding.end()) d->outstanding.erase(it);
    j->walked = false;
}

// Queue decoder job j's walked actions into batch bt.  Payloads are copied from S (host bytes the
// walk ran over), or, with dS (the device address of S in registered memory), gathered from there at
// flush.  On failure the batch's arrays go back to their sizes at entry (its other jobs stay valid).
// Snappy.decode's preamble (readPreamble, Snappy.java:404-420): the declared length, for sizing
// estimates only (65 536, the frame decoder's cap, when it is malformed or absent)
inline uint32_t snappy_declared_len(const uint8_t* p, size_t n) {
    uint32_t v = 0;
    for (size_t i = 0; i < n && i < 4; ++i) {
        v |= (uint32_t)(p[i] & 0x7f) << (7 * i);
        if ((p[i] & 0x80) == 0) return v < 65536u ? v : 65536u;
    }
    return 65536u;
}

int32_t enqueue_dec(Batch* bt, Job* j, const uint8_t* S, size_t walked, const uint8_t* dS, int64_t staged = -1) {
    const size_t n_act = bt->dact.size(), n_dc = bt->dc_off.size(), n_du = bt->du_off.size(), n_dir = bt->direct.size();
    const uint64_t dir_used = bt->direct_used, est0 = bt->est_out;
    auto fail = [&](int32_t code) -> int32_t {
        bt->est_out = est0;
        bt->dact.resize(n_act);
        bt->dact_direct.resize(n_act);
        bt->dc_off.resize(n_dc);
        bt->dc_len.resize(n_dc);
        bt->dc_crc.resize(n_dc);
        bt->dc_direct.resize(n_dc);
        bt->du_off.resize(n_du);
        bt->du_len.resize(n_du);
        bt->du_direct.resize(n_du);
        bt->direct.resize(n_dir);
        bt->direct_used = dir_used;
        return code;
    };
    uint64_t rbase = 0;
    if (dS && walked) {
        rbase = (bt->direct_used + 15) & ~15ull;
        bt->direct.push_back({S, dS, walked, rbase});
        bt->direct_used = rbase + walked;
    }
    DecJob J{};
    J.a0 = (uint32_t)bt->dact.size();
    J.validate = j->dec->validate ? 1u : 0u;
    size_t out_need = 0;
    for (const SnappyAction& a : j->acts) {
        if (a.kind != SAct::Uncomp && a.kind != SAct::Comp) continue;
        uint64_t off = 0;
        if (dS) {
            off = rbase + a.data;
        } else if (staged >= 0) {  // the walked bytes are already in the staging arena at `staged`
            off = (uint64_t)staged + a.data;
        } else {
            uint8_t* st = bt->stage(a.dlen, &off);
            if (!st) return fail(NX_ERR_HIP);
            nx::copy_bytes(st, S + a.data, a.dlen);
        }
        const uint8_t dir = dS ? 1 : 0;
        bt->dact_direct.push_back(dir);
        DecAct A{off, a.dlen, 0, 0, a.crc, a.dlen, 0};
        if (a.kind == SAct::Comp) {
            A.kind = 2;
            A.chunk = (uint32_t)bt->dc_off.size();
            bt->dc_off.push_back(off);
            bt->dc_len.push_back(a.dlen);
            bt->dc_crc.push_back(a.crc);
            bt->dc_direct.push_back(dir);
            if (j->dec->validate) bt->dc_validate = true;
            // the message's room: the preamble's length (never more than the bound); a chunk that
            // decodes longer (malformed, yet Java keeps it) spills (k_dec_finish, apply)
            A.cap = std::min<uint32_t>(snappy_declared_len(S + a.data, a.dlen), nx::bt::snappy_decoded_bound(a.dlen));
            out_need += A.cap;
            bt->est_out += A.cap;
        } else {
            A.kind = 1;
            A.chunk = (uint32_t)bt->du_off.size();
            bt->du_off.push_back(off);
            bt->du_len.push_back(a.dlen);
            bt->du_direct.push_back(dir);
            out_need += a.dlen;
            bt->est_out += a.dlen;
        }
        bt->dact.push_back(A);
    }
    J.na = (uint32_t)bt->dact.size() - J.a0;
    if (!bt->reserve_out(out_need + 16, &J.out_off)) return fail(NX_ERR_HIP);
    j->index = (uint32_t)bt->djob.size();
    bt->djob.push_back(J);
    bt->jobs.push_back(j);
    return NX_OK;
}

// The header walk of SnappyFrameDecoder.decode over S[0..n) from the decoder's state (:85-231); a
// header-level error ends it and is kept on the job, applied in order (the decoder turns corrupted then).
size_t walk(nx_snappy_frame_decoder* d, Job* j, const uint8_t* S, size_t n, bool& started, uint64_t& skip) {
    size_t p = 0;
    j->acts.clear();
    j->has_parse_err = false;
    j->parse_err.clear();
    while (p < n && nx::fr::snappy_parse_one(S, n, p, started, skip, d->validate, j->acts)) {
    }
    if (!j->acts.empty() && j->acts.back().kind == SAct::Error) {
        j->has_parse_err = true;
        j->parse_err = j->acts.back().err;
        p = j->acts.back().end;
        j->acts.pop_back();
    }
    return p;
}

bool has_gpu_work(const Job* j) {
    for (const SnappyAction& a : j->acts)
        if (a.kind == SAct::Uncomp || a.kind == SAct::Comp) return true;
    return false;
}

// Job j's compressed chunk decoded fewer bytes than its length, in validating mode: Java leaves the
// rest in the cumulation and parses it as the next chunk header (SnappyFrameDecoder.java:206-212).
// Walk the decoder's stream again from q (the first unread byte): every byte handed over so far, so
// the walks of the decoder's later, not yet applied jobs are void (new epoch; they deliver nothing and
// their bytes are covered here).  Returns true when j has GPU work again: it is queued into the
// collecting batch by queue_continuations() and completes there.
bool rewalk(nx_batcher* b, Batch* bt, Job* j, uint64_t q) {
    nx_snappy_frame_decoder* d = j->dec;
    d->epoch += 1;
    d->parse_failed = false;
    bool started = true;  // a compressed chunk was accepted (:180-183)
    uint64_t skip = 0;
    const uint8_t* S = d->hist.own_from(q);
    const size_t n = (size_t)(d->hist.end - q);
    const size_t p = walk(d, j, S, n, started, skip);
    d->started = started;
    d->skip = skip;
    d->parse_pos = q + p;
    if (j->has_parse_err) d->parse_failed = true;
    j->s_base = q;
    j->epoch = d->epoch;
    if (!has_gpu_work(j)) {
        if (j->has_parse_err) {
            j->status = NX_ERR_FRAME_CORRUPT;
            j->err = j->parse_err;
            d->corrupted = true;  // (:227-230)
        }
        return false;
    }
    // the messages so far live in bt's arena, which may be reused before j completes elsewhere
    for (nx_msg& m : j->msgs) {
        j->owned.emplace_back(m.data, m.data + m.len);
        m.data = j->owned.back().data();
    }
    d->outstanding.insert(q);
    j->walked = true;
    j->applied = false;
    b->cont.push_back({j, bt});
    return true;
}

// Launch everything `bt` collected (batcher lock held).
int32_t launch_inner(nx_batcher* b, Batch* bt) {
    NX_CLEAR_STALE_ERROR();
    const hipStream_t s = b->s[b->flushes % kStreams];
    const nx::NoGrowScope no_grow;  // the workspaces reserved at nx_batcher_new: a flush never allocates them
    const uint32_t nes = (uint32_t)bt->esl.size(), nej = (uint32_t)bt->ejob.size(), nda = (uint32_t)bt->dact.size();
    const uint32_t ndj = (uint32_t)bt->djob.size(), ndc = (uint32_t)bt->dc_off.size(), ndu = (uint32_t)bt->du_off.size();
    struct Lay {
        uint64_t at = 0;
        uint64_t put(uint64_t n) {
            const uint64_t r = (at + 15) & ~15ull;
            at = r + n;
            return r;
        }
    } Lh, Ld;
    // arrays the host fills (uploaded inside the staging arena)
    const uint64_t o_esl = Lh.put(sizeof(EncSlice) * nes), o_ein = Lh.put(8ull * nes), o_eslot = Lh.put(8ull * nes),
                   o_elen = Lh.put(4ull * nes), o_ejob = Lh.put(sizeof(EncJob) * nej), o_dact = Lh.put(sizeof(DecAct) * nda),
                   o_djob = Lh.put(sizeof(DecJob) * ndj), o_dcoff = Lh.put(8ull * ndc), o_dclen = Lh.put(4ull * ndc),
                   o_dccrc = Lh.put(4ull * ndc), o_dslot = Lh.put(8ull * ndc), o_duoff = Lh.put(8ull * ndu), o_dulen = Lh.put(4ull * ndu);
    // arrays the kernels fill (device only)
    const uint64_t o_eclen = Ld.put(4ull * nes), o_est = Ld.put(4ull * nes), o_ecrc = Ld.put(4ull * nes), o_dlen = Ld.put(4ull * ndc),
                   o_dcons = Ld.put(4ull * ndc), o_dst = Ld.put(4ull * ndc), o_dcrc = Ld.put(4ull * ndc), o_ducrc = Ld.put(4ull * ndu);
    // ---- FastLZ / LZF / LZ4 jobs: codec lists, decoder checksum lists, pieces
    const uint32_t nap = (uint32_t)bt->apc.size(), naj = (uint32_t)bt->ajob.size();
    Batch::AltList* AL[6] = {&bt->flz_e, &bt->lzf_e, &bt->lz4_e, &bt->flz_d, &bt->lzf_d, &bt->lz4_d};
    // LZ4 frame encode takes one compression level per launch: order its entries by level
    std::vector<uint32_t> lz4_perm(bt->lz4_e.size());
    for (uint32_t i = 0; i < lz4_perm.size(); ++i) lz4_perm[i] = i;
    std::stable_sort(lz4_perm.begin(), lz4_perm.end(), [&](uint32_t a, uint32_t c) { return bt->lz4_e.aux[a] < bt->lz4_e.aux[c]; });
    {
        Batch::AltList& Z = bt->lz4_e;
        Batch::AltList P;
        std::vector<uint32_t> pos(Z.size());
        for (uint32_t k = 0; k < lz4_perm.size(); ++k) {
            const uint32_t i = lz4_perm[k];
            pos[i] = k;
            P.off.push_back(Z.off[i]);
            P.slot.push_back(Z.slot[i]);
            P.len.push_back(Z.len[i]);
            P.aux.push_back(Z.aux[i]);
            P.lim.push_back(Z.lim[i]);
        }
        Z = std::move(P);
        for (nx::bt::AltPiece& q : bt->apc)
            if (q.kind == nx::bt::AK_LZ4_ENC) q.res = pos[q.res];
    }
    Batch::AltList ck[4];  // decoder checksums: Adler32 over slot / input, XXH32 over slot / input
    for (nx::bt::AltPiece& q : bt->apc) {
        if (q.kind < nx::bt::AK_DEC_FLZ || !q.pad) continue;
        const bool raw = q.kind == nx::bt::AK_DEC_RAW;
        const int li = (q.pad == 2 ? 2 : 0) + (raw ? 1 : 0);
        ck[li].off.push_back(raw ? q.src : q.slot);
        ck[li].len.push_back(raw ? q.len : q.olen);
        q.aux = (uint32_t)ck[li].off.size();  // 1-based within its list; made global below
    }
    const uint32_t nck[4] = {(uint32_t)ck[0].off.size(), (uint32_t)ck[1].off.size(), (uint32_t)ck[2].off.size(), (uint32_t)ck[3].off.size()};
    const uint32_t ck0[4] = {0, nck[0], nck[0] + nck[1], nck[0] + nck[1] + nck[2]};
    for (nx::bt::AltPiece& q : bt->apc) {
        if (q.kind < nx::bt::AK_DEC_FLZ || !q.pad) continue;
        const int li = (q.pad == 2 ? 2 : 0) + (q.kind == nx::bt::AK_DEC_RAW ? 1 : 0);
        q.aux += ck0[li];
    }
    const uint32_t ncks = ck0[3] + nck[3];
    uint64_t o_al[6][5], o_ck[4][2];
    for (int c = 0; c < 6; ++c) {
        const uint64_t m = AL[c]->size();
        o_al[c][0] = Lh.put(8 * m);
        o_al[c][1] = Lh.put(4 * m);
        o_al[c][2] = Lh.put(8 * m);
        o_al[c][3] = Lh.put(4 * m);
        o_al[c][4] = Lh.put(4 * m);
    }
    for (int c = 0; c < 4; ++c) {
        o_ck[c][0] = Lh.put(8ull * nck[c]);
        o_ck[c][1] = Lh.put(4ull * nck[c]);
    }
    const uint64_t o_apc = Lh.put(sizeof(nx::bt::AltPiece) * nap), o_ajob = Lh.put(sizeof(nx::bt::AltJobD) * naj);
    const uint32_t nfe = (uint32_t)bt->flz_e.size(), nle = (uint32_t)bt->lzf_e.size(), nze = (uint32_t)bt->lz4_e.size();
    const uint32_t nfd = (uint32_t)bt->flz_d.size(), nld = (uint32_t)bt->lzf_d.size(), nzd = (uint32_t)bt->lz4_d.size();
    const uint64_t o_fclen = Ld.put(4ull * nfe), o_fst = Ld.put(4ull * nfe), o_fadl = Ld.put(4ull * nfe), o_lolen = Ld.put(4ull * nle),
                   o_lst = Ld.put(4ull * nle), o_zolen = Ld.put(4ull * nze), o_zst = Ld.put(4ull * nze), o_dfr = Ld.put(4ull * nfd),
                   o_dlst = Ld.put(4ull * nld), o_dzst = Ld.put(4ull * nzd), o_dcks = Ld.put(4ull * ncks);
    uint64_t st_arr = 0;
    uint8_t* h = bt->stage(Lh.at + 16, &st_arr);
    if (!h) return NX_ERR_HIP;
    // device input arena: [staging bytes][direct region]
    const uint64_t d0 = (bt->st_used + 15) & ~15ull;
    for (uint32_t i = 0; i < nes; ++i)
        if (bt->esl_direct[i]) bt->esl[i].in_off += d0;
    for (uint32_t i = 0; i < nda; ++i)
        if (bt->dact_direct[i]) bt->dact[i].in_off += d0;
    for (uint32_t i = 0; i < ndc; ++i)
        if (bt->dc_direct[i]) bt->dc_off[i] += d0;
    for (uint32_t i = 0; i < ndu; ++i)
        if (bt->du_direct[i]) bt->du_off[i] += d0;
    std::vector<uint64_t> ein(nes), eslot(nes), dslot(ndc);
    std::vector<uint32_t> elen(nes);
    for (uint32_t i = 0; i < nes; ++i) {
        ein[i] = bt->esl[i].in_off;
        eslot[i] = bt->esl[i].slot_off;
        elen[i] = bt->esl[i].len;
    }
    uint64_t dslot_bytes = 0;
    for (uint32_t i = 0; i < ndc; ++i) {
        dslot[i] = dslot_bytes;
        dslot_bytes += nx::bt::dec_slot_bytes(bt->dc_len[i]);
    }
    bt->dslot_off = dslot;
    auto cp = [&](uint64_t off, const void* src, size_t n) {
        if (n) memcpy(h + off, src, n);
    };
    cp(o_esl, bt->esl.data(), sizeof(EncSlice) * nes);
    cp(o_ein, ein.data(), 8ull * nes);
    cp(o_eslot, eslot.data(), 8ull * nes);
    cp(o_elen, elen.data(), 4ull * nes);
    cp(o_ejob, bt->ejob.data(), sizeof(EncJob) * nej);
    cp(o_dact, bt->dact.data(), sizeof(DecAct) * nda);
    cp(o_djob, bt->djob.data(), sizeof(DecJob) * ndj);
    cp(o_dcoff, bt->dc_off.data(), 8ull * ndc);
    cp(o_dclen, bt->dc_len.data(), 4ull * ndc);
    cp(o_dccrc, bt->dc_crc.data(), 4ull * ndc);
    cp(o_dslot, dslot.data(), 8ull * ndc);
    cp(o_duoff, bt->du_off.data(), 8ull * ndu);
    cp(o_dulen, bt->du_len.data(), 4ull * ndu);
    // result records in the mapped arena, after the job outputs
    if (naj) {
        for (int c = 0; c < 6; ++c) {
            const Batch::AltList& L = *AL[c];
            const size_t m = L.size();
            cp(o_al[c][0], L.off.data(), 8 * m);
            cp(o_al[c][1], L.len.data(), 4 * m);
            cp(o_al[c][2], L.slot.data(), 8 * m);
            cp(o_al[c][3], L.aux.data(), 4 * m);
            cp(o_al[c][4], L.lim.data(), 4 * m);
        }
        for (int c = 0; c < 4; ++c) {
            cp(o_ck[c][0], ck[c].off.data(), 8ull * nck[c]);
            cp(o_ck[c][1], ck[c].len.data(), 4ull * nck[c]);
        }
        cp(o_apc, bt->apc.data(), sizeof(nx::bt::AltPiece) * nap);
        cp(o_ajob, bt->ajob.data(), sizeof(nx::bt::AltJobD) * naj);
        if (!bt->reserve_out(sizeof(nx::bt::AltRes) * nap + 8, &bt->res_alt)) return NX_ERR_HIP;
    }
    if (!bt->reserve_out(8ull * nej + 8, &bt->res_enc) || !bt->reserve_out(sizeof(DecRes) * nda + 8, &bt->res_dec)) return NX_ERR_HIP;
    // spill area: a chunk that decodes longer than its preamble said (Java grows its buffer up to
    // 65 536, SnappyFrameDecoder.java:203) has no room in its message reservation; k_dec_finish moves
    // it here, so apply() need not copy it from the device (only spills beyond this area do)
    const uint32_t spill_cap = (uint32_t)std::min<uint64_t>(nx::bt::kSpillBytes, 65536ull * ndc);
    if (ndc && !bt->reserve_out(spill_cap, &bt->res_spill)) return NX_ERR_HIP;
    const uint64_t o_spc = Ld.put(4);
    // Where the finish kernels write: straight into the mapped arena (their stores cross PCIe), or,
    // when the expected bytes fill most of a large arena (decoded messages: lengths known from the
    // preambles), into a device mirror that one DMA copy then moves.  The copy engine does not hold
    // CUs or flood the memory system with partial writes while the next batch parses (round 4 e2e:
    // the finish kernel's host writes ran at 53 GB/s and slowed a concurrent k_parse 2-3x).
    // The spill area is reserved for rare malformed chunks: it counts neither as expected bytes nor
    // against them (counted in out_used it leaned mid-sized flushes away from the DMA path).
    const uint64_t est = bt->est_out + 8ull * nej + sizeof(DecRes) * nda + sizeof(nx::bt::AltRes) * (naj ? bt->apc.size() : 0);
    const uint64_t spill_res = ndc ? spill_cap : 0;
    const uint64_t used_wo_spill = bt->out_used > spill_res ? bt->out_used - spill_res : 0;
    const bool dma_out = bt->out_used >= nx::bt::kDmaOutMin && est * 5 >= used_wo_spill * 4;
    nx::h::DevBuf& mirror = b->dmirror[b->flushes % kStreams];
    if (dma_out && !mirror.ensure(bt->out_used)) return NX_ERR_HIP;
    uint8_t* const ob = dma_out ? mirror.as<uint8_t>() : bt->out.d;
    if (!bt->din.ensure(d0 + bt->direct_used + 16) || !bt->slots.ensure(bt->eslots + dslot_bytes + bt->aslots + Ld.at + 128)) return NX_ERR_HIP;
    uint8_t* din = bt->din.as<uint8_t>();
    uint8_t* slots = bt->slots.as<uint8_t>();
    uint8_t* dslots = slots + bt->eslots;
    uint8_t* aslots = reinterpret_cast<uint8_t*>(((uintptr_t)(dslots + dslot_bytes) + 15) & ~(uintptr_t)15);
    uint8_t* D = aslots + bt->aslots;
    D = reinterpret_cast<uint8_t*>(((uintptr_t)D + 15) & ~(uintptr_t)15);
    // Host -> device.  Registered inputs (and a small staging arena) move in one gather launch that
    // reads the mapped pages, its op list itself read from pinned memory: no copy-engine work.  The
    // copy engines run the batches' result copies in order, and a descriptor copy queued behind the
    // previous batch's 500 MB result copy held this batch's gather (and, for an op list in pageable
    // memory, the submitting thread) until that copy ended (round 4 e2e trace).  A large staging
    // arena (payloads copied at submit) still goes by one DMA copy.
    // (round 5 measured the whole staging arena through the gather as well, profiles/r05/s10: no better)
    const bool dma_in = bt->direct.empty() && bt->st_used > nx::bt::kGatherStageMax;
    if (dma_in) {
        NX_HIP_CHECK(hipMemcpyAsync(din, bt->staging.h, bt->st_used, hipMemcpyHostToDevice, s));
    } else if (bt->st_used || !bt->direct.empty()) {
        const uint64_t piece = nx::bt::kGatherPiece;
        const uint32_t nst = (uint32_t)((bt->st_used + piece - 1) / piece);
        const uint32_t ng = nst + (uint32_t)bt->direct.size();
        if (!bt->gops.ensure(sizeof(nx::bt::GatherOp) * ng, 0)) return NX_ERR_HIP;
        nx::bt::GatherOp* ops = reinterpret_cast<nx::bt::GatherOp*>(bt->gops.h);
        for (uint32_t k = 0; k < nst; ++k) {
            const uint64_t o = (uint64_t)k * piece;
            ops[k] = {bt->staging.d + o, o, std::min<uint64_t>(piece, bt->st_used - o)};
        }
        for (uint32_t k = 0; k < (uint32_t)bt->direct.size(); ++k)
            ops[nst + k] = {bt->direct[k].dsrc, d0 + bt->direct[k].din_off, bt->direct[k].len};
        hipLaunchKernelGGL(nx::bt::k_gather_host, nx::bt::pcie_grid(ng), dim3(256), 0, s,
                           reinterpret_cast<const nx::bt::GatherOp*>(bt->gops.d), ng, din);
        NX_HIP_CHECK(hipGetLastError());
        b->launches += 1;
    }
    const uint8_t* A = din + st_arr;
    int32_t r;
    if (nes) {  // CRC32C + Snappy.encode of every encoder slice of every channel
        r = nx_crc32c_masked_batch(din, (const uint64_t*)(A + o_ein), (const uint32_t*)(A + o_elen), (uint32_t*)(D + o_ecrc), nes, s);
        if (r != NX_OK) return r;
        r = nx_snappy_encode_batch(din, (const uint64_t*)(A + o_ein), (const uint32_t*)(A + o_elen), slots, (const uint64_t*)(A + o_eslot),
                                   (uint32_t*)(D + o_eclen), (int32_t*)(D + o_est), nes, s);
        if (r != NX_OK) return r;
        hipLaunchKernelGGL(nx::bt::k_enc_finish, nx::bt::pcie_grid(nej), dim3(256), 0, s, din, slots, (const EncSlice*)(A + o_esl),
                           (const uint32_t*)(D + o_eclen), (const int32_t*)(D + o_est), (const uint32_t*)(D + o_ecrc),
                           (const EncJob*)(A + o_ejob), nej, ob, (int64_t*)(ob + bt->res_enc));
        NX_HIP_CHECK(hipGetLastError());
        b->launches += 3;
        b->chunks += nes;
    }
    if (ndj) {  // Snappy.decode (+ fused CRC verify) of every compressed chunk, CRC32C of uncompressed ones
        if (ndc) {
            r = nx_snappy_decode_batch(din, (const uint64_t*)(A + o_dcoff), (const uint32_t*)(A + o_dclen), dslots,
                                       (const uint64_t*)(A + o_dslot), nullptr, (uint32_t*)(D + o_dlen), (uint32_t*)(D + o_dcons),
                                       (int32_t*)(D + o_dst), bt->dc_validate ? (const uint32_t*)(A + o_dccrc) : nullptr,
                                       (uint32_t*)(D + o_dcrc), ndc, s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        if (ndu) {
            r = nx_crc32c_masked_batch(din, (const uint64_t*)(A + o_duoff), (const uint32_t*)(A + o_dulen), (uint32_t*)(D + o_ducrc), ndu, s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        if (ndc) NX_HIP_CHECK(hipMemsetAsync(D + o_spc, 0, 4, s));
        hipLaunchKernelGGL(nx::bt::k_dec_finish, nx::bt::pcie_grid(ndj), dim3(256), 0, s, din, dslots, (const uint64_t*)(A + o_dslot),
                           (const DecAct*)(A + o_dact),
                           (const DecJob*)(A + o_djob), ndj, (const uint32_t*)(D + o_dlen), (const uint32_t*)(D + o_dcons),
                           (const int32_t*)(D + o_dst), (const uint32_t*)(D + o_dcrc), (const uint32_t*)(D + o_ducrc), ob,
                           (DecRes*)(ob + bt->res_dec), bt->res_spill, ndc ? spill_cap : 0u, (uint32_t*)(D + o_spc));
        NX_HIP_CHECK(hipGetLastError());
        b->launches += 1;
        b->chunks += ndc + ndu;
    }
    if (naj) {  // FastLZ / LZF / LZ4: one launch per codec kernel for every job of every channel
        auto U64 = [&](int c, int f) { return (const uint64_t*)(A + o_al[c][f]); };
        auto U32 = [&](int c, int f) { return (const uint32_t*)(A + o_al[c][f]); };
        auto I32 = [&](int c, int f) { return (const int32_t*)(A + o_al[c][f]); };
        if (nfe) {  // FastLz.compress + the frame's Adler32 of every block (FastLzFrameEncoder.java:136-158)
            r = nx_fastlz_compress_batch(din, U64(0, 0), U32(0, 1), aslots, U64(0, 2), (uint32_t*)(D + o_fclen), I32(0, 3), I32(0, 4),
                                         (int32_t*)(D + o_fst), nfe, s);
            if (r != NX_OK) return r;
            r = nx_adler32_batch(din, U64(0, 0), U32(0, 1), (uint32_t*)(D + o_fadl), nfe, s);
            if (r != NX_OK) return r;
            b->launches += 2;
        }
        if (nle) {
            r = nx_lzf_encode_batch(din, U64(1, 0), U32(1, 1), aslots, U64(1, 2), (uint32_t*)(D + o_lolen), (int32_t*)(D + o_lst), nle, s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        for (uint32_t a0 = 0; a0 < nze;) {  // one launch per compression level (usually one)
            uint32_t a1 = a0;
            while (a1 < nze && bt->lz4_e.aux[a1] == bt->lz4_e.aux[a0]) ++a1;
            // aux = compressionLevel | highCompressor << 8: one launch per (level, compressor)
            r = nx_lz4_frame_encode_batch_ex(din, U64(2, 0) + a0, U32(2, 1) + a0, aslots, U64(2, 2) + a0, (uint32_t*)(D + o_zolen) + a0,
                                             (int32_t)(bt->lz4_e.aux[a0] & 0xFFu), (int32_t)(bt->lz4_e.aux[a0] >> 8),
                                             (int32_t*)(D + o_zst) + a0, a1 - a0, s);
            if (r != NX_OK) return r;
            b->launches += 1;
            a0 = a1;
        }
        if (nfd) {  // FastLz.decompress (in_avail = the cumulation's readable bytes from the block on)
            r = nx_fastlz_decompress_batch(din, U64(3, 0), U32(3, 1), U32(3, 3), aslots, U64(3, 2), (const uint32_t*)I32(3, 4),
                                           (int32_t*)(D + o_dfr), nfd, s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        if (nld) {
            r = nx_lzf_decode_batch(din, U64(4, 0), U32(4, 1), aslots, U64(4, 2), U32(4, 3), (int32_t*)(D + o_dlst), nld, s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        if (nzd) {
            r = nx_lz4_decode_batch(din, U64(5, 0), U32(5, 1), aslots, U64(5, 2), U32(5, 3), (int32_t*)(D + o_dzst), nzd, s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        uint32_t* dcks = (uint32_t*)(D + o_dcks);
        for (int c = 0; c < 4; ++c) {  // decoder checksums (after the decodes: stream order)
            if (!nck[c]) continue;
            const uint8_t* base = (c & 1) ? din : aslots;
            const uint64_t* co = (const uint64_t*)(A + o_ck[c][0]);
            const uint32_t* cl = (const uint32_t*)(A + o_ck[c][1]);
            r = c < 2 ? nx_adler32_batch(base, co, cl, dcks + ck0[c], nck[c], s)
                      : nx_xxhash32_batch(base, co, cl, nx::af::kLz4Seed, dcks + ck0[c], nck[c], s);
            if (r != NX_OK) return r;
            b->launches += 1;
        }
        const nx::bt::AltArrays R{(const uint32_t*)(D + o_fclen), (const int32_t*)(D + o_fst), (const uint32_t*)(D + o_fadl),
                                  (const uint32_t*)(D + o_lolen), (const int32_t*)(D + o_lst), (const uint32_t*)(D + o_zolen),
                                  (const int32_t*)(D + o_zst), (const int32_t*)(D + o_dfr), (const int32_t*)(D + o_dlst),
                                  (const int32_t*)(D + o_dzst), dcks};
        hipLaunchKernelGGL(nx::bt::k_alt_finish, nx::bt::pcie_grid(naj), dim3(256), 0, s, din, aslots, (const nx::bt::AltPiece*)(A + o_apc),
                           (const nx::bt::AltJobD*)(A + o_ajob), naj, R, ob, (nx::bt::AltRes*)(ob + bt->res_alt));
        NX_HIP_CHECK(hipGetLastError());
        b->launches += 1;
        b->chunks += nfe + nle + nze + nfd + nld + nzd;
    }
    if (dma_out) {
        NX_HIP_CHECK(hipMemcpyAsync(bt->out.h, ob, bt->out_used, hipMemcpyDeviceToHost, s));
        b->dma_flushes += 1;
        b->dma_bytes += bt->out_used;
    }
    NX_HIP_CHECK(hipEventRecord(bt->ev, s));
    bt->inflight = true;
    bt->seq = b->flushes;
    b->flushes += 1;
    return NX_OK;
}

// A launch that failed part-way: wait for whatever of it reached the stream, then complete every job
// of the batch with the error (each decoder it touched turns corrupted, as after the reference's
// exception), so poll() reports them done and result() returns the error.  The batch is not in the
// flush order (it never got a sequence number) and is reused once its jobs are released.
int32_t fail_batch(nx_batcher* b, Batch* bt, int32_t code) {
    (void)hipStreamSynchronize(b->s[b->flushes % kStreams]);
    for (Job* j : bt->jobs) {
        j->applied = true;
        j->status = code;
        j->err = "GPU batch launch failed";
        j->msgs.clear();
        if (j->kind == 1 && j->dec) {
            unwalk(j);
            j->dec->corrupted = true;
            trim_hist(j->dec);
        }
        if (j->kind == 3 && j->adec) j->adec->corrupted = true;
    }
    bt->inflight = false;
    bt->done = true;
    return code;
}

int32_t launch(nx_batcher* b, Batch* bt) {
    const int32_t r = launch_inner(b, bt);
    return r == NX_OK ? NX_OK : fail_batch(b, bt, r);
}

// An alt-codec job's result (its batch complete): an encoder's framed bytes as one message, or the
// decoder's messages in block order up to its first failure, with the reference's message
// (FastLzFrameDecoder.java:154-180, LzfDecoder.java:205, Lz4FrameDecoder.java:215-241); then the
// walk's header failure, if any.  A failure marks the decoder corrupted; jobs applied after that on
// the same decoder deliver nothing (Java skips all later input).
void apply_alt(Batch* bt, Job* j, const nx::bt::AltRes* ares) {
    using namespace nx::bt;
    j->applied = true;
    const AltJobD& J = bt->ajob[j->index];
    if (j->kind == 2) {  // encoder
        uint64_t total = 0;
        for (uint32_t k = J.p0; k < J.p0 + J.np; ++k) {
            if (ares[k].status != NX_OK) {
                j->status = ares[k].status;
                j->err = nx_status_string(ares[k].status);
                return;
            }
            total += ares[k].len;
        }
        j->msgs.push_back({bt->out.h + J.out_off, (size_t)total});
        return;
    }
    nx_alt_decoder_base* d = j->adec;
    if (d->corrupted) return;
    auto fail = [&](int32_t code, const std::string& msg) {
        j->status = code;
        j->err = msg;
        d->corrupted = true;
    };
    for (uint32_t i = 0; i < J.np; ++i) {
        const AltRes& R = ares[J.p0 + i];
        const AltPiece& P = bt->apc[J.p0 + i];
        const nx::af::Blk& B = j->ablk[i];
        if (R.status != NX_OK) {
            if (j->codec == 0) {
                int32_t code;
                std::string msg;
                const int32_t v = R.status == NX_ERR_FASTLZ_LENGTH_MISMATCH ? (int32_t)R.len : R.status;
                const uint8_t first = B.clen ? bt->staging.h[P.src] : 0;
                (void)nx::af::flz_block_error(v, B.olen, first, &code, &msg);
                fail(code, msg);
            } else {
                fail(R.status, j->codec == 1 ? nx::af::lzf_block_error() : nx::af::lz4_block_error());
            }
            return;
        }
        if (j->codec == 0 && B.has_cks && j->validate && R.cks != B.cks) {
            fail(NX_ERR_FASTLZ_CRC_MISMATCH, nx::af::flz_checksum_error(R.cks, B.cks));
            return;
        }
        if (j->codec == 2 && j->validate && (R.cks & 0x0FFFFFFFu) != B.cks) {
            fail(NX_ERR_LZ4_CHECKSUM_MISMATCH, nx::af::lz4_checksum_error(R.cks & 0x0FFFFFFFu, B.cks));
            return;
        }
        const bool emit = j->codec == 0 ? B.olen > 0 : (j->codec == 1 ? (B.comp || B.clen > 0) : true);
        if (emit) j->msgs.push_back({bt->out.h + R.off, (size_t)R.len});
    }
    if (j->awerr.set) fail(j->awerr.code, j->awerr.msg);
}

// The batch is complete: turn the result records into each job's messages, in submission order.
void apply(nx_batcher* b, Batch* bt) {
    const int64_t* res_len = reinterpret_cast<const int64_t*>(bt->out.h + bt->res_enc);
    const DecRes* dres = reinterpret_cast<const DecRes*>(bt->out.h + bt->res_dec);
    char buf[160];
    const nx::bt::AltRes* ares = reinterpret_cast<const nx::bt::AltRes*>(bt->out.h + bt->res_alt);
    for (Job* j : bt->jobs) {
        if (j->kind >= 2) {
            apply_alt(bt, j, ares);
            continue;
        }
        if (j->kind == 0) {
            const EncJob& E = bt->ejob[j->index];
            const int64_t r = res_len[j->index];
            if (r < 0) {  // a slice the encoder failed: the job fails (no framed bytes)
                j->status = (int32_t)r;
                j->err = nx_status_string((int32_t)r);
            } else {
                j->msgs.push_back({bt->out.h + E.out_off, (size_t)r});
            }
            j->applied = true;
            continue;
        }
        nx_snappy_frame_decoder* d = j->dec;
        j->applied = true;
        unwalk(j);
        // an earlier job of this decoder failed: Java skips later input (:86-89); or a re-walk after an
        // earlier job's leftover covered this job's bytes
        if (d->corrupted || (d->validate && j->epoch != d->epoch)) {
            trim_hist(d);
            continue;
        }
        const DecJob& J = bt->djob[j->index];
        uint32_t a = J.a0;
        bool failed = false, moved = false;
        for (const SnappyAction& act : j->acts) {
            if (act.kind != SAct::Uncomp && act.kind != SAct::Comp) {
                if (act.kind == SAct::Stream) d->started = true;
                continue;
            }
            const DecRes& R = dres[a];
            const DecAct& A = bt->dact[a];
            ++a;
            if (R.status != NX_OK) {
                j->status = R.status;
                if (R.status == NX_ERR_SNAPPY_CRC_MISMATCH) {
                    snprintf(buf, sizeof buf, "mismatching checksum: %x (expected: %x)", R.crc, A.crc);
                    j->err = buf;
                } else {
                    j->err = nx::fr::snappy_block_error(R.status, R.crc, nx_status_string);
                }
                failed = true;
                break;
            }
            if (R.off == nx::bt::kSpilled) {  // longer than its preamble said, beyond the spill area: from the decode slot (blocking)
                j->owned.emplace_back(R.len);
                const uint8_t* src = bt->slots.as<uint8_t>() + bt->eslots + bt->dslot_off[A.chunk];
                if (hipMemcpy(j->owned.back().data(), src, R.len, hipMemcpyDeviceToHost) != hipSuccess) {
                    j->status = NX_ERR_HIP;
                    j->err = nx_status_string(NX_ERR_HIP);
                    failed = true;
                    break;
                }
                j->msgs.push_back({j->owned.back().data(), (size_t)R.len});
            } else {
                j->msgs.push_back({bt->out.h + R.off, (size_t)R.len});
            }
            if (A.kind == 2 && J.validate && R.cons < A.len) {  // validating-mode leftover (:206-212)
                moved = rewalk(b, bt, j, j->s_base + act.data + R.cons);
                break;
            }
        }
        if (!failed && !moved && j->has_parse_err) {
            j->status = NX_ERR_FRAME_CORRUPT;
            j->err = j->parse_err;
            failed = true;
        }
        if (failed) d->corrupted = true;  // (:227-230)
        trim_hist(d);
    }
    bt->done = true;
}

// Queue the jobs apply() re-walked into the collecting batch (after every job already in it: those of
// the same decoder were walked before the re-walk and deliver nothing).  The next poll()/wait() launches it.
void queue_continuations(nx_batcher* b) {
    // take every moved job out of its batch first, and pin those batches (live) so that none is reset
    // for reuse below while a job listed here may still go back to it
    for (auto& [j, from] : b->cont) {
        for (size_t k = 0; k < from->jobs.size(); ++k)
            if (from->jobs[k] == j) {
                from->jobs.erase(from->jobs.begin() + (ptrdiff_t)k);
                break;
            }
        from->live += 1;
    }
    for (auto& [j, from] : b->cont) {
        Batch* to = b->cur ? b->cur : reuse_or_new_batch(b);
        nx_snappy_frame_decoder* d = j->dec;
        auto it = b->tickets.find(j->ticket);
        const bool live = it != b->tickets.end();
        const uint8_t* S = d->hist.at(j->s_base);  // the owned segment rewalk() made, from s_base on
        if (!to || !S || enqueue_dec(to, j, S, 0, nullptr) != NX_OK) {
            // cannot queue it: the job fails as a launch failure would (result() reports it)
            unwalk(j);
            j->applied = true;
            j->status = NX_ERR_HIP;
            j->err = "GPU batch launch failed";
            d->corrupted = true;
            trim_hist(d);
            from->jobs.push_back(j);  // stays owned by its batch
            continue;
        }
        b->cur = to;
        if (live) {
            if (from->live) from->live -= 1;
            to->live += 1;
            it->second.first = to;
        }
        b->kick = true;
    }
    for (auto& [j, from] : b->cont) from->live -= 1;
    b->cont.clear();
}

// Launch a collecting batch that holds re-walked jobs (their tickets are already out).
void kick(nx_batcher* b) {
    if (!b->kick) return;
    b->kick = false;
    Batch* bt = b->cur;
    if (!bt || bt->jobs.empty()) return;
    b->cur = nullptr;
    (void)launch(b, bt);  // a failed launch completes the batch's jobs with the error
}

// Apply completed batches in flush order up to (and including) sequence number `upto`; false if one
// of them is not complete (non-blocking) or failed.
bool advance(nx_batcher* b, uint64_t upto, bool block) {
    while (b->applied <= upto && b->applied < b->flushes) {
        Batch* bt = nullptr;
        for (Batch* x : b->all)
            if (x->inflight && x->seq == b->applied) bt = x;
        if (!bt) return false;  // unreachable: every launched batch stays in flight until applied
        const hipError_t e = block ? hipEventSynchronize(bt->ev) : hipEventQuery(bt->ev);
        if (e == hipErrorNotReady) (void)hipGetLastError();  // not an error: keep it from the next launch check
        if (e != hipSuccess) return false;
        apply(b, bt);
        bt->inflight = false;
        b->applied += 1;
        if (!b->cont.empty()) queue_continuations(b);
    }
    return true;
}

bool poll_batch(nx_batcher* b, Batch* bt, bool block) {
    if (bt->done) return true;
    if (!bt->inflight) return false;
    return advance(b, bt->seq, block) && bt->done;
}

// Hold the shared workspace of kind k for the batcher's flushes (they run in a NoGrowScope): the full
// reservation, or a smaller one when the device cannot spare it (a flush caps its grid to what is
// held).  Done by the first submit that needs the kind, or up front by nx_batcher_reserve.
bool ensure_held(nx_batcher* b, nx::WsKind k) {
    const uint32_t bit = 1u << (int)k;
    if (b->held & bit) return true;
    const uint32_t first = k == nx::WsKind::SnappyEnc ? nx::kBatcherEncHoldUnits
                         : k == nx::WsKind::DecRecords ? nx::kBatcherDecHoldUnits : nx::kBatcherHoldUnits;
    for (uint32_t u = first; u >= nx::kHandleHoldUnits; u /= 4) {
        if (nx::ws_hold(k, b->dev, u, b->s[0]) == NX_OK) {
            b->held |= bit;
            return true;
        }
    }
    return false;
}

// Auto-flush: launch the collecting batch once its input reaches the threshold (batcher lock held).
int32_t maybe_autoflush(nx_batcher* b, Batch* bt) {
    if (!b->flush_bytes || bt != b->cur || bt->st_used + bt->direct_used < b->flush_bytes) return NX_OK;
    b->cur = nullptr;
    return launch(b, bt);
}

}  // namespace

// ======================================================================= C-ABI
extern "C" nx_batcher* nx_batcher_new(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return nullptr;
    if (nx::crc_tables_init() != NX_OK) return nullptr;
    auto* b = new nx_batcher();
    for (int i = 0; i < kStreams; ++i) {
        if (hipStreamCreateWithFlags(&b->s[i], hipStreamNonBlocking) != hipSuccess) {
            for (int k = 0; k < i; ++k) (void)hipStreamDestroy(b->s[k]);
            delete b;
            return nullptr;
        }
    }
    // The workspaces (one per kind for the whole batcher, whichever of its streams a flush lands on)
    // are held by the first submit that needs them, or by nx_batcher_reserve.
    if (hipGetDevice(&b->dev) != hipSuccess) {
        nx_batcher_free(b);
        return nullptr;
    }
    return b;
}

extern "C" int32_t nx_batcher_reserve(nx_batcher* b, uint32_t kinds) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    for (int k = 0; k < (int)nx::WsKind::Count; ++k)
        if ((kinds >> k) & 1u)
            if (!ensure_held(b, (nx::WsKind)k)) return NX_ERR_HIP;
    return NX_OK;
}

extern "C" void nx_batcher_free(nx_batcher* b) {
    if (!b) return;
    for (int i = 0; i < kStreams; ++i) (void)hipStreamSynchronize(b->s[i]);
    for (Batch* x : b->all) delete x;
    for (int i = 0; i < kStreams; ++i) {
        nx::ws_forget_stream(b->s[i]);  // no workspace event may outlive its stream
        (void)hipStreamDestroy(b->s[i]);
    }
    for (int k = 0; k < (int)nx::WsKind::Count; ++k)
        if ((b->held >> k) & 1u) nx::ws_unhold((nx::WsKind)k, b->dev);
    delete b;
}

extern "C" int32_t nx_host_register(void* p, size_t n) {
    if (!p || !n) return NX_ERR_INVALID_ARG;
    if (hipHostRegister(p, n, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) return NX_ERR_HIP;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipHostUnregister(p);
        return NX_ERR_HIP;
    }
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[(uintptr_t)p] = {n, (uint8_t*)d};
    return NX_OK;
}

extern "C" int32_t nx_host_unregister(void* p) {
    if (!p) return NX_ERR_INVALID_ARG;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.erase((uintptr_t)p);
    }
    return hipHostUnregister(p) == hipSuccess ? NX_OK : NX_ERR_HIP;
}

extern "C" int64_t nx_snappy_frame_encoder_submit(nx_snappy_frame_encoder* e, nx_batcher* b, const uint8_t* in, size_t n,
                                                  int32_t in_registered) {
    if (!e || !b || (!in && n)) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (!ensure_held(b, nx::WsKind::SnappyEnc)) return NX_ERR_HIP;
    Batch* bt = collecting(b);
    if (!bt) return NX_ERR_HIP;
    Job* j = new Job();
    j->ticket = b->next_ticket++;
    j->kind = 0;
    EncJob E{};
    E.s0 = (uint32_t)bt->esl.size();
    if (!bt->reserve_out(nx_snappy_frame_max_encoded_length(n), &E.out_off)) {
        delete j;
        return NX_ERR_HIP;
    }
    if (n) {  // SnappyFrameEncoder.encode (:79-117): !in.isReadable() writes nothing
        E.stream_start = e->started ? 0u : 1u;  // e->started is set below, once the submit cannot fail
        uint64_t base = 0;
        const uint8_t* dsrc = in_registered ? registered_device_ptr(in, n) : nullptr;
        if (in_registered && !dsrc) {
            delete j;
            return NX_ERR_INVALID_ARG;  // not inside an nx_host_register'd range
        }
        const bool direct = dsrc != nullptr;
        if (direct) {  // DMA'd into the device arena's direct region at flush; adjacent inputs share one copy
            Batch::Direct* last = bt->direct.empty() ? nullptr : &bt->direct.back();
            if (last && last->src + last->len == in && last->din_off + last->len == bt->direct_used) {
                base = bt->direct_used;
                last->len += n;
            } else {
                base = (bt->direct_used + 15) & ~15ull;
                bt->direct.push_back({in, dsrc, n, base});
            }
            bt->direct_used = base + n;
        } else {
            uint8_t* st = bt->stage(n, &base);
            if (!st) {
                delete j;
                return NX_ERR_HIP;
            }
            nx::copy_bytes(st, in, n);
        }
        auto add = [&](uint64_t off, uint32_t len, bool comp) {
            EncSlice S{base + off, bt->eslots, len, comp ? 1u : 0u};
            bt->eslots += (nx_snappy_max_compressed_length(len) + 15) & ~(size_t)15;
            bt->esl.push_back(S);
            bt->esl_direct.push_back(direct ? 1 : 0);
        };
        int64_t dl = (int64_t)n;
        if (dl > 18) {  // MIN_COMPRESSIBLE_LENGTH (:46,90-113)
            uint64_t pos = 0;
            for (;;) {
                if (dl < 18) {
                    add(pos, (uint32_t)dl, false);
                    break;
                }
                const uint32_t len = dl > e->slice ? (uint32_t)e->slice : (uint32_t)dl;
                add(pos, len, true);
                pos += len;
                if (dl > e->slice) dl -= e->slice;
                else break;
            }
        } else {
            add(0, (uint32_t)n, false);
        }
        e->started = true;
    }
    E.ns = (uint32_t)bt->esl.size() - E.s0;
    j->index = (uint32_t)bt->ejob.size();
    bt->ejob.push_back(E);
    bt->jobs.push_back(j);
    bt->live += 1;
    b->tickets[j->ticket] = {bt, j};
    (void)maybe_autoflush(b, bt);  // a failed launch completes the job with the error (result())
    return (int64_t)j->ticket;
}

namespace {
int64_t decoder_submit(nx_snappy_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* consumed, bool registered) {
    if (!d || !b || (!in && n) || !consumed) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (!ensure_held(b, nx::WsKind::DecRecords)) return NX_ERR_HIP;
    Batch* bt = collecting(b);
    if (!bt) return NX_ERR_HIP;
    Job* j = new Job();
    j->ticket = b->next_ticket++;
    j->kind = 1;
    j->dec = d;
    size_t p = 0;  // bytes of `in` consumed
    // the chunk-header walk runs now, so the decoder's started/skip state advances in call order; it
    // is committed below, once the job is queued
    bool started = d->started;
    uint64_t skip = d->skip;
    const uint8_t* S = in;  // the walked bytes: a validating decoder's carried bytes, then `in`
    size_t carried = 0, walked = 0;
    std::vector<uint8_t> joined;
    const bool skipping = d->corrupted || d->parse_failed;  // (:86-89): an earlier input failed
    if (skipping) {
        p = n;
    } else {
        if (d->validate) {
            carried = (size_t)(d->hist.end - d->parse_pos);
            if (carried) {
                joined.reserve(carried + n);
                d->hist.copy_from(d->parse_pos, joined);
                joined.insert(joined.end(), in, in + n);
                S = joined.data();
            }
        }
        walked = walk(d, j, S, carried + n, started, skip);
        p = walked > carried ? walked - carried : 0;
    }
    // registered cumulation: the consumed bytes are gathered from the mapped pages at flush (the
    // caller keeps them valid until the job completes); else every payload is copied now
    const uint8_t* dS = nullptr;
    if (registered && walked && !carried) {
        dS = registered_device_ptr(in, walked);
        if (!dS) {  // not inside an nx_host_register'd range
            j->dec = nullptr;
            delete j;
            return NX_ERR_INVALID_ARG;
        }
    }
    // a validating decoder stages the walked bytes whole (headers too): the payloads are slices of
    // that copy, and its history references it instead of copying the bytes a second time
    int64_t staged = -1;
    if (d->validate && !dS && walked) {
        uint64_t off = 0;
        uint8_t* st = bt->stage(walked, &off);
        if (!st) {
            j->dec = nullptr;
            delete j;
            return NX_ERR_HIP;
        }
        nx::copy_bytes(st, S, walked);
        staged = (int64_t)off;
    }
    if (enqueue_dec(bt, j, S, walked, dS, staged) != NX_OK) {
        j->dec = nullptr;  // no reference taken yet
        delete j;
        return NX_ERR_HIP;
    }
    d->refs.fetch_add(1);  // released with the job (~Job)
    *consumed = p;
    if (!skipping) {
        d->started = started;
        d->skip = skip;
        // later submits skip their input (:227-230); the decoder turns corrupted when this job is
        // applied, after the jobs submitted before it have delivered their messages
        if (j->has_parse_err) d->parse_failed = true;
    }
    if (d->validate && !d->corrupted) {
        // every consumed byte is kept until no unapplied job can re-walk it (a leftover, :206-212);
        // skipped input too, since a re-walk may find that the failure was not reached after all
        // a registered cumulation stays valid until this job completes, and so does the job's copy in
        // the staging arena: referenced, not copied
        if (staged >= 0)
            d->hist.append_staged(&bt->staging.h, (uint64_t)staged + carried, p);
        else
            d->hist.append(in, p, !registered);
        if (!skipping) {
            j->s_base = d->parse_pos;
            j->epoch = d->epoch;
            j->walked = true;
            d->outstanding.insert(j->s_base);
            d->parse_pos += walked;
        }
    }
    bt->live += 1;
    b->tickets[j->ticket] = {bt, j};
    (void)maybe_autoflush(b, bt);  // a failed launch completes the job with the error (result())
    return (int64_t)j->ticket;
}
}  // namespace

extern "C" int64_t nx_snappy_frame_decoder_submit(nx_snappy_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                                  size_t* consumed) {
    return decoder_submit(d, b, in, n, consumed, false);
}

extern "C" int64_t nx_snappy_frame_decoder_submit_registered(nx_snappy_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                                             size_t* consumed) {
    return decoder_submit(d, b, in, n, consumed, true);
}

// ---------------------------------------------------------------- FastLZ / LZF / LZ4 submits
namespace {
using nx::bt::AltPiece;

inline uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

// Register job j (its pieces already in bt->apc from p0 on) with an output reservation of `out_need`.
int64_t queue_alt(nx_batcher* b, Batch* bt, Job* j, uint32_t p0, size_t out_need) {
    nx::bt::AltJobD J{};
    J.p0 = p0;
    J.np = (uint32_t)bt->apc.size() - p0;
    if (!bt->reserve_out(out_need + 16, &J.out_off)) return NX_ERR_HIP;
    j->index = (uint32_t)bt->ajob.size();
    bt->ajob.push_back(J);
    bt->jobs.push_back(j);
    bt->live += 1;
    b->tickets[j->ticket] = {bt, j};
    (void)maybe_autoflush(b, bt);  // a failed launch completes the job with the error (result())
    return (int64_t)j->ticket;
}

// Undo the pieces / list entries a failed submit added (the batch's other jobs stay valid).
struct AltMark {
    size_t apc, fe, le, ze, fd, ld, zd;
    uint64_t aslots;
    explicit AltMark(const Batch* bt)
        : apc(bt->apc.size()), fe(bt->flz_e.size()), le(bt->lzf_e.size()), ze(bt->lz4_e.size()), fd(bt->flz_d.size()),
          ld(bt->lzf_d.size()), zd(bt->lz4_d.size()), aslots(bt->aslots) {}
    void undo(Batch* bt) const {
        auto cut = [](Batch::AltList& L, size_t n) {
            L.off.resize(n);
            L.slot.resize(n);
            L.len.resize(n);
            L.aux.resize(n);
            if (!L.lim.empty()) L.lim.resize(n);
        };
        bt->apc.resize(apc);
        cut(bt->flz_e, fe);
        cut(bt->lzf_e, le);
        cut(bt->lz4_e, ze);
        cut(bt->flz_d, fd);
        cut(bt->lzf_d, ld);
        cut(bt->lz4_d, zd);
        bt->aslots = aslots;
    }
};

uint32_t push_list(Batch::AltList& L, uint64_t off, uint32_t len, uint64_t slot, uint32_t aux, int32_t lim = 0) {
    L.off.push_back(off);
    L.len.push_back(len);
    L.slot.push_back(slot);
    L.aux.push_back(aux);
    L.lim.push_back(lim);
    return (uint32_t)L.off.size() - 1;
}

Job* new_alt_job(nx_batcher* b, int kind, int codec) {
    Job* j = new Job();
    j->ticket = b->next_ticket++;
    j->kind = kind;
    j->codec = codec;
    return j;
}

// Decoder submit, shared by the three codecs: the header walk runs now (the decoder's state advances
// in call order, as ByteToMessageDecoder would call decode()); the walked bytes are staged; the blocks
// decode at flush; apply() delivers messages / the first failure in order.
template <class D, class St, class Walk>
int64_t alt_decoder_submit(D* d, St& st, nx_batcher* b, const uint8_t* in, size_t n, size_t* consumed, int codec, bool validate,
                           Walk walk) {
    if (!d || !b || (!in && n) || !consumed) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (!ensure_held(b, nx::WsKind::DecRecords)) return NX_ERR_HIP;
    Batch* bt = collecting(b);
    if (!bt) return NX_ERR_HIP;
    Job* j = new_alt_job(b, 3, codec);
    j->validate = validate;
    const AltMark mark(bt);
    const uint32_t p0 = (uint32_t)bt->apc.size();
    size_t p = n;
    size_t out_need = 0;
    St ns = st;
    const bool skipping = d->corrupted || d->parse_failed;  // an earlier input failed: Java skips everything
    if (!skipping) {
        p = walk(in, n, ns, j->ablk, j->awerr);
        if (j->awerr.set) p = n;  // the rest is skipped once the decoder is corrupted
    }
    if (!j->ablk.empty()) {
        // stage from the first block on; FastLZ's decompress() may read on to the end of the cumulation
        const size_t lo = j->ablk.front().data, hi = codec == 0 ? n : j->ablk.back().end;
        uint64_t off = 0;
        uint8_t* stg = bt->stage(hi - lo, &off);
        if (!stg) {
            delete j;
            return NX_ERR_HIP;
        }
        nx::copy_bytes(stg, in + lo, hi - lo);
        j->astage = off - lo;  // block b's payload is at staging offset astage + b.data
        for (const nx::af::Blk& k : j->ablk) {
            AltPiece P{};
            P.src = j->astage + k.data;
            P.len = k.clen;
            P.olen = k.olen;
            const bool cks = validate && k.has_cks;
            P.pad = cks ? (codec == 0 ? 1u : 2u) : 0u;  // checksum kind: 1 Adler32, 2 XXH32 (assigned at launch)
            if (!k.comp) {
                P.kind = nx::bt::AK_DEC_RAW;
            } else {
                P.slot = bt->aslots;
                bt->aslots += align16(k.olen) + 16;
                Batch::AltList& L = codec == 0 ? bt->flz_d : (codec == 1 ? bt->lzf_d : bt->lz4_d);
                // FastLZ: aux = in_avail (readable bytes from the block on), lim = originalLength;
                // LZF / LZ4: aux = the decoded length
                P.res = push_list(L, P.src, k.clen, P.slot, codec == 0 ? (uint32_t)(n - k.data) : k.olen, (int32_t)k.olen);
                P.kind = codec == 0 ? nx::bt::AK_DEC_FLZ : (codec == 1 ? nx::bt::AK_DEC_LZF : nx::bt::AK_DEC_LZ4);
            }
            bt->apc.push_back(P);
            out_need += align16(k.olen);
        }
    }
    const int64_t t = queue_alt(b, bt, j, p0, out_need);
    if (t < 0) {
        mark.undo(bt);
        delete j;
        return t;
    }
    j->adec = d;
    d->refs.fetch_add(1);  // released with the job (~Job)
    *consumed = p;
    if (!skipping) {
        st = ns;
        if (j->awerr.set) d->parse_failed = true;  // later submits skip; corrupted once applied
    }
    return t;
}
}  // namespace

extern "C" int64_t nx_fastlz_frame_decoder_submit(nx_fastlz_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                                  size_t* consumed) {
    if (!d) return NX_ERR_INVALID_ARG;
    return alt_decoder_submit(d, d->st, b, in, n, consumed, 0, d->validate, nx::af::flz_walk);
}

extern "C" int64_t nx_lzf_decoder_submit(nx_lzf_decoder* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* consumed) {
    if (!d) return NX_ERR_INVALID_ARG;
    return alt_decoder_submit(d, d->st, b, in, n, consumed, 1, false, nx::af::lzf_walk);
}

extern "C" int64_t nx_lz4_frame_decoder_submit(nx_lz4_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                               size_t* consumed) {
    if (!d || !b || (!in && n) || !consumed) return NX_ERR_INVALID_ARG;
    if (d->st.state == 2 && !d->corrupted && !d->parse_failed) {  // FINISHED: everything is skipped (:250-254)
        std::lock_guard<std::mutex> lk(b->mu);
        Batch* bt = collecting(b);
        if (!bt) return NX_ERR_HIP;
        Job* j = new_alt_job(b, 3, 2);
        const int64_t t = queue_alt(b, bt, j, (uint32_t)bt->apc.size(), 0);
        if (t < 0) {
            delete j;
            return t;
        }
        j->adec = d;
        d->refs.fetch_add(1);
        *consumed = n;
        return t;
    }
    return alt_decoder_submit(d, d->st, b, in, n, consumed, 2, d->validate, nx::af::lz4_walk);
}

// FastLzFrameEncoder.encode(ctx, in, out) over buf[r0 .. r0 + n) as a job (the reader index enters the
// readU16 quirk, FastLz.java:552-557).  The message is copied now.
extern "C" int64_t nx_fastlz_frame_encoder_submit(nx_fastlz_frame_encoder* e, nx_batcher* b, const uint8_t* buf, size_t r0, size_t n) {
    if (!e || !b || (!buf && n)) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (!ensure_held(b, nx::WsKind::FastLzEnc)) return NX_ERR_HIP;
    Batch* bt = collecting(b);
    if (!bt) return NX_ERR_HIP;
    Job* j = new_alt_job(b, 2, 0);
    const AltMark mark(bt);
    const uint32_t p0 = (uint32_t)bt->apc.size();
    if (n) {
        uint64_t off = 0;
        uint8_t* stg = bt->stage(n, &off);
        if (!stg) {
            delete j;
            return NX_ERR_HIP;
        }
        nx::copy_bytes(stg, buf + r0, n);
        std::vector<nx::af::FlzPlan> plan;
        nx::af::flz_plan(r0, n, plan);
        for (const nx::af::FlzPlan& q : plan) {
            AltPiece P{};
            P.kind = nx::bt::AK_FLZ_ENC;
            P.src = off + q.ioff;
            P.len = q.ilen;
            P.slot = bt->aslots;
            bt->aslots += align16(nx_fastlz_max_compressed_length(q.ilen) + 16);
            P.res = push_list(bt->flz_e, P.src, q.ilen, P.slot, (uint32_t)e->level, q.lim);
            P.aux = e->checksum ? 1u : 0u;
            bt->apc.push_back(P);
        }
    }
    const int64_t t = queue_alt(b, bt, j, p0, nx_fastlz_frame_max_encoded_length(n));
    if (t < 0) {
        mark.undo(bt);
        delete j;
    }
    return t;
}

// LzfEncoder.encode(ctx, in, out) as a job (LzfEncoder.java:169-246): below the compress threshold the
// message leaves as non-compressed blocks, else every 65535-byte chunk goes to the GPU encoder.
extern "C" int64_t nx_lzf_encoder_submit(nx_lzf_encoder* e, nx_batcher* b, const uint8_t* in, size_t n) {
    if (!e || !b || (!in && n)) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (!ensure_held(b, nx::WsKind::LzfEnc)) return NX_ERR_HIP;
    Batch* bt = collecting(b);
    if (!bt) return NX_ERR_HIP;
    Job* j = new_alt_job(b, 2, 1);
    const AltMark mark(bt);
    const uint32_t p0 = (uint32_t)bt->apc.size();
    uint64_t off = 0;
    if (n) {
        uint8_t* stg = bt->stage(n, &off);
        if (!stg) {
            delete j;
            return NX_ERR_HIP;
        }
        nx::copy_bytes(stg, in, n);
    }
    const bool comp = (int64_t)n >= e->threshold;
    size_t ip = 0;
    do {  // encodeNonCompress writes one (possibly empty) block even for n == 0 (:223-246)
        const uint32_t len = (uint32_t)((n - ip) < 65535 ? (n - ip) : 65535);
        AltPiece P{};
        P.src = off + ip;
        P.len = len;
        if (comp) {
            P.kind = nx::bt::AK_LZF_ENC;
            P.slot = bt->aslots;
            bt->aslots += align16(nx_lzf_max_compressed_length(len) + 16);
            P.res = push_list(bt->lzf_e, P.src, len, P.slot, 0);
        } else {
            P.kind = nx::bt::AK_LZF_RAW;
        }
        bt->apc.push_back(P);
        ip += len;
    } while (ip < n);
    const int64_t t = queue_alt(b, bt, j, p0, nx_lzf_frame_max_encoded_length(n));
    if (t < 0) {
        mark.undo(bt);
        delete j;
    }
    return t;
}

// Lz4FrameEncoder as jobs: op 0 = encode(in) (full blocks of the block buffer leave, :231-248), 1 =
// flush() (the partial block too, :291-300), 2 = close() (flush + the end block, :317-336; afterwards
// encode passes bytes through, :233-239).  The handle's block buffer advances at submit.
extern "C" int64_t nx_lz4_frame_encoder_submit(nx_lz4_frame_encoder* e, nx_batcher* b, const uint8_t* in, size_t n, int32_t op) {
    if (!e || !b || (!in && n) || op < 0 || op > 2) return NX_ERR_INVALID_ARG;
    // allocateBuffer's maxEncodeSize check (Lz4FrameEncoder.java:190-214): write() sizes the message
    // plus the buffered bytes; a bare flush (op 1, no bytes) sizes the buffer (:296-304); finishEncode
    // checks nothing (:306-315).  Nothing is queued or buffered when it fails.
    if (n > 0 || op == 0 || (op == 1 && !e->buf.empty())) {
        int32_t target = 0;
        int32_t r = nx_lz4_frame_encoder_check_size(e, (uint64_t)n + e->buf.size(), &target);
        if (r == NX_OK) r = nx_lz4_frame_encoder_check_finished(e, n, target);  // IllegalStateException after close
        if (r != NX_OK) return r;
    }
    std::lock_guard<std::mutex> lk(b->mu);
    if (!ensure_held(b, e->high ? nx::WsKind::Lz4HcEnc : nx::WsKind::Lz4Enc)) return NX_ERR_HIP;
    Batch* bt = collecting(b);
    if (!bt) return NX_ERR_HIP;
    Job* j = new_alt_job(b, 2, 2);
    const AltMark mark(bt);
    const uint32_t p0 = (uint32_t)bt->apc.size();
    std::vector<uint8_t> nbuf;  // the block buffer after this job
    size_t out_need = 0;
    auto fail = [&](int64_t code) {
        mark.undo(bt);
        delete j;
        return code;
    };
    if (e->finished) {  // pass-through (:233-239); flush / close after close write nothing
        if (n) {
            uint64_t off = 0;
            uint8_t* stg = bt->stage(n, &off);
            if (!stg) return fail(NX_ERR_HIP);
            nx::copy_bytes(stg, in, n);
            AltPiece P{};
            P.kind = nx::bt::AK_RAW;
            P.src = off;
            P.len = (uint32_t)n;
            bt->apc.push_back(P);
            out_need = n;
        }
        nbuf = e->buf;
    } else {
        const size_t have = e->buf.size(), total = have + n, bs = e->block_size;
        const size_t full = op == 0 ? total / bs * bs : total;  // flush / close take the partial block too
        if (full) {
            uint64_t off = 0;
            uint8_t* stg = bt->stage(full, &off);
            if (!stg) return fail(NX_ERR_HIP);
            const size_t from_buf = have < full ? have : full;
            nx::copy_bytes(stg, e->buf.data(), from_buf);
            if (full > from_buf) nx::copy_bytes(stg + from_buf, in, full - from_buf);
            for (size_t q = 0; q < full; q += bs) {
                const uint32_t len = (uint32_t)((full - q) < bs ? (full - q) : bs);
                AltPiece P{};
                P.kind = nx::bt::AK_LZ4_ENC;
                P.src = off + q;
                P.len = len;
                P.slot = bt->aslots;
                const uint64_t cap = nx::af::kLz4Header + nx_lz4_max_compressed_length(len);
                bt->aslots += align16(cap) + 16;
                P.res = push_list(bt->lz4_e, P.src, len, P.slot, (uint32_t)e->level | (e->high ? 0x100u : 0u));
                bt->apc.push_back(P);
                out_need += cap;
            }
        }
        if (full < have) nbuf.assign(e->buf.begin() + (ptrdiff_t)full, e->buf.end());  // (op 0 with a short input)
        if (full >= have) nbuf.assign(in + (full - have), in + n);
        else nbuf.insert(nbuf.end(), in, in + n);
        if (op == 2) {
            AltPiece P{};
            P.kind = nx::bt::AK_LZ4_END;
            P.aux = (uint32_t)e->level;
            bt->apc.push_back(P);
            out_need += nx::af::kLz4Header;
        }
    }
    const int64_t t = queue_alt(b, bt, j, p0, out_need);
    if (t < 0) return fail(t);
    if (!e->finished) e->buf.swap(nbuf);
    if (op == 2) e->finished = true;
    return t;
}

extern "C" int32_t nx_batcher_flush(nx_batcher* b) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    b->kick = false;
    Batch* bt = b->cur;
    if (!bt || bt->jobs.empty()) return NX_OK;
    b->cur = nullptr;
    return launch(b, bt);
}

extern "C" int32_t nx_batcher_poll(nx_batcher* b, int64_t ticket) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    auto it = b->tickets.find((uint64_t)ticket);
    if (it == b->tickets.end()) return NX_ERR_INVALID_ARG;
    Job* j = it->second.second;
    (void)poll_batch(b, it->second.first, false);
    kick(b);
    return j->applied ? 1 : 0;  // a re-walked job continues in a later batch
}

extern "C" int32_t nx_batcher_wait(nx_batcher* b, int64_t ticket) {
    if (!b) return NX_ERR_INVALID_ARG;
    for (;;) {  // more than one pass only when a re-walk moved the job to a later batch
        Batch* bt;
        Job* j;
        {
            std::lock_guard<std::mutex> lk(b->mu);
            auto it = b->tickets.find((uint64_t)ticket);
            if (it == b->tickets.end()) return NX_ERR_INVALID_ARG;
            bt = it->second.first;
            j = it->second.second;
            if (bt == b->cur) {  // not flushed yet: flush now
                b->cur = nullptr;
                (void)launch(b, bt);  // a failed launch completes the batch's jobs with the error
            }
            if (j->applied) return NX_OK;
        }
        if (hipEventSynchronize(bt->ev) != hipSuccess) return NX_ERR_HIP;
        std::lock_guard<std::mutex> lk(b->mu);
        // Unlocked, another thread's apply() may have moved the job into a continuation batch (a
        // re-walk), after which bt can be reset and reused: look the ticket up again, and wait on
        // its new batch if it moved.
        auto it = b->tickets.find((uint64_t)ticket);
        if (it == b->tickets.end()) return NX_ERR_INVALID_ARG;
        if (it->second.first != bt) continue;
        if (!poll_batch(b, bt, true)) return NX_ERR_HIP;
        kick(b);
        if (j->applied) return NX_OK;
    }
}

extern "C" int32_t nx_batcher_result(nx_batcher* b, int64_t ticket, const nx_msg** msgs, size_t* n_msgs, const char** err_msg) {
    if (!b || !msgs || !n_msgs) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    auto it = b->tickets.find((uint64_t)ticket);
    if (it == b->tickets.end()) return NX_ERR_INVALID_ARG;
    Job* j = it->second.second;
    if (!j->applied) return NX_ERR_INVALID_ARG;  // poll() / wait() first
    *msgs = j->msgs.data();
    *n_msgs = j->msgs.size();
    if (err_msg) *err_msg = j->err.empty() ? nullptr : j->err.c_str();
    return j->status;
}

extern "C" int32_t nx_batcher_release(nx_batcher* b, int64_t ticket) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    auto it = b->tickets.find((uint64_t)ticket);
    if (it == b->tickets.end()) return NX_ERR_INVALID_ARG;
    Batch* bt = it->second.first;
    b->tickets.erase(it);
    if (bt->live) bt->live -= 1;
    return NX_OK;
}

extern "C" int32_t nx_batcher_set_flush_bytes(nx_batcher* b, size_t bytes) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    b->flush_bytes = bytes;
    return NX_OK;
}

// Size the pinned arenas now: at least `nbatches` batch objects, each with a staging arena of
// staging_bytes and a result arena of out_bytes, so that submits (on the event loops) never call
// hipHostMalloc / hipHostFree once batches stay within those sizes (set the auto-flush threshold
// below staging_bytes).
extern "C" int32_t nx_batcher_reserve_arenas(nx_batcher* b, uint32_t nbatches, size_t staging_bytes, size_t out_bytes) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    std::vector<Batch*> made;
    while (b->all.size() < nbatches) {
        Batch* x = new Batch();
        if (hipEventCreateWithFlags(&x->ev, hipEventDisableTiming) != hipSuccess) {
            delete x;
            return NX_ERR_HIP;
        }
        x->staging.cnt = x->out.cnt = x->gops.cnt = &b->arena;
        b->all.push_back(x);
    }
    // A batch that holds jobs is left alone: an in-flight batch's arenas are being written, and the
    // results of an applied batch whose tickets are not all released (nx_batcher_result's messages),
    // or the staged bytes a collecting batch's jobs point into, live in its arenas; growing one
    // frees the old buffer under them.  Such a batch is sized when it is reused (reset, then staged).
    for (Batch* x : b->all)
        if (!x->inflight && x->live == 0 && x->jobs.empty() &&
            (!x->staging.ensure(staging_bytes, x->st_used) || !x->out.ensure(out_bytes, x->out_used) || !x->gops.ensure(1u << 20, 0)))
            return NX_ERR_HIP;
    return NX_OK;
}

extern "C" int32_t nx_batcher_arena_stats(nx_batcher* b, uint64_t* allocs, uint64_t* bytes, uint32_t* batches) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (allocs) *allocs = b->arena.allocs;
    if (bytes) *bytes = b->arena.bytes;
    if (batches) *batches = (uint32_t)b->all.size();
    return NX_OK;
}

extern "C" int32_t nx_batcher_dma_stats(nx_batcher* b, uint64_t* dma_flushes, uint64_t* dma_bytes) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (dma_flushes) *dma_flushes = b->dma_flushes;
    if (dma_bytes) *dma_bytes = b->dma_bytes;
    return NX_OK;
}

extern "C" int32_t nx_batcher_stats(nx_batcher* b, uint64_t* flushes, uint64_t* launches, uint64_t* chunks) {
    if (!b) return NX_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (flushes) *flushes = b->flushes;
    if (launches) *launches = b->launches;
    if (chunks) *chunks = b->chunks;
    return NX_OK;
}
