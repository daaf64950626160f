// snappy_frame_scan.hip — SnappyFrameDecoder's chunk walk over device-resident cumulations
// (SURVEY.md §8f row 1).
//
// Replaces the framing half of SnappyFrameDecoder.decode (SnappyFrameDecoder.java:85-231) as
// ByteToMessageDecoder.callDecode drives it (ByteToMessageDecoder.java:464-517: decode() again for
// as long as it reads bytes).  The data half — Snappy.decode + validateChecksum of each chunk — is
// nx_snappy_decode_batch (COMPRESSED_DATA) and nx_crc32c_masked_batch (UNCOMPRESSED_DATA), fed
// straight from the list this kernel writes, so a cumulation that is already in HBM never returns
// to the host to be framed.
//
// One lane per stream (one connection's cumulation).  The chunk chain is serial by construction —
// each header gives the position of the next — so the parallelism is across streams.  A lane reads
// 4 header bytes (plus the preamble varint of a compressed chunk) per chunk: at 64 KiB chunks that
// is ~0.01 % of the bytes the decoder moves.
//
// Data chunks go to one list of `cap` entries in structure-of-arrays form, so its arrays are the
// in_off / in_len / expected_masked_crc arguments of the batch kernels as they stand:
// COMPRESSED_DATA entries fill [0, counts[0]) and UNCOMPRESSED_DATA entries fill
// [cap - counts[1], cap).  Entries are claimed with atomics, so their order across streams is not
// fixed; chunk_stream / chunk_seq give each entry's stream and its position among that stream's
// data chunks.
#include <stdio.h>
#include <stdlib.h>
#include <mutex>
#include <vector>
#include "nx_common.hpp"
#include "../../include/netty_amd.h"

namespace nx {
namespace fscan {

typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
typedef v4u_ __attribute__((aligned(1))) v4uu_;
typedef __attribute__((address_space(1))) const v4uu_ gv4uu_;

// The 16 bytes at b[p, p + 16) as four LE dwords (one unaligned dwordx4 load), zero past len: a chunk
// header (type, length, masked CRC) and the preamble varint behind it in one memory round trip.
__device__ __forceinline__ uint4 hdr16(const uint8_t* __restrict__ b, uint64_t len, uint64_t p) {
    if (p + 16u <= len) {
        const v4u_ v = *(gv4uu_*)(b + p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < 16u && p + i < len; ++i) w[i >> 2] |= (uint32_t)b[p + i] << (8u * (i & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint32_t byte_of(const uint4& h, uint32_t i) {
    const uint32_t d = i < 4u ? h.x : (i < 8u ? h.y : (i < 12u ? h.z : h.w));
    return (d >> (8u * (i & 3u))) & 0xFFu;
}

// The chunk walk of SnappyFrameDecoder.decode (:85-231) from position w.p up to the first header at
// or after `stop` (or the end of the readable bytes, an error, or a list entry refused by `emit`).
// emit(type, header_pos, chunkLength, stored_crc) lists a data chunk and returns false when the list
// cannot take it (the walk then stops before the chunk).  k_frame_scan walks a whole cumulation with
// it; the segmented long-stream path below walks 1 MiB segments with it.
enum WalkEnd : uint32_t { kOpen = 0, kEnd = 1, kError = 2, kFull = 3 };
struct Walk {
    uint64_t p;
    uint64_t skip;  // numBytesToSkip (< 2^24: a chunk length)
    bool started;
    int32_t res;
};
template <class Emit>
__device__ WalkEnd walk(const uint8_t* __restrict__ b, uint64_t len, Walk& w, uint64_t stop, Emit&& emit) {
    uint64_t p = w.p, skip = w.skip;
    bool started = w.started;
    int32_t res = NX_OK;
    WalkEnd how = kEnd;
    while (p < len) {
        if (skip) {  // :91-99
            const uint64_t k = skip < len - p ? skip : len - p;
            p += k;
            skip -= k;
            continue;
        }
        if (p >= stop) {
            how = kOpen;
            break;
        }
        const uint64_t avail = len - p;
        if (avail < 4) break;  // :104-108
        const uint4 h = hdr16(b, len, p);
        const uint32_t type = h.x & 0xFFu;
        const uint32_t clen = h.x >> 8;
        if (type == 0xFFu) {  // STREAM_IDENTIFIER :115-136
            if (clen != 6u) {
                res = NX_ERR_SNAPPY_STREAM_ID_LENGTH;
                break;
            }
            if (avail < 10) break;
            p += 10;  // skipBytes(4 + 6) precede the content check (:124-133)
            if (h.y != 0x50614E73u || (h.z & 0xFFFFu) != 0x5970u) {  // "sNaPpY"

                res = NX_ERR_SNAPPY_STREAM_ID_CONTENT;
                break;
            }
            started = true;
            continue;
        }
        if (type & 0x80u) {  // RESERVED_SKIPPABLE :137-151
            if (!started) {
                res = NX_ERR_SNAPPY_SKIPPABLE_BEFORE_ID;
                break;
            }
            p += 4;
            const uint64_t k = clen < len - p ? (uint64_t)clen : len - p;
            p += k;
            skip = clen - k;
            continue;
        }
        if (type > 1u) {  // RESERVED_UNSKIPPABLE :152-157
            res = NX_ERR_SNAPPY_UNSKIPPABLE;
            break;
        }
        if (!started) {  // :159-161, :181-183
            res = type ? NX_ERR_SNAPPY_UNCOMPRESSED_BEFORE_ID : NX_ERR_SNAPPY_COMPRESSED_BEFORE_ID;
            break;
        }
        if (type == 1u && clen > 65536u + 4u) {  // :162-165
            res = NX_ERR_SNAPPY_UNCOMPRESSED_TOO_LARGE;
            break;
        }
        if (avail < 4ull + clen) break;  // :167-169, :190-192
        if (clen < 4u) {  // the 4-byte checksum does not fit the chunk
            res = NX_ERR_SNAPPY_CHUNK_TOO_SHORT;
            break;
        }
        if (type == 0u) {
            // snappy.getPreamble(in) reads the varint from the cumulation, not the chunk
            // (Snappy.java:404-441), then :197-201 bounds it.
            uint32_t ulen = 0;
            bool complete = false;
            for (uint32_t i = 0; i < 4u && p + 8 + i < len; ++i) {
                const uint32_t c = byte_of(h, 8u + i);
                ulen |= (c & 0x7Fu) << (7u * i);
                if (!(c & 0x80u)) {
                    complete = true;
                    break;
                }
                if (i == 3u) res = NX_ERR_SNAPPY_PREAMBLE_TOO_LONG;
            }
            if (res) break;
            if (!complete) ulen = 0;
            if (ulen > 65536u) {
                res = NX_ERR_SNAPPY_DECOMPRESSED_TOO_LARGE;
                break;
            }
        }
        if (!emit(type, p, clen, h.y)) {  // a full list stops the stream before this chunk
            res = NX_SCAN_LIST_FULL;
            how = kFull;
            break;
        }
        p += 4ull + clen;
    }
    if (res < 0) how = kError;
    w.p = p;
    w.skip = skip;
    w.started = started;
    w.res = res;
    return how;
}

// One lane per cumulation.
__global__ void __launch_bounds__(256) k_frame_scan(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                    const uint64_t* __restrict__ in_len, uint32_t* __restrict__ state,
                                                    uint64_t* __restrict__ consumed, int32_t* __restrict__ status,
                                                    uint64_t* __restrict__ data_off, uint32_t* __restrict__ data_len,
                                                    uint32_t* __restrict__ masked_crc, uint32_t* __restrict__ chunk_stream,
                                                    uint32_t* __restrict__ chunk_seq, uint32_t* __restrict__ counts,
                                                    uint32_t cap, uint32_t n) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint64_t base = in_off[s];
    const uint8_t* b = in + base;
    const uint64_t len = in_len[s];
    const uint32_t st = state[s];
    bool corrupted = (st >> 1) & 1u;
    Walk w{0, st >> 8, (st & 1u) != 0, NX_OK};
    uint32_t seq = 0;
    if (corrupted) {  // :86-89 — everything readable is discarded
        w.p = len;
    } else {
        walk(b, len, w, ~0ull, [&](uint32_t type, uint64_t p, uint32_t clen, uint32_t crc) {
            if (atomicAdd(&counts[2], 1u) >= cap) return false;
            const uint32_t k = type == 0u ? atomicAdd(&counts[0], 1u) : cap - 1u - atomicAdd(&counts[1], 1u);
            data_off[k] = base + p + 8;
            data_len[k] = clen - 4u;
            masked_crc[k] = crc;
            chunk_stream[k] = s;
            chunk_seq[k] = seq++;
            return true;
        });
    }
    if (w.res < 0) corrupted = true;  // :227-230
    consumed[s] = w.p;
    status[s] = w.res;
    state[s] = (w.started ? 1u : 0u) | (corrupted ? 2u : 0u) | ((uint32_t)w.skip << 8);
}

// ------------------------------------------------------------------------------------------------
// Segmented walk of ONE long cumulation (round 5).  The chain is serial — each
// header gives the next header's position — so a lone lane needs one dependent memory round trip
// per chunk (~35 K for 1 GiB of 30 KB chunks).  Here the cumulation is cut into segments of SEG bytes:
//   k_seg_guess  — one workgroup per segment j >= 1 finds the first position q >= j*SEG from which
//                  four consecutive hops are plausible data-chunk headers (type 0 or 1, lengths and
//                  preamble within the decoder's limits).  A guess is only a speculation;
//   k_seg_count  — one lane per segment walks (walk() above, the exact decoder semantics) from its
//                  guess (segment 0: from 0 with the caller's state) to the first header at or past
//                  the segment's end, counting data chunks;
//   k_seg_stitch — one workgroup follows the true chain through the segments: the walk of segment
//                  j is accepted only if it started exactly where the previous accepted walk left
//                  off; otherwise (a wrong or missing guess) the workgroup re-walks the segment from
//                  the true position.  It prefix-sums the accepted segments' counts, claims list
//                  entries (stopping at the list capacity as the lane walk does) and writes the
//                  cumulation's consumed / status / state;
//   k_seg_emit   — one lane per accepted segment walks it again and writes its list entries.
// The result equals the lane walk's whatever the guesses: they decide only how much is walked twice.
constexpr uint64_t kSegBytes = 1ull << 20;
constexpr uint32_t kSegMax = 1024;          // segments per cumulation (the segment size doubles beyond 1 GiB)
constexpr uint32_t kGuessWindow = 1u << 17; // guesses are searched in the first 128 KiB of a segment
constexpr uint64_t kNone = ~0ull;

struct SegInfo {
    uint64_t entry;  // where the segment's walk started (kNone: no guess)
    uint64_t exit;   // its Walk.p at the end
    uint64_t skip;
    uint32_t ncomp, nunc;
    uint32_t how;    // WalkEnd
    int32_t res;
    uint32_t started;
    uint32_t pad;
};
struct SegStep {     // one accepted segment, in chain order
    uint32_t seg, o0, o1, pad;  // its first compressed / uncompressed entry among the stream's
};
struct SegPath {
    uint32_t nseg;         // accepted segments
    uint32_t base0, base1; // list slots of the stream's first compressed / uncompressed entry
    uint32_t limit;        // data chunks that get entries (fewer than the chain's when the list fills)
    uint32_t state_in;     // the cumulation's decoder state before the walk
    uint32_t stats[3];     // diagnostics (NX_SCAN_STATS): straight prefix J, parallel re-walks, serial re-walks
};

// A plausible data-chunk header: type 0 / 1, a length the decoder accepts for that type (a
// compressed chunk no longer than Snappy's bound for 64 KiB plus its checksum), a compressed chunk's
// preamble a varint of at most 3 bytes and <= 65536.  Only a speculation filter: the stitch accepts
// nothing it has not walked exactly.
constexpr uint32_t kMaxCompChunk = 4u + 32u + 65536u + 65536u / 6u;
__device__ __forceinline__ bool hop_ok(uint32_t type, uint32_t clen, uint32_t v0, uint32_t v1, uint32_t v2) {
    if (type > 1u || clen < 5u || clen > (type ? 65540u : kMaxCompChunk)) return false;
    if (type == 0u) {
        uint32_t ulen = v0 & 0x7Fu;
        if (v0 & 0x80u) {
            ulen |= (v1 & 0x7Fu) << 7;
            if (v1 & 0x80u) {
                if (v2 & 0x80u) return false;
                ulen |= v2 << 14;
            }
        }
        if (ulen > 65536u) return false;
    }
    return true;
}

// Do the chunks after the one at q (of total size 4 + clen) continue plausibly for three more hops?
// Reaching the end exactly counts as plausible.
__device__ __forceinline__ bool plausible_tail(const uint8_t* __restrict__ b, uint64_t len, uint64_t q) {
    for (int h = 1; h < 4; ++h) {
        if (q == len) return true;
        if (q > len) return h > 1;  // the candidate's own chunk must fit; a later one may be cut off
        if (q + 9 > len) return true;
        const uint4 x = hdr16(b, len, q);
        const uint32_t type = x.x & 0xFFu, clen = x.x >> 8;
        if (!hop_ok(type, clen, x.z & 0xFFu, (x.z >> 8) & 0xFFu, (x.z >> 16) & 0xFFu)) return false;
        q += 4ull + clen;
    }
    return true;
}

// One workgroup (4 waves) per segment j >= 1: the first plausible position in [j*seg, j*seg +
// kGuessWindow).  Each wave stages a 16 KiB window of the segment in LDS (16-byte loads), so the
// workgroup covers 64 KiB per pass; lane l tests positions 64 t + l of its wave's window against the
// whole first-hop rule from LDS, follows the rare survivors' next three hops in HBM, and keeps its
// lowest; the workgroup's lowest wins.
constexpr uint32_t kGuessWin = 16384;
__global__ void __launch_bounds__(256) k_seg_guess(const uint8_t* __restrict__ b, uint64_t len, uint64_t seg, uint32_t nseg,
                                                   SegInfo* __restrict__ info) {
    __shared__ __attribute__((aligned(16))) uint8_t win[4][kGuessWin + 16];
    __shared__ unsigned long long best;
    const uint32_t j = blockIdx.x + 1u;
    if (j >= nseg) return;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t lo = (uint64_t)j * seg;
    const uint64_t hi = min(len, lo + (uint64_t)kGuessWindow);
    if (threadIdx.x == 0) best = kNone;
    uint8_t* w8 = win[wv];
    for (uint64_t pass = lo; pass < hi; pass += 4ull * kGuessWin) {
        const uint64_t q0 = pass + (uint64_t)wv * kGuessWin;
        if (q0 < hi) {
            for (uint32_t u = lane; u <= kGuessWin / 16u; u += 64u) {
                const uint4 d = hdr16(b, len, q0 + 16ull * u);
                *reinterpret_cast<uint4*>(w8 + 16u * u) = d;
            }
        }
        __syncthreads();
        uint64_t mine = kNone;
        if (q0 < hi) {
            const uint32_t nq = (uint32_t)min((uint64_t)kGuessWin, hi - q0);
            for (uint32_t o = lane; o < nq; o += 64u) {
                const uint32_t type = w8[o];
                const uint32_t clen = (uint32_t)w8[o + 1] | ((uint32_t)w8[o + 2] << 8) | ((uint32_t)w8[o + 3] << 16);
                if (hop_ok(type, clen, w8[o + 8], w8[o + 9], w8[o + 10]) && q0 + o + 9 <= len &&
                    plausible_tail(b, len, q0 + o + 4ull + clen)) {
                    mine = q0 + o;
                    break;
                }
            }
        }
        if (mine != kNone) atomicMin(&best, (unsigned long long)mine);
        __syncthreads();
        if (best != kNone) break;
    }
    if (threadIdx.x == 0) info[j].entry = best;
}

__global__ void __launch_bounds__(256) k_seg_count(const uint8_t* __restrict__ b, uint64_t len, uint64_t seg, uint32_t nseg,
                                                   const uint32_t* __restrict__ state_p, SegInfo* __restrict__ info) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nseg) return;
    SegInfo I = info[j];
    Walk w{0, 0, true, NX_OK};
    if (j == 0) {
        const uint32_t st = *state_p;
        I.entry = 0;
        w.skip = st >> 8;
        w.started = (st & 1u) != 0;
    } else if (I.entry == kNone) {
        I.how = kEnd;
        info[j] = I;
        return;
    } else {
        w.p = I.entry;
    }
    uint32_t nc = 0, nu = 0;
    const uint64_t stop = j + 1u < nseg ? (uint64_t)(j + 1u) * seg : ~0ull;
    I.how = walk(b, len, w, stop, [&](uint32_t type, uint64_t, uint32_t, uint32_t) {
        (type == 0u ? nc : nu) += 1u;
        return true;
    });
    I.exit = w.p;
    I.skip = w.skip;
    I.res = w.res;
    I.started = w.started;
    I.ncomp = nc;
    I.nunc = nu;
    info[j] = I;
}

// One workgroup: follows the true chain through the segments (in LDS).  The straight prefix — segments
// 0..J whose walks each ended in the next segment exactly where its guess started — is found and
// prefix-summed in parallel; from J on, one lane follows the chain, re-walking any segment whose
// speculative walk did not start where the chain entered it.  Then list entries are claimed as the
// lane walk would (one per data chunk until the list is full).
__global__ void __launch_bounds__(256) k_seg_stitch(const uint8_t* __restrict__ b, uint64_t len, uint64_t seg, uint32_t nseg,
                                                    SegInfo* __restrict__ info, SegStep* __restrict__ path, SegPath* __restrict__ P,
                                                    uint32_t* __restrict__ counts, uint32_t cap, uint32_t* __restrict__ state_p,
                                                    uint64_t* __restrict__ consumed_p, int32_t* __restrict__ status_p) {
    __shared__ SegInfo si[kSegMax];
    __shared__ uint32_t first_bad;
    __shared__ uint32_t s0[256], s1[256];
    const uint32_t t = threadIdx.x;
    const uint32_t st_in = *state_p;
    if ((st_in >> 1) & 1u) {  // corrupted (:86-89): everything readable is discarded
        if (t == 0) {
            P->state_in = st_in;
            P->nseg = 0;
            *consumed_p = len;
            *status_p = NX_OK;
        }
        return;
    }
    __shared__ uint32_t nfix;
    for (uint32_t i = t; i < nseg; i += blockDim.x) si[i] = info[i];
    if (t == 0) nfix = 0;
    __syncthreads();
    // a wrong or missing guess for segment i + 1 whose predecessor's walk ended inside it: re-walk it
    // from there, all such segments at once (twice, for a fix whose own exit then disagrees); the
    // serial pass below accepts a segment only where the chain really enters it
    for (int it = 0; it < 2; ++it) {
        bool fix = false;
        uint32_t fi = 0;
        for (uint32_t i = t; i + 1u < nseg; i += blockDim.x) {
            const SegInfo& c = si[i];
            if (c.how == kOpen && c.exit / seg == (uint64_t)(i + 1u) && si[i + 1u].entry != c.exit && !fix) {
                fix = true;
                fi = i;
            }
        }
        __syncthreads();
        SegInfo R;
        if (fix) {
            const SegInfo& c = si[fi];
            Walk w{c.exit, 0, c.started != 0, NX_OK};
            uint32_t nc = 0, nu = 0;
            const uint64_t stop = fi + 2u < nseg ? (uint64_t)(fi + 2u) * seg : ~0ull;
            R.how = walk(b, len, w, stop, [&](uint32_t type, uint64_t, uint32_t, uint32_t) {
                (type == 0u ? nc : nu) += 1u;
                return true;
            });
            R.entry = c.exit;
            R.exit = w.p;
            R.skip = w.skip;
            R.res = w.res;
            R.started = w.started;
            R.ncomp = nc;
            R.nunc = nu;
            R.pad = 0;
        }
        __syncthreads();  // every fixing thread has read its predecessor before any segment changes
        if (fix) {
            si[fi + 1u] = R;
            info[fi + 1u] = R;
            atomicAdd(&nfix, 1u);
        }
        __syncthreads();
    }
    if (t == 0) first_bad = nseg - 1u;
    __syncthreads();
    for (uint32_t i = t; i + 1u < nseg; i += blockDim.x) {
        const SegInfo& c = si[i];
        const bool straight = c.how == kOpen && c.exit / seg == (uint64_t)(i + 1u) && si[i + 1u].entry == c.exit;
        if (!straight) atomicMin(&first_bad, i);
    }
    __syncthreads();
    const uint32_t J = first_bad;
    // inclusive prefix sums over segments 0..J: four per thread, then a scan of the 256 partials
    uint32_t a0 = 0, a1 = 0;
    for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t i = 4u * t + k;
        if (i <= J && i < nseg) {
            a0 += si[i].ncomp;
            a1 += si[i].nunc;
        }
    }
    s0[t] = a0;
    s1[t] = a1;
    __syncthreads();
    for (uint32_t d = 1; d < 256u; d <<= 1) {
        const uint32_t x0 = t >= d ? s0[t - d] : 0u, x1 = t >= d ? s1[t - d] : 0u;
        __syncthreads();
        s0[t] += x0;
        s1[t] += x1;
        __syncthreads();
    }
    {
        uint32_t c0 = s0[t] - a0, c1 = s1[t] - a1;  // exclusive: before segment 4t
        for (uint32_t k = 0; k < 4u; ++k) {
            const uint32_t i = 4u * t + k;
            if (i <= J && i < nseg) {
                path[i] = SegStep{i, c0, c1, 0u};
                c0 += si[i].ncomp;
                c1 += si[i].nunc;
            }
        }
    }
    __syncthreads();
    if (t != 0) return;
    P->state_in = st_in;
    P->stats[0] = J;
    P->stats[1] = nfix;
    uint32_t nser = 0;
    uint32_t j = J, np = J + 1u, c0 = s0[255], c1 = s1[255];
    for (;;) {
        const SegInfo& cur = si[j];
        if (cur.how != kOpen) break;
        const uint32_t nj = (uint32_t)min((uint64_t)(nseg - 1u), cur.exit / seg);
        if (si[nj].entry != cur.exit) {  // a wrong or missing guess: walk it from the true position
            Walk w{cur.exit, 0, cur.started != 0, NX_OK};
            uint32_t nc = 0, nu = 0;
            const uint64_t stop = nj + 1u < nseg ? (uint64_t)(nj + 1u) * seg : ~0ull;
            SegInfo R;
            R.how = walk(b, len, w, stop, [&](uint32_t type, uint64_t, uint32_t, uint32_t) {
                (type == 0u ? nc : nu) += 1u;
                return true;
            });
            R.entry = cur.exit;
            R.exit = w.p;
            R.skip = w.skip;
            R.res = w.res;
            R.started = w.started;
            R.ncomp = nc;
            R.nunc = nu;
            R.pad = 0;
            si[nj] = R;
            info[nj] = R;
            ++nser;
        }
        j = nj;
        path[np++] = SegStep{j, c0, c1, 0u};
        c0 += si[j].ncomp;
        c1 += si[j].nunc;
    }
    P->stats[2] = nser;
    const uint32_t tot = c0 + c1;
    const uint32_t used = counts[2];
    const uint32_t room = used < cap ? cap - used : 0u;
    const uint32_t limit = tot < room ? tot : room;
    P->nseg = np;
    P->limit = limit;
    P->base0 = counts[0];
    P->base1 = counts[1];
    counts[2] = used + limit + (limit < tot ? 1u : 0u);  // the lane walk's refused claim counts too
    if (limit == tot) {
        counts[0] = P->base0 + c0;
        counts[1] = P->base1 + c1;
        const SegInfo& L = si[j];
        *consumed_p = L.exit;
        *status_p = L.res;
        *state_p = (L.started ? 1u : 0u) | (L.res < 0 ? 2u : 0u) | ((uint32_t)L.skip << 8);
    }
    // else k_seg_emit's segment holding chunk `limit` stops before it and writes the rest
}

// One lane per accepted segment: walks it again and writes its list entries.
__global__ void __launch_bounds__(256) k_seg_emit(const uint8_t* __restrict__ b, uint64_t base, uint64_t len, uint64_t seg,
                                                  uint32_t nseg, uint32_t s, const SegInfo* __restrict__ info,
                                                  const SegStep* __restrict__ path, const SegPath* __restrict__ P,
                                                  uint64_t* __restrict__ data_off, uint32_t* __restrict__ data_len,
                                                  uint32_t* __restrict__ masked_crc, uint32_t* __restrict__ chunk_stream,
                                                  uint32_t* __restrict__ chunk_seq, uint32_t* __restrict__ counts, uint32_t cap,
                                                  uint32_t* __restrict__ state_p, uint64_t* __restrict__ consumed_p,
                                                  int32_t* __restrict__ status_p) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P->nseg) return;
    const SegStep S = path[k];
    const SegInfo I = info[S.seg];
    const uint32_t first = S.o0 + S.o1, n = I.ncomp + I.nunc, limit = P->limit;
    // segments wholly past the cut list nothing; the one holding chunk `limit` stops before it
    if (first > limit || (first == limit && !(limit < first + n))) return;
    Walk w{I.entry, 0, true, NX_OK};
    if (k == 0) {
        w.skip = P->state_in >> 8;
        w.started = (P->state_in & 1u) != 0;
    }
    const uint64_t stop = S.seg + 1u < nseg ? (uint64_t)(S.seg + 1u) * seg : ~0ull;
    uint32_t n0 = S.o0, n1 = S.o1;
    const WalkEnd how = walk(b, len, w, stop, [&](uint32_t type, uint64_t p, uint32_t clen, uint32_t crc) {
        if (n0 + n1 >= limit) return false;
        const uint32_t e = type == 0u ? P->base0 + n0++ : cap - 1u - (P->base1 + n1++);
        data_off[e] = base + p + 8;
        data_len[e] = clen - 4u;
        masked_crc[e] = crc;
        chunk_stream[e] = s;
        chunk_seq[e] = n0 + n1 - 1u;
        return true;
    });
    if (how == kFull) {  // the list filled up here: the lane walk stops before this chunk
        counts[0] = P->base0 + n0;
        counts[1] = P->base1 + n1;
        *consumed_p = w.p;
        *status_p = NX_SCAN_LIST_FULL;
        *state_p = (w.started ? 1u : 0u) | ((uint32_t)w.skip << 8);
    }
}

}  // namespace fscan
}  // namespace nx

extern "C" int32_t nx_snappy_frame_scan_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                              uint32_t* state, uint64_t* consumed, int32_t* status, uint64_t* data_off,
                                              uint32_t* data_len, uint32_t* masked_crc, uint32_t* chunk_stream,
                                              uint32_t* chunk_seq, uint32_t* counts, uint32_t cap, uint32_t n,
                                              void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (!counts || (n && (!in || !in_off || !in_len || !state || !consumed || !status)) ||
        (cap && (!data_off || !data_len || !masked_crc || !chunk_stream || !chunk_seq)))
        return NX_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    NX_HIP_CHECK(hipMemsetAsync(counts, 0, 3 * sizeof(uint32_t), st));
    if (n == 0) return NX_OK;
    hipLaunchKernelGGL(nx::fscan::k_frame_scan, dim3((n + 255) / 256), dim3(256), 0, st, in, in_off, in_len, state,
                       consumed, status, data_off, data_len, masked_crc, chunk_stream, chunk_seq, counts, cap, n);
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}

// One long cumulation in[0, len) (its length a host value, as a ByteBuf's readableBytes is): the
// segmented walk.  Same outputs as nx_snappy_frame_scan_batch with n = 1 (stream index 0), counts
// zeroed first; asynchronous on `stream` (its 2 KiB-per-segment scratch is stream-ordered).
extern "C" int32_t nx_snappy_frame_scan_long(const uint8_t* in, uint64_t len, uint32_t* state, uint64_t* consumed, int32_t* status,
                                             uint64_t* data_off, uint32_t* data_len, uint32_t* masked_crc, uint32_t* chunk_stream,
                                             uint32_t* chunk_seq, uint32_t* counts, uint32_t cap, void* stream) {
    NX_CLEAR_STALE_ERROR();
    using namespace nx::fscan;
    if (!counts || !state || !consumed || !status || (len && !in) ||
        (cap && (!data_off || !data_len || !masked_crc || !chunk_stream || !chunk_seq)))
        return NX_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    NX_HIP_CHECK(hipMemsetAsync(counts, 0, 3 * sizeof(uint32_t), st));
    uint64_t seg = kSegBytes;
    while ((len + seg - 1) / seg > kSegMax) seg *= 2;
    const uint32_t nseg = len ? (uint32_t)((len + seg - 1) / seg) : 1u;
    static std::once_flag keep;  // keep freed stream-ordered scratch in the pool rather than returning it at each sync
    std::call_once(keep, [] {
        int dev = 0;
        hipMemPool_t pool = nullptr;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
            uint64_t thr = 64ull << 20;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
        }
    });
    void* scratch = nullptr;
    const size_t sb = sizeof(SegInfo) * nseg + sizeof(SegStep) * nseg + sizeof(SegPath);
    NX_HIP_CHECK(hipMallocAsync(&scratch, sb, st));
    SegInfo* info = static_cast<SegInfo*>(scratch);
    SegStep* path = reinterpret_cast<SegStep*>(info + nseg);
    SegPath* P = reinterpret_cast<SegPath*>(path + nseg);
    if (nseg > 1) hipLaunchKernelGGL(k_seg_guess, dim3(nseg - 1), dim3(256), 0, st, in, len, seg, nseg, info);
    hipLaunchKernelGGL(k_seg_count, dim3((nseg + 255) / 256), dim3(256), 0, st, in, len, seg, nseg, state, info);
    hipLaunchKernelGGL(k_seg_stitch, dim3(1), dim3(256), 0, st, in, len, seg, nseg, info, path, P, counts, cap, state, consumed,
                       status);
    hipLaunchKernelGGL(k_seg_emit, dim3((nseg + 255) / 256), dim3(256), 0, st, in, (uint64_t)0, len, seg, nseg, 0u, info, path, P,
                       data_off, data_len, masked_crc, chunk_stream, chunk_seq, counts, cap, state, consumed, status);
    NX_HIP_CHECK(hipGetLastError());
    static const bool stats = getenv("NX_SCAN_STATS") != nullptr;
    if (stats) {  // diagnostics only: synchronous
        SegPath h{};
        NX_HIP_CHECK(hipMemcpyAsync(&h, P, sizeof(h), hipMemcpyDeviceToHost, st));
        NX_HIP_CHECK(hipStreamSynchronize(st));
        fprintf(stderr, "nx_snappy_frame_scan_long: %u segments, straight prefix to %u, %u parallel and %u serial re-walks, %u on the path\n",
                nseg, h.stats[0], h.stats[1], h.stats[2], h.nseg);
    }
    NX_HIP_CHECK(hipFreeAsync(scratch, st));
    return NX_OK;
}
