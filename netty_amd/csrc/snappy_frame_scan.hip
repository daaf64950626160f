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
#include "nx_common.hpp"
#include "../../include/netty_amd.h"

namespace nx {
namespace fscan {

__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

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
    bool started = st & 1u;
    bool corrupted = (st >> 1) & 1u;
    uint64_t skip = st >> 8;  // numBytesToSkip (< 2^24: a chunk length)
    uint64_t p = 0;
    int32_t res = NX_OK;
    uint32_t seq = 0;
    if (corrupted) {  // :86-89 — everything readable is discarded
        p = len;
    } else {
        while (p < len) {
            if (skip) {  // :91-99
                const uint64_t k = skip < len - p ? skip : len - p;
                p += k;
                skip -= k;
                continue;
            }
            const uint64_t avail = len - p;
            if (avail < 4) break;  // :104-108
            const uint32_t type = b[p];
            const uint32_t clen = (uint32_t)b[p + 1] | ((uint32_t)b[p + 2] << 8) | ((uint32_t)b[p + 3] << 16);
            if (type == 0xFFu) {  // STREAM_IDENTIFIER :115-136
                if (clen != 6u) {
                    res = NX_ERR_SNAPPY_STREAM_ID_LENGTH;
                    break;
                }
                if (avail < 10) break;
                const uint8_t* q = b + p + 4;
                p += 10;  // skipBytes(4 + 6) precede the content check (:124-133)
                if (q[0] != 's' || q[1] != 'N' || q[2] != 'a' || q[3] != 'P' || q[4] != 'p' || q[5] != 'Y') {
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
                    const uint32_t c = b[p + 8 + i];
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
            // claim a list entry; a full list stops the stream before this chunk
            if (atomicAdd(&counts[2], 1u) >= cap) {
                res = NX_SCAN_LIST_FULL;
                break;
            }
            const uint32_t k = type == 0u ? atomicAdd(&counts[0], 1u) : cap - 1u - atomicAdd(&counts[1], 1u);
            data_off[k] = base + p + 8;
            data_len[k] = clen - 4u;
            masked_crc[k] = le32(b + p + 4);
            chunk_stream[k] = s;
            chunk_seq[k] = seq++;
            p += 4ull + clen;
        }
    }
    if (res < 0) corrupted = true;  // :227-230
    consumed[s] = p;
    status[s] = res;
    state[s] = (started ? 1u : 0u) | (corrupted ? 2u : 0u) | ((uint32_t)skip << 8);
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
