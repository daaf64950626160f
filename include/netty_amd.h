/*
 * netty_amd.h — C-ABI of the MI355X-native codec-compression hot path (libnetty_amd.so).
 *
 * Plain pointers and sizes only (no torch / HIP types in the signatures; `stream` is a
 * hipStream_t passed as void*, NULL = default stream).  Two layers:
 *
 *  (1) Device batch kernels — thousands of independent chunks per launch, all buffers
 *      device-resident.  Each replaces the per-ByteBuf Java call named in its comment.
 *      Chunk i reads in[in_off[i] .. in_off[i]+in_len[i]) and writes out[out_off[i] ..].
 *      Every entry point is asynchronous on `stream`, returns NX_OK or NX_ERR_INVALID_ARG /
 *      NX_ERR_HIP for launch problems, and reports per-chunk results in device arrays
 *      (status[i] >= 0 ok, < 0 = include/netty_amd_status.h).
 *
 *  (2) Host handler layer — the framing state machines of SnappyFrameEncoder/Decoder,
 *      FastLzFrameEncoder/Decoder and LzfEncoder/Decoder over host memory (a direct
 *      ByteBuf's memoryAddress(), ByteBuf.java:2395-2403), batching every chunk of a call
 *      into one GPU launch (H2D → kernel → D2H).  This is what the JNI glue in
 *      INTEGRATION.md binds, one native handle per Netty handler instance.
 *
 * Reference paths below are relative to
 * /root/reference/codec-compression/src/main/java/io/netty/handler/codec/compression/.
 */
#ifndef NETTY_AMD_H
#define NETTY_AMD_H
#include <stddef.h>
#include <stdint.h>
#include "netty_amd_status.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ library */
const char* nx_version(void);
const char* nx_status_string(int32_t status);
/* Number of visible GPUs (0 when none); never initialises more than hipGetDeviceCount. */
int32_t nx_device_count(void);
/* Upper bound of Snappy.encode output for `n` input bytes (buffer sizing, cf. Snappy.java:82). */
size_t nx_snappy_max_compressed_length(size_t n);
/* FastLz.calculateOutputBufferLength (FastLz.java:84-87) + FastLZ tail slack. */
size_t nx_fastlz_max_compressed_length(size_t n);
size_t nx_lzf_max_compressed_length(size_t n);

/* ------------------------------------------------------------------ (1) device batch kernels */

/* Replaces Snappy.encode(ByteBuf in, ByteBuf out, int length)  Snappy.java:82-165
 * (in.readerIndex()==0, as SnappyFrameEncoder's readSlice gives).  in_len[i] <= 65536.
 * out capacity per chunk >= nx_snappy_max_compressed_length(in_len[i]).
 * out_len[i] = bytes written (preamble + tags), status[i] = NX_OK. */
int32_t nx_snappy_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                               uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                               int32_t* status, uint32_t n, void* stream);

/* Device workspaces (no reference counterpart: Snappy.java:187-211 allocates its table per call).
 * The encoders' hash tables and the decoder's record slots live in one workspace per device and
 * kind, shared by every stream: a batch's launches wait on the device for the previous batch's (the
 * host never blocks).  The standalone batch calls grow a workspace on demand (blocking, once per
 * size); batchers and handles reserve their share when created (nx_batcher_new, nx_*_new), never
 * grow it in submit / flush / encode / decode (a larger batch caps its grid to the reserved slots),
 * and the last of them to be freed frees it.
 *
 * nx_snappy_encoder_reserve places and zeroes the Snappy table workspace for batches of up to
 * max_chunks chunks now (a server calls it at start-up, before allocating its own buffers, so the
 * placement choice has memory to draw candidates from); kept until trimmed.
 * nx_workspaces_trim frees, on the current device, every workspace no batcher or handle holds.
 * nx_workspace_info reports the bytes and owners of one kind (NX_WS_*).
 * The workspaces remember an event on the stream of each batch call that used them (later batches
 * wait on it).  A caller that destroys a stream it passed to a batch call first calls
 * nx_workspaces_forget_stream(stream): it waits for the stream and drops those events, so no later
 * call waits on an event whose stream is gone.  Batchers and handles do this for their own streams. */
#define NX_WS_SNAPPY_ENC 0
#define NX_WS_LZ4_ENC 1
#define NX_WS_FASTLZ_ENC 2
#define NX_WS_LZF_ENC 3
#define NX_WS_DEC_RECORDS 4
#define NX_WS_LZ4HC_ENC 5
int32_t nx_snappy_encoder_reserve(uint32_t max_chunks, void* stream);
/* The same with a bound (round 6): max_bytes caps the Snappy table workspace for good (0: no cap; 128
 * KiB per lane, whole blocks of 256 lanes above 16 384): batches of any size then run on those lanes
 * and the standalone calls never grow it past the cap until nx_workspaces_trim frees it.  Returns
 * NX_ERR_INVALID_ARG when max_bytes holds no lane or the workspace is already larger.  *bytes = the
 * workspace's bytes, *peak = the most bytes its placement held at once (both nullable). */
int32_t nx_snappy_encoder_reserve_ex(uint32_t max_chunks, uint64_t max_bytes, void* stream,
                                     uint64_t* bytes, uint64_t* peak);
/* Placement bound of every later large (>= 2 GiB) encoder workspace: peak_bytes = the
 * bytes its candidate allocations may hold at once (0: half of the device's memory, the default;
 * UINT64_MAX: all but 8 GiB of free memory), max_candidates = candidates drawn in all (0: 24). */
int32_t nx_workspace_placement_config(uint64_t peak_bytes, int32_t max_candidates);
/* The launches nx_snappy_encode_batch makes for n chunks on the current device and its present
 * Snappy workspace: *count launches of sizes[0..*count) chunks (at most cap written).  Equal
 * full-occupancy launches (1 638 400 chunks: 5 x 327 680 on 256 CUs); a caller cutting a large job
 * into calls (bench.py) makes each call one of them. */
int32_t nx_snappy_encode_plan(uint32_t n, uint32_t* sizes, uint32_t cap, uint32_t* count);
/* The same plan for `slots` resident lanes on `cus` CUs, host arithmetic only (no device is touched):
 * k = ceil(n / slots) launches, equal in steps of cus x 128 chunks, the rest below one step on the last. */
int32_t nx_snappy_encode_plan_for(uint32_t n, uint32_t slots, int32_t cus, uint32_t* sizes, uint32_t cap,
                                  uint32_t* count);
int32_t nx_workspaces_trim(void);
int32_t nx_workspaces_forget_stream(void* stream);
int32_t nx_workspace_info(int32_t kind, uint64_t* bytes, int32_t* owners);

/* Diagnostics (no reference counterpart): the probe times in ms of the candidate workspace placements
 * the encoder's last large hash-table workspace was chosen from, and the index kept
 * (DESIGN.md §3).  *n = 0 before any such workspace exists. */
int32_t nx_snappy_encode_placement(float* probe_ms, int32_t cap, int32_t* n, int32_t* pick);

/* Replaces Snappy.decode(ByteBuf in, ByteBuf out)  Snappy.java:315-393 as driven by
 * SnappyFrameDecoder.decode for one COMPRESSED_DATA chunk (SnappyFrameDecoder.java:194-224),
 * fused with Snappy.validateChecksum over the output (Snappy.java:700-707).
 *   out_cap[i]   — output ByteBuf max capacity (65536 in the frame decoder, :203); NULL = 65536;
 *                  must be <= 2^24 (Snappy blocks; the out buffer needs out_cap[i] bytes).
 *   out_len[i]   — bytes produced (partial output on a silently truncated chunk, as Java).
 *   consumed[i]  — input bytes consumed by the decoder state machine (nullable).
 *   expected_masked_crc — NULL: no verification; else status NX_ERR_SNAPPY_CRC_MISMATCH on mismatch.
 *   crc_out[i]   — masked CRC32C of the produced output (nullable). */
int32_t nx_snappy_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                               uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                               uint32_t* out_len, uint32_t* consumed, int32_t* status,
                               const uint32_t* expected_masked_crc, uint32_t* crc_out,
                               uint32_t n, void* stream);

/* Same contract as nx_snappy_decode_batch, single-kernel variant: each wave parses its frame's tag
 * stream itself (speculative 64-byte windows) and expands it.  nx_snappy_decode_batch takes this path
 * for batches of up to 32768 frames (a lone frame decodes in ~0.9 ms instead of the lane-serial
 * parse's ~4 ms) and for frames of more than 16384 output-producing tags. */
int32_t nx_snappy_decode_batch_fused(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                     uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                     uint32_t* out_len, uint32_t* consumed, int32_t* status,
                                     const uint32_t* expected_masked_crc, uint32_t* crc_out,
                                     uint32_t n, void* stream);

/* Same contract, always the throughput pair (lane-serial parse to records, then the record
 * expander) whatever the batch size: what nx_snappy_decode_batch runs above 32768 frames.  Exported so
 * the parity tests and A/B tools exercise the pair on small batches too. */
int32_t nx_snappy_decode_batch_pair(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                    uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                    uint32_t* out_len, uint32_t* consumed, int32_t* status,
                                    const uint32_t* expected_masked_crc, uint32_t* crc_out,
                                    uint32_t n, void* stream);


/* Replaces the chunk walk of SnappyFrameDecoder.decode (SnappyFrameDecoder.java:85-231) as
 * ByteToMessageDecoder.callDecode runs it over a cumulation (ByteToMessageDecoder.java:464-517),
 * for n device-resident cumulations at once (one per stream/connection).
 *   in[in_off[s] .. +in_len[s]) — stream s's readable bytes.
 *   state[s]    (in/out) — started (bit 0) | corrupted (bit 1) | numBytesToSkip << 8; 0 for a new decoder.
 *   consumed[s] — bytes read (the cumulation's new readerIndex).  On a frame error: the start of the
 *                 failing chunk (the end of a stream identifier whose contents mismatch).
 *   status[s]   — NX_OK; NX_SCAN_LIST_FULL (the list filled up before this stream's next data chunk:
 *                 call again from consumed[s]); < 0 = NX_ERR_SNAPPY_* frame error (the decoder is now
 *                 corrupted, as :227-230).
 * Data chunks are listed in device arrays of `cap` entries: COMPRESSED_DATA at [0, counts[0]),
 * UNCOMPRESSED_DATA at [cap - counts[1], cap).  Entry k: data_off[k] = absolute position in `in` of
 * the payload (after the 4-byte checksum), data_len[k] = chunkLength - 4, masked_crc[k] = the stored
 * checksum, chunk_stream[k] = s, chunk_seq[k] = the chunk's index among stream s's data chunks.
 * The first counts[0] entries of data_off / data_len / masked_crc are nx_snappy_decode_batch's
 * in_off / in_len / expected_masked_crc as they stand.  The call zeroes counts[0..2] (counts[2] counts
 * claims, which may exceed cap).
 * A compressed chunk's Snappy errors (and any checksum mismatch) surface in the decode batch; the
 * caller drops the stream's chunks after the first failing one, as Java stops at the exception. */
int32_t nx_snappy_frame_scan_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                   uint32_t* state, uint64_t* consumed, int32_t* status,
                                   uint64_t* data_off, uint32_t* data_len, uint32_t* masked_crc,
                                   uint32_t* chunk_stream, uint32_t* chunk_seq, uint32_t* counts,
                                   uint32_t cap, uint32_t n, void* stream);

/* The same walk for ONE long cumulation in[0, len) whose length the caller holds on the host (a
 * ByteBuf's readableBytes): outputs as nx_snappy_frame_scan_batch with n = 1 (chunk_stream 0).  The
 * cumulation is cut into 1 MiB segments (more when it exceeds 1 GiB); a wave per segment guesses
 * where the chain enters it (four consecutive plausible data-chunk headers), a lane per segment walks
 * it with the decoder's exact semantics, one workgroup stitches the true chain (re-walking any
 * segment whose guess was wrong) and a lane per segment writes its entries: the result equals the
 * serial walk's whatever the guesses.  A 1 GiB stream takes well under a millisecond where one lane
 * needs ~35 K dependent header loads.  Asynchronous on `stream`. */
int32_t nx_snappy_frame_scan_long(const uint8_t* in, uint64_t len, uint32_t* state, uint64_t* consumed, int32_t* status,
                                  uint64_t* data_off, uint32_t* data_len, uint32_t* masked_crc, uint32_t* chunk_stream,
                                  uint32_t* chunk_seq, uint32_t* counts, uint32_t cap, void* stream);

/* Replaces Snappy.calculateChecksum(ByteBuf, off, len)  Snappy.java:668-676
 * (Crc32c.java:105-124 + maskChecksum :720-722).  masked_out[i] = mask(crc32c(chunk i)). */
int32_t nx_crc32c_masked_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len,
                               uint32_t* masked_out, uint32_t n, void* stream);

/* Replaces FastLz.compress(input, inOffset, inLength, output, outOffset, level)
 * FastLz.java:96-399.  level[i] in {0,1,2} (0 = AUTO); u16_limit[i] = readableBytes() - inOffset
 * of the Java call (the readU16 quirk, FastLz.java:552-557; NULL = in_len[i]); when
 * u16_limit[i] > in_len[i] the bytes following the chunk in `in` must be readable.
 * out_len[i] = compress return value. */
int32_t nx_fastlz_compress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                 uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                 const int32_t* level, const int32_t* u16_limit, int32_t* status,
                                 uint32_t n, void* stream);

/* Replaces FastLz.decompress(input, inOffset, inLength, output, outOffset, outLength)
 * FastLz.java:409-543.  out_len_limit[i] = originalLength; in_avail[i] = readable bytes from
 * the chunk start (NULL = in_len[i]).  result[i] = Java return value (0 on overflow/underflow)
 * or NX_ERR_FASTLZ_BAD_LEVEL / NX_ERR_FASTLZ_INPUT_OOB. */
int32_t nx_fastlz_decompress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                   const uint32_t* in_avail, uint8_t* out, const uint64_t* out_off,
                                   const uint32_t* out_len_limit, int32_t* result,
                                   uint32_t n, void* stream);

/* java.util.zip.Adler32 over each chunk (FastLzFrameEncoder.java:142-146 / Decoder :171-180). */
int32_t nx_adler32_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len,
                         uint32_t* out, uint32_t n, void* stream);

/* Replaces ChunkEncoder.appendEncodedChunk(...) as LZFEncoder.appendEncoded calls it per 65535-byte
 * chunk (LzfEncoder.java:218-221; compress-lzf 1.0.3 ChunkEncoder.tryCompress): writes a complete
 * "ZV" block (compressed if it saves bytes, else non-compressed).  in_len[i] <= 65535.  Each chunk
 * gets a fresh table, which writes exactly what LzfEncoder's long-lived table (kept across chunks and
 * messages, LzfEncoder.java:57,161-163) writes: no stale entry can pass tryCompress's 3-byte check
 * (oracle/netty_oracle.c, above lzf_try_compress).
 * PARITY UNPINNED vs com.ning:compress-lzf (third-party, not in the reference). */
int32_t nx_lzf_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                            uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                            int32_t* status, uint32_t n, void* stream);

/* Replaces ChunkDecoder.decodeChunk(in, inPos, out, outPos, outEnd)  LzfDecoder.java:205:
 * decodes one compressed LZF body into exactly out_len[i] bytes. status NX_OK / NX_ERR_LZF_CORRUPT. */
int32_t nx_lzf_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                            uint8_t* out, const uint64_t* out_off, const uint32_t* out_len,
                            int32_t* status, uint32_t n, void* stream);

/* Replaces LZ4Compressor.compress as Lz4FrameEncoder.flushBufferedData calls it for one block
 * (Lz4FrameEncoder.java:259-275; fastCompressor() = liblz4's LZ4_compress_default through
 * lz4-java's JNI, :125,163,273).  in_len[i] <= 2^25 (MAX_BLOCK_SIZE); out capacity >=
 * nx_lz4_max_compressed_length (= LZ4_compressBound).  Bit-exact with LZ4_compress_default: the
 * oracle's restatement is pinned byte-for-byte against pyarrow's bundled liblz4. */
size_t nx_lz4_max_compressed_length(size_t n);
int32_t nx_lz4_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                            const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream);

/* Same contract for lz4-java's highCompressor() (Lz4FrameEncoder(highCompressor = true),
 * Lz4FrameEncoder.java:123-125,161-163): liblz4's LZ4_compress_HC at level 9 (hash-chain match finder,
 * 256 candidates, pattern analysis, lazy three-match parse), bit-exact with the oracle's restatement,
 * which is pinned byte-for-byte against pyarrow's liblz4 at level 9.  One block per wave (lane 0) with
 * 256 KiB of tables in HBM per wave, on at most 2 waves per CU: the NX_WS_LZ4HC_ENC workspace never
 * exceeds CUs x 2 x 256 KiB (128 MiB on 256 CUs).  A compatibility path, far slower than the fast
 * compressor (below a 16-core host's liblz4; INTEGRATION.md keeps HC on the JVM). */
int32_t nx_lz4hc_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                              const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream);

/* Replaces LZ4FastDecompressor.decompress as Lz4FrameDecoder.decode calls it for one
 * BLOCK_TYPE_COMPRESSED block (Lz4FrameDecoder.java:199-208; lz4-java 1.8.0 = liblz4's
 * LZ4_decompress_fast, restated from the published block format): block i = in[in_off[i] .. +in_len[i]) must decode to exactly out_len[i] bytes at
 * out + out_off[i].  status NX_OK / NX_ERR_LZ4_MALFORMED.  Same parse/expand kernels as Snappy. */
int32_t nx_lz4_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                            const uint64_t* out_off, const uint32_t* out_len, int32_t* status, uint32_t n, void* stream);

/* Replaces Lz4XXHash32.update + getValue (Lz4XXHash32.java:37-102; XXH32 of lz4-java 1.8.0,
 * third-party, restated from the published algorithm): out[i] = XXH32(block i, seed), unmasked
 * (the frame stores out[i] & 0x0FFFFFFF, :101).  Lz4FrameDecoder with validateChecksums compares it
 * with the header's checksum (Lz4FrameDecoder.java:226-228). */
int32_t nx_xxhash32_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t seed,
                          uint32_t* out, uint32_t n, void* stream);

/* Replaces Lz4FrameEncoder.flushBufferedData (Lz4FrameEncoder.java:248-284) for n buffered blocks:
 * slot i = out[out_off[i] .. + 21 + nx_lz4_max_compressed_length(in_len[i])) receives the 21-byte
 * header (magic, token = blockType | compression_level, LE compressedLength, LE decompressedLength,
 * LE XXH32 & 0x0FFFFFFF) and the block (compressed, or raw when not smaller, :270-273).
 * out_len[i] = bytes written (0 for an empty block, as :249).  compression_level as
 * Lz4FrameEncoder.compressionLevel(blockSize) (:158-166): 6 for the default 64 KiB; in_len[i] < 2^25.
 * The end block of close() (:326-335) is 21 host-written bytes. */
int32_t nx_lz4_frame_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                  uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                  int32_t compression_level, int32_t* status, uint32_t n, void* stream);
/* The same with the block compressor chosen as the encoder's highCompressor flag (0: fast, else HC). */
int32_t nx_lz4_frame_encode_batch_ex(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                     uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                     int32_t compression_level, int32_t high_compressor, int32_t* status,
                                     uint32_t n, void* stream);

/* Replaces the block walk of Lz4FrameDecoder.decode (Lz4FrameDecoder.java:121-261) under
 * ByteToMessageDecoder.callDecode, for n device-resident cumulations (one per stream).
 *   state[s] (in/out) — finished (bit 0) | corrupted (bit 1); 0 for a new decoder.
 *   consumed[s] — bytes read.  A block whose payload is not all readable stops the walk at its
 *                 header (Java has read the header and waits in DECOMPRESS_DATA; re-reading it next
 *                 call gives the same result).  On an error: the start of the failing block.  After
 *                 the end block: all of in_len (FINISHED discards the rest, :251-254).
 *   status[s]   — NX_OK; NX_SCAN_LIST_FULL (call again from consumed[s]); < 0 = NX_ERR_LZ4_* header
 *                 error (the decoder is now corrupted, :257-259).
 * Blocks are listed as the Snappy scan lists chunks: BLOCK_TYPE_COMPRESSED at [0, counts[0]),
 * BLOCK_TYPE_NON_COMPRESSED at [cap - counts[1], cap).  Entry k: data_off[k] = absolute payload
 * position in `in`, comp_len / decomp_len / checksum = the header's fields, block_stream[k] = s,
 * block_seq[k] = the block's index within stream s.  The first counts[0] entries of data_off /
 * comp_len / decomp_len are nx_lz4_decode_batch's in_off / in_len / out_len as they stand. */
int32_t nx_lz4_frame_scan_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                uint32_t* state, uint64_t* consumed, int32_t* status, uint64_t* data_off,
                                uint32_t* comp_len, uint32_t* decomp_len, uint32_t* checksum,
                                uint32_t* block_stream, uint32_t* block_seq, uint32_t* counts, uint32_t cap,
                                uint32_t n, void* stream);

/* Bench/test data: the text-like generator of include/netty_amd_textgen.h on the device.
 * Chunk k (global index first_chunk + k) is written to out + k*chunk_len. */
int32_t nx_textgen_device(uint8_t* out, uint64_t first_chunk, uint32_t n_chunks, uint32_t chunk_len,
                          void* stream);

/* Device-memory helpers for callers without their own allocator (ctypes tests, JNI). */
void* nx_device_alloc(size_t bytes);
int32_t nx_device_free(void* p);
int32_t nx_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int32_t nx_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int32_t nx_stream_sync(void* stream);

/* Gather chunk i from src[src_off[i] .. +len[i]) to dst[dst_off[i] ..): packs fixed-capacity
 * output slots into one contiguous stream so a batch returns to host memory in one D2H copy
 * (the per-message `out` buffers of MessageToByteEncoder.write, MessageToByteEncoder.java:105-117). */
int32_t nx_pack_batch(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint8_t* dst,
                      const uint64_t* dst_off, uint32_t n, void* stream);

/* ------------------------------------------------------------------ (2) host handler layer */
/* Output list of one decode()/encode() call: messages are views into an arena owned by the
 * handle (valid until the next call on the same handle). */
typedef struct {
    const uint8_t* data;
    size_t len;
} nx_msg;

/* SnappyFrameEncoder / snappyEncoderWithJumboFrames()  SnappyFrameEncoder.java:60-117 */
typedef struct nx_snappy_frame_encoder nx_snappy_frame_encoder;
nx_snappy_frame_encoder* nx_snappy_frame_encoder_new(int32_t jumbo);
void nx_snappy_frame_encoder_free(nx_snappy_frame_encoder* e);
size_t nx_snappy_frame_max_encoded_length(size_t n);
/* encode(ctx, in, out): appends the framed bytes for `in` to out (capacity out_cap).
 * Returns bytes written (>= 0) or a negative status. */
int64_t nx_snappy_frame_encoder_encode(nx_snappy_frame_encoder* e, const uint8_t* in, size_t n,
                                       uint8_t* out, size_t out_cap);

/* SnappyFrameDecoder(boolean validateChecksums)  SnappyFrameDecoder.java:67-231.
 * decode(): runs ByteToMessageDecoder.callDecode over the cumulation in[0..n)
 * (ByteToMessageDecoder.java:464-517): *consumed = bytes read; msgs/n_msgs = decoded messages.
 * Returns NX_OK or a negative status (the decoder is then corrupted, :227-230); *err_msg gets the
 * reference's exception message. */
typedef struct nx_snappy_frame_decoder nx_snappy_frame_decoder;
nx_snappy_frame_decoder* nx_snappy_frame_decoder_new(int32_t validate_checksums);
void nx_snappy_frame_decoder_free(nx_snappy_frame_decoder* d);
int32_t nx_snappy_frame_decoder_decode(nx_snappy_frame_decoder* d, const uint8_t* in, size_t n,
                                       size_t* consumed, const nx_msg** msgs, size_t* n_msgs,
                                       const char** err_msg);

/* FastLzFrameEncoder(level, checksum)  FastLzFrameEncoder.java:100-172.
 * reader_index = in.readerIndex() of the Java message (enters the readU16 quirk). */
typedef struct nx_fastlz_frame_encoder nx_fastlz_frame_encoder;
nx_fastlz_frame_encoder* nx_fastlz_frame_encoder_new(int32_t level, int32_t checksum);
void nx_fastlz_frame_encoder_free(nx_fastlz_frame_encoder* e);
size_t nx_fastlz_frame_max_encoded_length(size_t n);
int64_t nx_fastlz_frame_encoder_encode(nx_fastlz_frame_encoder* e, const uint8_t* buf, size_t reader_index,
                                       size_t n, uint8_t* out, size_t out_cap);

/* FastLzFrameDecoder(checksum)  FastLzFrameDecoder.java:113-207 */
typedef struct nx_fastlz_frame_decoder nx_fastlz_frame_decoder;
nx_fastlz_frame_decoder* nx_fastlz_frame_decoder_new(int32_t validate_checksums);
void nx_fastlz_frame_decoder_free(nx_fastlz_frame_decoder* d);
int32_t nx_fastlz_frame_decoder_decode(nx_fastlz_frame_decoder* d, const uint8_t* in, size_t n,
                                       size_t* consumed, const nx_msg** msgs, size_t* n_msgs,
                                       const char** err_msg);

/* LzfEncoder(totalLength, compressThreshold)  LzfEncoder.java:127-216.  nx_lzf_encoder_new(t) =
 * LzfEncoder(MAX_CHUNK_LEN, t); _new_ex(total_length, t) = LzfEncoder(totalLength, compressThreshold).
 * NULL when totalLength is outside 16..65535 (:147-150) or compressThreshold < 16 (:152-156).
 * totalLength does not change the output: it sizes compress-lzf's hash table, which the
 * non-allocating ChunkEncoder LzfEncoder uses (:161-163) takes from max(totalLength, 65535)
 * (16384 entries always).  The deprecated safeInstance flag selects an encoder with
 * the same output (UnsafeChunkEncoderLE vs ChunkEncoder) and is not carried. */
typedef struct nx_lzf_encoder nx_lzf_encoder;
nx_lzf_encoder* nx_lzf_encoder_new(int32_t compress_threshold);
nx_lzf_encoder* nx_lzf_encoder_new_ex(int32_t total_length, int32_t compress_threshold);
void nx_lzf_encoder_free(nx_lzf_encoder* e);
size_t nx_lzf_frame_max_encoded_length(size_t n);
int64_t nx_lzf_encoder_encode(nx_lzf_encoder* e, const uint8_t* in, size_t n, uint8_t* out, size_t out_cap);

/* LzfDecoder  LzfDecoder.java:112-241 */
typedef struct nx_lzf_decoder nx_lzf_decoder;
nx_lzf_decoder* nx_lzf_decoder_new(void);
void nx_lzf_decoder_free(nx_lzf_decoder* d);
int32_t nx_lzf_decoder_decode(nx_lzf_decoder* d, const uint8_t* in, size_t n, size_t* consumed,
                              const nx_msg** msgs, size_t* n_msgs, const char** err_msg);

/* Lz4FrameEncoder(LZ4Factory.fastestInstance(), highCompressor, blockSize, new Lz4XXHash32(DEFAULT_SEED),
 * maxEncodeSize)  Lz4FrameEncoder.java:121-170; blockSize in [64, 2^25) (MAX_BLOCK_SIZE 2^25 itself
 * is refused).  nx_lz4_frame_encoder_new(b) = _new_ex(b, 0, INT32_MAX) (:140-141, DEFAULT_MAX_ENCODE_SIZE).
 * _new_ex returns NULL for max_encode_size <= 0 (checkPositive, :168) or a bad block size.
 * encode buffers a partial block (:231-248) and returns the bytes of every full block it flushed;
 * flush() writes the partial block (:291-300); close() flushes and appends the end block (:317-336),
 * after which encode passes bytes through (:233-239).  encode and flush first size the output as
 * allocateBuffer does (:190-214: sum over the pending bytes' blocks of LZ4_compressBound + 21) and
 * fail with NX_ERR_LZ4_ENCODE_SIZE, changing nothing, when that exceeds maxEncodeSize; close does not
 * (finishEncode allocates its footer directly, :306-315).  nx_lz4_frame_encoder_error: the last
 * failure's message (the reference's EncoderException text), or NULL. */
typedef struct nx_lz4_frame_encoder nx_lz4_frame_encoder;
nx_lz4_frame_encoder* nx_lz4_frame_encoder_new(int32_t block_size);
nx_lz4_frame_encoder* nx_lz4_frame_encoder_new_ex(int32_t block_size, int32_t high_compressor, int32_t max_encode_size);
const char* nx_lz4_frame_encoder_error(nx_lz4_frame_encoder* e);
void nx_lz4_frame_encoder_free(nx_lz4_frame_encoder* e);
size_t nx_lz4_frame_max_encoded_length(size_t n, int32_t block_size);
int64_t nx_lz4_frame_encoder_encode(nx_lz4_frame_encoder* e, const uint8_t* in, size_t n, uint8_t* out, size_t out_cap);
int64_t nx_lz4_frame_encoder_flush(nx_lz4_frame_encoder* e, uint8_t* out, size_t out_cap);
int64_t nx_lz4_frame_encoder_close(nx_lz4_frame_encoder* e, uint8_t* out, size_t out_cap);

/* Lz4FrameDecoder(validateChecksums)  Lz4FrameDecoder.java:95-261.  Returns NX_OK or the
 * NX_ERR_LZ4_* code of the first failure (err_msg = the reference's message; the decoder is then
 * corrupted and discards what follows, :251-259). */
typedef struct nx_lz4_frame_decoder nx_lz4_frame_decoder;
nx_lz4_frame_decoder* nx_lz4_frame_decoder_new(int32_t validate_checksums);
void nx_lz4_frame_decoder_free(nx_lz4_frame_decoder* d);
int32_t nx_lz4_frame_decoder_decode(nx_lz4_frame_decoder* d, const uint8_t* in, size_t n, size_t* consumed,
                                    const nx_msg** msgs, size_t* n_msgs, const char** err_msg);

/* ------------------------------------------------------------------ (3) asynchronous cross-channel batcher
 * Netty calls one handler per channel on that channel's event loop (ByteToMessageDecoder.java:194-196),
 * which must never block (BlockHound, common/.../internal/Hidden.java:38), and one call carries only a
 * few chunks.  A batcher turns the encode()/decode() calls of MANY handles into jobs of one GPU launch:
 * submit() runs the handle's framing at once (its stream state advances in call order) and returns a
 * ticket without touching the GPU; flush() launches every pending job (CRC32C + Snappy.encode of all
 * encoder slices, Snappy.decode + CRC verify of all decoder chunks, one finish kernel writing each
 * job's result straight into mapped pinned host memory); poll() never blocks; result() gives zero-copy
 * views valid until release().  Thread-safe. */
typedef struct nx_batcher nx_batcher;
nx_batcher* nx_batcher_new(void);
void nx_batcher_free(nx_batcher* b);
/* Page-lock a pooled direct ByteBuf's memory (ByteBuf.memoryAddress(), ByteBuf.java:2395-2403) so
 * encoder inputs in it are DMA'd to the device without a staging copy. */
int32_t nx_host_register(void* ptr, size_t len);
int32_t nx_host_unregister(void* ptr);
/* SnappyFrameEncoder.encode(ctx, in, out) as a job.  in_registered != 0: `in` lies in registered
 * memory and stays valid until the job completes (DMA'd at flush); else it is copied now (the caller
 * may release it, as MessageToByteEncoder.java:109 does).  Result: one message, the framed bytes.
 * Returns the ticket (> 0) or a negative status. */
int64_t nx_snappy_frame_encoder_submit(nx_snappy_frame_encoder* e, nx_batcher* b, const uint8_t* in, size_t n,
                                       int32_t in_registered);
/* SnappyFrameDecoder.decode(ctx, in, out) over the cumulation in[0..n) as a job: *consumed = bytes the
 * caller discards now (the chunk payloads are copied).  Result: the decoded messages in order, then
 * (status < 0) the first failure's message; a failed job marks the decoder corrupted (:227-230).
 * The decoder may be freed (nx_snappy_frame_decoder_free, a handler removed) while its jobs are in
 * flight: each job holds a reference to it until the job's batch is reused or the batcher is freed.
 * A validating decoder whose compressed chunk decodes short (a leftover, SnappyFrameDecoder.java:
 * 206-212) walks its stream again at apply time: the messages of bytes that later jobs had consumed
 * arrive on the earlier job's ticket, so read every ticket of a decoder before releasing it. */
int64_t nx_snappy_frame_decoder_submit(nx_snappy_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                       size_t* consumed);
/* The same for a cumulation in registered memory (a pooled direct buffer the socket read into): the
 * consumed bytes in[0..*consumed) are not copied; they stay valid until the job completes (a Java
 * caller keeps a retained slice) and the chunk payloads are gathered from the mapped pages at flush. */
int64_t nx_snappy_frame_decoder_submit_registered(nx_snappy_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                                  size_t* consumed);
int32_t nx_batcher_flush(nx_batcher* b);
int32_t nx_batcher_poll(nx_batcher* b, int64_t ticket);  /* 1 done, 0 pending, < 0 error; never blocks */
int32_t nx_batcher_wait(nx_batcher* b, int64_t ticket);  /* blocks (flushes first if needed): NX_OK */
int32_t nx_batcher_result(nx_batcher* b, int64_t ticket, const nx_msg** msgs, size_t* n_msgs, const char** err_msg);
int32_t nx_batcher_release(nx_batcher* b, int64_t ticket);
int32_t nx_batcher_stats(nx_batcher* b, uint64_t* flushes, uint64_t* launches, uint64_t* chunks);
/* Auto-flush: once the collecting batch holds `bytes` of input (copied payloads + registered ranges),
 * the submit that crossed the threshold launches it (0 = off, the default: only flush() launches).
 * Flushes rotate over four HIP streams, so a launched batch's PCIe traffic (gather from registered
 * pages, results into mapped memory) overlaps the next batch's kernels; results are applied in flush
 * order, so per-decoder semantics are those of one serial execution. */
int32_t nx_batcher_set_flush_bytes(nx_batcher* b, size_t bytes);
/* Hold the device workspaces of the given kinds (bit NX_WS_* per kind) for this batcher now, so that
 * no submit pays for it: a server calls it at start-up.  Otherwise the first submit that needs a kind
 * holds it (Snappy tables for 65 536 lanes, records for 65 536 frames, 16 384 lanes of the other
 * encoders' tables; a quarter of that, and so on down to 1 024, when the device cannot spare it).
 * nx_batcher_new itself reserves nothing (a decode-only batcher never holds encoder tables). */
int32_t nx_batcher_reserve(nx_batcher* b, uint32_t kinds);
/* Pinned host arenas (the staging copy of submitted bytes and the mapped result memory) grow inside
 * submit when a batch outgrows them.  nx_batcher_reserve_arenas sizes them up front: at least
 * `nbatches` batch objects with staging_bytes / out_bytes each, so that submits of a server whose
 * auto-flush threshold stays below staging_bytes never allocate (ByteToMessageDecoder.java:286-341
 * runs on the event loop).  nx_batcher_arena_stats reports the allocations made so far (growth
 * included), the pinned bytes held and the number of batch objects. */
int32_t nx_batcher_reserve_arenas(nx_batcher* b, uint32_t nbatches, size_t staging_bytes, size_t out_bytes);
int32_t nx_batcher_arena_stats(nx_batcher* b, uint64_t* allocs, uint64_t* bytes, uint32_t* batches);
/* Flushes whose results went to host memory by one DMA copy from a device mirror (large batches of
 * decoded messages; one mirror per batcher stream, grown to the largest such flush and kept until
 * nx_batcher_free) instead of through the finish kernels' mapped stores, and the bytes copied. */
int32_t nx_batcher_dma_stats(nx_batcher* b, uint64_t* dma_flushes, uint64_t* dma_bytes);

/* The FastLZ, LZF and LZ4 handlers as batcher jobs, with the Snappy jobs' contract (one launch per
 * codec kernel per flush for every job of every channel; results applied in submission order per
 * handle, a failing decoder job marking the decoder corrupted; the handle may be freed while its jobs
 * are in flight).  Inputs are copied at submit.
 *   FastLzFrameEncoder.encode (FastLzFrameEncoder.java:111-172) over buf[reader_index .. + n): one
 *     message, the framed blocks.
 *   LzfEncoder.encode (LzfEncoder.java:169-246): one message.
 *   Lz4FrameEncoder (Lz4FrameEncoder.java:221-336): op 0 = encode(in) — the full blocks of the handle's
 *     block buffer leave, the rest stays buffered; op 1 = encode(in) then flush() (the partial block
 *     too); op 2 = encode(in) then close() (flush + the end block; later jobs pass bytes through).
 *   FastLzFrameDecoder / LzfDecoder / Lz4FrameDecoder .decode over the cumulation in[0..n):
 *     *consumed = bytes the caller discards now; result: the decoded messages, then the failure. */
int64_t nx_fastlz_frame_encoder_submit(nx_fastlz_frame_encoder* e, nx_batcher* b, const uint8_t* buf, size_t reader_index,
                                       size_t n);
int64_t nx_lzf_encoder_submit(nx_lzf_encoder* e, nx_batcher* b, const uint8_t* in, size_t n);
int64_t nx_lz4_frame_encoder_submit(nx_lz4_frame_encoder* e, nx_batcher* b, const uint8_t* in, size_t n, int32_t op);
int64_t nx_fastlz_frame_decoder_submit(nx_fastlz_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                       size_t* consumed);
int64_t nx_lzf_decoder_submit(nx_lzf_decoder* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* consumed);
int64_t nx_lz4_frame_decoder_submit(nx_lz4_frame_decoder* d, nx_batcher* b, const uint8_t* in, size_t n,
                                    size_t* consumed);

#ifdef __cplusplus
}
#endif
#endif
