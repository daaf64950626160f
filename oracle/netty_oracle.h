/*
 * netty_oracle.h — CPU restatement of Netty's codec-compression hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / the CPU baseline.
 * The product path (netty_amd/) never links or calls it.
 *
 * Pinned by the reference's own known-answer vectors (tests/test_oracle_kat.py); see
 * oracle/netty_oracle.c for the file:line each function follows.
 */
#ifndef NETTY_ORACLE_H
#define NETTY_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/netty_amd_status.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- CRC32C (Crc32c.java) + Snappy mask (Snappy.java:658-722) ---- */
uint32_t orc_crc32c(const uint8_t* p, size_t n);
uint32_t orc_crc32c_update(uint32_t state, const uint8_t* p, size_t n); /* raw state, init 0xFFFFFFFF */
uint32_t orc_mask_checksum(uint32_t crc);
uint32_t orc_snappy_checksum(const uint8_t* p, size_t n);

/* ---- Snappy raw block (Snappy.java:82-393) ---- */
size_t orc_snappy_max_compressed_length(size_t n);
/* encode(in, out, length) with in.readerIndex()==0 (the framing encoder's readSlice). Returns bytes written. */
size_t orc_snappy_encode(const uint8_t* in, int32_t length, uint8_t* out);
/* orc_snappy_encode plus a census of its table traffic (test-only; netty_oracle.c snappy_encode_impl):
 * census[0..3] += probes, inserts, matches, matches of 7+ bytes. */
size_t orc_snappy_encode_census(const uint8_t* in, int32_t length, uint8_t* out, uint64_t* census);
/* One-shot decode of a complete chunk payload, as SnappyFrameDecoder drives Snappy.decode.
 * out_cap = output ByteBuf max capacity (65536 in the frame decoder).
 * Returns status (NX_OK or NX_ERR_*); *out_len = bytes produced (partial on silent truncation);
 * *consumed = input bytes consumed by the state machine (differs from in_len on truncation). */
int32_t orc_snappy_decode(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_cap,
                          size_t* out_len, size_t* consumed);
/* Snappy.getPreamble: returns the varint (0 if incomplete), or NX_ERR_SNAPPY_PREAMBLE_TOO_LONG. */
int64_t orc_snappy_get_preamble(const uint8_t* in, size_t in_len);

/* ---- Snappy framing (SnappyFrameEncoder.java:79-152) ---- */
size_t orc_snappy_frame_max_encoded(size_t n);
/* One encode(ctx,in,out) call.  *started is the per-encoder 'started' flag. */
size_t orc_snappy_frame_encode(const uint8_t* in, size_t n, int jumbo, int* started, uint8_t* out);

/* ---- FastLZ (FastLz.java:96-557) ---- */
/* compress(input, inOffset, inLength, output, outOffset, level).
 * in points at the chunk start; readU16's readableBytes() quirk is expressed as
 * u16_limit = readableBytes() - inOffset (relative to the chunk start; may be <= 0):
 * readU16(o) returns only in[o] when o + 1 >= u16_limit.  Bytes in[inLength .. u16_limit)
 * must be readable (they are the rest of the message). */
int32_t orc_fastlz_compress(const uint8_t* in, int32_t in_len, uint8_t* out, int32_t level,
                            int32_t u16_limit);
/* decompress(input, inOffset, inLength, output, outOffset, outLength).  in_avail = readable bytes
 * from the chunk start (>= in_len; reads beyond it raise NX_ERR_FASTLZ_INPUT_OOB). Returns the
 * Java return value (>= 0, 0 on overflow/underflow) or a negative status. */
int32_t orc_fastlz_decompress(const uint8_t* in, int32_t in_len, int32_t in_avail, uint8_t* out,
                              int32_t out_len);
uint32_t orc_adler32(const uint8_t* p, size_t n);
/* FastLzFrameEncoder.encode over one message buffer; reader index r0, writer index r0+n.
 * level 0/1/2; checksum 0/1 (Adler32).  Returns bytes written. */
size_t orc_fastlz_frame_encode(const uint8_t* buf, size_t r0, size_t n, int level, int checksum,
                               uint8_t* out);
size_t orc_fastlz_frame_max_encoded(size_t n);

/* ---- LZF (LzfEncoder/LzfDecoder framing; chunk codec restates the LZF format) ---- */
/* Encode one chunk (<= 65535 bytes) to an LZF "ZV" block (compressed if it saves bytes). */
size_t orc_lzf_encode_chunk(const uint8_t* in, int32_t in_len, uint8_t* out);
/* LZF compressed-chunk body decoder (ChunkDecoder.decodeChunk semantics). Returns NX_OK or
 * NX_ERR_LZF_CORRUPT; writes exactly out_len bytes on success. */
int32_t orc_lzf_decode_chunk(const uint8_t* in, int32_t in_len, uint8_t* out, int32_t out_len);
/* Raw LZF body compressor (compress-lzf 1.0.3 ChunkEncoder.tryCompress) used by orc_lzf_encode_chunk;
 * returns body length (may exceed in_len). */
int32_t orc_lzf_compress_body(const uint8_t* in, int32_t in_len, uint8_t* out);
size_t orc_lzf_frame_encode(const uint8_t* in, size_t n, int32_t compress_threshold, uint8_t* out);
/* One LzfEncoder instance: its ChunkEncoder table persists across encode() calls. */
typedef struct orc_lzf_encoder orc_lzf_encoder;
orc_lzf_encoder* orc_lzf_encoder_new(int32_t compress_threshold);
void orc_lzf_encoder_free(orc_lzf_encoder* e);
size_t orc_lzf_encoder_encode(orc_lzf_encoder* e, const uint8_t* in, size_t n, uint8_t* out);
size_t orc_lzf_frame_max_encoded(size_t n);

/* LZ4 block format (lz4-java 1.8.0, a third-party dependency absent from the reference: pom.xml
 * 946-950; Lz4FrameDecoder.java:203-208 calls its decompressor with the exact decompressed length).
 * Restated from the published block format: sequences of token | literal-length extension |
 * literals | 2-byte LE offset | match-length extension (+4), the last sequence literals only.
 * PARITY UNPINNED against lz4-java: no fixtures for it exist in the reference.
 * orc_lz4_decompress returns NX_OK when exactly out_len bytes are produced from all in_len bytes,
 * else NX_ERR_LZ4_MALFORMED.  orc_lz4_compress is a greedy single-probe compressor (LZ4's skip acceleration: the step over
 * misses grows by one every 64 misses) producing valid
 * blocks for tests (last 5 bytes literals, no match starting in the last 12). */
int32_t orc_lz4_decompress(const uint8_t* in, int32_t in_len, uint8_t* out, int32_t out_len);
int32_t orc_lz4_compress(const uint8_t* in, int32_t n, uint8_t* out);
size_t orc_lz4_max_compressed(size_t n);
/* LZ4_compress_HC level 9 (lz4-java highCompressor(), Lz4FrameEncoder.java:123-125,161-163): the
 * hash-chain match finder (256 candidates, pattern analysis) and lazy three-match parse of liblz4's
 * lz4hc.c.  Pinned against pyarrow's liblz4 Codec('lz4_raw', compression_level=9). */
int32_t orc_lz4hc_compress(const uint8_t* in, int32_t n, uint8_t* out);

/* XXHash32 (lz4-java 1.8.0 XXHash32.hash, third-party; restated from the published XXH32
 * algorithm: four lane accumulators over 16-byte stripes, then 4-byte and 1-byte tails and the
 * avalanche).  Pinned by Lz4FrameDecoderTest.java:33-41 ("Netty" -> 0x0F79E486 after the
 * Lz4XXHash32.java:101 mask) and by the independent python-xxhash package in tests. */
uint32_t orc_xxhash32(const uint8_t* p, size_t n, uint32_t seed);
/* One Lz4FrameEncoder.flushBufferedData block (Lz4FrameEncoder.java:248-284): 21-byte header
 * (magic "LZ4Block", token = blockType | compressionLevel, LE compressedLength, LE decompressedLength,
 * LE checksum = XXH32(seed 0x9747b28c) & 0x0FFFFFFF) then the compressed block, or the raw bytes
 * when compression does not shrink them.  n >= 1.  Returns bytes written (<= 21 + max_compressed). */
size_t orc_lz4_frame_block(const uint8_t* in, int32_t n, int32_t compression_level, uint8_t* out);
/* The same with the block compressor of Lz4FrameEncoder(highCompressor = high) (:161-163). */
size_t orc_lz4_frame_block_ex(const uint8_t* in, int32_t n, int32_t compression_level, int32_t high, uint8_t* out);

/* ---- Test data: java.util.Random restatement and the text-like generator ---- */
void orc_java_random_bytes(int64_t seed, uint8_t* out, size_t n);
int64_t orc_java_random_next_long(int64_t* state_seed); /* state already scrambled */
int64_t orc_java_random_scramble(int64_t seed);
/* Text-like chunk generator (BASELINE config 2/3); must equal the device generator. */
void orc_textgen_init(void);
void orc_textgen_chunk(uint64_t chunk_index, uint8_t* out, size_t n);
const uint8_t* orc_textgen_vocab(uint32_t* n_words, const uint32_t** offsets, const uint32_t** cdf);

#ifdef __cplusplus
}
#endif
#endif
