/*
 * netty_amd_status.h — per-chunk status codes shared by the C-ABI (include/netty_amd.h)
 * and the CPU oracle (oracle/netty_oracle.c).
 *
 * Netty's codecs signal failure with Java exceptions; Netty's own JNI layer returns
 * negative errno-style ints that the Java side turns into exceptions
 * (transport-native-unix-common/src/main/c/netty_unix_filedescriptor.c:115-117 →
 * FileDescriptor.java:105-110).  This build follows that convention: every batch entry
 * point writes one int32 status per chunk, >= 0 on success, < 0 = one of the codes below.
 * Each code maps 1:1 to a reference throw site (file:line relative to
 * codec-compression/src/main/java/io/netty/handler/codec/compression/).
 */
#ifndef NETTY_AMD_STATUS_H
#define NETTY_AMD_STATUS_H

#define NX_OK 0

/* Snappy.java:414-416  "Preamble is greater than 4 bytes" */
#define NX_ERR_SNAPPY_PREAMBLE_TOO_LONG   (-1)
/* Snappy.java:638-640  "Offset is less than minimum permissible value" */
#define NX_ERR_SNAPPY_OFFSET_ZERO         (-2)
/* Snappy.java:642-645  "Offset is greater than maximum value supported by this implementation" */
#define NX_ERR_SNAPPY_OFFSET_NEGATIVE     (-3)
/* Snappy.java:647-649  "Offset exceeds size of chunk" */
#define NX_ERR_SNAPPY_OFFSET_BEYOND       (-4)
/* SnappyFrameDecoder.java:203 buffer(…, 65536) max capacity → IndexOutOfBoundsException */
#define NX_ERR_SNAPPY_OUTPUT_OVERFLOW     (-5)
/* Snappy.java:480-492: code-63 literal length negative as Java int → IllegalArgumentException */
#define NX_ERR_SNAPPY_LITERAL_LEN_INVALID (-6)
/* Snappy.java:700-706  "mismatching checksum: %x (expected: %x)" */
#define NX_ERR_SNAPPY_CRC_MISMATCH        (-7)

/* FastLz.java:412-416  "invalid level: %d (expected: %d or %d)" */
#define NX_ERR_FASTLZ_BAD_LEVEL           (-20)
/* FastLz.java:444-465: match bytes read past the readable input → IndexOutOfBoundsException */
#define NX_ERR_FASTLZ_INPUT_OOB           (-21)
/* FastLzFrameDecoder.java:160-164  originalLength/actual length mismatch */
#define NX_ERR_FASTLZ_LENGTH_MISMATCH     (-22)
/* FastLzFrameDecoder.java:171-179  "stream corrupted: mismatching checksum" */
#define NX_ERR_FASTLZ_CRC_MISMATCH        (-23)

/* LzfDecoder.java:205 → ChunkDecoder.decodeChunk throws on corrupt data (3rd-party) */
#define NX_ERR_LZF_CORRUPT                (-30)

/* Frame-level format errors raised by the host framing state machines (SnappyFrameDecoder.java:
 * 116-118,128-133,138-140,152-157,159-165,181-201; FastLzFrameDecoder.java:121-124;
 * LzfDecoder.java:120-122,134-137).  The handle's err_msg carries the reference message. */
#define NX_ERR_FRAME_CORRUPT              (-40)

/* Lz4FrameDecoder.java:203-217: the LZ4 decompressor's LZ4Exception ("Malformed input at %d",
 * lz4-java 1.8.0, third-party) → DecompressionException.  Raised for a block that reads past its
 * input, copies from before the output start (offset 0 or > bytes produced), or does not produce
 * exactly the frame's decompressedLength. */
#define NX_ERR_LZ4_MALFORMED              (-50)

/* Device LZ4 frame scan (nx_lz4_frame_scan_batch), one code per Lz4FrameDecoder throw site: */
/* :127-130  "unexpected block identifier" */
#define NX_ERR_LZ4_BAD_MAGIC              (-51)
/* :136-141  "invalid compressedLength: %d (expected: 0-%d)" */
#define NX_ERR_LZ4_COMPRESSED_LENGTH      (-52)
/* :143-149  "invalid decompressedLength: %d (expected: 0-%d)" */
#define NX_ERR_LZ4_DECOMPRESSED_LENGTH    (-53)
/* :150-156  "stream corrupted: compressedLength(%d) and decompressedLength(%d) mismatch" */
#define NX_ERR_LZ4_LENGTH_MISMATCH        (-54)
/* :209-213  "unexpected blockType: %d (expected: %d or %d)" */
#define NX_ERR_LZ4_BLOCK_TYPE             (-55)
/* :226-228 → CompressionUtil.checkChecksum  "stream corrupted: mismatching checksum: %d (expected: %d)" */
#define NX_ERR_LZ4_CHECKSUM_MISMATCH      (-56)
/* :160-162  "stream corrupted: checksum error" (end block with a non-zero checksum) */
#define NX_ERR_LZ4_END_CHECKSUM           (-57)
/* Lz4FrameEncoder.allocateBuffer (Lz4FrameEncoder.java:190-214): EncoderException "requested encode
 * buffer size (%d bytes) exceeds the maximum allowable size (%d bytes)" when the blocks of the pending
 * bytes need more than maxEncodeSize (nx_lz4_frame_encoder_error has the message). */
#define NX_ERR_LZ4_ENCODE_SIZE            (-58)
/* Lz4FrameEncoder.encode after close() (Lz4FrameEncoder.java:233-239): IllegalStateException "encode
 * finished and not enough space to write remaining data" when allocateBuffer(allowEmptyReturn) returned
 * EMPTY_BUFFER, i.e. the message's blocks need fewer than blockSize bytes (:216-218). */
#define NX_ERR_LZ4_ENCODE_FINISHED        (-59)

/* Device frame scan (nx_snappy_frame_scan_batch), one code per SnappyFrameDecoder throw site: */
/* :116-118  "Unexpected length of stream identifier: %d" */
#define NX_ERR_SNAPPY_STREAM_ID_LENGTH        (-41)
/* :128-133 → checkByte :233-238  "Unexpected stream identifier contents. Mismatched snappy protocol version?" */
#define NX_ERR_SNAPPY_STREAM_ID_CONTENT       (-42)
/* :181-183  "Received COMPRESSED_DATA tag before STREAM_IDENTIFIER" */
#define NX_ERR_SNAPPY_COMPRESSED_BEFORE_ID    (-43)
/* :159-161  "Received UNCOMPRESSED_DATA tag before STREAM_IDENTIFIER" */
#define NX_ERR_SNAPPY_UNCOMPRESSED_BEFORE_ID  (-44)
/* :138-140  "Received RESERVED_SKIPPABLE tag before STREAM_IDENTIFIER" */
#define NX_ERR_SNAPPY_SKIPPABLE_BEFORE_ID     (-45)
/* :162-165  "Received UNCOMPRESSED_DATA larger than 65540 bytes" */
#define NX_ERR_SNAPPY_UNCOMPRESSED_TOO_LARGE  (-46)
/* :198-201  "Received COMPRESSED_DATA that contains uncompressed data that exceeds 65536 bytes" */
#define NX_ERR_SNAPPY_DECOMPRESSED_TOO_LARGE  (-47)
/* chunk length < 4: the checksum read runs past the chunk (:171-177, :194-195 throw from ByteBuf) */
#define NX_ERR_SNAPPY_CHUNK_TOO_SHORT         (-48)
/* :152-157  "Found reserved unskippable chunk type: 0x%x" */
#define NX_ERR_SNAPPY_UNSKIPPABLE             (-49)
/* Not an error: the frame scan's chunk list is full; the stream stopped before a data chunk and
 * continues from consumed[i] on the next call. */
#define NX_SCAN_LIST_FULL                     1

#define NX_ERR_INVALID_ARG                (-100)
#define NX_ERR_HIP                        (-101)
#define NX_ERR_NO_DEVICE                  (-102)
/* A kernel's own loop bound tripped (a bug guard: the kernel stopped instead of spinning). */
#define NX_ERR_INTERNAL                   (-103)

#endif
