// frame_parse.hpp — SnappyFrameDecoder's chunk-header walk over host memory (SnappyFrameDecoder.java:85-258),
// shared by the synchronous handler (handlers.cpp) and the cross-channel batcher (batcher.cpp).
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../include/netty_amd_status.h"

namespace nx {
namespace fr {

inline uint32_t le24(const uint8_t* p) { return p[0] | (p[1] << 8) | ((uint32_t)p[2] << 16); }
inline uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

// AbstractByteBuf.checkReadableBytes0's IndexOutOfBoundsException (AbstractByteBuf.java:1465-1471), as
// ByteToMessageDecoder's DecoderException(cause) reports it; the buffer's toString() is omitted.
inline const char* bytebuf_oob(char* buf, size_t cap, size_t reader, int len, size_t writer) {
    snprintf(buf, cap, "java.lang.IndexOutOfBoundsException: readerIndex(%zu) + length(%d) exceeds writerIndex(%zu)", reader, len,
             writer);
    return buf;
}
// Snappy.decode's failure as SnappyFrameDecoder.decode() throws it: the DecompressionException texts
// (nx_status_string), except a code-63 literal whose Java int length + 1 is negative.  There
// decodeLiteral's out.writeBytes(in, length) fails in ensureWritable's argument check
// (Snappy.java:480-492, AbstractByteBuf.java:279-281), an IllegalArgumentException that
// ByteToMessageDecoder wraps in a DecoderException; `field` = the literal's 4 length bytes (LE).
inline std::string snappy_block_error(int32_t st, uint32_t field, const char* (*status_string)(int32_t)) {
    if (st == NX_ERR_SNAPPY_LITERAL_LEN_INVALID) {
        char buf[96];
        snprintf(buf, sizeof buf, "java.lang.IllegalArgumentException: minWritableBytes : %d (expected: >= 0)", (int32_t)(field + 1u));
        return buf;
    }
    return status_string(st);
}

enum class SAct { Stream, Skip, Uncomp, Comp, Error };
struct SnappyAction {
    SAct kind;
    size_t data = 0;     // payload position (after the 4-byte masked checksum)
    uint32_t dlen = 0;   // payload bytes
    uint32_t crc = 0;    // stored masked checksum
    size_t end = 0;      // reader index after this action
    uint64_t skip = 0;   // numBytesToSkip after this action
    int job = -1;        // GPU job index
    std::string err;     // Error action: the reference exception message
};

// One SnappyFrameDecoder.decode() call over in[p..n) (SnappyFrameDecoder.java:85-231), with the
// chunk work deferred.  Returns false when decode() would return without consuming (need more).
inline bool snappy_parse_one(const uint8_t* in, size_t n, size_t& p, bool& started, uint64_t& skip, bool validate,
                      std::vector<SnappyAction>& acts) {
    if (skip) {  // :91-99
        uint64_t s = skip < (uint64_t)(n - p) ? skip : (uint64_t)(n - p);
        p += s;
        skip -= s;
        SnappyAction a{SAct::Skip};
        a.end = p;
        a.skip = skip;
        acts.push_back(a);
        return s > 0;
    }
    const size_t inSize = n - p;
    if (inSize < 4) return false;
    const uint8_t type = in[p];
    const uint32_t chunkLength = le24(in + p + 1);
    SnappyAction a{SAct::Error};
    a.end = p;
    a.skip = skip;
    char buf[160];
    auto fail = [&](const char* msg) {
        a.kind = SAct::Error;
        a.err = msg;
        acts.push_back(a);
        return false;
    };
    if (type == 0xff) {  // STREAM_IDENTIFIER (:115-136)
        if (chunkLength != 6) {
            snprintf(buf, sizeof buf, "Unexpected length of stream identifier: %u", chunkLength);
            return fail(buf);
        }
        if (inSize < 10) return false;
        a.end = p + 10;
        if (memcmp(in + p + 4, "sNaPpY", 6) != 0) return fail("Unexpected stream identifier contents. Mismatched snappy protocol version?");
        started = true;
        p += 10;
        a.kind = SAct::Stream;
        acts.push_back(a);
        return true;
    }
    if (type == 0) {  // COMPRESSED_DATA (:180-224)
        if (!started) return fail("Received COMPRESSED_DATA tag before STREAM_IDENTIFIER");
        if (inSize < 4 + (size_t)chunkLength) return false;
        if (chunkLength < 4) {
            // No DecompressionException in the reference: skipBytes(4) then readIntLE() run past the
            // chunk (:194-195), and the negative slice fails in ByteBuf (:208 / :215), wrapped as a
            // DecoderException (ByteToMessageDecoder.java:297-300).  The preamble check comes first.
            if (inSize < 8) return fail(bytebuf_oob(buf, sizeof buf, p + 4, 4, n));
            uint32_t pre = 0;
            int bi = 0;
            bool done = false;
            for (size_t q = p + 8; q < n; ++q) {
                pre |= (uint32_t)(in[q] & 0x7f) << (bi++ * 7);
                if (!(in[q] & 0x80)) {
                    done = true;
                    break;
                }
                if (bi >= 4) return fail("Preamble is greater than 4 bytes");
            }
            if (done && pre > 65536) return fail("Received COMPRESSED_DATA that contains uncompressed data that exceeds 65536 bytes");
            if (validate) {  // in.writerIndex(readerIndex + chunkLength - 4) below the reader index (:208)
                snprintf(buf, sizeof buf,
                         "java.lang.IndexOutOfBoundsException: readerIndex: %zu, writerIndex: %zu "
                         "(expected: 0 <= readerIndex <= writerIndex <= capacity)", p + 8, p + 4 + (size_t)chunkLength);
                return fail(buf);
            }
            snprintf(buf, sizeof buf, "java.lang.IllegalArgumentException: minimumReadableBytes : %d (expected: >= 0)",
                     (int)chunkLength - 4);  // in.readSlice(chunkLength - 4) (:215)
            return fail(buf);
        }
        a.crc = le32(in + p + 4);
        // snappy.getPreamble(in): the varint is read from the cumulation (Snappy.java:404-441)
        uint32_t ulen = 0;
        int bi = 0;
        bool complete = false;
        for (size_t q = p + 8; q < n; ++q) {
            const uint32_t cur = in[q];
            ulen |= (cur & 0x7f) << (bi++ * 7);
            if ((cur & 0x80) == 0) {
                complete = true;
                break;
            }
            if (bi >= 4) return fail("Preamble is greater than 4 bytes");
        }
        if (!complete) ulen = 0;
        if (ulen > 65536) return fail("Received COMPRESSED_DATA that contains uncompressed data that exceeds 65536 bytes");
        a.kind = SAct::Comp;
        a.data = p + 8;
        a.dlen = chunkLength - 4;
        p += 4 + chunkLength;
        a.end = p;
        acts.push_back(a);
        return true;
    }
    if (type == 1) {  // UNCOMPRESSED_DATA (:158-179)
        if (!started) return fail("Received UNCOMPRESSED_DATA tag before STREAM_IDENTIFIER");
        if (chunkLength > 65536 + 4) return fail("Received UNCOMPRESSED_DATA larger than 65540 bytes");
        if (inSize < 4 + (size_t)chunkLength) return false;
        if (chunkLength < 4) {
            // (:171-178) readIntLE / skipBytes(4) run past the chunk; with validation the CRC32C of a
            // negative length is the empty CRC (Crc32c.update's loop does not run, mask(0) =
            // 0xa282ead8, DecompressionException unless the 4 bytes read happen to equal it); then
            // readRetainedSlice(chunkLength - 4) fails in ByteBuf.  Heap-buffer behaviour.
            if (inSize < 8) return fail(bytebuf_oob(buf, sizeof buf, p + 4, 4, n));
            const uint32_t ck = le32(in + p + 4);
            if (validate && ck != 0xa282ead8u) {
                snprintf(buf, sizeof buf, "mismatching checksum: a282ead8 (expected: %x)", ck);
                return fail(buf);
            }
            snprintf(buf, sizeof buf, "java.lang.IllegalArgumentException: minimumReadableBytes : %d (expected: >= 0)",
                     (int)chunkLength - 4);
            return fail(buf);
        }
        a.kind = SAct::Uncomp;
        a.crc = le32(in + p + 4);
        a.data = p + 8;
        a.dlen = chunkLength - 4;
        p += 4 + chunkLength;
        a.end = p;
        acts.push_back(a);
        return true;
    }
    if (type & 0x80) {  // RESERVED_SKIPPABLE (:137-150)
        if (!started) return fail("Received RESERVED_SKIPPABLE tag before STREAM_IDENTIFIER");
        p += 4;
        const uint64_t s = chunkLength < (uint64_t)(n - p) ? chunkLength : (uint64_t)(n - p);
        p += s;
        if (s != chunkLength) skip = chunkLength - s;
        a.kind = SAct::Skip;
        a.end = p;
        a.skip = skip;
        acts.push_back(a);
        return true;
    }
    snprintf(buf, sizeof buf, "Found reserved unskippable chunk type: 0x%x", (unsigned)type);  // :151-157
    return fail(buf);
}

}  // namespace fr
}  // namespace nx
