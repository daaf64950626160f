// alt_frames.hpp — the FastLZ / LZF / LZ4 framing shared by the synchronous handlers (handlers.cpp)
// and the asynchronous batcher (batcher.cpp): the handles' state, the header walks of their decode()
// methods over host memory, the encoders' block plans and the failure texts.  Private to the library.
//
//   FastLzFrameDecoder.decode   FastLzFrameDecoder.java:113-207
//   LzfDecoder.decode           LzfDecoder.java:112-241
//   Lz4FrameDecoder.decode      Lz4FrameDecoder.java:150-261
//   FastLzFrameEncoder.encode   FastLzFrameEncoder.java:111-172
//   LzfEncoder.encode           LzfEncoder.java:169-246
//   Lz4FrameEncoder             Lz4FrameEncoder.java:221-336
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <string>
#include <vector>
#include "../../include/netty_amd.h"
#include "handles.hpp"

namespace nx {
namespace af {

inline uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
inline uint32_t be24(const uint8_t* p) { return ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2]; }
inline uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

constexpr uint8_t kLz4Magic[8] = {'L', 'Z', '4', 'B', 'l', 'o', 'c', 'k'};
constexpr uint32_t kLz4Header = 21;
constexpr uint32_t kLz4Seed = 0x9747b28cu;  // Lz4Constants.java:70

// One data block a decoder walk found complete: payload in[data .. data + clen).
struct Blk {
    size_t data = 0, end = 0;
    uint32_t clen = 0;  // payload bytes
    uint32_t olen = 0;  // decoded bytes (= clen for a raw block)
    uint32_t cks = 0;   // the header's checksum
    bool comp = false, has_cks = false;
    uint32_t type = 0;  // LZ4: blockType
};

// The first header-level failure of a walk (the decoder turns corrupted there).
struct WalkErr {
    bool set = false;
    int32_t code = NX_OK;
    std::string msg;
    size_t at = 0;  // reader index at the throw
};

// ---------------------------------------------------------------------------- FastLZ decoder
struct FlzState {
    int state = 0;  // 0 INIT_BLOCK, 1 INIT_BLOCK_PARAMS, 2 DECOMPRESS_DATA, 3 CORRUPTED
    uint32_t chunkLength = 0, originalLength = 0, currentChecksum = 0;
    bool isCompressed = false, hasChecksum = false;
};

// callDecode over in[0..n) from state s (not CORRUPTED): complete blocks into `blks`; returns the bytes
// read (the header bytes of an incomplete block included, as Java reads them into its state).
inline size_t flz_walk(const uint8_t* in, size_t n, FlzState& s, std::vector<Blk>& blks, WalkErr& err) {
    size_t p = 0;
    for (;;) {
        if (s.state == 0) {  // :116-131
            if (n - p < 4) break;
            if (be24(in + p) != (('F' << 16) | ('L' << 8) | 'Z')) {
                err = {true, NX_ERR_FRAME_CORRUPT, "unexpected block identifier", p + 3};
                break;
            }
            const uint8_t options = in[p + 3];
            s.isCompressed = (options & 0x01) == 1;
            s.hasChecksum = (options & 0x10) == 0x10;
            p += 4;
            s.state = 1;
        }
        if (s.state == 1) {  // :132-141
            const size_t need = 2 + (s.isCompressed ? 2 : 0) + (s.hasChecksum ? 4 : 0);
            if (n - p < need) break;
            s.currentChecksum = s.hasChecksum ? be32(in + p) : 0;
            p += s.hasChecksum ? 4 : 0;
            s.chunkLength = be16(in + p);
            p += 2;
            s.originalLength = s.isCompressed ? be16(in + p) : s.chunkLength;
            p += s.isCompressed ? 2 : 0;
            s.state = 2;
        }
        if (s.state == 2) {  // :142-196
            if (n - p < s.chunkLength) break;
            Blk b;
            b.data = p;
            b.end = p + s.chunkLength;
            b.clen = s.chunkLength;
            b.olen = s.originalLength;
            b.cks = s.currentChecksum;
            b.comp = s.isCompressed;
            b.has_cks = s.hasChecksum;
            blks.push_back(b);
            p += s.chunkLength;
            s.state = 0;
        }
    }
    return p;
}

// A compressed block's decompress() result r against originalLength (:155-164, FastLz.java:412-416).
// `first` = the block's first byte (the level bits).  Empty when the block decoded.
inline bool flz_block_error(int32_t r, uint32_t olen, uint8_t first, int32_t* code, std::string* msg) {
    if (r >= 0 && (uint32_t)r == olen) return false;
    char buf[160];
    if (r == NX_ERR_FASTLZ_BAD_LEVEL) {
        snprintf(buf, sizeof buf, "invalid level: %d (expected: %d or %d)", ((int8_t)first >> 5) + 1, 1, 2);
        *code = r;
    } else if (r < 0) {
        snprintf(buf, sizeof buf, "%s", nx_status_string(r));
        *code = r;
    } else {
        snprintf(buf, sizeof buf, "stream corrupted: originalLength(%u) and actual length(%d) mismatch", olen, r);
        *code = NX_ERR_FASTLZ_LENGTH_MISMATCH;
    }
    *msg = buf;
    return true;
}

inline std::string flz_checksum_error(uint32_t got, uint32_t want) {  // :171-180
    char buf[160];
    snprintf(buf, sizeof buf, "stream corrupted: mismatching checksum: %d (expected: %d)", (int32_t)got, (int32_t)want);
    return buf;
}

// ---------------------------------------------------------------------------- LZF decoder
struct LzfState {
    int state = 0;  // 0 INIT_BLOCK, 1 INIT_ORIGINAL_LENGTH, 2 DECOMPRESS_DATA, 3 CORRUPTED
    uint32_t chunkLength = 0, originalLength = 0;
    bool isCompressed = false;
};

// One decode() call per turn, as callDecode drives it (ByteToMessageDecoder.java:464-517): LzfDecoder
// reads a non-compressed block's header in one call and its payload in the next (:150-152 breaks
// out of the switch), so a zero-length non-compressed block is a call that reads nothing and adds
// nothing — callDecode stops there and the rest waits for the next channelRead.
inline size_t lzf_walk(const uint8_t* in, size_t n, LzfState& s, std::vector<Blk>& blks, WalkErr& err) {
    size_t p = 0;
    while (p < n) {  // in.isReadable()
        const size_t p0 = p;
        bool added = false;
        if (s.state == 0) {  // :115-153
            if (n - p < 5) break;  // HEADER_LEN_NOT_COMPRESSED
            if (be16(in + p) != (('Z' << 8) | 'V')) {
                err = {true, NX_ERR_FRAME_CORRUPT, "unexpected block identifier", p + 2};
                break;
            }
            const int8_t type = (int8_t)in[p + 2];
            if (type != 0 && type != 1) {
                char buf[96];
                snprintf(buf, sizeof buf, "unknown type of chunk: %d (expected: %d or %d)", (int)type, 0, 1);
                err = {true, NX_ERR_FRAME_CORRUPT, buf, p + 3};
                break;
            }
            s.isCompressed = type == 1;
            s.chunkLength = be16(in + p + 3);
            p += 5;
            s.state = s.isCompressed ? 1 : 2;
            if (!s.isCompressed) continue;  // this decode() call ends here (it read the header)
        }
        if (s.state == 1) {  // :154-169
            if (n - p < 2) {
                if (p == p0) break;
                continue;
            }
            s.originalLength = be16(in + p);
            p += 2;
            s.state = 2;
        }
        if (s.state == 2) {  // :171-228
            if (n - p >= s.chunkLength) {
                Blk b;
                b.data = p;
                b.end = p + s.chunkLength;
                b.clen = s.chunkLength;
                b.olen = s.isCompressed ? s.originalLength : s.chunkLength;
                b.comp = s.isCompressed;
                blks.push_back(b);
                added = s.isCompressed || s.chunkLength > 0;
                p += s.chunkLength;
                s.state = 0;
            }
        }
        if (!added && p == p0) break;  // no progress (:494-500)
    }
    return p;
}

// compress-lzf's ChunkDecoder failure (a third-party LZFException): a fixed text.
inline const char* lzf_block_error() { return "Corrupt LZF data"; }

// ---------------------------------------------------------------------------- LZ4 decoder
struct Lz4State {
    int state = 0;  // 0 INIT_BLOCK, 1 DECOMPRESS_DATA, 2 FINISHED, 3 CORRUPTED
    uint32_t blockType = 0, compressedLength = 0, decompressedLength = 0, currentChecksum = 0;
};

inline size_t lz4_walk(const uint8_t* in, size_t n, Lz4State& s, std::vector<Blk>& blks, WalkErr& err) {
    size_t p = 0;
    char mbuf[160];
    while (s.state < 2) {
        if (s.state == 0) {
            if (n - p < kLz4Header) break;  // :153-155
            const uint8_t* h = in + p;
            if (memcmp(h, kLz4Magic, 8) != 0) {  // :156-159
                err = {true, NX_ERR_LZ4_BAD_MAGIC, "unexpected block identifier", p + 8};
                break;
            }
            const uint32_t token = h[8];
            const uint32_t level = (token & 0x0Fu) + 10u;
            s.blockType = token & 0xF0u;
            const int32_t c = (int32_t)le32(h + 9), u = (int32_t)le32(h + 13);
            if (c < 0 || c > (1 << 25)) {  // :165-169
                snprintf(mbuf, sizeof mbuf, "invalid compressedLength: %d (expected: 0-%d)", c, 1 << 25);
                err = {true, NX_ERR_LZ4_COMPRESSED_LENGTH, mbuf, p + 13};
                break;
            }
            const int64_t maxd = (int64_t)1 << level;
            if (u < 0 || u > maxd) {  // :171-176
                snprintf(mbuf, sizeof mbuf, "invalid decompressedLength: %d (expected: 0-%lld)", u, (long long)maxd);
                err = {true, NX_ERR_LZ4_DECOMPRESSED_LENGTH, mbuf, p + 17};
                break;
            }
            if ((u == 0) != (c == 0) || (s.blockType == 0x10u && u != c)) {  // :177-183
                snprintf(mbuf, sizeof mbuf, "stream corrupted: compressedLength(%d) and decompressedLength(%d) mismatch", c, u);
                err = {true, NX_ERR_LZ4_LENGTH_MISMATCH, mbuf, p + 17};
                break;
            }
            s.currentChecksum = le32(h + 17);
            p += kLz4Header;
            s.compressedLength = (uint32_t)c;
            s.decompressedLength = (uint32_t)u;
            if (u == 0) {  // the end block (:185-193)
                if (s.currentChecksum != 0u) {
                    err = {true, NX_ERR_LZ4_END_CHECKSUM, "stream corrupted: checksum error", p};
                    break;
                }
                s.state = 2;
                p = n;  // callDecode runs decode() again; FINISHED skips the rest (:250-254)
                break;
            }
            s.state = 1;
        }
        if (s.state == 1) {
            if (n - p < s.compressedLength) break;  // :204-206
            if (s.blockType != 0x10u && s.blockType != 0x20u) {  // :230-234
                snprintf(mbuf, sizeof mbuf, "unexpected blockType: %u (expected: %d or %d)", s.blockType, 0x10, 0x20);
                err = {true, NX_ERR_LZ4_BLOCK_TYPE, mbuf, p};
                break;
            }
            Blk b;
            b.data = p;
            b.end = p + s.compressedLength;
            b.clen = s.compressedLength;
            b.olen = s.decompressedLength;
            b.cks = s.currentChecksum;
            b.comp = s.blockType == 0x20u;
            b.has_cks = true;
            b.type = s.blockType;
            blks.push_back(b);
            p += s.compressedLength;
            s.state = 0;
        }
    }
    return p;
}

// lz4-java's LZ4Exception (third-party), wrapped in a DecompressionException (:240-241): a fixed text.
inline const char* lz4_block_error() { return "LZ4 block decompression failed: malformed input"; }

inline std::string lz4_checksum_error(uint32_t got, uint32_t want) {  // CompressionUtil.checkChecksum
    char buf[160];
    snprintf(buf, sizeof buf, "stream corrupted: mismatching checksum: %d (expected: %d)", (int32_t)got, (int32_t)want);
    return buf;
}

// ---------------------------------------------------------------------------- encoder plans
// FastLzFrameEncoder.encode over buf[r0 .. r0 + n): blocks of up to 65535 bytes; block i reads the
// readU16 limit readableBytes() - inOffset of the Java call (FastLz.java:552-557).
struct FlzPlan {
    uint64_t ioff;  // relative to the message start
    uint32_t ilen;
    int32_t lim;
};
inline void flz_plan(size_t r0, size_t n, std::vector<FlzPlan>& out) {
    const size_t w = r0 + n;
    const uint32_t nc = (uint32_t)((n + 65534) / 65535);
    for (uint32_t i = 0; i < nc; ++i) {
        const size_t r = r0 + (size_t)i * 65535;
        FlzPlan p;
        p.ioff = (uint64_t)i * 65535;
        p.ilen = (uint32_t)((n - p.ioff) < 65535 ? (n - p.ioff) : 65535);
        const int64_t l64 = (int64_t)(w - r) - (int64_t)r;  // readableBytes() - inOffset
        p.lim = l64 < -0x40000000 ? -0x40000000 : (int32_t)l64;
        out.push_back(p);
    }
}

// LZ4 compressionLevel(blockSize) (Lz4FrameEncoder.java:158-166)
inline int32_t lz4_level(uint32_t block_size) {
    const int32_t ceil_log2 = 32 - __builtin_clz(block_size - 1u);
    return ceil_log2 - 10 > 0 ? ceil_log2 - 10 : 0;
}

}  // namespace af
}  // namespace nx

// ------------------------------------------------------------------------------ handles
// The handles of the FastLZ / LZF / LZ4 handlers.  A batcher job holds a reference to its handle
// (refs), so a handler may be removed while its jobs are in flight; parse_failed = a submitted input
// failed its header walk (later submits skip their input; the decoder turns corrupted when that job
// is applied, in order).
struct nx_fastlz_frame_encoder {
    nx::h::Gpu g;
    int32_t level;
    bool checksum;
};

struct nx_lzf_encoder {
    nx::h::Gpu g;
    int32_t threshold;
};

struct nx_lz4_frame_encoder {
    nx::h::Gpu g;
    uint32_t block_size = 65536;
    int32_t level = 6;
    bool high = false;                  // highCompressor (Lz4FrameEncoder.java:161-163)
    int32_t max_encode_size = 0x7FFFFFFF;  // maxEncodeSize (:168), DEFAULT_MAX_ENCODE_SIZE
    std::string err;                    // the last failure's message
    bool finished = false;
    std::vector<uint8_t> buf;  // the block buffer (Lz4FrameEncoder.java:221-226)
};

// allocateBuffer's maxEncodeSize check (handlers.cpp; the batcher's submit runs it too)
int32_t nx_lz4_frame_encoder_check_size(nx_lz4_frame_encoder* e, uint64_t remaining, int32_t* target_out = nullptr);
int32_t nx_lz4_frame_encoder_check_finished(nx_lz4_frame_encoder* e, size_t n, int32_t target);

struct nx_alt_decoder_base {
    nx::h::Gpu g;
    nx::h::MsgList ml;
    bool corrupted = false;     // batcher: set when a failing job is applied
    bool parse_failed = false;  // batcher: a submitted input failed its header walk
    std::atomic<int> refs{1};
    virtual ~nx_alt_decoder_base() = default;
};

struct nx_fastlz_frame_decoder : nx_alt_decoder_base {
    bool validate = false;
    nx::af::FlzState st;
};

struct nx_lzf_decoder : nx_alt_decoder_base {
    nx::af::LzfState st;
};

struct nx_lz4_frame_decoder : nx_alt_decoder_base {
    bool validate = false;
    nx::af::Lz4State st;
};

inline void nx_alt_decoder_unref(nx_alt_decoder_base* d) {
    if (d && d->refs.fetch_sub(1) == 1) delete d;
}
