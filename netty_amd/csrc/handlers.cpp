// handlers.cpp — host handler layer: Netty's framing state machines over host memory, with every
// chunk of one encode()/decode() call batched into a single GPU launch.
//
//   SnappyFrameEncoder   SnappyFrameEncoder.java:79-152
//   SnappyFrameDecoder   SnappyFrameDecoder.java:85-258 (+ ByteToMessageDecoder.callDecode :464-517)
//   FastLzFrameEncoder   FastLzFrameEncoder.java:111-172
//   FastLzFrameDecoder   FastLzFrameDecoder.java:113-207
//   LzfEncoder           LzfEncoder.java:169-246
//   LzfDecoder           LzfDecoder.java:112-241
//
// Headers are parsed on the host exactly as the Java decode() does (they are a few bytes per
// chunk); the per-chunk arithmetic (Snappy/FastLZ/LZF, CRC32C, Adler32) runs on the GPU.  Results
// are applied in stream order, so the first failing chunk truncates the message list and marks the
// decoder corrupted just like the reference's exception path.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../include/netty_amd.h"
#include "nx_common.hpp"
#include "frame_parse.hpp"
#include "handles.hpp"
#include "alt_frames.hpp"

extern "C" int32_t nx_snappy_decode_batch(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*, const uint64_t*,
                                          const uint32_t*, uint32_t*, uint32_t*, int32_t*, const uint32_t*, uint32_t*, uint32_t,
                                          void*);

namespace {
using nx::h::DevBuf;
using nx::h::Gpu;
using nx::h::MsgList;
using nx::h::kStreamStart;

inline uint32_t le24(const uint8_t* p) { return p[0] | (p[1] << 8) | ((uint32_t)p[2] << 16); }
inline uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
inline uint32_t be24(const uint8_t* p) { return ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2]; }
inline uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

}  // namespace

// ======================================================================= Snappy frame encoder

extern "C" nx_snappy_frame_encoder* nx_snappy_frame_encoder_new(int32_t jumbo) {
    auto* e = new nx_snappy_frame_encoder();
    if (!e->g.hold(nx::WsKind::SnappyEnc)) {
        delete e;
        return nullptr;
    }
    e->slice = jumbo ? 65535 : 32767;  // SnappyFrameEncoder.java:31,39
    return e;
}
extern "C" void nx_snappy_frame_encoder_free(nx_snappy_frame_encoder* e) { delete e; }
extern "C" size_t nx_snappy_frame_max_encoded_length(size_t n) { return 10 + (n / 32767 + 2) * 8 + 32 + n + n / 6; }

extern "C" int64_t nx_snappy_frame_encoder_encode(nx_snappy_frame_encoder* e, const uint8_t* in, size_t n, uint8_t* out,
                                                  size_t out_cap) {
    const nx::NoGrowScope no_grow;
    if (!e) return NX_ERR_INVALID_ARG;
    if (n == 0) return 0;  // !in.isReadable()
    if (out_cap < nx_snappy_frame_max_encoded_length(n)) return NX_ERR_INVALID_ARG;
    size_t op = 0;
    if (!e->started) {
        e->started = true;
        memcpy(out, kStreamStart, 10);
        op = 10;
    }
    struct Sl {
        uint64_t off;
        uint32_t len;
        bool comp;
    };
    std::vector<Sl> sl;
    int64_t dl = (int64_t)n;
    if (dl > 18) {  // MIN_COMPRESSIBLE_LENGTH (:46,90-113)
        uint64_t pos = 0;
        for (;;) {
            if (dl < 18) {
                sl.push_back({pos, (uint32_t)dl, false});
                break;
            }
            uint32_t len = dl > e->slice ? (uint32_t)e->slice : (uint32_t)dl;
            sl.push_back({pos, len, true});
            pos += len;
            if (dl > e->slice) dl -= e->slice; else break;
        }
    } else {
        sl.push_back({0, (uint32_t)n, false});
    }
    const uint32_t ns = (uint32_t)sl.size();
    std::vector<uint64_t> ioff(ns), ooff(ns);
    std::vector<uint32_t> ilen(ns);
    uint64_t ocur = 0;
    for (uint32_t i = 0; i < ns; ++i) {
        ioff[i] = sl[i].off;
        ilen[i] = sl[i].len;
        ooff[i] = ocur;
        ocur += nx_snappy_max_compressed_length(sl[i].len);
        ocur = (ocur + 15) & ~15ull;
    }
    Gpu& g = e->g;
    if (!g.din.ensure(n) || !g.dout.ensure(ocur) || !g.a0.ensure(8ull * ns) || !g.a1.ensure(8ull * ns) ||
        !g.a2.ensure(4ull * ns) || !g.a3.ensure(4ull * ns) || !g.a4.ensure(4ull * ns) || !g.a5.ensure(4ull * ns))
        return NX_ERR_HIP;
    bool ok = g.h2d(g.din.p, in, n) && g.h2d(g.a0.p, ioff.data(), 8ull * ns) && g.h2d(g.a1.p, ooff.data(), 8ull * ns) &&
              g.h2d(g.a2.p, ilen.data(), 4ull * ns);
    if (!ok) return NX_ERR_HIP;
    // masked CRC32C of every slice (calculateAndWriteChecksum :150-152, writeUnencodedChunk :119-124)
    int32_t r = nx_crc32c_masked_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.a5.as<uint32_t>(), ns, g.s);
    if (r != NX_OK) return r;
    // Snappy.encode of every slice (uncompressed slices are encoded too but ignored: keeps one launch)
    r = nx_snappy_encode_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                               g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), g.a4.as<int32_t>(), ns, g.s);
    if (r != NX_OK) return r;
    std::vector<uint32_t> clen(ns), crc(ns);
    ok = g.d2h(clen.data(), g.a3.p, 4ull * ns) && g.d2h(crc.data(), g.a5.p, 4ull * ns) && g.sync();
    if (!ok) return NX_ERR_HIP;
    // the framed layout is known once the lengths are: each compressed chunk's bytes (and nothing
    // else of its slot) go straight to their place in `out`
    for (uint32_t i = 0; i < ns; ++i)
        if (sl[i].comp && ((clen[i] + 4) >> 24)) return NX_ERR_INVALID_ARG;  // setChunkLength (:126-132)
    {
        size_t q = op;
        for (uint32_t i = 0; i < ns && ok; ++i) {
            if (sl[i].comp) {
                ok = g.d2h(out + q + 8, g.dout.as<uint8_t>() + ooff[i], clen[i]);
                q += 8 + clen[i];
            } else {
                q += 8 + sl[i].len;
            }
        }
        if (!g.sync() || !ok) return NX_ERR_HIP;
    }
    for (uint32_t i = 0; i < ns; ++i) {
        if (sl[i].comp) {
            const uint32_t chunkLength = clen[i] + 4;  // setChunkLength (:126-132)
            if (chunkLength >> 24) return NX_ERR_INVALID_ARG;
            out[op++] = 0;
            out[op++] = (uint8_t)chunkLength;
            out[op++] = (uint8_t)(chunkLength >> 8);
            out[op++] = (uint8_t)(chunkLength >> 16);
            memcpy(out + op, &crc[i], 4);
            op += 4 + clen[i];  // payload already copied from the device
        } else {
            const uint32_t cl = sl[i].len + 4;
            out[op++] = 1;
            out[op++] = (uint8_t)cl;
            out[op++] = (uint8_t)(cl >> 8);
            out[op++] = (uint8_t)(cl >> 16);
            memcpy(out + op, &crc[i], 4);
            op += 4;
            nx::copy_bytes(out + op, in + sl[i].off, sl[i].len);
            op += sl[i].len;
        }
    }
    return (int64_t)op;
}

// ======================================================================= Snappy frame decoder

extern "C" nx_snappy_frame_decoder* nx_snappy_frame_decoder_new(int32_t validate) {
    auto* d = new nx_snappy_frame_decoder();
    if (!d->g.hold(nx::WsKind::DecRecords)) {
        delete d;
        return nullptr;
    }
    d->validate = validate != 0;
    return d;
}
extern "C" void nx_snappy_frame_decoder_free(nx_snappy_frame_decoder* d) { nx_decoder_unref(d); }

using nx::fr::SAct;
using nx::fr::SnappyAction;
using nx::fr::snappy_parse_one;

extern "C" int32_t nx_snappy_frame_decoder_decode(nx_snappy_frame_decoder* d, const uint8_t* in, size_t n, size_t* consumed,
                                                  const nx_msg** msgs, size_t* n_msgs, const char** err_msg) {
    const nx::NoGrowScope no_grow;
    if (!d || (!in && n)) return NX_ERR_INVALID_ARG;
    MsgList& ml = d->ml;
    ml.clear();
    size_t rd = 0;
    auto finish = [&](int32_t r) {
        *consumed = rd;
        *msgs = ml.msgs.data();
        *n_msgs = ml.msgs.size();
        if (err_msg) *err_msg = ml.err.empty() ? nullptr : ml.err.c_str();
        return r;
    };
    auto corrupt = [&](size_t at, int32_t code, const std::string& msg) {
        ml.err = msg;
        d->corrupted = true;  // :227-230
        rd = at;
        return finish(code);
    };
    if (d->corrupted) {  // :86-89
        rd = n;
        return finish(NX_OK);
    }
    for (;;) {  // loops again only for the validating-mode leftover case below
        std::vector<SnappyAction> acts;
        size_t p = rd;
        bool started = d->started;
        uint64_t skip = d->skip;
        while (p < n && snappy_parse_one(in, n, p, started, skip, d->validate, acts)) {
        }
        // ---- one GPU batch: decode every compressed chunk; CRC every uncompressed one if validating
        std::vector<int> comp_idx, unc_idx;
        size_t lo = (size_t)-1, hi = 0;
        for (size_t i = 0; i < acts.size(); ++i) {
            SnappyAction& a = acts[i];
            if (a.kind == SAct::Comp) {
                a.job = (int)comp_idx.size();
                comp_idx.push_back((int)i);
            } else if (a.kind == SAct::Uncomp && d->validate) {
                a.job = (int)unc_idx.size();
                unc_idx.push_back((int)i);
            } else {
                continue;
            }
            lo = a.data < lo ? a.data : lo;
            hi = a.data + a.dlen > hi ? a.data + a.dlen : hi;
        }
        const uint32_t ncomp = (uint32_t)comp_idx.size(), nunc = (uint32_t)unc_idx.size(), nj = ncomp + nunc;
        std::vector<uint32_t> olen(ncomp), cons(ncomp), ucrc(nunc);
        std::vector<int32_t> st(ncomp);
        std::vector<std::vector<uint8_t>> outs(ncomp);  // each decoded chunk, exactly olen bytes
        Gpu& g = d->g;
        if (nj) {
            const size_t span = hi - lo;
            std::vector<uint64_t> ioff(nj), ooff(ncomp);
            std::vector<uint32_t> ilen(nj), expect(ncomp);
            for (uint32_t j = 0; j < ncomp; ++j) {
                const SnappyAction& a = acts[comp_idx[j]];
                ioff[j] = a.data - lo;
                ilen[j] = a.dlen;
                ooff[j] = (uint64_t)j * 65536;
                expect[j] = a.crc;
            }
            for (uint32_t j = 0; j < nunc; ++j) {
                const SnappyAction& a = acts[unc_idx[j]];
                ioff[ncomp + j] = a.data - lo;
                ilen[ncomp + j] = a.dlen;
            }
            if (!g.din.ensure(span + 1) || !g.dout.ensure((size_t)ncomp * 65536 + 16) || !g.a0.ensure(8ull * nj) ||
                !g.a1.ensure(8ull * ncomp + 8) || !g.a2.ensure(4ull * nj) || !g.a3.ensure(4ull * ncomp + 4) ||
                !g.a4.ensure(4ull * ncomp + 4) || !g.a5.ensure(4ull * ncomp + 4) || !g.a6.ensure(4ull * nj + 4))
                return finish(NX_ERR_HIP);
            bool ok = g.h2d(g.din.p, in + lo, span) && g.h2d(g.a0.p, ioff.data(), 8ull * nj) && g.h2d(g.a2.p, ilen.data(), 4ull * nj) &&
                      g.h2d(g.a1.p, ooff.data(), 8ull * ncomp) && g.h2d(g.a5.p, expect.data(), 4ull * ncomp);
            if (!ok) return finish(NX_ERR_HIP);
            int32_t* d_st = g.a6.as<int32_t>();
            uint32_t* d_ucrc = g.a6.as<uint32_t>() + ncomp;
            if (ncomp) {
                int32_t r = nx_snappy_decode_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                                                   g.a1.as<uint64_t>(), nullptr, g.a3.as<uint32_t>(), g.a4.as<uint32_t>(), d_st,
                                                   d->validate ? g.a5.as<uint32_t>() : nullptr, nullptr, ncomp, g.s);
                if (r != NX_OK) return finish(r);
            }
            if (nunc) {
                int32_t r = nx_crc32c_masked_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>() + ncomp, g.a2.as<uint32_t>() + ncomp, d_ucrc,
                                                   nunc, g.s);
                if (r != NX_OK) return finish(r);
            }
            ok = g.d2h(olen.data(), g.a3.p, 4ull * ncomp) && g.d2h(cons.data(), g.a4.p, 4ull * ncomp) &&
                 g.d2h(st.data(), d_st, 4ull * ncomp) && g.d2h(ucrc.data(), d_ucrc, 4ull * nunc) && g.sync();
            if (!ok) return finish(NX_ERR_HIP);
            // only the bytes each chunk produced cross PCIe (a message's olen, not its 64 KiB slot)
            for (uint32_t j = 0; j < ncomp && ok; ++j) {
                if (st[j] != NX_OK && st[j] != NX_ERR_SNAPPY_CRC_MISMATCH) continue;
                outs[j].resize(olen[j]);
                ok = g.d2h(outs[j].data(), g.dout.as<uint8_t>() + (size_t)j * 65536, olen[j]);
            }
            if (!g.sync() || !ok) return finish(NX_ERR_HIP);
        }
        // ---- apply in stream order (the first failing chunk ends the call, as the Java exception does)
        bool reparse = false;
        char buf[128];
        for (const SnappyAction& a : acts) {
            if (a.kind == SAct::Error) return corrupt(a.end, NX_ERR_FRAME_CORRUPT, a.err);
            if (a.kind == SAct::Stream) {
                d->started = true;
            } else if (a.kind == SAct::Uncomp) {
                if (d->validate && ucrc[a.job] != a.crc) {  // :171-175
                    snprintf(buf, sizeof buf, "mismatching checksum: %x (expected: %x)", ucrc[a.job], a.crc);
                    return corrupt(a.end, NX_ERR_SNAPPY_CRC_MISMATCH, buf);
                }
                ml.msgs.push_back({in + a.data, a.dlen});  // readRetainedSlice: a view of the cumulation
            } else if (a.kind == SAct::Comp) {
                const int j = a.job;
                if (st[j] == NX_ERR_SNAPPY_CRC_MISMATCH) {
                    snprintf(buf, sizeof buf, "mismatching checksum: %x (expected: %x)",
                             nx::host_mask(nx::host_crc32c(outs[j].data(), olen[j])), a.crc);
                    return corrupt(a.end, st[j], buf);
                }
                if (st[j] != NX_OK)
                    return corrupt(a.end, st[j], nx::fr::snappy_block_error(st[j], cons[j] >= 4 ? le32(in + a.data + cons[j] - 4) : 0u,
                                                                           nx_status_string));
                ml.owned.push_back(std::move(outs[j]));
                ml.msgs.push_back({ml.owned.back().data(), olen[j]});
                if (d->validate && cons[j] < a.dlen) {
                    // validating mode restores the writer index and leaves the unread chunk bytes in
                    // the cumulation (:206-212); they are parsed again as the next chunk header.
                    rd = a.data + cons[j];
                    d->skip = 0;
                    reparse = true;
                    break;
                }
            }
            rd = a.end;
            d->skip = a.skip;
        }
        if (!reparse) break;
    }
    return finish(NX_OK);
}

// ======================================================================= FastLZ frame encoder

extern "C" nx_fastlz_frame_encoder* nx_fastlz_frame_encoder_new(int32_t level, int32_t checksum) {
    if (level != 0 && level != 1 && level != 2) return nullptr;  // FastLzFrameEncoder.java:101-105
    auto* e = new nx_fastlz_frame_encoder();
    if (!e->g.hold(nx::WsKind::FastLzEnc)) {
        delete e;
        return nullptr;
    }
    e->level = level;
    e->checksum = checksum != 0;
    return e;
}
extern "C" void nx_fastlz_frame_encoder_free(nx_fastlz_frame_encoder* e) { delete e; }
extern "C" size_t nx_fastlz_frame_max_encoded_length(size_t n) { return (n / 65535 + 1) * (12 + 82) + n + n / 16; }

extern "C" int64_t nx_fastlz_frame_encoder_encode(nx_fastlz_frame_encoder* e, const uint8_t* buf, size_t r0, size_t n,
                                                  uint8_t* out, size_t out_cap) {
    const nx::NoGrowScope no_grow;
    if (!e) return NX_ERR_INVALID_ARG;
    if (n == 0) return 0;
    if (out_cap < nx_fastlz_frame_max_encoded_length(n)) return NX_ERR_INVALID_ARG;
    const uint8_t* in = buf + r0;
    const size_t w = r0 + n;
    const uint32_t nc = (uint32_t)((n + 65534) / 65535);
    std::vector<uint64_t> ioff(nc), ooff(nc);
    std::vector<uint32_t> ilen(nc);
    std::vector<int32_t> lim(nc), lvl(nc, e->level);
    uint64_t oc = 0;
    for (uint32_t i = 0; i < nc; ++i) {
        const size_t r = r0 + (size_t)i * 65535;
        ioff[i] = (uint64_t)i * 65535;
        ilen[i] = (uint32_t)((n - ioff[i]) < 65535 ? (n - ioff[i]) : 65535);
        const int64_t l64 = (int64_t)(w - r) - (int64_t)r;  // readableBytes() - inOffset (FastLz.java:552-557)
        lim[i] = l64 < -0x40000000 ? -0x40000000 : (int32_t)l64;
        ooff[i] = oc;
        oc += nx_fastlz_max_compressed_length(ilen[i]) + 16;
    }
    Gpu& g = e->g;
    if (!g.din.ensure(n) || !g.dout.ensure(oc) || !g.a0.ensure(8ull * nc) || !g.a1.ensure(8ull * nc) || !g.a2.ensure(4ull * nc) ||
        !g.a3.ensure(4ull * nc) || !g.a4.ensure(4ull * nc) || !g.a5.ensure(4ull * nc) || !g.a6.ensure(8ull * nc))
        return NX_ERR_HIP;
    bool ok = g.h2d(g.din.p, in, n) && g.h2d(g.a0.p, ioff.data(), 8ull * nc) && g.h2d(g.a1.p, ooff.data(), 8ull * nc) &&
              g.h2d(g.a2.p, ilen.data(), 4ull * nc) && g.h2d(g.a5.p, lim.data(), 4ull * nc) &&
              g.h2d(g.a6.p, lvl.data(), 4ull * nc);
    if (!ok) return NX_ERR_HIP;
    int32_t r = nx_fastlz_compress_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                                         g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), g.a6.as<int32_t>(), g.a5.as<int32_t>(),
                                         g.a4.as<int32_t>(), nc, g.s);
    if (r != NX_OK) return r;
    std::vector<uint32_t> ad(nc);
    if (e->checksum) {
        // reuse a4 (status no longer needed after the compress kernel ran: stream-ordered)
        r = nx_adler32_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.a4.as<uint32_t>(), nc, g.s);
        if (r != NX_OK) return r;
    }
    std::vector<uint32_t> clen(nc);
    ok = g.d2h(clen.data(), g.a3.p, 4ull * nc) && (!e->checksum || g.d2h(ad.data(), g.a4.p, 4ull * nc)) && g.sync();
    if (!ok) return NX_ERR_HIP;
    size_t op = 0;
    for (uint32_t i = 0; i < nc; ++i) {
        const uint32_t length = ilen[i];
        const size_t outputIdx = op;
        out[op] = 'F';
        out[op + 1] = 'L';
        out[op + 2] = 'Z';
        size_t outputOffset = outputIdx + 4 + (e->checksum ? 4 : 0);
        if (e->checksum) {
            const uint32_t c = ad[i];
            out[outputIdx + 4] = (uint8_t)(c >> 24);
            out[outputIdx + 5] = (uint8_t)(c >> 16);
            out[outputIdx + 6] = (uint8_t)(c >> 8);
            out[outputIdx + 7] = (uint8_t)c;
        }
        uint8_t blockType;
        uint32_t chunkLength;
        if (length >= 32 && clen[i] < length) {  // MIN_LENGTH_TO_COMPRESSION (FastLz.java:59), :153-158
            blockType = 1;
            chunkLength = clen[i];
            out[outputOffset] = (uint8_t)(chunkLength >> 8);
            out[outputOffset + 1] = (uint8_t)chunkLength;
            outputOffset += 2;
            // only the compressed bytes cross PCIe, straight into their framed position
            ok = ok && g.d2h(out + outputOffset + 2, g.dout.as<uint8_t>() + ooff[i], chunkLength);
        } else {
            blockType = 0;
            chunkLength = length;
            nx::copy_bytes(out + outputOffset + 2, in + ioff[i], length);
        }
        out[outputOffset] = (uint8_t)(length >> 8);
        out[outputOffset + 1] = (uint8_t)length;
        out[outputIdx + 3] = (uint8_t)(blockType | (e->checksum ? 0x10 : 0));
        op = outputOffset + 2 + chunkLength;
    }
    if (!g.sync() || !ok) return NX_ERR_HIP;  // every queued copy has landed (or failed) before returning
    return (int64_t)op;
}

// ======================================================================= FastLZ frame decoder
extern "C" nx_fastlz_frame_decoder* nx_fastlz_frame_decoder_new(int32_t validate) {
    auto* d = new nx_fastlz_frame_decoder();
    if (!d->g.hold(nx::WsKind::DecRecords)) {  // FastLZ blocks decode through the record expander
        delete d;
        return nullptr;
    }
    d->validate = validate != 0;
    return d;
}
extern "C" void nx_fastlz_frame_decoder_free(nx_fastlz_frame_decoder* d) { nx_alt_decoder_unref(d); }

extern "C" int32_t nx_fastlz_frame_decoder_decode(nx_fastlz_frame_decoder* d, const uint8_t* in, size_t n, size_t* consumed,
                                                  const nx_msg** msgs, size_t* n_msgs, const char** err_msg) {
    const nx::NoGrowScope no_grow;
    if (!d || (!in && n)) return NX_ERR_INVALID_ARG;
    MsgList& ml = d->ml;
    ml.clear();
    size_t rd = 0;
    auto finish = [&](int32_t r) {
        *consumed = rd;
        *msgs = ml.msgs.data();
        *n_msgs = ml.msgs.size();
        if (err_msg) *err_msg = ml.err.empty() ? nullptr : ml.err.c_str();
        return r;
    };
    if (d->corrupted || d->st.state == 3) {  // CORRUPTED (:197-199)
        rd = n;
        return finish(NX_OK);
    }
    struct Blk : nx::af::Blk {
        int job = -1;
    };
    // host parse (FastLzFrameDecoder.decode as driven by callDecode); persistent header state
    nx::af::FlzState ns = d->st;
    std::vector<nx::af::Blk> walked;
    nx::af::WalkErr werr;
    const size_t p = nx::af::flz_walk(in, n, ns, walked, werr);
    std::vector<Blk> blks(walked.size());
    for (size_t i = 0; i < walked.size(); ++i) static_cast<nx::af::Blk&>(blks[i]) = walked[i];
    // GPU: decompress every compressed block; Adler32 over every produced block if verifying
    // (decompressed blocks in dout, raw blocks straight from the staged cumulation in din)
    uint32_t nz = 0;
    for (auto& b : blks)
        if (b.comp) b.job = (int)nz++;
    const uint32_t nb = (uint32_t)blks.size();
    const bool want_cks = d->validate;
    std::vector<int32_t> res(nz);
    std::vector<uint32_t> adl(nb);
    std::vector<uint64_t> ooff(nz);
    uint64_t ocap = 0;
    for (auto& b : blks)
        if (b.comp) {
            ooff[b.job] = ocap;
            ocap += ((uint64_t)b.olen + 15) & ~15ull;
        }
    std::vector<uint8_t> hout(ocap);
    Gpu& g = d->g;
    uint32_t ncks = 0;
    for (auto& b : blks) ncks += (b.has_cks && want_cks) ? 1u : 0u;
    if (nz || ncks) {
        const size_t lo = blks.front().data;
        const size_t span = n - lo;  // decompress may read past its chunk (in_avail = readable bytes)
        std::vector<uint64_t> ioff(nz);
        std::vector<uint32_t> ilen(nz), iav(nz), olim(nz);
        for (auto& b : blks)
            if (b.comp) {
                ioff[b.job] = b.data - lo;
                ilen[b.job] = b.clen;
                iav[b.job] = (uint32_t)(n - b.data);
                olim[b.job] = b.olen;
            }
        // checksum jobs: compressed → (dout, ooff, olen); raw → (din, data-lo, clen)
        std::vector<uint64_t> czoff, croff;
        std::vector<uint32_t> czlen, crlen;
        std::vector<uint32_t> cz_blk, cr_blk;
        for (uint32_t i = 0; i < nb; ++i) {
            const Blk& b = blks[i];
            if (!(b.has_cks && want_cks)) continue;
            if (b.comp) {
                czoff.push_back(ooff[b.job]);
                czlen.push_back(b.olen);
                cz_blk.push_back(i);
            } else {
                croff.push_back(b.data - lo);
                crlen.push_back(b.clen);
                cr_blk.push_back(i);
            }
        }
        const uint32_t ncz = (uint32_t)czoff.size(), ncr = (uint32_t)croff.size();
        if (!g.din.ensure(span + 1) || !g.dout.ensure(ocap + 16) || !g.a0.ensure(8ull * nz + 8) || !g.a1.ensure(8ull * nz + 8) ||
            !g.a2.ensure(4ull * nz + 4) || !g.a3.ensure(4ull * nz + 4) || !g.a4.ensure(4ull * nz + 4) || !g.a5.ensure(4ull * nz + 4) ||
            !g.a6.ensure(16ull * (ncz + ncr) + 16))
            return finish(NX_ERR_HIP);
        uint64_t* d_coff = g.a6.as<uint64_t>();
        uint32_t* d_clen = reinterpret_cast<uint32_t*>(d_coff + ncz + ncr);
        uint32_t* d_cval = d_clen + ncz + ncr;
        std::vector<uint64_t> coff(czoff);
        coff.insert(coff.end(), croff.begin(), croff.end());
        std::vector<uint32_t> clen(czlen);
        clen.insert(clen.end(), crlen.begin(), crlen.end());
        bool ok = g.h2d(g.din.p, in + lo, span) && g.h2d(g.a0.p, ioff.data(), 8ull * nz) && g.h2d(g.a1.p, ooff.data(), 8ull * nz) &&
                  g.h2d(g.a2.p, ilen.data(), 4ull * nz) && g.h2d(g.a3.p, iav.data(), 4ull * nz) && g.h2d(g.a4.p, olim.data(), 4ull * nz) &&
                  g.h2d(d_coff, coff.data(), 8ull * (ncz + ncr)) && g.h2d(d_clen, clen.data(), 4ull * (ncz + ncr));
        if (!ok) return finish(NX_ERR_HIP);
        if (nz) {
            int32_t r = nx_fastlz_decompress_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.a3.as<uint32_t>(),
                                                   g.dout.as<uint8_t>(), g.a1.as<uint64_t>(), g.a4.as<uint32_t>(), g.a5.as<int32_t>(),
                                                   nz, g.s);
            if (r != NX_OK) return finish(r);
        }
        if (ncz) {
            int32_t r = nx_adler32_batch(g.dout.as<uint8_t>(), d_coff, d_clen, d_cval, ncz, g.s);
            if (r != NX_OK) return finish(r);
        }
        if (ncr) {
            int32_t r = nx_adler32_batch(g.din.as<uint8_t>(), d_coff + ncz, d_clen + ncz, d_cval + ncz, ncr, g.s);
            if (r != NX_OK) return finish(r);
        }
        std::vector<uint32_t> cval(ncz + ncr);
        ok = g.d2h(res.data(), g.a5.p, 4ull * nz) && g.d2h(hout.data(), g.dout.p, ocap) && g.d2h(cval.data(), d_cval, 4ull * (ncz + ncr)) &&
             g.sync();
        if (!ok) return finish(NX_ERR_HIP);
        for (uint32_t k = 0; k < ncz; ++k) adl[cz_blk[k]] = cval[k];
        for (uint32_t k = 0; k < ncr; ++k) adl[cr_blk[k]] = cval[ncz + k];
    }
    // apply in order
    for (uint32_t i = 0; i < nb; ++i) {
        Blk& b = blks[i];
        const uint8_t* data;
        uint32_t len;
        if (b.comp) {
            const int32_t r = res[b.job];
            int32_t code;
            std::string emsg;
            if (nx::af::flz_block_error(r, b.olen, b.data < n ? in[b.data] : 0, &code, &emsg)) {
                ml.err = emsg;
                d->st.state = 3;
                d->corrupted = true;
                rd = b.data;
                return finish(code);
            }
            data = hout.data() + ooff[b.job];
            len = b.olen;
        } else {
            data = in + b.data;
            len = b.clen;
        }
        if (b.has_cks && want_cks && adl[i] != b.cks) {  // FastLzFrameDecoder.java:171-180
            ml.err = nx::af::flz_checksum_error(adl[i], b.cks);
            d->st.state = 3;
            d->corrupted = true;
            rd = b.data;
            return finish(NX_ERR_FASTLZ_CRC_MISMATCH);
        }
        if (len > 0) {
            if (b.comp) {
                ml.owned.emplace_back(data, data + len);
                ml.msgs.push_back({ml.owned.back().data(), len});
            } else {
                ml.msgs.push_back({data, len});
            }
        }
        rd = b.end;
    }
    if (werr.set) {
        ml.err = werr.msg;
        d->st.state = 3;
        d->corrupted = true;
        rd = werr.at;
        return finish(werr.code);
    }
    rd = p;
    d->st = ns;
    return finish(NX_OK);
}

// ======================================================================= LZF encoder / decoder
// LzfEncoder(totalLength, compressThreshold) (LzfEncoder.java:127-166).  totalLength is validated as
// :147-150 does (MIN_BLOCK_TO_COMPRESS 16 .. MAX_CHUNK_LEN 65535) and does not change the bytes: it
// only sizes the ChunkEncoder's hash table, and the non-allocating encoders LzfEncoder takes
// (ChunkEncoderFactory.optimalNonAllocatingInstance / safeNonAllocatingInstance, :161-163) size it from
// max(totalLength, MAX_CHUNK_LEN), i.e. the 16384-entry table for every totalLength (compress-lzf
// 1.0.3 ChunkEncoder(int, BufferRecycler, boolean); DESIGN.md §2: restated, not pinned).
extern "C" nx_lzf_encoder* nx_lzf_encoder_new_ex(int32_t total_length, int32_t compress_threshold) {
    if (total_length < 16 || total_length > 65535) return nullptr;  // :147-150
    return nx_lzf_encoder_new(compress_threshold);
}

extern "C" nx_lzf_encoder* nx_lzf_encoder_new(int32_t compress_threshold) {
    if (compress_threshold < 16) return nullptr;  // LzfEncoder.java:152-156
    auto* e = new nx_lzf_encoder();
    if (!e->g.hold(nx::WsKind::LzfEnc)) {
        delete e;
        return nullptr;
    }
    e->threshold = compress_threshold;
    return e;
}
extern "C" void nx_lzf_encoder_free(nx_lzf_encoder* e) { delete e; }
extern "C" size_t nx_lzf_frame_max_encoded_length(size_t n) { return (n / 65535 + 1) * 7 + n + n / 32 + 64; }

extern "C" int64_t nx_lzf_encoder_encode(nx_lzf_encoder* e, const uint8_t* in, size_t n, uint8_t* out, size_t out_cap) {
    const nx::NoGrowScope no_grow;
    if (!e) return NX_ERR_INVALID_ARG;
    if (out_cap < nx_lzf_frame_max_encoded_length(n)) return NX_ERR_INVALID_ARG;
    if ((int64_t)n < e->threshold) {  // encodeNonCompress (LzfEncoder.java:197-203,223-246)
        size_t op = 0, ip = 0;
        do {
            const uint32_t len = (uint32_t)((n - ip) < 65535 ? (n - ip) : 65535);
            out[op] = 'Z';
            out[op + 1] = 'V';
            out[op + 2] = 0;
            out[op + 3] = (uint8_t)(len >> 8);
            out[op + 4] = (uint8_t)len;
            nx::copy_bytes(out + op + 5, in + ip, len);
            op += 5 + len;
            ip += len;
        } while (ip < n);
        return (int64_t)op;
    }
    const uint32_t nc = (uint32_t)((n + 65534) / 65535);
    std::vector<uint64_t> ioff(nc), ooff(nc);
    std::vector<uint32_t> ilen(nc);
    uint64_t oc = 0;
    for (uint32_t i = 0; i < nc; ++i) {
        ioff[i] = (uint64_t)i * 65535;
        ilen[i] = (uint32_t)((n - ioff[i]) < 65535 ? (n - ioff[i]) : 65535);
        ooff[i] = oc;
        oc += nx_lzf_max_compressed_length(ilen[i]) + 16;
    }
    Gpu& g = e->g;
    if (!g.din.ensure(n) || !g.dout.ensure(oc) || !g.a0.ensure(8ull * nc) || !g.a1.ensure(8ull * nc) || !g.a2.ensure(4ull * nc) ||
        !g.a3.ensure(4ull * nc) || !g.a4.ensure(4ull * nc))
        return NX_ERR_HIP;
    bool ok = g.h2d(g.din.p, in, n) && g.h2d(g.a0.p, ioff.data(), 8ull * nc) && g.h2d(g.a1.p, ooff.data(), 8ull * nc) &&
              g.h2d(g.a2.p, ilen.data(), 4ull * nc);
    if (!ok) return NX_ERR_HIP;
    int32_t r = nx_lzf_encode_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                                    g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), g.a4.as<int32_t>(), nc, g.s);
    if (r != NX_OK) return r;
    std::vector<uint32_t> olen(nc);
    ok = g.d2h(olen.data(), g.a3.p, 4ull * nc) && g.sync();
    if (!ok) return NX_ERR_HIP;
    size_t op = 0;
    for (uint32_t i = 0; i < nc && ok; ++i) {  // each block's bytes only, concatenated in place
        ok = g.d2h(out + op, g.dout.as<uint8_t>() + ooff[i], olen[i]);
        op += olen[i];
    }
    if (!g.sync() || !ok) return NX_ERR_HIP;
    return (int64_t)op;
}

extern "C" nx_lzf_decoder* nx_lzf_decoder_new(void) {
    auto* d = new nx_lzf_decoder();
    if (!d->g.hold(nx::WsKind::DecRecords)) {  // LZF blocks decode through the record expander
        delete d;
        return nullptr;
    }
    return d;
}
extern "C" void nx_lzf_decoder_free(nx_lzf_decoder* d) { nx_alt_decoder_unref(d); }

extern "C" int32_t nx_lzf_decoder_decode(nx_lzf_decoder* d, const uint8_t* in, size_t n, size_t* consumed, const nx_msg** msgs,
                                         size_t* n_msgs, const char** err_msg) {
    const nx::NoGrowScope no_grow;
    if (!d || (!in && n)) return NX_ERR_INVALID_ARG;
    MsgList& ml = d->ml;
    ml.clear();
    size_t rd = 0;
    auto finish = [&](int32_t r) {
        *consumed = rd;
        *msgs = ml.msgs.data();
        *n_msgs = ml.msgs.size();
        if (err_msg) *err_msg = ml.err.empty() ? nullptr : ml.err.c_str();
        return r;
    };
    if (d->corrupted || d->st.state == 3) {  // CORRUPTED (:229-231)
        rd = n;
        return finish(NX_OK);
    }
    struct Blk : nx::af::Blk {
        int job = -1;
    };
    nx::af::LzfState ns = d->st;
    std::vector<nx::af::Blk> walked;
    nx::af::WalkErr werr;
    const size_t p = nx::af::lzf_walk(in, n, ns, walked, werr);
    std::vector<Blk> blks(walked.size());
    for (size_t i = 0; i < walked.size(); ++i) static_cast<nx::af::Blk&>(blks[i]) = walked[i];
    uint32_t nz = 0;
    uint64_t ocap = 0;
    std::vector<uint64_t> ooff;
    for (auto& b : blks)
        if (b.comp) {
            b.job = (int)nz++;
            ooff.push_back(ocap);
            ocap += ((uint64_t)b.olen + 15) & ~15ull;
        }
    std::vector<int32_t> st(nz);
    std::vector<uint8_t> hout(ocap);
    Gpu& g = d->g;
    if (nz) {
        const size_t lo = blks.front().data;
        const size_t span = p - lo;
        std::vector<uint64_t> ioff(nz);
        std::vector<uint32_t> ilen(nz), olen(nz);
        for (auto& b : blks)
            if (b.comp) {
                ioff[b.job] = b.data - lo;
                ilen[b.job] = b.clen;
                olen[b.job] = b.olen;
            }
        if (!g.din.ensure(span + 1) || !g.dout.ensure(ocap + 16) || !g.a0.ensure(8ull * nz) || !g.a1.ensure(8ull * nz) ||
            !g.a2.ensure(4ull * nz) || !g.a3.ensure(4ull * nz) || !g.a4.ensure(4ull * nz))
            return finish(NX_ERR_HIP);
        bool ok = g.h2d(g.din.p, in + lo, span) && g.h2d(g.a0.p, ioff.data(), 8ull * nz) && g.h2d(g.a1.p, ooff.data(), 8ull * nz) &&
                  g.h2d(g.a2.p, ilen.data(), 4ull * nz) && g.h2d(g.a3.p, olen.data(), 4ull * nz);
        if (!ok) return finish(NX_ERR_HIP);
        int32_t r = nx_lzf_decode_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                                        g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), g.a4.as<int32_t>(), nz, g.s);
        if (r != NX_OK) return finish(r);
        ok = g.d2h(st.data(), g.a4.p, 4ull * nz) && g.d2h(hout.data(), g.dout.p, ocap) && g.sync();
        if (!ok) return finish(NX_ERR_HIP);
    }
    for (auto& b : blks) {
        if (b.comp) {
            if (st[b.job] != NX_OK) {
                ml.err = nx::af::lzf_block_error();
                d->st.state = 3;
                d->corrupted = true;
                rd = b.data;
                return finish(st[b.job]);
            }
            ml.owned.emplace_back(hout.begin() + ooff[b.job], hout.begin() + ooff[b.job] + b.olen);
            ml.msgs.push_back({ml.owned.back().data(), b.olen});
        } else if (b.clen > 0) {
            ml.msgs.push_back({in + b.data, b.clen});
        }
        rd = b.end;
    }
    if (werr.set) {
        ml.err = werr.msg;
        d->st.state = 3;
        d->corrupted = true;
        rd = werr.at;
        return finish(werr.code);
    }
    rd = p;
    d->st = ns;
    return finish(NX_OK);
}

// ======================================================================= LZ4 frame encoder / decoder
//   Lz4FrameEncoder   Lz4FrameEncoder.java:231-336 (encode, flushBufferedData, finishEncode)
//   Lz4FrameDecoder   Lz4FrameDecoder.java:121-261
// Every full block of one encode() call (and every block of one decode() call) goes to the GPU in
// one batch: nx_lz4_frame_encode_batch / nx_lz4_decode_batch + nx_xxhash32_batch.
using nx::af::kLz4Header;
using nx::af::kLz4Magic;
using nx::af::kLz4Seed;


extern "C" nx_lz4_frame_encoder* nx_lz4_frame_encoder_new_ex(int32_t block_size, int32_t high_compressor, int32_t max_encode_size) {
    // compressionLevel(blockSize) :158-166; the device block encoder takes blocks below 32 MiB
    if (block_size < 64 || block_size > (1 << 25) || max_encode_size <= 0) return nullptr;
    auto* e = new nx_lz4_frame_encoder();
    e->high = high_compressor != 0;
    if (!e->g.hold(e->high ? nx::WsKind::Lz4HcEnc : nx::WsKind::Lz4Enc)) {
        delete e;
        return nullptr;
    }
    e->max_encode_size = max_encode_size;
    e->block_size = (uint32_t)block_size;
    const int32_t ceil_log2 = 32 - __builtin_clz((uint32_t)block_size - 1u);
    e->level = ceil_log2 - 10 > 0 ? ceil_log2 - 10 : 0;
    e->buf.reserve(block_size);
    return e;
}
extern "C" nx_lz4_frame_encoder* nx_lz4_frame_encoder_new(int32_t block_size) {
    return nx_lz4_frame_encoder_new_ex(block_size, 0, 0x7FFFFFFF);
}
extern "C" void nx_lz4_frame_encoder_free(nx_lz4_frame_encoder* e) { delete e; }
extern "C" const char* nx_lz4_frame_encoder_error(nx_lz4_frame_encoder* e) { return e && !e->err.empty() ? e->err.c_str() : nullptr; }
extern "C" size_t nx_lz4_frame_max_encoded_length(size_t n, int32_t block_size) {
    const size_t bs = block_size > 0 ? (size_t)block_size : 65536;
    return (n / bs + 2) * (kLz4Header + 16 + bs / 255) + n + kLz4Header;
}

namespace {
// flushBufferedData (:248-284) for nb consecutive blocks of `src` (the last may be short).
int64_t lz4_flush_blocks(nx_lz4_frame_encoder* e, const uint8_t* src, size_t n, uint8_t* out, size_t out_cap) {
    if (n == 0) return 0;
    const uint32_t bs = e->block_size;
    const uint32_t nb = (uint32_t)((n + bs - 1) / bs);
    std::vector<uint64_t> ioff(nb), ooff(nb);
    std::vector<uint32_t> ilen(nb);
    uint64_t oc = 0;
    for (uint32_t i = 0; i < nb; ++i) {
        ioff[i] = (uint64_t)i * bs;
        ilen[i] = (uint32_t)((n - ioff[i]) < bs ? (n - ioff[i]) : bs);
        ooff[i] = oc;
        oc += kLz4Header + nx_lz4_max_compressed_length(ilen[i]);
    }
    Gpu& g = e->g;
    if (!g.din.ensure(n) || !g.dout.ensure(oc) || !g.a0.ensure(8ull * nb) || !g.a1.ensure(8ull * nb) || !g.a2.ensure(4ull * nb) ||
        !g.a3.ensure(4ull * nb) || !g.a4.ensure(4ull * nb))
        return NX_ERR_HIP;
    bool ok = g.h2d(g.din.p, src, n) && g.h2d(g.a0.p, ioff.data(), 8ull * nb) && g.h2d(g.a1.p, ooff.data(), 8ull * nb) &&
              g.h2d(g.a2.p, ilen.data(), 4ull * nb);
    if (!ok) return NX_ERR_HIP;
    int32_t r = nx_lz4_frame_encode_batch_ex(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                                             g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), e->level, e->high ? 1 : 0, g.a4.as<int32_t>(), nb,
                                             g.s);
    if (r != NX_OK) return r;
    std::vector<uint32_t> olen(nb);
    std::vector<int32_t> st(nb);
    ok = g.d2h(olen.data(), g.a3.p, 4ull * nb) && g.d2h(st.data(), g.a4.p, 4ull * nb) && g.sync();
    if (!ok) return NX_ERR_HIP;
    size_t op = 0;
    for (uint32_t i = 0; i < nb; ++i) {
        if (st[i] != NX_OK) return st[i];
        if (op + olen[i] > out_cap) return NX_ERR_INVALID_ARG;
        op += olen[i];
    }
    op = 0;
    for (uint32_t i = 0; i < nb && ok; ++i) {  // each framed block's bytes only, concatenated in place
        ok = g.d2h(out + op, g.dout.as<uint8_t>() + ooff[i], olen[i]);
        op += olen[i];
    }
    if (!g.sync() || !ok) return NX_ERR_HIP;
    return (int64_t)op;
}
}  // namespace

// allocateBuffer's size check (:190-214): the blocks of `remaining` pending bytes, each
// maxCompressedLength(curSize) + HEADER_LENGTH, against maxEncodeSize (Java int arithmetic: a sum
// that overflows is negative and fails too).  Returns NX_OK or NX_ERR_LZ4_ENCODE_SIZE with the message.
int32_t nx_lz4_frame_encoder_check_size(nx_lz4_frame_encoder* e, uint64_t remaining, int32_t* target_out) {
    if (target_out) *target_out = 0;
    if (remaining > 0x7FFFFFFFull) {  // int remaining < 0 (:195-197)
        e->err = "too much data to allocate a buffer for compression";
        return NX_ERR_LZ4_ENCODE_SIZE;
    }
    int64_t target = 0;
    while (remaining > 0) {
        const uint64_t cur = remaining < e->block_size ? remaining : e->block_size;
        remaining -= cur;
        target += (int64_t)nx_lz4_max_compressed_length(cur) + (int64_t)kLz4Header;
    }
    const int32_t t32 = (int32_t)(uint32_t)(uint64_t)target;  // the Java int sum
    if (t32 > e->max_encode_size || t32 < 0) {
        char buf[160];
        snprintf(buf, sizeof buf, "requested encode buffer size (%d bytes) exceeds the maximum allowable size (%d bytes)", t32,
                 e->max_encode_size);
        e->err = buf;
        return NX_ERR_LZ4_ENCODE_SIZE;
    }
    if (target_out) *target_out = t32;
    return NX_OK;
}

// encode() after close() (:233-239): write()'s allocateBuffer(allowEmptyReturn = true) hands encode an
// EMPTY_BUFFER when the message's blocks need fewer than blockSize bytes (:216-218), and encode then
// throws; a larger message gets a buffer of its size and passes through.
int32_t nx_lz4_frame_encoder_check_finished(nx_lz4_frame_encoder* e, size_t n, int32_t target) {
    if (!e->finished || n == 0 || target >= (int32_t)e->block_size) return NX_OK;
    e->err = "encode finished and not enough space to write remaining data";
    return NX_ERR_LZ4_ENCODE_FINISHED;
}

extern "C" int64_t nx_lz4_frame_encoder_encode(nx_lz4_frame_encoder* e, const uint8_t* in, size_t n, uint8_t* out,
                                               size_t out_cap) {
    const nx::NoGrowScope no_grow;
    if (!e || (!in && n)) return NX_ERR_INVALID_ARG;
    {   // MessageToByteEncoder.write: allocateBuffer before encode (:190-214), also after close()
        int32_t target = 0;
        int32_t r = nx_lz4_frame_encoder_check_size(e, (uint64_t)n + e->buf.size(), &target);
        if (r == NX_OK) r = nx_lz4_frame_encoder_check_finished(e, n, target);
        if (r != NX_OK) return r;
    }
    if (e->finished) {  // :233-239 — after close() a message of at least a block's buffer passes through
        if (out_cap < n) return NX_ERR_INVALID_ARG;
        if (n) memcpy(out, in, n);
        return (int64_t)n;
    }
    // :241-248 — fill the block buffer; every full buffer is flushed
    const size_t have = e->buf.size();
    const size_t total = have + n;
    const size_t full = total / e->block_size * e->block_size;
    if (full == 0) {
        e->buf.insert(e->buf.end(), in, in + n);
        return 0;
    }
    std::vector<uint8_t> joined;
    const uint8_t* src = in;
    if (have) {
        joined.reserve(full);
        joined.insert(joined.end(), e->buf.begin(), e->buf.end());
        joined.insert(joined.end(), in, in + (full - have));
        src = joined.data();
    }
    const int64_t w = lz4_flush_blocks(e, src, full, out, out_cap);
    if (w < 0) return w;
    e->buf.assign(in + (full - have), in + n);
    return w;
}

static int64_t lz4_flush_buffer(nx_lz4_frame_encoder* e, uint8_t* out, size_t out_cap) {
    const int64_t w = lz4_flush_blocks(e, e->buf.data(), e->buf.size(), out, out_cap);
    if (w >= 0) e->buf.clear();
    return w;
}

extern "C" int64_t nx_lz4_frame_encoder_flush(nx_lz4_frame_encoder* e, uint8_t* out, size_t out_cap) {
    const nx::NoGrowScope no_grow;
    if (!e) return NX_ERR_INVALID_ARG;  // flush() :296-304: allocateBuffer(ctx, EMPTY_BUFFER, .., false) first
    if (!e->buf.empty()) {
        const int32_t r = nx_lz4_frame_encoder_check_size(e, e->buf.size());
        if (r != NX_OK) return r;
    }
    return lz4_flush_buffer(e, out, out_cap);
}

extern "C" int64_t nx_lz4_frame_encoder_close(nx_lz4_frame_encoder* e, uint8_t* out, size_t out_cap) {
    const nx::NoGrowScope no_grow;
    if (!e) return NX_ERR_INVALID_ARG;
    if (e->finished) return 0;  // finishEncode :306-310
    const int64_t w = lz4_flush_buffer(e, out, out_cap);  // the footer buffer: no maxEncodeSize check (:313-315)
    if (w < 0) return w;
    if ((size_t)w + kLz4Header > out_cap) return NX_ERR_INVALID_ARG;
    uint8_t* f = out + w;  // the end block :326-335
    memcpy(f, kLz4Magic, 8);
    f[8] = (uint8_t)(0x10 | e->level);
    memset(f + 9, 0, 12);
    e->finished = true;
    return w + kLz4Header;
}

extern "C" nx_lz4_frame_decoder* nx_lz4_frame_decoder_new(int32_t validate_checksums) {
    auto* d = new nx_lz4_frame_decoder();
    if (!d->g.hold(nx::WsKind::DecRecords)) {
        delete d;
        return nullptr;
    }
    d->validate = validate_checksums != 0;
    return d;
}
extern "C" void nx_lz4_frame_decoder_free(nx_lz4_frame_decoder* d) { nx_alt_decoder_unref(d); }

extern "C" int32_t nx_lz4_frame_decoder_decode(nx_lz4_frame_decoder* d, const uint8_t* in, size_t n, size_t* consumed,
                                               const nx_msg** msgs, size_t* n_msgs, const char** err_msg) {
    const nx::NoGrowScope no_grow;
    if (!d || (!in && n) || !consumed || !msgs || !n_msgs) return NX_ERR_INVALID_ARG;
    MsgList& ml = d->ml;
    ml.clear();
    size_t rd = 0;
    auto finish = [&](int32_t r) {
        *consumed = rd;
        *msgs = ml.msgs.data();
        *n_msgs = ml.msgs.size();
        if (err_msg) *err_msg = ml.err.empty() ? nullptr : ml.err.c_str();
        return r;
    };
    if (d->corrupted || d->st.state >= 2) {  // FINISHED / CORRUPTED :250-254
        rd = n;
        return finish(NX_OK);
    }
    struct Blk : nx::af::Blk {
        int job = -1;
    };
    nx::af::Lz4State ns = d->st;
    std::vector<nx::af::Blk> walked;
    nx::af::WalkErr werr;
    const size_t p = nx::af::lz4_walk(in, n, ns, walked, werr);
    std::vector<Blk> blks(walked.size());
    for (size_t i = 0; i < walked.size(); ++i) static_cast<nx::af::Blk&>(blks[i]) = walked[i];
    // GPU: decode the compressed blocks; hash every block's bytes when validating
    uint32_t nz = 0;
    uint64_t ocap = 0;
    std::vector<uint64_t> ooff;
    for (auto& b : blks)
        if (b.type == 0x20u) {
            b.job = (int)nz++;
            ooff.push_back(ocap);
            ocap += ((uint64_t)b.olen + 15) & ~15ull;
        }
    const uint32_t nb = (uint32_t)blks.size();
    std::vector<int32_t> st(nz);
    std::vector<uint32_t> hz(nz), hr(nb);
    std::vector<uint8_t> hout(ocap);
    Gpu& g = d->g;
    if (nb) {
        const size_t lo = blks.front().data, span = blks.back().end - lo;
        std::vector<uint64_t> ioff(nz), roff(nb);
        std::vector<uint32_t> ilen(nz), olen(nz), rlen(nb);
        for (uint32_t k = 0; k < nb; ++k) {
            const Blk& b = blks[k];
            roff[k] = b.data - lo;
            rlen[k] = b.type == 0x10u ? b.clen : 0u;
            if (b.job >= 0) {
                ioff[b.job] = b.data - lo;
                ilen[b.job] = b.clen;
                olen[b.job] = b.olen;
            }
        }
        if (!g.din.ensure(span + 1) || !g.dout.ensure(ocap + 16) || !g.a0.ensure(8ull * nb) || !g.a1.ensure(8ull * nb) ||
            !g.a2.ensure(4ull * nb) || !g.a3.ensure(4ull * nb) || !g.a4.ensure(4ull * nb) || !g.a5.ensure(4ull * nb) ||
            !g.a6.ensure(4ull * nb))
            return finish(NX_ERR_HIP);
        bool ok = g.h2d(g.din.p, in + lo, span);
        if (nz)
            ok = ok && g.h2d(g.a0.p, ioff.data(), 8ull * nz) && g.h2d(g.a1.p, ooff.data(), 8ull * nz) &&
                 g.h2d(g.a2.p, ilen.data(), 4ull * nz) && g.h2d(g.a3.p, olen.data(), 4ull * nz);
        if (!ok) return finish(NX_ERR_HIP);
        if (nz) {
            int32_t r = nx_lz4_decode_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), g.dout.as<uint8_t>(),
                                            g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), g.a4.as<int32_t>(), nz, g.s);
            if (r != NX_OK) return finish(r);
            if (d->validate) {
                r = nx_xxhash32_batch(g.dout.as<uint8_t>(), g.a1.as<uint64_t>(), g.a3.as<uint32_t>(), kLz4Seed, g.a5.as<uint32_t>(),
                                      nz, g.s);
                if (r != NX_OK) return finish(r);
                ok = g.d2h(hz.data(), g.a5.p, 4ull * nz);
            }
            ok = ok && g.d2h(st.data(), g.a4.p, 4ull * nz) && g.d2h(hout.data(), g.dout.p, ocap);
        }
        if (ok && d->validate) {  // non-compressed blocks are hashed where they lie (retainedSlice :197-199)
            ok = g.sync() && g.h2d(g.a0.p, roff.data(), 8ull * nb) && g.h2d(g.a2.p, rlen.data(), 4ull * nb);
            if (ok) {
                int32_t r = nx_xxhash32_batch(g.din.as<uint8_t>(), g.a0.as<uint64_t>(), g.a2.as<uint32_t>(), kLz4Seed,
                                              g.a6.as<uint32_t>(), nb, g.s);
                if (r != NX_OK) return finish(r);
                ok = g.d2h(hr.data(), g.a6.p, 4ull * nb);
            }
        }
        ok = ok && g.sync();
        if (!ok) return finish(NX_ERR_HIP);
    }
    for (uint32_t k = 0; k < nb; ++k) {
        const Blk& b = blks[k];
        const uint8_t* data;
        if (b.job >= 0) {
            if (st[b.job] != NX_OK) {  // LZ4Exception → DecompressionException (:240-241)
                ml.err = nx::af::lz4_block_error();
                d->st.state = 3;
                d->corrupted = true;
                rd = b.data;
                return finish(st[b.job]);
            }
            data = hout.data() + ooff[b.job];
        } else {
            data = in + b.data;
        }
        if (d->validate) {  // CompressionUtil.checkChecksum (:226-228; Lz4XXHash32.getValue masks, :101)
            const uint32_t got = (b.job >= 0 ? hz[b.job] : hr[k]) & 0x0FFFFFFFu;
            if (got != b.cks) {
                ml.err = nx::af::lz4_checksum_error(got, b.cks);
                d->st.state = 3;
                d->corrupted = true;
                rd = b.end;
                return finish(NX_ERR_LZ4_CHECKSUM_MISMATCH);
            }
        }
        if (b.job >= 0) {
            ml.owned.emplace_back(data, data + b.olen);
            ml.msgs.push_back({ml.owned.back().data(), b.olen});
        } else {
            ml.msgs.push_back({in + b.data, b.olen});
        }
        rd = b.end;
    }
    if (werr.set) {
        ml.err = werr.msg;
        d->st.state = 3;
        d->corrupted = true;
        rd = werr.at;
        return finish(werr.code);
    }
    rd = p;
    d->st = ns;
    return finish(NX_OK);
}
