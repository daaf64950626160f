// handles.hpp — device context and the Snappy handler handles shared by the synchronous handler layer
// (handlers.cpp) and the asynchronous cross-channel batcher (batcher.cpp).  Private to the library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <atomic>
#include <deque>
#include <set>
#include <string>
#include <vector>
#include "../../include/netty_amd.h"
#include "nx_common.hpp"
#include "workspace.hpp"

namespace nx {

// memcpy of n bytes that may be zero with a null source (an empty message or cumulation: memcpy's
// arguments must be valid pointers even for n = 0; found by the UBSan run, profiles/r05/s35)
inline void copy_bytes(void* dst, const void* src, size_t n) {
    if (n) memcpy(dst, src, n);
}

namespace h {

// ------------------------------------------------------------------ device context
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n) {
        if (n <= cap) return true;
        size_t c = cap ? cap : 4096;
        while (c < n) c += c / 2 + 4096;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, c) != hipSuccess) return false;
        cap = c;
        return true;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

struct Gpu {
    hipStream_t s = nullptr;
    int dev = 0;
    bool ok = false;
    uint32_t held = 0;  // bit per WsKind whose shared workspace this handle holds (workspace.hpp)
    DevBuf din, dout, a0, a1, a2, a3, a4, a5, a6;
    Gpu() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return;
        if (hipGetDevice(&dev) != hipSuccess) return;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
        ok = nx::crc_tables_init() == NX_OK;
    }
    // Reserve the device workspace of kind k for this handle's launches, at construction (its
    // encode/decode calls then never allocate: they run in a NoGrowScope).
    bool hold(WsKind k) {
        if (!ok || ws_hold(k, dev, kHandleHoldUnits, s) != NX_OK) return false;
        held |= 1u << (int)k;
        return true;
    }
    ~Gpu() {
        if (s) (void)hipStreamSynchronize(s);
        for (int k = 0; k < (int)WsKind::Count; ++k)
            if (held & (1u << k)) ws_unhold((WsKind)k, dev);
        if (s) {
            ws_forget_stream(s);
            (void)hipStreamDestroy(s);
        }
    }
    bool h2d(void* d, const void* h, size_t n) { return n == 0 || hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s) == hipSuccess; }
    bool d2h(void* h, const void* d, size_t n) { return n == 0 || hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s) == hipSuccess; }
    bool sync() { return hipStreamSynchronize(s) == hipSuccess; }
};

struct MsgList {
    std::vector<nx_msg> msgs;
    std::vector<std::vector<uint8_t>> owned;  // decoded payloads (stable storage)
    std::string err;
    void clear() {
        msgs.clear();
        owned.clear();
        err.clear();
    }
};

inline constexpr uint8_t kStreamStart[10] = {0xff, 0x06, 0x00, 0x00, 0x73, 0x4e, 0x61, 0x50, 0x70, 0x59};

// A validating batcher decoder's handed-over stream bytes, as segments in stream order: a reference to
// a registered cumulation or to the job's copy in its batch's staging arena (both valid while the job
// that consumed them is unapplied, which is as long as a re-walk can need them; a staging arena may
// be reallocated while its batch collects, so that reference is the arena's pointer + offset), or an
// owned copy.
struct StreamHist {
    struct Seg {
        uint64_t pos;
        const uint8_t* p;
        size_t n;
        std::vector<uint8_t> own;
        uint8_t* const* base = nullptr;  // staging reference: bytes at *base + off
        uint64_t off = 0;
        const uint8_t* data() const { return base ? *base + off : p; }
    };
    std::deque<Seg> segs;
    uint64_t end = 0;  // stream position after the last byte handed over
    void append(const uint8_t* p, size_t n, bool copy) {
        if (!n) return;
        Seg s{end, p, n, {}};
        if (copy) {
            s.own.assign(p, p + n);
            s.p = s.own.data();
        }
        segs.push_back(std::move(s));
        end += n;
    }
    void append_staged(uint8_t* const* base, uint64_t off, size_t n) {
        if (!n) return;
        Seg s{end, nullptr, n, {}, base, off};
        segs.push_back(std::move(s));
        end += n;
    }
    // [a, end) into `out` (appended)
    void copy_from(uint64_t a, std::vector<uint8_t>& out) const {
        for (const Seg& s : segs) {
            if (s.pos + s.n <= a) continue;
            const size_t o = a > s.pos ? (size_t)(a - s.pos) : 0;
            out.insert(out.end(), s.data() + o, s.data() + s.n);
        }
    }
    // Make [a, end) one owned, contiguous segment and return its bytes (a re-walk: what it leaves
    // carried outlives the jobs whose registered memory it was in).
    const uint8_t* own_from(uint64_t a) {
        std::vector<uint8_t> v;
        copy_from(a, v);
        while (!segs.empty() && segs.back().pos >= a) segs.pop_back();
        if (!segs.empty() && segs.back().pos + segs.back().n > a) {  // split the segment holding a
            Seg& s = segs.back();
            s.n = (size_t)(a - s.pos);
            if (!s.own.empty()) s.own.resize(s.n);  // (p stays valid: shrinking keeps the buffer)
        }
        Seg t{a, nullptr, v.size(), std::move(v)};
        t.p = t.own.data();
        segs.push_back(std::move(t));
        return segs.back().p;
    }
    // bytes at stream position a, contiguous to the end of its segment
    const uint8_t* at(uint64_t a) const {
        for (const Seg& s : segs)
            if (a >= s.pos && a < s.pos + s.n) return s.data() + (a - s.pos);
        return nullptr;
    }
    void drop_before(uint64_t a) {  // whole segments that end at or below a
        while (!segs.empty() && segs.front().pos + segs.front().n <= a) segs.pop_front();
    }
    void clear(uint64_t at_pos) {
        segs.clear();
        end = at_pos;
    }
};

}  // namespace h
}  // namespace nx

struct nx_snappy_frame_encoder {
    nx::h::Gpu g;
    bool started = false;
    int32_t slice;
};

struct nx_snappy_frame_decoder {
    nx::h::Gpu g;
    bool validate;
    bool started = false;
    bool corrupted = false;
    bool parse_failed = false;  // batcher: a submitted input failed its header walk (applied later, in order)
    uint64_t skip = 0;  // numBytesToSkip
    nx::h::MsgList ml;
    // Batcher, validating decoders only.  A compressed chunk that decodes fewer bytes than its length
    // leaves the rest to be parsed again as the next chunk header (SnappyFrameDecoder.java:206-212),
    // which is only known once the chunk is decoded.  So the handed-over byte stream is kept from the
    // first byte a not-yet-applied job walked (absolute positions in the decoder's stream): a leftover
    // found at apply() re-walks it from there.
    nx::h::StreamHist hist;            // stream bytes from the first an unapplied job walked to hist.end
    uint64_t parse_pos = 0;            // the header walk has reached here; [parse_pos, end) is carried into the next submit
    uint64_t epoch = 0;                // bumped by each re-walk: jobs walked under an older epoch deliver nothing
    std::multiset<uint64_t> outstanding;  // walk starts of jobs submitted and not yet applied
    // the owner's reference plus one per batcher job: nx_snappy_frame_decoder_free drops the owner's,
    // and the handle is deleted when the last job referring to it is deleted (a handler removed while
    // its jobs are in flight)
    std::atomic<int> refs{1};
};

inline void nx_decoder_unref(nx_snappy_frame_decoder* d) {
    if (d && d->refs.fetch_sub(1) == 1) delete d;
}
