// handles.hpp — device context and the Snappy handler handles shared by the synchronous handler layer
// (handlers.cpp) and the asynchronous cross-channel batcher (batcher.cpp).  Private to the library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <set>
#include <string>
#include <vector>
#include "../../include/netty_amd.h"
#include "nx_common.hpp"
#include "workspace.hpp"

namespace nx {
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
        if (s) (void)hipStreamDestroy(s);
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
    std::vector<uint8_t> hist;         // stream bytes [hist_base, hist_base + hist.size())
    uint64_t hist_base = 0;
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
