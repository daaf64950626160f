// workspace.hip — storage, growth and ownership of the shared device workspaces (workspace.hpp).
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include "workspace.hpp"

namespace nx {
namespace {
constexpr int kMaxDevices = 64;
SharedWs g_ws[(int)WsKind::Count][kMaxDevices];
thread_local bool t_no_grow = false;

// Free W (waits for its last use first: nothing may still read or write it).
hipError_t ws_drop(SharedWs& W) {
    hipError_t e = hipSuccess;
    static const bool dbg = getenv("NX_HIP_DEBUG") != nullptr;
    for (const WsUse& u : W.uses) {
        const hipError_t f = hipEventSynchronize(u.ev);
        if (f != hipSuccess && dbg) fprintf(stderr, "netty_amd: ws_drop: part-use event sync: %s\n", hipGetErrorString(f));
        if (e == hipSuccess) e = f;
        W.spare.push_back(u.ev);
    }
    W.uses.clear();
    W.cursor = 0;
    if (W.p) {
        const hipError_t f = W.used ? hipEventSynchronize(W.ev) : hipSuccess;
        if (f != hipSuccess && dbg) fprintf(stderr, "netty_amd: ws_drop: last-use event sync: %s\n", hipGetErrorString(f));
        if (e == hipSuccess) e = f;
        const hipError_t g = hipFree(W.p);
        if (g != hipSuccess && dbg) fprintf(stderr, "netty_amd: ws_drop: hipFree(%p): %s\n", W.p, hipGetErrorString(g));
        if (e == hipSuccess) e = g;
    }
    W.p = nullptr;
    W.slots = 0;
    W.stamp = 0;
    W.used = false;
    return e;
}

hipError_t ws_mark(SharedWs& W, hipStream_t st) {
    if (!W.ev) {
        const hipError_t e = hipEventCreateWithFlags(&W.ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    W.used = true;
    W.ev_st = st;
    return hipEventRecord(W.ev, st);
}

// Reallocate W with at least `slots` slots (caller holds W.mu).  Blocking: set-up only.
hipError_t ws_grow(WsKind k, SharedWs& W, size_t slots, hipStream_t st) {
    if (W.p && W.slots >= slots) return hipSuccess;
    hipError_t e = ws_drop(W);
    if (e != hipSuccess) return e;
    void* p = nullptr;
    if (k == WsKind::DecRecords) {
        e = hipMalloc(&p, slots * kDecSlotBytes);  // records are written before they are read: no zeroing
    } else {
        const WsSpec& s = kWsSpec[(int)k];
        if (s.entry_bytes == 8) {
            uint64_t* q = nullptr;
            e = alloc_placed_workspace<uint64_t>(slots, s.lg, st, &q, &W.place);
            p = q;
        } else {
            uint32_t* q = nullptr;
            e = alloc_placed_workspace<uint32_t>(slots, s.lg, st, &q, &W.place);
            p = q;
        }
    }
    if (e != hipSuccess) return e;
    W.p = p;
    W.slots = slots;
    W.stamp = 0;
    return ws_mark(W, st);  // users on other streams wait for the zeroing
}
}  // namespace

SharedWs& shared_ws(WsKind k, int dev) { return g_ws[(int)k][dev < 0 || dev >= kMaxDevices ? 0 : dev]; }

// LZ4 HC: always one block per wave on at most cus * waves_per_cu waves (128 MiB of
// tables on 256 CUs).  Its dense form would hold 32 768 lanes x 256 KiB = 8 GiB (and draw placement
// candidates of that size) for a compatibility path whose 256-candidate chains run no faster dense.
size_t hc_slots(uint32_t n, int cus) { return std::min<size_t>(n, (size_t)cus * kWsSpec[(int)WsKind::Lz4HcEnc].waves_per_cu); }

size_t ws_want(WsKind k, uint32_t n, int cus) {
    if (k == WsKind::DecRecords) return std::min<uint32_t>(n, kDecMaxFrames);
    if (k == WsKind::Lz4HcEnc) return hc_slots(n, cus);
    return lane_grid(n, cus, kWsSpec[(int)k].waves_per_cu).slots;
}

LaneGrid ws_grid(WsKind k, uint32_t n, int cus, size_t have) {
    const unsigned wpcu = kWsSpec[(int)k].waves_per_cu;
    if (k == WsKind::Lz4HcEnc) {
        LaneGrid g;
        g.spread = true;
        g.block = 64;
        g.slots = std::max<size_t>(1, std::min(hc_slots(n, cus), have));
        g.grid = (unsigned)g.slots;
        return g;
    }
    LaneGrid g = lane_grid(n, cus, wpcu);
    if (g.slots <= have) return g;
    if (!g.spread && have >= kSpreadMaxChunks) {
        g.slots = have / 256 * 256;
        g.grid = (unsigned)(g.slots / 256);
        return g;
    }
    g.spread = true;
    g.block = 64;
    g.slots = std::min<size_t>(std::min<size_t>(have, (size_t)cus * wpcu), n);
    g.grid = (unsigned)g.slots;
    return g;
}

NoGrowScope::NoGrowScope() : prev(t_no_grow) { t_no_grow = true; }
NoGrowScope::~NoGrowScope() { t_no_grow = prev; }
bool ws_no_grow() { return t_no_grow; }

WsLease::WsLease(WsKind k, int dev, hipStream_t st) : k_(k), W_(shared_ws(k, dev)), lk_(W_.mu), st_(st) {}

WsLease::~WsLease() {
    if (!acquired_) return;
    if (part_) {  // the next users of slots [a_, b_) wait for this batch's launches
        hipEvent_t ev = nullptr;
        if (!W_.spare.empty()) {
            ev = W_.spare.back();
            W_.spare.pop_back();
        } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            ev = nullptr;
        }
        if (ev && hipEventRecord(ev, st_) == hipSuccess) {
            // uses inside [a_, b_) are covered: this stream waited for them before its launches
            size_t k = 0;
            for (const WsUse& u : W_.uses) {
                if (u.a >= a_ && u.b <= b_) W_.spare.push_back(u.ev);
                else W_.uses[k++] = u;
            }
            W_.uses.resize(k);
            W_.uses.push_back({a_, b_, ev, st_});
            return;
        }
        if (ev) W_.spare.push_back(ev);
        // no event: fall back to the whole-workspace mark below (every later user waits for it)
    } else {
        for (const WsUse& u : W_.uses) W_.spare.push_back(u.ev);  // this stream waited for all of them
        W_.uses.clear();
    }
    (void)ws_mark(W_, st_);
}

hipError_t WsLease::acquire(size_t want) {
    want = ws_capped(W_, want);
    if (!W_.p || (!t_no_grow && W_.slots < want)) {
        const hipError_t e = ws_grow(k_, W_, std::max(want, W_.slots), st_);
        if (e != hipSuccess) return e;
        W_.kept = true;
    }
    acquired_ = true;
    for (const WsUse& u : W_.uses) {
        const hipError_t e = hipStreamWaitEvent(st_, u.ev, 0);
        if (e != hipSuccess) return e;
    }
    return W_.used ? hipStreamWaitEvent(st_, W_.ev, 0) : hipSuccess;
}

hipError_t WsLease::acquire_part(size_t want, size_t* first, size_t* count) {
    want = ws_capped(W_, want);
    if (!W_.p || (!t_no_grow && W_.slots < want)) {
        const hipError_t e = ws_grow(k_, W_, std::max(want, W_.slots), st_);
        if (e != hipSuccess) return e;
        W_.kept = true;
    }
    const size_t n = std::max<size_t>(1, std::min(want, W_.slots));
    if (W_.cursor + n > W_.slots) W_.cursor = 0;
    a_ = W_.cursor;
    b_ = a_ + n;
    W_.cursor = b_ == W_.slots ? 0 : b_;
    acquired_ = true;
    part_ = true;
    *first = a_;
    *count = n;
    if (W_.uses.size() > 32) {  // forget the completed ones
        size_t k = 0;
        for (const WsUse& u : W_.uses) {
            if (hipEventQuery(u.ev) == hipSuccess) W_.spare.push_back(u.ev);
            else W_.uses[k++] = u;
        }
        (void)hipGetLastError();  // hipErrorNotReady is kept as the thread's last error: a launch check would see it
        W_.uses.resize(k);
    }
    for (const WsUse& u : W_.uses) {
        if (u.b <= a_ || u.a >= b_) continue;
        const hipError_t e = hipStreamWaitEvent(st_, u.ev, 0);
        if (e != hipSuccess) return e;
    }
    return W_.used ? hipStreamWaitEvent(st_, W_.ev, 0) : hipSuccess;
}

void ws_forget_stream(hipStream_t st) {
    if (!st) return;
    for (int k = 0; k < (int)WsKind::Count; ++k)
        for (int d = 0; d < kMaxDevices; ++d) {
            SharedWs& W = g_ws[k][d];
            std::lock_guard<std::mutex> lk(W.mu);
            size_t j = 0;
            for (const WsUse& u : W.uses) {
                if (u.st == st) W.spare.push_back(u.ev);
                else W.uses[j++] = u;
            }
            W.uses.resize(j);
            if (W.used && W.ev_st == st) {
                W.used = false;  // its work is complete: nothing later needs to wait for it
                W.ev_st = nullptr;
            }
        }
}

int32_t ws_hold(WsKind k, int dev, uint32_t units, hipStream_t st) {
    int cus = 256;
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    SharedWs& W = shared_ws(k, dev);
    std::lock_guard<std::mutex> lk(W.mu);
    NX_HIP_CHECK(ws_grow(k, W, std::max(ws_capped(W, ws_want(k, units, cus)), W.slots), st));
    W.owners += 1;
    return NX_OK;
}

void ws_unhold(WsKind k, int dev) {
    SharedWs& W = shared_ws(k, dev);
    std::lock_guard<std::mutex> lk(W.mu);
    if (W.owners > 0) W.owners -= 1;
    if (W.owners == 0 && !W.kept) (void)ws_drop(W);
}

}  // namespace nx

// Free, on the current device, every workspace no batcher or handle holds (those grown by the
// standalone batch API or nx_snappy_encoder_reserve included); held ones stay, and are freed when
// their last owner is.  Blocks until their last launches complete.
extern "C" int32_t nx_workspaces_trim(void) {
    int dev = 0;
    NX_HIP_CHECK(hipGetDevice(&dev));
    int32_t r = NX_OK;
    for (int k = 0; k < (int)nx::WsKind::Count; ++k) {
        nx::SharedWs& W = nx::shared_ws((nx::WsKind)k, dev);
        std::lock_guard<std::mutex> lk(W.mu);
        W.kept = false;
        if (W.owners == 0) {
            W.cap = 0;  // a reserve's cap lasts until its workspace is freed
            const hipError_t e = nx::ws_drop(W);
            if (e != hipSuccess) r = nx_hip_fail(e, __FILE__, __LINE__ + k * 1000);  // line + 1000 * kind under NX_HIP_DEBUG
        }
    }
    return r;
}

// Before a caller destroys a stream it passed to batch calls (netty_amd.h): wait for it, then drop
// the workspace events recorded on it.
extern "C" int32_t nx_workspaces_forget_stream(void* stream) {
    if (!stream) return NX_OK;  // the null stream is never destroyed
    NX_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    nx::ws_forget_stream((hipStream_t)stream);
    return NX_OK;
}

// Bytes of the workspace of `kind` (NX_WS_* in netty_amd.h) on the current device and its owners.
extern "C" int32_t nx_workspace_info(int32_t kind, uint64_t* bytes, int32_t* owners) {
    if (kind < 0 || kind >= (int32_t)nx::WsKind::Count || !bytes || !owners) return NX_ERR_INVALID_ARG;
    int dev = 0;
    NX_HIP_CHECK(hipGetDevice(&dev));
    nx::SharedWs& W = nx::shared_ws((nx::WsKind)kind, dev);
    std::lock_guard<std::mutex> lk(W.mu);
    const nx::WsSpec& s = nx::kWsSpec[kind];
    *bytes = kind == (int32_t)nx::WsKind::DecRecords ? W.slots * nx::kDecSlotBytes : W.slots * ((size_t)s.entry_bytes << s.lg);
    *owners = W.owners;
    return NX_OK;
}

// The placement bound of every later large workspace (nx_common.hpp placement_peak_cap /
// placement_max_candidates): peak_bytes = the bytes the candidates of one workspace may hold at once
// (0: half of the device's memory, the default; UINT64_MAX: all but 8 GiB of free memory), and
// max_candidates = the candidates drawn in all (0: the default 24; 1: no placement choice).
extern "C" int32_t nx_workspace_placement_config(uint64_t peak_bytes, int32_t max_candidates) {
    if (max_candidates < 0) return NX_ERR_INVALID_ARG;
    nx::placement_peak_cap() = peak_bytes;
    nx::placement_max_candidates() = max_candidates;
    return NX_OK;
}
