// workspace.hpp — the device workspaces of the batch kernels (the encoders' per-lane hash tables,
// the decoder's per-frame record slots): one per device and kind, shared by every stream.
//
// Launches that use a workspace are ordered on the device: a batch waits (hipStreamWaitEvent) for
// the event the previous batch recorded after its launches, so the host never blocks and any number
// of streams (the batcher's four, every handle's own) share one allocation.  The decoder's record
// slots are leased by PART (WsLease::acquire_part): a batch of m frames takes the next m slots of a
// ring over the workspace and waits only for the earlier batches whose slots it reuses, so the
// parse / expand of batches on different streams overlap (round 4: with one lease for the whole
// workspace, a batcher's auto-flushed batches ran their decodes strictly one after another).  A workspace grows only
// where growth is allowed: in the standalone batch entry points (nx_*_batch called directly) and at
// set-up (nx_snappy_encoder_reserve, nx_batcher_new and the handle constructors, which hold it).
// Batches submitted by a batcher or a handle run inside a NoGrowScope: they use the slots the owner
// reserved and cap their grid to them, so a flush never allocates, frees or probes.  The last owner
// to let go frees it unless the standalone API grew it (then nx_workspaces_trim does).
#pragma once
#include <mutex>
#include <vector>
#include "nx_common.hpp"

namespace nx {

enum class WsKind : int { SnappyEnc = 0, Lz4Enc, FastLzEnc, LzfEnc, DecRecords, Lz4HcEnc, Count };

// Table geometry per encoder kind (entry bytes, log2 entries per table, waves per CU of its launch);
// each codec static_asserts its own constants against this.
struct WsSpec {
    uint32_t entry_bytes;
    uint32_t lg;
    unsigned waves_per_cu;
};
// SnappyEnc: 20 waves per CU (5 blocks of 256, 327 680 lanes on 256 CUs: 40 GiB of tables; round 6).
// Lz4HcEnc: 2^15 x 8 bytes = liblz4's HC tables per lane (u32 hashTable[2^15] + u16 chainTable[2^16]),
// 2 waves per CU, always one block per wave (kHcMaxSlots: at most cus * 2 tables, 128 MiB on 256 CUs).
#ifndef NX_LZ4_WPCU  // build options for A/B runs of the alt encoders' occupancy (scripts/build_lib_variant.sh; LZ4 at 20: level)
#define NX_LZ4_WPCU 16
#endif
#ifndef NX_FLZ_WPCU  // FastLZ: 16 waves per CU since round 6 (profiles/r06/s4: 310 vs 351-360 ms per 262 144 chunks)
#define NX_FLZ_WPCU 16
#endif
#ifndef NX_LZF_WPCU  // LZF: 16 waves per CU measured level with 8 (profiles/r06/s4), so the smaller workspace stays
#define NX_LZF_WPCU 8
#endif
constexpr WsSpec kWsSpec[] = {{8, 14, 20}, {8, 13, NX_LZ4_WPCU}, {8, 13, NX_FLZ_WPCU}, {8, 14, NX_LZF_WPCU}, {0, 0, 0}, {8, 15, 2}};
constexpr size_t kDecSlotBytes = 16384u * 4u + 8u;  // records of one frame + its count and length
#ifndef NX_DEC_MAX_FRAMES  // build option for A/B runs (scripts/build_lib_variant.sh)
#define NX_DEC_MAX_FRAMES 262144
#endif
constexpr uint32_t kDecMaxFrames = NX_DEC_MAX_FRAMES;  // frames per parse/expand launch pair

struct WsUse {  // an in-flight part lease: slots [a, b), done when ev completes
    size_t a, b;
    hipEvent_t ev;
    hipStream_t st;  // the stream ev was recorded on (ws_forget_stream)
};
struct SharedWs {
    std::mutex mu;
    std::vector<WsUse> uses;        // part leases not yet known to be complete
    std::vector<hipEvent_t> spare;  // their recycled events
    size_t cursor = 0;              // next part lease starts here (wraps to 0)
    void* p = nullptr;
    size_t slots = 0;    // tables (lanes or waves) or frames
    uint32_t stamp = 0;  // encoders: last stamp used
    hipEvent_t ev = nullptr;
    hipStream_t ev_st = nullptr;  // the stream ev was last recorded on
    bool used = false;   // ev has been recorded
    int owners = 0;      // batchers and handles holding it
    bool kept = false;   // grown by the standalone API or a reserve: kept until nx_workspaces_trim
    size_t cap = 0;      // most slots it may ever grow to (nx_snappy_encoder_reserve_ex; 0: no cap)
    PlacementReport place;
};
// the slots a grow to `want` may take under W's cap
inline size_t ws_capped(const SharedWs& W, size_t want) { return W.cap && want > W.cap ? W.cap : want; }

SharedWs& shared_ws(WsKind k, int dev);
// slots a batch of n units asks for: the encoders' lane_grid slots, the decoder's frames per launch
size_t ws_want(WsKind k, uint32_t n, int cus);
// The lane-per-chunk grid for n chunks over at most `have` table slots: the dense form while it has
// at least kSpreadMaxChunks lanes (a dense wave does the work of ~16 spread waves), else one chunk
// per wave on up to cus * waves_per_cu waves.
LaneGrid ws_grid(WsKind k, uint32_t n, int cus, size_t have);

struct NoGrowScope {
    NoGrowScope();
    ~NoGrowScope();
    bool prev;
};
bool ws_no_grow();

// One batch's use of a workspace: holds its lock from acquire() to destruction.
class WsLease {
  public:
    WsLease(WsKind k, int dev, hipStream_t st);
    ~WsLease();
    // Grow to `want` slots when growth is allowed (blocking, set-up only), allocate if there is no
    // workspace yet, then order the stream after the previous user's launches.
    hipError_t acquire(size_t want);
    // The same for min(want, slots) slots [*first, *first + *count) of the ring: the stream waits for
    // the last whole-workspace user and for the part leases that overlap them.
    hipError_t acquire_part(size_t want, size_t* first, size_t* count);
    SharedWs& ws() { return W_; }

  private:
    WsKind k_;
    SharedWs& W_;
    std::unique_lock<std::mutex> lk_;
    hipStream_t st_;
    bool acquired_ = false;
    bool part_ = false;
    size_t a_ = 0, b_ = 0;
};

// Owners: hold at creation (grows to `units` now), unhold at destruction (the last one frees).
int32_t ws_hold(WsKind k, int dev, uint32_t units, hipStream_t st);
void ws_unhold(WsKind k, int dev);
// A stream the library created is about to be destroyed, and its work is complete (the caller has
// synchronized it): forget the workspace events recorded on it, so that no later wait or drop
// touches an event whose stream no longer exists (the HIP runtime looks at that stream's capture
// state in hipEventSynchronize / hipStreamWaitEvent).
void ws_forget_stream(hipStream_t st);

// Owner sizes: a handle encodes a message of up to 1024 slices without waiting on another slot; a
// batcher flush of up to 16384 slices / frames runs at full grid.
constexpr uint32_t kHandleHoldUnits = 1024;
constexpr uint32_t kBatcherHoldUnits = 16384;
// A batcher's reservations.  Snappy tables in the DENSE form for 65 536 lanes (8 GiB): a flush of more
// than kSpreadMaxChunks slices runs lane-per-chunk on 256 blocks, one per CU (the table request rate
// saturates from ~32 K lanes; 16 640 lanes were only 65 blocks, and a reservation below
// kSpreadMaxChunks lanes runs one chunk per wave on 4 096 waves).  Records for 65 536 frames (4 GiB), so
// k_parse's lane-per-frame launch of a sub-batch fills every CU as well.
constexpr uint32_t kBatcherEncHoldUnits = 65536;
constexpr uint32_t kBatcherDecHoldUnits = 65536;

}  // namespace nx
