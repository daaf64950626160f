// records.hpp — the record expander (snappy_decode.hip: k_expand) as a service for the other LZ77
// decoders.  A codec's parse kernel walks a block per lane and emits k_expand's 32-bit records
// (bit 31 copy | bits 30..25 length-1 | bits 24..0 input position or copy distance); k_expand writes
// the bytes a wave per block.  The parse only takes blocks that decode cleanly with every read inside
// the block; any other block (an error, a read past in_len, more records than a slot holds) is left
// with status kNeedSerial and the codec's lane-serial kernel decodes it, so results and statuses stay
// exactly the serial decoder's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nx {
namespace dec {

constexpr int32_t kNeedSerial = -1000;  // = k_parse's kNeedFused: the block goes to the lane-serial path

enum class RecCodec { FastLz, Lzf };

// Called once per sub-batch [base, base + m) after its expand launch, on the same stream: launches
// the codec's finish kernel (its lane-serial decoder for status kNeedSerial blocks, the result fix-up
// for the others).  olen[i] = bytes the parse produced for block base + i.
using RecAfter = hipError_t (*)(uint32_t base, uint32_t m, const uint32_t* olen, void* ctx, hipStream_t st);

// Parse + expand of n blocks: block i = in[in_off[i] .. + in_len[i]), at most lim[i] output bytes
// (FastLZ: outLength; LZF: exactly lim[i]) to out + out_off[i]; avail (FastLZ, nullable): readable
// bytes from the block start.  status[i] is the parse/expand status (NX_OK or kNeedSerial) when
// `after` runs.
int32_t decode_records(RecCodec codec, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* avail,
                       const uint32_t* lim,
                       uint8_t* out, const uint64_t* out_off, int32_t* status, uint32_t n, hipStream_t st, RecAfter after,
                       void* ctx);

}  // namespace dec
}  // namespace nx
