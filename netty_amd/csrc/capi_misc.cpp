// capi_misc.cpp — library-level C-ABI entry points (version, status strings, sizing, device helpers).
#include <hip/hip_runtime.h>
#include "../../include/netty_amd.h"

extern "C" const char* nx_version(void) { return "netty_amd 0.1.0 (gfx950)"; }

extern "C" const char* nx_status_string(int32_t s) {
    switch (s) {
        case NX_OK: return "ok";
        case NX_ERR_LZ4_BAD_MAGIC: return "unexpected block identifier";
        case NX_ERR_LZ4_COMPRESSED_LENGTH: return "invalid compressedLength";
        case NX_ERR_LZ4_DECOMPRESSED_LENGTH: return "invalid decompressedLength";
        case NX_ERR_LZ4_LENGTH_MISMATCH: return "stream corrupted: compressedLength and decompressedLength mismatch";
        case NX_ERR_LZ4_BLOCK_TYPE: return "unexpected blockType";
        case NX_ERR_LZ4_CHECKSUM_MISMATCH: return "stream corrupted: mismatching checksum";
        case NX_ERR_LZ4_END_CHECKSUM: return "stream corrupted: checksum error";
        case NX_ERR_LZ4_ENCODE_SIZE: return "requested encode buffer size exceeds the maximum allowable size";
        case NX_ERR_LZ4_ENCODE_FINISHED: return "encode finished and not enough space to write remaining data";
        case NX_ERR_SNAPPY_PREAMBLE_TOO_LONG: return "Preamble is greater than 4 bytes";
        case NX_ERR_SNAPPY_OFFSET_ZERO: return "Offset is less than minimum permissible value";
        case NX_ERR_SNAPPY_OFFSET_NEGATIVE: return "Offset is greater than maximum value supported by this implementation";
        case NX_ERR_SNAPPY_OFFSET_BEYOND: return "Offset exceeds size of chunk";
        case NX_ERR_SNAPPY_OUTPUT_OVERFLOW: return "decoded data exceeds the output buffer's maximum capacity";
        case NX_ERR_SNAPPY_LITERAL_LEN_INVALID: return "literal length is negative";
        case NX_ERR_SNAPPY_CRC_MISMATCH: return "mismatching checksum";
        case NX_ERR_FASTLZ_BAD_LEVEL: return "invalid level";
        case NX_ERR_FASTLZ_INPUT_OOB: return "compressed data references bytes past the readable input";
        case NX_ERR_FASTLZ_LENGTH_MISMATCH: return "stream corrupted: originalLength and actual length mismatch";
        case NX_ERR_FASTLZ_CRC_MISMATCH: return "stream corrupted: mismatching checksum";
        case NX_ERR_LZF_CORRUPT: return "Corrupt LZF data";
        case NX_ERR_FRAME_CORRUPT: return "corrupted frame";
        case NX_ERR_SNAPPY_STREAM_ID_LENGTH: return "Unexpected length of stream identifier";
        case NX_ERR_SNAPPY_STREAM_ID_CONTENT: return "Unexpected stream identifier contents. Mismatched snappy protocol version?";
        case NX_ERR_SNAPPY_COMPRESSED_BEFORE_ID: return "Received COMPRESSED_DATA tag before STREAM_IDENTIFIER";
        case NX_ERR_SNAPPY_UNCOMPRESSED_BEFORE_ID: return "Received UNCOMPRESSED_DATA tag before STREAM_IDENTIFIER";
        case NX_ERR_SNAPPY_SKIPPABLE_BEFORE_ID: return "Received RESERVED_SKIPPABLE tag before STREAM_IDENTIFIER";
        case NX_ERR_SNAPPY_UNCOMPRESSED_TOO_LARGE: return "Received UNCOMPRESSED_DATA larger than 65540 bytes";
        case NX_ERR_SNAPPY_DECOMPRESSED_TOO_LARGE: return "Received COMPRESSED_DATA that contains uncompressed data that exceeds 65536 bytes";
        case NX_ERR_SNAPPY_CHUNK_TOO_SHORT:  // not a DecompressionException: ByteBuf fails (SnappyFrameDecoder.java:171-215)
            return "java.lang.IllegalArgumentException: data chunk shorter than its 4-byte checksum (ByteBuf read past the chunk)";
        case NX_ERR_SNAPPY_UNSKIPPABLE: return "Found reserved unskippable chunk type";
        case NX_ERR_LZ4_MALFORMED: return "Malformed LZ4 input";
        case NX_SCAN_LIST_FULL: return "chunk list full (call again from consumed)";
        case NX_ERR_INVALID_ARG: return "invalid argument";
        case NX_ERR_HIP: return "HIP runtime error";
        case NX_ERR_NO_DEVICE: return "no GPU device";
        case NX_ERR_INTERNAL: return "kernel loop guard tripped (internal error)";
        default: return "unknown status";
    }
}

extern "C" int32_t nx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" size_t nx_snappy_max_compressed_length(size_t n) { return 32 + n + n / 6; }
extern "C" size_t nx_fastlz_max_compressed_length(size_t n) {
    size_t a = (size_t)((double)n * 1.06);  // FastLz.calculateOutputBufferLength (FastLz.java:84-87)
    if (a < 66) a = 66;
    return a + 16;
}
extern "C" size_t nx_lzf_max_compressed_length(size_t n) { return n + n / 32 + 16; }

extern "C" void* nx_device_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
    return p;
}
extern "C" int32_t nx_device_free(void* p) { return hipFree(p) == hipSuccess ? NX_OK : NX_ERR_HIP; }
extern "C" int32_t nx_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream) == hipSuccess ? NX_OK : NX_ERR_HIP;
}
extern "C" int32_t nx_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream) == hipSuccess ? NX_OK : NX_ERR_HIP;
}
extern "C" int32_t nx_stream_sync(void* stream) {
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? NX_OK : NX_ERR_HIP;
}

// Diagnostics only: with NX_SEGV_TRACE set when the library loads, a segmentation fault prints the
// native call stack (addresses resolve with addr2line against this library) before the previous
// handler (Python's faulthandler under pytest) runs.
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
namespace {
struct sigaction g_prev_segv;
void nx_segv_trace(int sig, siginfo_t* si, void* ctx) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char hdr[] = "netty_amd: SIGSEGV, native stack:\n";
    (void)!write(2, hdr, sizeof hdr - 1);
    backtrace_symbols_fd(frames, n, 2);
    sigaction(SIGSEGV, &g_prev_segv, nullptr);
    if (g_prev_segv.sa_flags & SA_SIGINFO) {
        if (g_prev_segv.sa_sigaction) g_prev_segv.sa_sigaction(sig, si, ctx);
    } else if (g_prev_segv.sa_handler != SIG_DFL && g_prev_segv.sa_handler != SIG_IGN) {
        g_prev_segv.sa_handler(sig);
    }
    raise(sig);
}
struct SegvTraceInit {
    SegvTraceInit() {
        if (!getenv("NX_SEGV_TRACE")) return;
        struct sigaction sa;
        memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = nx_segv_trace;
        sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigaction(SIGSEGV, &sa, &g_prev_segv);
    }
} g_segv_trace_init;
}  // namespace
