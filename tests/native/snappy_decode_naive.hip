// snappy_decode_naive.hip — thread-per-chunk Snappy decoder (reference-structured baseline).
//
// Executes Snappy.decode's state machine (Snappy.java:315-650) once per complete chunk, as
// SnappyFrameDecoder drives it (SnappyFrameDecoder.java:194-224), one chunk per lane, output
// straight to HBM.  TEST-ONLY (tests/native/libnx_test_naive.so, not part of libnetty_amd.so): a
// second GPU implementation the product decoder (snappy_decode.hip) is cross-checked against, with
// nx_snappy_decode_batch's contract.
#include "../../netty_amd/csrc/nx_common.hpp"

namespace nx {

// Returns status; *olen/*cons as the oracle (oracle/netty_oracle.c orc_snappy_decode).
__device__ int32_t snappy_decode_serial(const uint8_t* __restrict__ in, uint32_t in_len, uint8_t* __restrict__ out,
                                        uint32_t out_cap, uint32_t* olen, uint32_t* cons) {
    uint32_t ip = 0, op = 0;
    *olen = 0;
    *cons = 0;
    if (in_len == 0) return NX_OK;
    uint32_t ulen = 0;
    {
        int byteIndex = 0;
        bool complete = false;
        while (ip < in_len) {
            uint32_t cur = in[ip++];
            ulen |= (cur & 0x7f) << (byteIndex++ * 7);
            if ((cur & 0x80) == 0) { complete = true; break; }
            if (byteIndex >= 4) { *cons = ip; return NX_ERR_SNAPPY_PREAMBLE_TOO_LONG; }
        }
        if (!complete || ulen == 0) { *cons = ip; return NX_OK; }
        if (ulen > out_cap) { *cons = ip; return NX_ERR_SNAPPY_OUTPUT_OVERFLOW; }
    }
    int32_t st = NX_OK;
    while (ip < in_len) {
        uint32_t tag = in[ip++];
        uint32_t after_tag = ip;
        uint32_t type = tag & 3u;
        if (type == 0) {
            uint32_t code = tag >> 2;
            int64_t length;
            if (code < 60) {
                length = code;
            } else {
                uint32_t nb = code - 59;
                if (in_len - ip < nb) { ip = after_tag; break; }
                uint32_t v = 0;
                for (uint32_t k = 0; k < nb; ++k) v |= (uint32_t)in[ip + k] << (8 * k);
                ip += nb;
                length = (nb == 4) ? (int64_t)(int32_t)v : (int64_t)v;
            }
            int32_t jlen = (int32_t)((uint32_t)length + 1u);
            if (jlen >= 0 && in_len - ip < (uint32_t)jlen) { ip = after_tag; break; }
            if (jlen < 0) { st = NX_ERR_SNAPPY_LITERAL_LEN_INVALID; break; }
            if ((uint64_t)op + (uint32_t)jlen > out_cap) { st = NX_ERR_SNAPPY_OUTPUT_OVERFLOW; break; }
            for (int32_t k = 0; k < jlen; ++k) out[op + k] = in[ip + k];
            ip += jlen;
            op += jlen;
        } else {
            int64_t length, offset;
            if (type == 1) {
                if (in_len - ip < 1) break;
                length = 4 + ((tag & 0x1c) >> 2);
                offset = ((int64_t)(tag & 0xe0) << 3) | in[ip];
                ip += 1;
            } else if (type == 2) {
                if (in_len - ip < 2) break;
                length = 1 + (tag >> 2);
                offset = (int64_t)in[ip] | ((int64_t)in[ip + 1] << 8);
                ip += 2;
            } else {
                if (in_len - ip < 4) break;
                length = 1 + (tag >> 2);
                uint32_t v = (uint32_t)in[ip] | ((uint32_t)in[ip + 1] << 8) | ((uint32_t)in[ip + 2] << 16) |
                             ((uint32_t)in[ip + 3] << 24);
                offset = (int64_t)(int32_t)v;
                ip += 4;
            }
            if (offset == 0) { st = NX_ERR_SNAPPY_OFFSET_ZERO; break; }
            if (offset < 0) { st = NX_ERR_SNAPPY_OFFSET_NEGATIVE; break; }
            if ((uint64_t)offset > op) { st = NX_ERR_SNAPPY_OFFSET_BEYOND; break; }
            if ((uint64_t)op + (uint64_t)length > out_cap) { st = NX_ERR_SNAPPY_OUTPUT_OVERFLOW; break; }
            for (int64_t k = 0; k < length; ++k) out[op + k] = out[op + k - offset];
            op += (uint32_t)length;
        }
    }
    *olen = op;
    *cons = ip;
    return st;
}

__global__ void __launch_bounds__(256) k_snappy_decode_naive(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                             const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                                                             uint32_t* __restrict__ out_len, uint32_t* __restrict__ consumed,
                                                             int32_t* __restrict__ status, const uint32_t* __restrict__ expect,
                                                             uint32_t* __restrict__ crc_out, uint32_t n,
                                                             const CrcTables* __restrict__ tabs) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nthreads = gridDim.x * blockDim.x;
    for (uint32_t c = tid; c < n; c += nthreads) {
        uint32_t cap = out_cap ? out_cap[c] : 65536u;
        uint32_t olen, cons;
        uint8_t* o = out + out_off[c];
        int32_t st = snappy_decode_serial(in + in_off[c], in_len[c], o, cap, &olen, &cons);
        if (st == NX_OK && (expect || crc_out)) {
            uint32_t crc = 0xFFFFFFFFu;
            for (uint32_t i = 0; i < olen; ++i) crc = (crc >> 8) ^ tabs->T8[0][(crc ^ o[i]) & 0xFFu];
            uint32_t m = mask_checksum(~crc);
            if (crc_out) crc_out[c] = m;
            if (expect && m != expect[c]) st = NX_ERR_SNAPPY_CRC_MISMATCH;
        }
        out_len[c] = olen;
        if (consumed) consumed[c] = cons;
        status[c] = st;
    }
}

}  // namespace nx

extern "C" int32_t nx_snappy_decode_batch_naive(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                                uint32_t* out_len, uint32_t* consumed, int32_t* status,
                                                const uint32_t* expected_masked_crc, uint32_t* crc_out, uint32_t n,
                                                void* stream) {
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    if (nx::crc_tables_init() != NX_OK) return NX_ERR_HIP;
    unsigned grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(nx::k_snappy_decode_naive, dim3(grid), dim3(256), 0, (hipStream_t)stream, in, in_off, in_len, out, out_off,
                       out_cap, out_len, consumed, status, expected_masked_crc, crc_out, n, nx::crc_tables_dev());
    NX_HIP_CHECK(hipGetLastError());
    return NX_OK;
}
