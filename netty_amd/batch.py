"""Device-resident batch API (thin wrappers over the C-ABI batch kernels).

All tensors are torch tensors on the same HIP device; torch is used only as the device
allocator / stream provider.  Chunk i is ``data[off[i] : off[i] + length[i]]``.  Calls are
asynchronous on torch's current stream.
"""
from __future__ import annotations

import torch

from . import _lib


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {rc} ({_lib.status_string(rc)})")


# Shared device workspaces (include/netty_amd.h NX_WS_*; csrc/workspace.hpp)
WS_SNAPPY_ENC, WS_LZ4_ENC, WS_FASTLZ_ENC, WS_LZF_ENC, WS_DEC_RECORDS, WS_LZ4HC_ENC = range(6)


def workspace_info(kind: int) -> tuple[int, int]:
    """(bytes, owners) of the current device's workspace of `kind`."""
    import ctypes as C
    b, o = C.c_uint64(0), C.c_int32(0)
    _chk(_lib.load().nx_workspace_info(kind, C.byref(b), C.byref(o)), "nx_workspace_info")
    return b.value, o.value


def workspaces_trim():
    """Free the current device's workspaces that no batcher or handle holds."""
    _chk(_lib.load().nx_workspaces_trim(), "nx_workspaces_trim")


def snappy_encoder_reserve(max_chunks: int, max_bytes: int = 0) -> tuple[int, int]:
    """nx_snappy_encoder_reserve_ex: place the Snappy table workspace now, capped at max_bytes for good
    (0: no cap).  Returns (workspace bytes, most bytes its placement held at once)."""
    import ctypes as C
    b, p = C.c_uint64(0), C.c_uint64(0)
    _chk(_lib.load().nx_snappy_encoder_reserve_ex(max_chunks, max_bytes, _stream(), C.byref(b), C.byref(p)),
         "nx_snappy_encoder_reserve_ex")
    return b.value, p.value


def workspace_placement_config(peak_bytes: int = 0, max_candidates: int = 0):
    """nx_workspace_placement_config: the bytes a large workspace's placement candidates may hold at once
    (0: half the device; 2**64 - 1: all but 8 GiB free) and the candidates drawn in all (0: 24)."""
    _chk(_lib.load().nx_workspace_placement_config(peak_bytes, max_candidates), "nx_workspace_placement_config")


def snappy_max_compressed_length(n: int) -> int:
    return _lib.load().nx_snappy_max_compressed_length(n)


def fastlz_max_compressed_length(n: int) -> int:
    return _lib.load().nx_fastlz_max_compressed_length(n)


def lzf_max_compressed_length(n: int) -> int:
    return _lib.load().nx_lzf_max_compressed_length(n)


def snappy_encode(inp, in_off, in_len, out, out_off, out_len=None, status=None):
    """Snappy.encode per chunk (Snappy.java:82-165).  Returns (out_len, status) int tensors."""
    n = in_len.numel()
    dev = inp.device
    out_len = torch.empty(n, dtype=torch.int32, device=dev) if out_len is None else out_len
    status = torch.empty(n, dtype=torch.int32, device=dev) if status is None else status
    _chk(_lib.load().nx_snappy_encode_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_len),
                                            _ptr(status), n, _stream()), "nx_snappy_encode_batch")
    return out_len, status


def snappy_decode(inp, in_off, in_len, out, out_off, out_cap=None, expected_crc=None, want_crc=False, consumed=False,
                  out_len=None, status=None, variant="auto", fn=None):
    """Snappy.decode per chunk (+ fused masked-CRC32C verify).  Returns dict of tensors.

    variant: "auto" (the fused decoder up to 32768 frames, the parse/expand pair above), "pair" (always
    the parse/expand kernel pair) or "fused" (always the single-kernel wave decoder), same contract; fn: another entry point of that contract (the tests' lane-per-chunk cross-check kernel)."""
    n = in_len.numel()
    dev = inp.device
    out_len = torch.empty(n, dtype=torch.int32, device=dev) if out_len is None else out_len
    status = torch.empty(n, dtype=torch.int32, device=dev) if status is None else status
    cons = torch.empty(n, dtype=torch.int32, device=dev) if consumed else None
    crc = torch.empty(n, dtype=torch.int32, device=dev) if want_crc else None
    lib = _lib.load()
    if fn is None:
        fn = {"auto": lib.nx_snappy_decode_batch, "fused": lib.nx_snappy_decode_batch_fused,
              "pair": lib.nx_snappy_decode_batch_pair}[variant]
    _chk(fn(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(cons),
            _ptr(status), _ptr(expected_crc), _ptr(crc), n, _stream()), "nx_snappy_decode_batch")
    return {"out_len": out_len, "status": status, "consumed": cons, "crc": crc}


def snappy_frame_scan(inp, in_off, in_len, state, cap: int):
    """SnappyFrameDecoder's chunk walk over device cumulations (nx_snappy_frame_scan_batch).

    in_off / in_len: int64 tensors (one cumulation per stream); state: int32 tensor, updated in place
    (started | corrupted << 1 | numBytesToSkip << 8).  Returns a dict of tensors: consumed, status,
    counts [compressed, uncompressed, claims], and the list arrays data_off, data_len, masked_crc,
    stream, seq (compressed entries at [0, counts[0]), uncompressed at [cap - counts[1], cap))."""
    n = in_len.numel()
    dev = inp.device
    c = max(int(cap), 1)
    r = {"consumed": torch.empty(n, dtype=torch.int64, device=dev),
         "status": torch.empty(n, dtype=torch.int32, device=dev),
         "data_off": torch.empty(c, dtype=torch.int64, device=dev),
         "data_len": torch.empty(c, dtype=torch.int32, device=dev),
         "masked_crc": torch.empty(c, dtype=torch.int32, device=dev),
         "stream": torch.empty(c, dtype=torch.int32, device=dev),
         "seq": torch.empty(c, dtype=torch.int32, device=dev),
         "counts": torch.empty(3, dtype=torch.int32, device=dev)}
    _chk(_lib.load().nx_snappy_frame_scan_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(state), _ptr(r["consumed"]),
                                                _ptr(r["status"]), _ptr(r["data_off"]), _ptr(r["data_len"]),
                                                _ptr(r["masked_crc"]), _ptr(r["stream"]), _ptr(r["seq"]), _ptr(r["counts"]),
                                                int(cap), n, _stream()), "nx_snappy_frame_scan_batch")
    return r


def snappy_frame_scan_long(inp, length: int, state, cap: int, offset: int = 0):
    """The segmented walk of ONE long cumulation inp[offset, offset + length) (nx_snappy_frame_scan_long);
    state: a one-element int32 tensor, updated in place.  Same result dict as snappy_frame_scan with
    n = 1 (data_off relative to inp[offset])."""
    dev = inp.device
    c = max(int(cap), 1)
    r = {"consumed": torch.empty(1, dtype=torch.int64, device=dev),
         "status": torch.empty(1, dtype=torch.int32, device=dev),
         "data_off": torch.empty(c, dtype=torch.int64, device=dev),
         "data_len": torch.empty(c, dtype=torch.int32, device=dev),
         "masked_crc": torch.empty(c, dtype=torch.int32, device=dev),
         "stream": torch.empty(c, dtype=torch.int32, device=dev),
         "seq": torch.empty(c, dtype=torch.int32, device=dev),
         "counts": torch.empty(3, dtype=torch.int32, device=dev)}
    _chk(_lib.load().nx_snappy_frame_scan_long(_ptr(inp) + int(offset), int(length), _ptr(state), _ptr(r["consumed"]),
                                               _ptr(r["status"]), _ptr(r["data_off"]), _ptr(r["data_len"]),
                                               _ptr(r["masked_crc"]), _ptr(r["stream"]), _ptr(r["seq"]), _ptr(r["counts"]),
                                               int(cap), _stream()), "nx_snappy_frame_scan_long")
    return r


def crc32c_masked(inp, off, length, out=None):
    """Snappy.calculateChecksum per chunk (Snappy.java:668-676)."""
    n = length.numel()
    out = torch.empty(n, dtype=torch.int32, device=inp.device) if out is None else out
    _chk(_lib.load().nx_crc32c_masked_batch(_ptr(inp), _ptr(off), _ptr(length), _ptr(out), n, _stream()),
         "nx_crc32c_masked_batch")
    return out


def fastlz_compress(inp, in_off, in_len, out, out_off, level=None, u16_limit=None):
    n = in_len.numel()
    dev = inp.device
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    _chk(_lib.load().nx_fastlz_compress_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_len),
                                              _ptr(level), _ptr(u16_limit), _ptr(status), n, _stream()),
         "nx_fastlz_compress_batch")
    return out_len, status


def fastlz_decompress(inp, in_off, in_len, out, out_off, out_len_limit, in_avail=None):
    n = in_len.numel()
    res = torch.empty(n, dtype=torch.int32, device=inp.device)
    _chk(_lib.load().nx_fastlz_decompress_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(in_avail), _ptr(out),
                                                _ptr(out_off), _ptr(out_len_limit), _ptr(res), n, _stream()),
         "nx_fastlz_decompress_batch")
    return res


def adler32(inp, off, length):
    n = length.numel()
    out = torch.empty(n, dtype=torch.int32, device=inp.device)
    _chk(_lib.load().nx_adler32_batch(_ptr(inp), _ptr(off), _ptr(length), _ptr(out), n, _stream()), "nx_adler32_batch")
    return out


def lzf_encode(inp, in_off, in_len, out, out_off):
    n = in_len.numel()
    dev = inp.device
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    _chk(_lib.load().nx_lzf_encode_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_len),
                                         _ptr(status), n, _stream()), "nx_lzf_encode_batch")
    return out_len, status


def lzf_decode(inp, in_off, in_len, out, out_off, out_len):
    n = in_len.numel()
    status = torch.empty(n, dtype=torch.int32, device=inp.device)
    _chk(_lib.load().nx_lzf_decode_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_len),
                                         _ptr(status), n, _stream()), "nx_lzf_decode_batch")
    return status


def lz4_max_compressed_length(n: int) -> int:
    return _lib.load().nx_lz4_max_compressed_length(n)


def lz4_encode(inp, in_off, in_len, out, out_off, high: bool = False):
    """LZ4 block encode per chunk (nx_lz4_encode_batch; high: lz4-java's highCompressor(), liblz4's
    LZ4_compress_HC level 9, nx_lz4hc_encode_batch).  Returns (out_len, status)."""
    n = in_len.numel()
    dev = inp.device
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    name = "nx_lz4hc_encode_batch" if high else "nx_lz4_encode_batch"
    _chk(getattr(_lib.load(), name)(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_len),
                                    _ptr(status), n, _stream()), name)
    return out_len, status


def lz4_decode(inp, in_off, in_len, out, out_off, out_len):
    """LZ4 block decode per chunk to exactly out_len[i] bytes (nx_lz4_decode_batch).  Returns status."""
    n = in_len.numel()
    status = torch.empty(n, dtype=torch.int32, device=inp.device)
    _chk(_lib.load().nx_lz4_decode_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off), _ptr(out_len),
                                         _ptr(status), n, _stream()), "nx_lz4_decode_batch")
    return status


LZ4_DEFAULT_SEED = 0x9747B28C  # Lz4Constants.java:70


def xxhash32(inp, off, length, seed: int = LZ4_DEFAULT_SEED, out=None):
    """XXH32 per block (nx_xxhash32_batch), unmasked; Lz4XXHash32.getValue() is this & 0x0FFFFFFF."""
    n = length.numel()
    out = torch.empty(n, dtype=torch.int32, device=inp.device) if out is None else out
    _chk(_lib.load().nx_xxhash32_batch(_ptr(inp), _ptr(off), _ptr(length), seed & 0xFFFFFFFF, _ptr(out), n, _stream()),
         "nx_xxhash32_batch")
    return out


def lz4_frame_encode(inp, in_off, in_len, out, out_off, compression_level: int = 6, high: bool = False):
    """Lz4FrameEncoder.flushBufferedData per block (nx_lz4_frame_encode_batch_ex): header + block in each
    out slot (capacity 21 + lz4_max_compressed_length); high = the highCompressor flag.
    Returns (out_len, status)."""
    n = in_len.numel()
    dev = inp.device
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    _chk(_lib.load().nx_lz4_frame_encode_batch_ex(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(out), _ptr(out_off),
                                                  _ptr(out_len), int(compression_level), int(bool(high)), _ptr(status), n,
                                                  _stream()),
         "nx_lz4_frame_encode_batch_ex")
    return out_len, status


def lz4_frame_scan(inp, in_off, in_len, state, cap: int):
    """Lz4FrameDecoder's block walk over device cumulations (nx_lz4_frame_scan_batch).  state: int32
    tensor (finished | corrupted << 1), updated in place.  Returns a dict of tensors: consumed, status,
    counts [compressed, non-compressed, claims] and the list arrays data_off, comp_len, decomp_len,
    checksum, stream, seq (compressed at [0, counts[0]), non-compressed at [cap - counts[1], cap))."""
    n = in_len.numel()
    dev = inp.device
    c = max(int(cap), 1)
    r = {"consumed": torch.empty(n, dtype=torch.int64, device=dev),
         "status": torch.empty(n, dtype=torch.int32, device=dev),
         "data_off": torch.empty(c, dtype=torch.int64, device=dev),
         "comp_len": torch.empty(c, dtype=torch.int32, device=dev),
         "decomp_len": torch.empty(c, dtype=torch.int32, device=dev),
         "checksum": torch.empty(c, dtype=torch.int32, device=dev),
         "stream": torch.empty(c, dtype=torch.int32, device=dev),
         "seq": torch.empty(c, dtype=torch.int32, device=dev),
         "counts": torch.empty(3, dtype=torch.int32, device=dev)}
    _chk(_lib.load().nx_lz4_frame_scan_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), _ptr(state), _ptr(r["consumed"]),
                                             _ptr(r["status"]), _ptr(r["data_off"]), _ptr(r["comp_len"]),
                                             _ptr(r["decomp_len"]), _ptr(r["checksum"]), _ptr(r["stream"]), _ptr(r["seq"]),
                                             _ptr(r["counts"]), int(cap), n, _stream()), "nx_lz4_frame_scan_batch")
    return r


def lz4_frame_decode(inp, scan: dict, cap: int, validate_checksums: bool = True):
    """The data half of Lz4FrameDecoder.decode (Lz4FrameDecoder.java:184-229) for the blocks a scan listed:
    compressed blocks are decoded into one output buffer (slots packed by decomp_len), non-compressed
    blocks stay where they are in `inp` (Java's retainedSlice, :197-199).  With validate_checksums the
    masked XXH32 of every block's bytes is compared with its header (:226-228).
    Returns {"compressed": (out, out_off, status), "raw": (data_off, len, status)} over the two list ranges."""
    nc, nu = (int(v) for v in scan["counts"][:2].tolist())
    dev = inp.device
    dl = scan["decomp_len"][:nc].to(torch.int64)
    out_off = torch.cumsum(dl, 0) - dl
    total = int(dl.sum().item()) if nc else 0
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    st_c = lz4_decode(inp, scan["data_off"][:nc], scan["comp_len"][:nc], out, out_off, scan["decomp_len"][:nc]) if nc \
        else torch.empty(0, dtype=torch.int32, device=dev)
    lo = cap - nu
    r_off, r_len = scan["data_off"][lo:cap], scan["decomp_len"][lo:cap]
    st_u = torch.zeros(nu, dtype=torch.int32, device=dev)
    if validate_checksums:
        bad = torch.tensor(-56, dtype=torch.int32, device=dev)  # NX_ERR_LZ4_CHECKSUM_MISMATCH
        if nc:
            hc = xxhash32(out, out_off, scan["decomp_len"][:nc]) & 0x0FFFFFFF
            st_c = torch.where((st_c == 0) & (hc != scan["checksum"][:nc]), bad, st_c)
        if nu:
            hu = xxhash32(inp, r_off, r_len) & 0x0FFFFFFF
            st_u = torch.where(hu != scan["checksum"][lo:cap], bad, st_u)
    return {"compressed": (out, out_off, st_c), "raw": (r_off, r_len, st_u)}


def textgen(out, first_chunk: int, n_chunks: int, chunk_len: int):
    """Fill out[k*chunk_len:(k+1)*chunk_len] with text-like chunk first_chunk+k."""
    _chk(_lib.load().nx_textgen_device(_ptr(out), first_chunk, n_chunks, chunk_len, _stream()), "nx_textgen_device")
    return out


def gather(src, src_off, length, dst=None, dst_off=None):
    """Pack chunk i = src[src_off[i] : +length[i]] contiguously (nx_pack_batch).  dst_off defaults
    to the exclusive scan of length.  Returns (dst, dst_off)."""
    n = length.numel()
    if dst_off is None:
        dst_off = torch.zeros(n, dtype=torch.int64, device=src.device)
        if n > 1:
            torch.cumsum(length[:-1].to(torch.int64), 0, out=dst_off[1:])
    if dst is None:
        total = int((dst_off[-1] + length[-1].to(torch.int64)).item()) if n else 0
        dst = torch.empty(max(total, 1), dtype=torch.uint8, device=src.device)
    _chk(_lib.load().nx_pack_batch(_ptr(src), _ptr(src_off), _ptr(length), _ptr(dst), _ptr(dst_off), n, _stream()),
         "nx_pack_batch")
    return dst, dst_off


def pack(chunks: list[bytes], device, align: int = 16, pad: int = 0):
    """Pack host chunks into one device tensor; returns (data, off[int64], len[int32])."""
    offs, cur = [], 0
    for c in chunks:
        offs.append(cur)
        cur += (len(c) + align - 1) // align * align
    buf = bytearray(cur + pad + 16)
    for o, c in zip(offs, chunks):
        buf[o:o + len(c)] = c
    data = torch.frombuffer(buf, dtype=torch.uint8).to(device)  # buf is a fresh bytearray, copied by .to()
    off = torch.tensor(offs, dtype=torch.int64, device=device)
    ln = torch.tensor([len(c) for c in chunks], dtype=torch.int32, device=device)
    return data, off, ln


def out_slots(lengths: list[int], device, align: int = 16):
    offs, cur = [], 0
    for n in lengths:
        offs.append(cur)
        cur += (n + align - 1) // align * align
    data = torch.zeros(cur + 16, dtype=torch.uint8, device=device)
    return data, torch.tensor(offs, dtype=torch.int64, device=device)
