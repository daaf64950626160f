"""ctypes binding of the CPU parity oracle (oracle/netty_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package ``netty_amd`` never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u8p = C.POINTER(C.c_uint8)


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        L.orc_crc32c.restype = C.c_uint32
        L.orc_crc32c.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_mask_checksum.restype = C.c_uint32
        L.orc_mask_checksum.argtypes = [C.c_uint32]
        L.orc_snappy_checksum.restype = C.c_uint32
        L.orc_snappy_checksum.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_snappy_max_compressed_length.restype = C.c_size_t
        L.orc_snappy_max_compressed_length.argtypes = [C.c_size_t]
        L.orc_snappy_encode.restype = C.c_size_t
        L.orc_snappy_encode.argtypes = [C.c_char_p, C.c_int32, C.c_void_p]
        L.orc_snappy_decode.restype = C.c_int32
        L.orc_snappy_decode.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                        C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.orc_snappy_get_preamble.restype = C.c_int64
        L.orc_snappy_get_preamble.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_snappy_frame_max_encoded.restype = C.c_size_t
        L.orc_snappy_frame_max_encoded.argtypes = [C.c_size_t]
        L.orc_snappy_frame_encode.restype = C.c_size_t
        L.orc_snappy_frame_encode.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.POINTER(C.c_int),
                                              C.c_void_p]
        L.orc_fastlz_compress.restype = C.c_int32
        L.orc_fastlz_compress.argtypes = [C.c_char_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.orc_fastlz_decompress.restype = C.c_int32
        L.orc_fastlz_decompress.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32]
        L.orc_adler32.restype = C.c_uint32
        L.orc_adler32.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_fastlz_frame_encode.restype = C.c_size_t
        L.orc_fastlz_frame_encode.argtypes = [C.c_char_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                              C.c_void_p]
        L.orc_fastlz_frame_max_encoded.restype = C.c_size_t
        L.orc_fastlz_frame_max_encoded.argtypes = [C.c_size_t]
        L.orc_lzf_encode_chunk.restype = C.c_size_t
        L.orc_lzf_encode_chunk.argtypes = [C.c_char_p, C.c_int32, C.c_void_p]
        L.orc_lzf_decode_chunk.restype = C.c_int32
        L.orc_lzf_decode_chunk.argtypes = [C.c_char_p, C.c_int32, C.c_void_p, C.c_int32]
        L.orc_lzf_compress_body.restype = C.c_int32
        L.orc_lzf_compress_body.argtypes = [C.c_char_p, C.c_int32, C.c_void_p]
        L.orc_lzf_frame_encode.restype = C.c_size_t
        L.orc_lzf_frame_encode.argtypes = [C.c_char_p, C.c_size_t, C.c_int32, C.c_void_p]
        L.orc_lzf_frame_max_encoded.restype = C.c_size_t
        L.orc_lzf_frame_max_encoded.argtypes = [C.c_size_t]
        L.orc_java_random_bytes.restype = None
        L.orc_java_random_bytes.argtypes = [C.c_int64, C.c_void_p, C.c_size_t]
        L.orc_java_random_scramble.restype = C.c_int64
        L.orc_java_random_scramble.argtypes = [C.c_int64]
        L.orc_java_random_next_long.restype = C.c_int64
        L.orc_java_random_next_long.argtypes = [C.POINTER(C.c_int64)]
        L.orc_textgen_chunk.restype = None
        L.orc_textgen_chunk.argtypes = [C.c_uint64, C.c_void_p, C.c_size_t]
        _lib = L
    return _lib


def _buf(n: int):
    return (C.c_uint8 * max(n, 1))()


# ---------------------------------------------------------------- CRC32C
def crc32c(data: bytes) -> int:
    return lib().orc_crc32c(bytes(data), len(data))


def mask_checksum(c: int) -> int:
    return lib().orc_mask_checksum(c & 0xFFFFFFFF)


def snappy_checksum(data: bytes) -> int:
    return lib().orc_snappy_checksum(bytes(data), len(data))


# ---------------------------------------------------------------- Snappy
def snappy_encode(data: bytes) -> bytes:
    L = lib()
    out = _buf(L.orc_snappy_max_compressed_length(len(data)))
    n = L.orc_snappy_encode(bytes(data), len(data), out)
    return bytes(out[:n])


def snappy_decode(data: bytes, out_cap: int = 1 << 31):
    """Returns (status, output bytes, consumed)."""
    L = lib()
    cap = out_cap
    pre = L.orc_snappy_get_preamble(bytes(data), len(data))
    alloc = min(cap, max(pre, 0) if pre > 0 else 0)
    # the output can exceed the preamble (never checked); size by the worst case
    worst = min(cap, len(data) * 64 + 64)
    out = _buf(max(alloc, worst))
    olen = C.c_size_t(0)
    cons = C.c_size_t(0)
    st = L.orc_snappy_decode(bytes(data), len(data), out, min(cap, len(out)), C.byref(olen), C.byref(cons))
    return st, bytes(out[:olen.value]), cons.value


def snappy_get_preamble(data: bytes) -> int:
    return lib().orc_snappy_get_preamble(bytes(data), len(data))


def snappy_frame_encode(data: bytes, jumbo: bool = False, started: bool = False):
    """One SnappyFrameEncoder.encode() call.  Returns (bytes, started_after)."""
    L = lib()
    out = _buf(L.orc_snappy_frame_max_encoded(len(data)))
    st = C.c_int(1 if started else 0)
    n = L.orc_snappy_frame_encode(bytes(data), len(data), 1 if jumbo else 0, C.byref(st), out)
    return bytes(out[:n]), bool(st.value)


# ---------------------------------------------------------------- FastLZ
def fastlz_compress(data: bytes, level: int, u16_limit: int | None = None, tail: bytes = b"") -> bytes:
    L = lib()
    buf = bytes(data) + bytes(tail)
    lim = len(data) if u16_limit is None else u16_limit
    out = _buf(max(int(len(data) * 1.06), 66) + 16)
    n = L.orc_fastlz_compress(buf, len(data), out, level, lim)
    return bytes(out[:n])


def fastlz_decompress(data: bytes, out_len: int, in_avail: int | None = None):
    """Returns (java return value or negative status, output bytes)."""
    L = lib()
    avail = len(data) if in_avail is None else in_avail
    out = _buf(out_len)
    r = L.orc_fastlz_decompress(bytes(data), len(data), avail, out, out_len)
    return r, bytes(out[:max(r, 0)])


def adler32(data: bytes) -> int:
    return lib().orc_adler32(bytes(data), len(data))


def fastlz_frame_encode(data: bytes, level: int = 0, checksum: bool = False, r0: int = 0,
                        prefix: bytes | None = None) -> bytes:
    L = lib()
    buf = (prefix if prefix is not None else bytes(r0)) + bytes(data)
    out = _buf(L.orc_fastlz_frame_max_encoded(len(data)))
    n = L.orc_fastlz_frame_encode(buf, r0, len(data), level, 1 if checksum else 0, out)
    return bytes(out[:n])


# ---------------------------------------------------------------- LZF
def lzf_encode_chunk(data: bytes) -> bytes:
    out = _buf(len(data) + len(data) // 32 + 64)
    n = lib().orc_lzf_encode_chunk(bytes(data), len(data), out)
    return bytes(out[:n])


def lzf_compress_body(data: bytes) -> bytes:
    out = _buf(len(data) + len(data) // 32 + 64)
    n = lib().orc_lzf_compress_body(bytes(data), len(data), out)
    return bytes(out[:n])


def lzf_decode_chunk(body: bytes, out_len: int):
    out = _buf(out_len)
    st = lib().orc_lzf_decode_chunk(bytes(body), len(body), out, out_len)
    return st, bytes(out[:out_len]) if st == 0 else b""


def lzf_frame_encode(data: bytes, compress_threshold: int = 16) -> bytes:
    L = lib()
    out = _buf(L.orc_lzf_frame_max_encoded(len(data)))
    n = L.orc_lzf_frame_encode(bytes(data), len(data), compress_threshold, out)
    return bytes(out[:n])


# ---------------------------------------------------------------- data
def java_random_bytes(seed: int, n: int) -> bytes:
    out = _buf(n)
    lib().orc_java_random_bytes(C.c_int64(seed), out, n)
    return bytes(out[:n])


class JavaRandom:
    """java.util.Random restatement (nextLong only; nextBytes via java_random_bytes)."""

    def __init__(self, seed: int):
        self._s = C.c_int64(lib().orc_java_random_scramble(C.c_int64(seed)))

    def next_long(self) -> int:
        return lib().orc_java_random_next_long(C.byref(self._s))


def textgen_chunk(index: int, n: int = 65536) -> bytes:
    out = _buf(n)
    lib().orc_textgen_chunk(index, out, n)
    return bytes(out[:n])
