"""ctypes binding of libnetty_amd.so (the C-ABI of include/netty_amd.h).

The library is built in-tree by ``make -C netty_amd`` (or ``__graft_entry__.build()``).  There is
no fallback: if the shared object is missing or cannot be loaded, importing the product API
raises, so a GPU run can never silently route through a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnetty_amd.so")

_lib = None

vp = C.c_void_p
u32 = C.c_uint32
i32 = C.c_int32
u64 = C.c_uint64
sz = C.c_size_t
i64 = C.c_int64


class NxMsg(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("len", C.c_size_t)]


_SIGS = {
    "nx_version": (C.c_char_p, []),
    "nx_status_string": (C.c_char_p, [i32]),
    "nx_device_count": (i32, []),
    "nx_snappy_max_compressed_length": (sz, [sz]),
    "nx_fastlz_max_compressed_length": (sz, [sz]),
    "nx_lzf_max_compressed_length": (sz, [sz]),
    "nx_snappy_encode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_snappy_decode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_snappy_decode_batch_fused": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_snappy_decode_batch_pair": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_crc32c_masked_batch": (i32, [vp, vp, vp, vp, u32, vp]),
    "nx_snappy_frame_scan_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]),
    "nx_snappy_frame_scan_long": (i32, [vp, C.c_uint64, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_fastlz_compress_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_fastlz_decompress_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_adler32_batch": (i32, [vp, vp, vp, vp, u32, vp]),
    "nx_lzf_encode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_lzf_decode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_lz4_decode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_lz4_encode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_lz4hc_encode_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
    "nx_lz4_max_compressed_length": (sz, [sz]),
    "nx_xxhash32_batch": (i32, [vp, vp, vp, u32, vp, u32, vp]),
    "nx_lz4_frame_encode_batch": (i32, [vp, vp, vp, vp, vp, vp, i32, vp, u32, vp]),
    "nx_lz4_frame_encode_batch_ex": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, vp, u32, vp]),
    "nx_lz4_frame_scan_batch": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]),
    "nx_textgen_device": (i32, [vp, u64, u32, u32, vp]),
    "nx_pack_batch": (i32, [vp, vp, vp, vp, vp, u32, vp]),
    "nx_device_alloc": (vp, [sz]),
    "nx_device_free": (i32, [vp]),
    "nx_memcpy_h2d": (i32, [vp, vp, sz, vp]),
    "nx_memcpy_d2h": (i32, [vp, vp, sz, vp]),
    "nx_stream_sync": (i32, [vp]),
    # asynchronous cross-channel batcher
    "nx_batcher_new": (vp, []),
    "nx_batcher_free": (None, [vp]),
    "nx_host_register": (i32, [vp, sz]),
    "nx_host_unregister": (i32, [vp]),
    "nx_snappy_frame_encoder_submit": (i64, [vp, vp, vp, sz, i32]),
    "nx_snappy_frame_decoder_submit": (i64, [vp, vp, vp, sz, C.POINTER(sz)]),
    "nx_snappy_frame_decoder_submit_registered": (i64, [vp, vp, vp, sz, C.POINTER(sz)]),
    "nx_batcher_flush": (i32, [vp]),
    "nx_batcher_poll": (i32, [vp, i64]),
    "nx_batcher_wait": (i32, [vp, i64]),
    "nx_batcher_result": (i32, [vp, i64, C.POINTER(C.POINTER(NxMsg)), C.POINTER(sz), C.POINTER(C.c_char_p)]),
    "nx_batcher_release": (i32, [vp, i64]),
    "nx_batcher_stats": (i32, [vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]),
    "nx_batcher_set_flush_bytes": (i32, [vp, sz]),
    "nx_batcher_reserve": (i32, [vp, C.c_uint32]),
    "nx_batcher_reserve_arenas": (i32, [vp, C.c_uint32, sz, sz]),
    "nx_batcher_arena_stats": (i32, [vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(C.c_uint32)]),
    "nx_batcher_dma_stats": (i32, [vp, C.POINTER(u64), C.POINTER(u64)]),
    "nx_fastlz_frame_encoder_submit": (i64, [vp, vp, vp, sz, sz]),
    "nx_lzf_encoder_submit": (i64, [vp, vp, vp, sz]),
    "nx_lz4_frame_encoder_submit": (i64, [vp, vp, vp, sz, i32]),
    "nx_fastlz_frame_decoder_submit": (i64, [vp, vp, vp, sz, C.POINTER(sz)]),
    "nx_lzf_decoder_submit": (i64, [vp, vp, vp, sz, C.POINTER(sz)]),
    "nx_lz4_frame_decoder_submit": (i64, [vp, vp, vp, sz, C.POINTER(sz)]),
    # host handler layer
    "nx_snappy_frame_encoder_new": (vp, [i32]),
    "nx_snappy_frame_encoder_free": (None, [vp]),
    "nx_snappy_frame_max_encoded_length": (sz, [sz]),
    "nx_snappy_frame_encoder_encode": (i64, [vp, C.c_char_p, sz, vp, sz]),
    "nx_snappy_frame_decoder_new": (vp, [i32]),
    "nx_snappy_frame_decoder_free": (None, [vp]),
    "nx_snappy_frame_decoder_decode": (i32, [vp, C.c_char_p, sz, C.POINTER(sz), C.POINTER(C.POINTER(NxMsg)),
                                             C.POINTER(sz), C.POINTER(C.c_char_p)]),
    "nx_fastlz_frame_encoder_new": (vp, [i32, i32]),
    "nx_fastlz_frame_encoder_free": (None, [vp]),
    "nx_fastlz_frame_max_encoded_length": (sz, [sz]),
    "nx_fastlz_frame_encoder_encode": (i64, [vp, C.c_char_p, sz, sz, vp, sz]),
    "nx_fastlz_frame_decoder_new": (vp, [i32]),
    "nx_fastlz_frame_decoder_free": (None, [vp]),
    "nx_fastlz_frame_decoder_decode": (i32, [vp, C.c_char_p, sz, C.POINTER(sz), C.POINTER(C.POINTER(NxMsg)),
                                             C.POINTER(sz), C.POINTER(C.c_char_p)]),
    "nx_lzf_encoder_new": (vp, [i32]),
    "nx_lzf_encoder_new_ex": (vp, [i32, i32]),
    "nx_lzf_encoder_free": (None, [vp]),
    "nx_lzf_frame_max_encoded_length": (sz, [sz]),
    "nx_lzf_encoder_encode": (i64, [vp, C.c_char_p, sz, vp, sz]),
    "nx_lz4_frame_encoder_new": (vp, [i32]),
    "nx_lz4_frame_encoder_new_ex": (vp, [i32, i32, i32]),
    "nx_lz4_frame_encoder_error": (C.c_char_p, [vp]),
    "nx_lz4_frame_encoder_free": (None, [vp]),
    "nx_lz4_frame_max_encoded_length": (sz, [sz, i32]),
    "nx_lz4_frame_encoder_encode": (i64, [vp, C.c_char_p, sz, vp, sz]),
    "nx_lz4_frame_encoder_flush": (i64, [vp, vp, sz]),
    "nx_lz4_frame_encoder_close": (i64, [vp, vp, sz]),
    "nx_lz4_frame_decoder_new": (vp, [i32]),
    "nx_lz4_frame_decoder_free": (None, [vp]),
    "nx_lz4_frame_decoder_decode": (i32, [vp, C.c_char_p, sz, C.POINTER(sz), C.POINTER(C.POINTER(NxMsg)),
                                         C.POINTER(sz), C.POINTER(C.c_char_p)]),
    "nx_snappy_encoder_reserve": (i32, [u32, vp]),
    "nx_snappy_encoder_reserve_ex": (i32, [u32, u64, vp, C.POINTER(u64), C.POINTER(u64)]),
    "nx_snappy_encode_plan": (i32, [u32, C.POINTER(u32), u32, C.POINTER(u32)]),
    "nx_snappy_encode_plan_for": (i32, [u32, u32, i32, C.POINTER(u32), u32, C.POINTER(u32)]),
    "nx_workspace_placement_config": (i32, [u64, i32]),
    "nx_snappy_encode_placement": (i32, [C.POINTER(C.c_float), i32, C.POINTER(i32), C.POINTER(i32)]),
    "nx_workspaces_trim": (i32, []),
    "nx_workspaces_forget_stream": (i32, [vp]),
    "nx_workspace_info": (i32, [i32, C.POINTER(C.c_uint64), C.POINTER(i32)]),
    "nx_lzf_decoder_new": (vp, []),
    "nx_lzf_decoder_free": (None, [vp]),
    "nx_lzf_decoder_decode": (i32, [vp, C.c_char_p, sz, C.POINTER(sz), C.POINTER(C.POINTER(NxMsg)),
                                    C.POINTER(sz), C.POINTER(C.c_char_p)]),
}

EXPORTED = tuple(_SIGS.keys())


def load():
    """Load libnetty_amd.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"netty_amd: {LIB_PATH} is not built (run `make -C netty_amd` or "
                          f"__graft_entry__.build()); the HIP path has no CPU fallback")
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def status_string(code: int) -> str:
    return load().nx_status_string(code).decode()


def check(code: int, what: str = "netty_amd call"):
    if code != 0:
        raise RuntimeError(f"{what} failed: {code} ({status_string(code)})")
