"""netty_amd — MI355X-native (gfx950 HIP) implementation of Netty's codec-compression hot path.

Snappy (block + framing, masked CRC32C), FastLZ (level 1/2 + framing, Adler32), LZF and LZ4
(block + framing, XXHash32) codecs, with the per-chunk arithmetic in hand-written HIP kernels (libnetty_amd.so) behind
the reference's handler API (see ``netty_amd.handlers``) and a device-resident batch API
(``netty_amd.batch``).  The C-ABI is declared in ``include/netty_amd.h``.
"""
from ._lib import load as _load_lib  # noqa: F401  (raises if the HIP library is not built)
from .handlers import (  # noqa: F401
    Batcher,
    CompressionException,
    DecoderException,
    DecompressionException,
    EmbeddedChannel,
    EncoderException,
    FastLzFrameDecoder,
    FastLzFrameEncoder,
    IllegalStateException,
    Lz4FrameDecoder,
    Lz4FrameEncoder,
    LzfDecoder,
    LzfEncoder,
    SnappyFrameDecoder,
    SnappyFrameEncoder,
    SnappyFramedDecoder,
    SnappyFramedEncoder,
)

__version__ = "0.1.0"

_load_lib()
