"""HTTP content-coding hooks for the snappy codec.

Netty's HTTP codec reaches this package's hot path at two decision points.  Both are restated here
so that a pipeline can route `content-encoding: snappy` bodies through the GPU handlers.  The HTTP
codec itself stays Netty's: message objects, header parsing, chunked transfer.

- ``new_content_decoder`` restates HttpContentDecompressor.newContentDecoder
  (codec-http/.../HttpContentDecompressor.java:90-145).  "snappy" (ASCII case-insensitive) gets a
  channel around SnappyFrameDecoder (:124-130); gzip/deflate/br/zstd are not in scope and return None.
- ``HttpContentCompressor.determine_encoding`` restates determineEncoding
  (HttpContentCompressor.java:295-365), the Accept-Encoding q-value negotiation that picks "snappy".
  ``new_content_encoder`` is the snappy encoder factory (:232-233, :470-474).

Reference paths are relative to /root/reference/codec-http/src/main/java/io/netty/handler/codec/http/.
"""
from __future__ import annotations

import re
import struct

from .handlers import EmbeddedChannel, SnappyFrameDecoder, SnappyFrameEncoder

SNAPPY = "snappy"  # HttpHeaderValues.SNAPPY (HttpHeaderValues.java:124-126)

# java.lang.Float.parseFloat's decimal grammar (FloatingDecimal): optional sign, NaN / Infinity,
# or digits with an optional exponent and an optional f/F/d/D suffix.  Java's hex-float forms are
# not accepted here: they read as NumberFormatException, so q = 0.
_JAVA_FLOAT = re.compile(r"[+-]?(NaN|Infinity|((\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)[fFdD]?)")


def _java_parse_float(s: str) -> float:
    """Float.parseFloat: trims chars <= ' ' (String.trim), raises ValueError like NumberFormatException,
    and rounds to float32."""
    t = s.strip("".join(chr(c) for c in range(33)))
    if not _JAVA_FLOAT.fullmatch(t):
        raise ValueError(s)
    t = t.rstrip("fFdD") if not t.endswith("Infinity") else t
    v = float(t.replace("Infinity", "inf").replace("NaN", "nan"))
    try:
        return struct.unpack("f", struct.pack("f", v))[0]
    except OverflowError:  # beyond float32: Java rounds to +-Infinity
        return float("inf") if v > 0 else float("-inf")


def _ascii_eq_ignore_case(a: str, b: str) -> bool:
    return len(a) == len(b) and all(x == y or (x.isascii() and y.isascii() and x.lower() == y.lower())
                                    for x, y in zip(a, b))


def new_content_decoder(content_encoding: str):
    """HttpContentDecompressor.newContentDecoder for the snappy coding (HttpContentDecompressor.java:124-130).
    Returns an EmbeddedChannel around SnappyFrameDecoder for "snappy", None for anything else."""
    if _ascii_eq_ignore_case(content_encoding, SNAPPY):
        return EmbeddedChannel(SnappyFrameDecoder())
    return None


class HttpContentCompressor:
    """Encoding negotiation of HttpContentCompressor (HttpContentCompressor.java:170-245, 295-365).
    Each flag stands for the StandardCompressionOptions entry being configured; the default is every
    option, as the no-argument constructor gives when brotli and zstd are available (:236-245)."""

    def __init__(self, br: bool = True, zstd: bool = True, snappy: bool = True, gzip: bool = True,
                 deflate: bool = True):
        self.br, self.zstd, self.snappy, self.gzip, self.deflate = br, zstd, snappy, gzip, deflate

    def determine_encoding(self, accept_encoding: str) -> str | None:
        star_q = br_q = zstd_q = snappy_q = gzip_q = deflate_q = -1.0
        start, length = 0, len(accept_encoding)
        while start < length:
            comma = accept_encoding.find(",", start)
            if comma == -1:
                comma = length
            encoding = accept_encoding[start:comma]
            q = 1.0
            eq = encoding.find("=")
            if eq != -1:
                try:
                    q = _java_parse_float(encoding[eq + 1:])
                except ValueError:
                    q = 0.0  # ignore the encoding
            if "*" in encoding:
                star_q = q
            elif "br" in encoding and q > br_q:
                br_q = q
            elif "zstd" in encoding and q > zstd_q:
                zstd_q = q
            elif "snappy" in encoding and q > snappy_q:
                snappy_q = q
            elif "gzip" in encoding and q > gzip_q:
                gzip_q = q
            elif "deflate" in encoding and q > deflate_q:
                deflate_q = q
            start = comma + 1
        if br_q > 0.0 or zstd_q > 0.0 or snappy_q > 0.0 or gzip_q > 0.0 or deflate_q > 0.0:
            if br_q != -1.0 and br_q >= zstd_q and self.br:
                return "br"
            elif zstd_q != -1.0 and zstd_q >= snappy_q and self.zstd:
                return "zstd"
            elif snappy_q != -1.0 and snappy_q >= gzip_q and self.snappy:
                return "snappy"
            elif gzip_q != -1.0 and gzip_q >= deflate_q and self.gzip:
                return "gzip"
            elif deflate_q != -1.0 and self.deflate:
                return "deflate"
        if star_q > 0.0:
            if br_q == -1.0 and self.br:
                return "br"
            if zstd_q == -1.0 and self.zstd:
                return "zstd"
            if snappy_q == -1.0 and self.snappy:
                return "snappy"
            if gzip_q == -1.0 and self.gzip:
                return "gzip"
            if deflate_q == -1.0 and self.deflate:
                return "deflate"
        return None

    def new_content_encoder(self, accept_encoding: str):
        """(content-encoding, EmbeddedChannel around the encoder) when the negotiation picks snappy
        (SnappyEncoderFactory, :470-474); (encoding, None) for codings outside this package."""
        enc = self.determine_encoding(accept_encoding)
        if enc == SNAPPY:
            return enc, EmbeddedChannel(SnappyFrameEncoder())
        return enc, None
