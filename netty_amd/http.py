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

- ``SnappyHttpBodyEncoder`` / ``SnappyHttpBodyDecoder`` are the NON-BLOCKING snappy body path over the
  cross-channel batcher: HttpContentEncoder / HttpContentDecoder run their
  codec through an EmbeddedChannel synchronously (HttpContentEncoder.java:336-343,
  HttpContentDecoder.java:165-175), so a GPU codec there would have to block the event loop.  These
  handlers instead submit each body content as a batcher job and release messages strictly in
  arrival order once their jobs complete (poll() never blocks), with the header rewriting those two
  classes do for a coded body.

Reference paths are relative to /root/reference/codec-http/src/main/java/io/netty/handler/codec/http/.
"""
from __future__ import annotations

import collections
import re
import struct
from dataclasses import dataclass, field

from .handlers import DecoderException, Batcher, EmbeddedChannel, SnappyFrameDecoder, SnappyFrameEncoder

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


# ------------------------------------------------------------------ non-blocking snappy body path
@dataclass
class HttpMessage:
    """The head of a request or response (headers by lower-case name)."""
    headers: dict = field(default_factory=dict)


@dataclass
class HttpContent:
    content: bytes = b""


@dataclass
class LastHttpContent(HttpContent):
    trailers: dict = field(default_factory=dict)


class _Ordered:
    """A channel's messages in arrival order: ready ones, or batcher tickets still running."""

    def __init__(self, batcher: Batcher):
        self.b = batcher
        self.q = collections.deque()  # [ticket or None, message or builder]

    def push_ready(self, msg):
        self.q.append([None, msg])

    def push_job(self, ticket, build):
        self.q.append([ticket, build])

    def poll(self) -> list:
        """Messages whose turn has come (a running job stops the release; never blocks).

        A job that failed (a corrupted body) raises its DecoderException once, after its entry has
        left the queue: ``e.messages`` holds what this poll released before it plus the contents the
        job decoded before the failure (its LastHttpContent is not released: the reference's exception
        leaves HttpContentDecoder.decode before finishDecode).  The messages queued behind it come out
        on the next polls; the body's later contents decode to nothing, as the corrupted decoder skips
        its input (SnappyFrameDecoder.java:86-89), and its LastHttpContent still ends the message."""
        out = []
        while self.q:
            t, m = self.q[0]
            if t is not None:
                if not self.b.poll(t):
                    break
                self.q.popleft()
                try:
                    r = self.b.result(t)
                except DecoderException as e:
                    e.messages = out + [x for x in m(list(getattr(e, "decoded", []))) if not isinstance(x, LastHttpContent)]
                    raise
                out.extend(m(r))
                continue
            self.q.popleft()
            out.extend(m if isinstance(m, list) else [m])
        return out


class SnappyHttpBodyEncoder:
    """Outbound, for a response whose coding HttpContentCompressor negotiated as snappy
    (determineEncoding :295-365; SnappyEncoderFactory :470-474 makes one SnappyFrameEncoder per
    response).  Header rewriting as HttpContentEncoder.encode does for a coded body
    (HttpContentEncoder.java:181-196): Content-Encoding set, Content-Length removed, chunked transfer.
    Each content's bytes become one batcher job; the framed bytes replace the content when it is done."""

    def __init__(self, batcher: Batcher):
        self.b = batcher
        self.o = _Ordered(batcher)
        self.enc = None

    def write(self, msg, encoding: str | None = None):
        """encoding: the negotiated coding for a response head (None = pass the body through)."""
        if isinstance(msg, HttpMessage):
            if encoding == SNAPPY:
                h = dict(msg.headers)
                h["content-encoding"] = SNAPPY
                h.pop("content-length", None)
                h["transfer-encoding"] = "chunked"
                msg = HttpMessage(h)
                self.enc = SnappyFrameEncoder()
            self.o.push_ready(msg)
            return
        if self.enc is None:  # an identity body
            self.o.push_ready(msg)
            return
        t = self.b.submit_encode(self.enc, msg.content)
        # fetchEncoderOutput (:352-366) drops an empty buffer: an empty content yields no chunk
        framed = lambda r: [HttpContent(x) for x in r if x]  # noqa: E731
        if isinstance(msg, LastHttpContent):
            trailers = msg.trailers
            self.enc = None  # finishEncode: SnappyFrameEncoder adds nothing at the end of the body (:345-350)
            self.o.push_job(t, lambda r: framed(r) + [LastHttpContent(b"", trailers)])  # encodeContent (:271-290)
        else:
            self.o.push_job(t, framed)

    def poll(self) -> list:
        return self.o.poll()


class SnappyHttpBodyDecoder:
    """Inbound, ahead of HttpContentDecompressor: a message whose Content-Encoding is snappy
    (newContentDecoder :124-130, ASCII case-insensitive) is decoded here, with HttpContentDecoder's
    header rewriting (HttpContentDecoder.java:89-137: the trimmed Content-Encoding picks the decoder,
    Content-Length is removed for chunked transfer, the identity target coding removes
    Content-Encoding); every other message passes through in order.  One DefaultHttpContent per
    non-empty decoded chunk, as ByteBufForwarder (:286-294) fires them, then the last content with the
    trailers (:174-187)."""

    def __init__(self, batcher: Batcher, validate_checksums: bool = False):
        self.b = batcher
        self.o = _Ordered(batcher)
        self.dec = None
        self.validate = validate_checksums

    def read(self, msg):
        if isinstance(msg, HttpMessage):
            ce = msg.headers.get("content-encoding", "")
            if _ascii_eq_ignore_case(ce.strip(), SNAPPY):
                h = dict(msg.headers)
                if "content-length" in h:
                    del h["content-length"]
                    h["transfer-encoding"] = "chunked"
                h.pop("content-encoding", None)
                msg = HttpMessage(h)
                self.dec = SnappyFrameDecoder(self.validate)
            self.o.push_ready(msg)
            return
        if self.dec is None:
            self.o.push_ready(msg)
            return
        t = self.b.submit_decode(self.dec, msg.content)
        if isinstance(msg, LastHttpContent):
            trailers = msg.trailers
            self.dec = None
            self.o.push_job(t, lambda r: [HttpContent(x) for x in r if x] + [LastHttpContent(b"", trailers)])
        else:
            self.o.push_job(t, lambda r: [HttpContent(x) for x in r if x])

    def poll(self) -> list:
        return self.o.poll()
