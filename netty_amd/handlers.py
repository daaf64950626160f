"""Netty's codec-compression handler API over the GPU path.

Mirrors the public surface of the reference handlers (same names, constructor options,
encode/decode contracts and error behaviour):

* ``SnappyFrameEncoder()`` / ``SnappyFrameEncoder.snappy_encoder_with_jumbo_frames()``
  — SnappyFrameEncoder.java:60-117
* ``SnappyFrameDecoder(validate_checksums=False)`` — SnappyFrameDecoder.java:67-231
* ``FastLzFrameEncoder(level=0, checksum=False)`` — FastLzFrameEncoder.java:58-172
* ``FastLzFrameDecoder(validate_checksums=False)`` — FastLzFrameDecoder.java:90-207
* ``LzfEncoder(compress_threshold=16)`` / ``LzfDecoder()`` — LzfEncoder.java / LzfDecoder.java

Encoders follow ``MessageToByteEncoder.write`` (MessageToByteEncoder.java:99-131): one call per
outbound message, empty output replaced by an empty buffer.  Decoders follow
``ByteToMessageDecoder.channelRead`` (ByteToMessageDecoder.java:286-341): inbound bytes are
cumulated, ``decode`` runs until it stops making progress, consumed bytes are discarded, and a
failure raises ``DecompressionException`` and leaves the decoder corrupted (all later input is
skipped).  The per-chunk work runs in libnetty_amd.so (HIP kernels); headers are parsed by the
native host layer exactly as the Java decode() does.
"""
from __future__ import annotations

import ctypes as C

from . import _lib


class DecoderException(Exception):
    """io.netty.handler.codec.DecoderException"""


class EncoderException(Exception):
    """io.netty.handler.codec.EncoderException"""


class DecompressionException(DecoderException):
    """DecompressionException.java:23"""


class IllegalStateException(Exception):
    """java.lang.IllegalStateException (Lz4FrameEncoder.encode after close, Lz4FrameEncoder.java:233-239)"""


class CompressionException(EncoderException):
    """CompressionException.java:23"""


def _new(handle, what):
    if not handle:
        raise RuntimeError(f"{what}: native handle creation failed (no GPU visible, or invalid options); "
                           f"the HIP path has no CPU fallback")
    return handle


class _Encoder:
    """MessageToByteEncoder<ByteBuf> template (MessageToByteEncoder.java:99-160)."""

    _free = None

    def encode(self, data: bytes) -> bytes:  # pragma: no cover - overridden
        raise NotImplementedError

    def write(self, msg) -> bytes:
        return self.encode(bytes(msg))

    def close(self):
        if getattr(self, "_h", None):
            getattr(_lib.load(), self._free)(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Decoder:
    """ByteToMessageDecoder template (ByteToMessageDecoder.java:286-341, callDecode :464-517)."""

    _free = None
    _decode_fn = None

    def __init__(self):
        self._cum = bytearray()

    def channel_read(self, data) -> list[bytes]:
        L = _lib.load()
        self._cum += bytes(data)
        buf = bytes(self._cum)
        consumed = C.c_size_t(0)
        msgs = C.POINTER(_lib.NxMsg)()
        nmsg = C.c_size_t(0)
        err = C.c_char_p()
        rc = getattr(L, self._decode_fn)(self._h, buf, len(buf), C.byref(consumed), C.byref(msgs), C.byref(nmsg),
                                         C.byref(err))
        out = [C.string_at(msgs[i].data, msgs[i].len) if msgs[i].len else b"" for i in range(nmsg.value)]
        del self._cum[:consumed.value]
        if rc != 0:
            if rc in (-100, -101, -102, -103):
                raise RuntimeError(f"{type(self).__name__}: native failure {rc} ({_lib.status_string(rc)})")
            msg = err.value.decode() if err.value else _lib.status_string(rc)
            # a ByteBuf failure (IndexOutOfBounds / IllegalArgument) reaches the pipeline as the
            # DecoderException ByteToMessageDecoder wraps it in (ByteToMessageDecoder.java:297-300)
            e = DecoderException(msg) if msg.startswith("java.lang.") else DecompressionException(msg)
            e.decoded = out  # messages fired before the failing chunk
            e.status = rc
            raise e
        return out

    def readable_bytes(self) -> int:
        return len(self._cum)

    def close(self):
        if getattr(self, "_h", None):
            getattr(_lib.load(), self._free)(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------------------------- Snappy
class SnappyFrameEncoder(_Encoder):
    """SnappyFrameEncoder.java:29-153 — 32767-byte slices (65535 with jumbo frames)."""

    _free = "nx_snappy_frame_encoder_free"

    def __init__(self, jumbo: bool = False):
        self._h = _new(_lib.load().nx_snappy_frame_encoder_new(1 if jumbo else 0), "SnappyFrameEncoder")

    @classmethod
    def snappy_encoder_with_jumbo_frames(cls) -> "SnappyFrameEncoder":
        return cls(jumbo=True)

    def encode(self, data: bytes) -> bytes:
        L = _lib.load()
        cap = L.nx_snappy_frame_max_encoded_length(len(data))
        out = (C.c_uint8 * max(cap, 1))()
        n = L.nx_snappy_frame_encoder_encode(self._h, data, len(data), out, cap)
        if n < 0:
            raise CompressionException(_lib.status_string(n))
        return bytes(out[:n])


class SnappyFrameDecoder(_Decoder):
    """SnappyFrameDecoder.java:37-259 (validateChecksums defaults to false, :67-69)."""

    _free = "nx_snappy_frame_decoder_free"
    _decode_fn = "nx_snappy_frame_decoder_decode"

    def __init__(self, validate_checksums: bool = False):
        super().__init__()
        self._h = _new(_lib.load().nx_snappy_frame_decoder_new(1 if validate_checksums else 0), "SnappyFrameDecoder")


# Deprecated aliases kept by the reference (SnappyFramedEncoder.java:22, SnappyFramedDecoder.java:22)
SnappyFramedEncoder = SnappyFrameEncoder
SnappyFramedDecoder = SnappyFrameDecoder


# ------------------------------------------------------------------------------------- FastLZ
LEVEL_AUTO, LEVEL_1, LEVEL_2 = 0, 1, 2


class FastLzFrameEncoder(_Encoder):
    """FastLzFrameEncoder.java:45-173.  ``reader_index`` of encode() reproduces the readU16 quirk."""

    _free = "nx_fastlz_frame_encoder_free"

    def __init__(self, level: int = LEVEL_AUTO, checksum: bool = False):
        if level not in (LEVEL_AUTO, LEVEL_1, LEVEL_2):
            raise ValueError(f"level: {level} (expected: {LEVEL_AUTO} or {LEVEL_1} or {LEVEL_2})")
        self._h = _new(_lib.load().nx_fastlz_frame_encoder_new(level, 1 if checksum else 0), "FastLzFrameEncoder")

    def encode(self, data: bytes, reader_index: int = 0, buffer: bytes | None = None) -> bytes:
        """Encode ``data``; if ``buffer``/``reader_index`` are given, data = buffer[reader_index:]."""
        L = _lib.load()
        if buffer is None:
            buffer, reader_index = bytes(reader_index) + bytes(data), reader_index
        n = len(buffer) - reader_index
        cap = L.nx_fastlz_frame_max_encoded_length(n)
        out = (C.c_uint8 * max(cap, 1))()
        r = L.nx_fastlz_frame_encoder_encode(self._h, bytes(buffer), reader_index, n, out, cap)
        if r < 0:
            raise CompressionException(_lib.status_string(r))
        return bytes(out[:r])


class FastLzFrameDecoder(_Decoder):
    """FastLzFrameDecoder.java:36-208."""

    _free = "nx_fastlz_frame_decoder_free"
    _decode_fn = "nx_fastlz_frame_decoder_decode"

    def __init__(self, validate_checksums: bool = False):
        super().__init__()
        self._h = _new(_lib.load().nx_fastlz_frame_decoder_new(1 if validate_checksums else 0), "FastLzFrameDecoder")


# ------------------------------------------------------------------------------------- LZF
class LzfEncoder(_Encoder):
    """LzfEncoder.java:36-253: LzfEncoder(totalLength = MAX_CHUNK_LEN, compressThreshold = 16)
    (:111-166).  total_length is validated as the reference does and does not change the bytes
    (include/netty_amd.h, nx_lzf_encoder_new_ex)."""

    _free = "nx_lzf_encoder_free"
    MAX_CHUNK_LEN = 65535  # LZFChunk.MAX_CHUNK_LEN
    MIN_BLOCK_TO_COMPRESS = 16  # LzfEncoder.java:42

    def __init__(self, compress_threshold: int = 16, total_length: int = MAX_CHUNK_LEN):
        if total_length < 16 or total_length > 65535:  # :147-150
            raise ValueError(f"totalLength: {total_length} (expected: 16-65535)")
        if compress_threshold < 16:  # :152-156
            raise ValueError(f"compressThreshold:{compress_threshold} expected >=16")
        self._h = _new(_lib.load().nx_lzf_encoder_new_ex(total_length, compress_threshold), "LzfEncoder")

    def encode(self, data: bytes) -> bytes:
        L = _lib.load()
        cap = L.nx_lzf_frame_max_encoded_length(len(data))
        out = (C.c_uint8 * max(cap, 1))()
        r = L.nx_lzf_encoder_encode(self._h, data, len(data), out, cap)
        if r < 0:
            raise CompressionException(_lib.status_string(r))
        return bytes(out[:r])


class LzfDecoder(_Decoder):
    """LzfDecoder.java:40-242."""

    _free = "nx_lzf_decoder_free"
    _decode_fn = "nx_lzf_decoder_decode"

    def __init__(self):
        super().__init__()
        self._h = _new(_lib.load().nx_lzf_decoder_new(), "LzfDecoder")


class Lz4FrameEncoder(_Encoder):
    """Lz4FrameEncoder.java:61-403 (XXHash32 seed 0x9747b28c).  high_compressor selects lz4-java's
    highCompressor() (liblz4 LZ4_compress_HC level 9) over fastCompressor() (:121-125,161-163);
    max_encode_size is the maxEncodeSize constructor argument (:150-170, default Integer.MAX_VALUE).
    encode() returns the full blocks it flushed (a partial block stays buffered, :231-248); flush()
    writes the partial block (:296-304); finish_encode() = close(): flush + end block (:306-330).
    encode() and flush() raise EncoderException when the pending bytes' output would exceed
    max_encode_size (allocateBuffer, :190-214), leaving the encoder unchanged."""

    _free = "nx_lz4_frame_encoder_free"
    MAX_ENCODE_SIZE = (1 << 31) - 1  # DEFAULT_MAX_ENCODE_SIZE (:68)

    def __init__(self, block_size: int = 1 << 16, high_compressor: bool = False, max_encode_size: int = MAX_ENCODE_SIZE):
        if not 64 <= block_size <= 1 << 25:
            raise ValueError(f"blockSize: {block_size} (expected: 64-{1 << 25})")
        if max_encode_size <= 0:  # ObjectUtil.checkPositive (:168)
            raise ValueError(f"maxEncodeSize : {max_encode_size} (expected: > 0)")
        self.block_size = block_size
        self.high_compressor = bool(high_compressor)
        self.max_encode_size = int(max_encode_size)
        self._h = _new(_lib.load().nx_lz4_frame_encoder_new_ex(block_size, int(self.high_compressor), self.max_encode_size),
                       "Lz4FrameEncoder")

    def _out(self, n: int):
        cap = _lib.load().nx_lz4_frame_max_encoded_length(n, self.block_size)
        return (C.c_uint8 * cap)(), cap

    def raise_for(self, r):
        """the reference's exception for a handle status: NX_ERR_LZ4_ENCODE_SIZE (-58) is allocateBuffer's
        EncoderException, NX_ERR_LZ4_ENCODE_FINISHED (-59) encode's IllegalStateException after close"""
        if r == -58:
            raise EncoderException(_lib.load().nx_lz4_frame_encoder_error(self._h).decode())
        if r == -59:
            raise IllegalStateException(_lib.load().nx_lz4_frame_encoder_error(self._h).decode())

    def _ret(self, r, out) -> bytes:
        self.raise_for(r)
        if r < 0:
            raise CompressionException(_lib.status_string(r))
        return bytes(out[:r])

    def encode(self, data: bytes) -> bytes:
        out, cap = self._out(len(data) + self.block_size)
        return self._ret(_lib.load().nx_lz4_frame_encoder_encode(self._h, data, len(data), out, cap), out)

    def flush(self) -> bytes:
        out, cap = self._out(self.block_size)
        return self._ret(_lib.load().nx_lz4_frame_encoder_flush(self._h, out, cap), out)

    def finish_encode(self) -> bytes:
        out, cap = self._out(self.block_size)
        return self._ret(_lib.load().nx_lz4_frame_encoder_close(self._h, out, cap), out)


class Lz4FrameDecoder(_Decoder):
    """Lz4FrameDecoder.java:36-277 (validateChecksums default false, :100-102)."""

    _free = "nx_lz4_frame_decoder_free"
    _decode_fn = "nx_lz4_frame_decoder_decode"

    def __init__(self, validate_checksums: bool = False):
        super().__init__()
        self._h = _new(_lib.load().nx_lz4_frame_decoder_new(int(validate_checksums)), "Lz4FrameDecoder")


# ------------------------------------------------------------------------------------- harness
class EmbeddedChannel:
    """The subset of io.netty.channel.embedded.EmbeddedChannel the codec tests use
    (EmbeddedChannel.java:337-483): one handler, outbound/inbound message queues."""

    def __init__(self, handler):
        self.handler = handler
        self._outbound: list[bytes] = []
        self._inbound: list[bytes] = []

    def write_outbound(self, *msgs) -> bool:
        for m in msgs:
            # MessageToByteEncoder.write: empty output is replaced by EMPTY_BUFFER (:112-117)
            self._outbound.append(self.handler.write(m))
        return bool(self._outbound)

    def write_inbound(self, *msgs) -> bool:
        for m in msgs:
            self._inbound.extend(self.handler.channel_read(m))
        return bool(self._inbound)

    def read_outbound(self):
        return self._outbound.pop(0) if self._outbound else None

    def read_inbound(self):
        return self._inbound.pop(0) if self._inbound else None

    def finish(self) -> bool:
        return bool(self._outbound or self._inbound)


class Batcher:
    """Asynchronous cross-channel batching executor (include/netty_amd.h section 3, csrc/batcher.cpp):
    encode()/decode() calls of many SnappyFrameEncoder / SnappyFrameDecoder instances become jobs of
    one GPU launch per flush().  submit_* never touches the GPU; poll() never blocks."""

    def __init__(self, flush_bytes: int = 0):
        self._h = _new(_lib.load().nx_batcher_new(), "Batcher")
        if flush_bytes:
            self.set_flush_bytes(flush_bytes)

    def set_flush_bytes(self, n: int):
        """Auto-flush once the collecting batch holds n input bytes (0 = only flush())."""
        _lib.load().nx_batcher_set_flush_bytes(self._h, n)

    def close(self):
        if self._h:
            _lib.load().nx_batcher_free(self._h)
            self._h = None

    __del__ = close

    def reserve(self, kinds: int = 0x1F):
        """Hold the device workspaces of the given kinds now (bit NX_WS_* per kind; default all), so no
        submit pays for them (nx_batcher_reserve)."""
        r = _lib.load().nx_batcher_reserve(self._h, kinds)
        if r != 0:
            raise RuntimeError(f"nx_batcher_reserve: {_lib.status_string(r)}")

    def reserve_arenas(self, nbatches: int, staging_bytes: int, out_bytes: int):
        """Size the pinned arenas now (nx_batcher_reserve_arenas): submits then never allocate."""
        r = _lib.load().nx_batcher_reserve_arenas(self._h, nbatches, staging_bytes, out_bytes)
        if r != 0:
            raise RuntimeError(f"nx_batcher_reserve_arenas: {_lib.status_string(r)}")

    def arena_stats(self) -> dict:
        a, n = C.c_uint64(0), C.c_uint64(0)
        k = C.c_uint32(0)
        _lib.load().nx_batcher_arena_stats(self._h, C.byref(a), C.byref(n), C.byref(k))
        return {"allocs": a.value, "bytes": n.value, "batches": k.value}

    def _ticket(self, t, what):
        if t < 0:
            raise RuntimeError(f"{what}: {_lib.status_string(t)}")
        return t

    def submit_encode(self, encoder, data, registered_ptr: int | None = None, reader_index: int = 0, op: int = 0) -> int:
        """encode() of any encoder handler as a job: SnappyFrameEncoder (with registered_ptr, an address
        inside memory passed to register(), the bytes are DMA'd from there at flush and must stay valid
        until completion), FastLzFrameEncoder (``reader_index`` as in encode()), LzfEncoder,
        Lz4FrameEncoder (``op`` 0 encode, 1 encode + flush, 2 encode + close)."""
        L = _lib.load()
        if isinstance(encoder, FastLzFrameEncoder):
            buf = bytes(reader_index) + bytes(data)
            return self._ticket(L.nx_fastlz_frame_encoder_submit(encoder._h, self._h, buf, reader_index, len(data)),
                                "nx_fastlz_frame_encoder_submit")
        if isinstance(encoder, LzfEncoder):
            buf = bytes(data)
            return self._ticket(L.nx_lzf_encoder_submit(encoder._h, self._h, buf, len(buf)), "nx_lzf_encoder_submit")
        if isinstance(encoder, Lz4FrameEncoder):
            buf = bytes(data)
            t = L.nx_lz4_frame_encoder_submit(encoder._h, self._h, buf, len(buf), op)
            encoder.raise_for(t)
            return self._ticket(t, "nx_lz4_frame_encoder_submit")
        if registered_ptr is not None:
            t = L.nx_snappy_frame_encoder_submit(encoder._h, self._h, C.c_void_p(registered_ptr), len(data), 1)
        else:
            buf = bytes(data)
            t = L.nx_snappy_frame_encoder_submit(encoder._h, self._h, buf, len(buf), 0)
        if t < 0:
            raise RuntimeError(f"nx_snappy_frame_encoder_submit: {_lib.status_string(t)}")
        return t

    _DECODE_SUBMIT = {"SnappyFrameDecoder": "nx_snappy_frame_decoder_submit",
                      "FastLzFrameDecoder": "nx_fastlz_frame_decoder_submit",
                      "LzfDecoder": "nx_lzf_decoder_submit",
                      "Lz4FrameDecoder": "nx_lz4_frame_decoder_submit"}

    def submit_decode(self, decoder, data) -> int:
        """decode() of any decoder handler over its cumulation + data as a job; the consumed bytes leave
        the cumulation now (ByteToMessageDecoder.channelRead)."""
        L = _lib.load()
        fn = next(v for k, v in self._DECODE_SUBMIT.items() if type(decoder).__name__ == k or
                  any(c.__name__ == k for c in type(decoder).__mro__))
        decoder._cum += bytes(data)
        buf = bytes(decoder._cum)
        consumed = C.c_size_t(0)
        t = self._ticket(getattr(L, fn)(decoder._h, self._h, buf, len(buf), C.byref(consumed)), fn)
        del decoder._cum[:consumed.value]
        return t

    def submit_decode_registered(self, decoder: "SnappyFrameDecoder", ptr: int, n: int) -> tuple[int, int]:
        """SnappyFrameDecoder.decode over a cumulation the caller holds in registered memory
        (register()): nothing is copied; bytes [ptr, ptr + consumed) must stay valid until the job
        completes.  Returns (ticket, consumed); the caller discards the consumed bytes afterwards."""
        consumed = C.c_size_t(0)
        t = _lib.load().nx_snappy_frame_decoder_submit_registered(decoder._h, self._h, C.c_void_p(ptr), n, C.byref(consumed))
        if t < 0:
            raise RuntimeError(f"nx_snappy_frame_decoder_submit_registered: {_lib.status_string(t)}")
        return t, consumed.value

    def flush(self):
        r = _lib.load().nx_batcher_flush(self._h)
        if r != 0:
            raise RuntimeError(f"nx_batcher_flush: {_lib.status_string(r)}")

    def poll(self, ticket: int) -> bool:
        r = _lib.load().nx_batcher_poll(self._h, ticket)
        if r < 0:
            raise RuntimeError(f"nx_batcher_poll: {_lib.status_string(r)}")
        return r == 1

    def wait(self, ticket: int):
        r = _lib.load().nx_batcher_wait(self._h, ticket)
        if r != 0:
            raise RuntimeError(f"nx_batcher_wait: {_lib.status_string(r)}")

    def result(self, ticket: int, release: bool = True):
        """The job's messages (list of bytes); a failed decoder job raises like decode() would, with
        the messages decoded before the failure attached as .decoded."""
        L = _lib.load()
        msgs = C.POINTER(_lib.NxMsg)()
        n = C.c_size_t(0)
        err = C.c_char_p()
        rc = L.nx_batcher_result(self._h, ticket, C.byref(msgs), C.byref(n), C.byref(err))
        out = [C.string_at(msgs[i].data, msgs[i].len) if msgs[i].len else b"" for i in range(n.value)]
        if release:
            L.nx_batcher_release(self._h, ticket)
        if rc != 0:
            if rc in (-100, -101, -102, -103):
                raise RuntimeError(f"Batcher: native failure {rc} ({_lib.status_string(rc)})")
            msg = err.value.decode() if err.value else _lib.status_string(rc)
            e = DecoderException(msg) if msg.startswith("java.lang.") else DecompressionException(msg)
            e.decoded = out
            raise e
        return out

    def stats(self) -> dict:
        f, l_, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        _lib.load().nx_batcher_stats(self._h, C.byref(f), C.byref(l_), C.byref(c))
        df, db = C.c_uint64(0), C.c_uint64(0)
        _lib.load().nx_batcher_dma_stats(self._h, C.byref(df), C.byref(db))
        return {"flushes": f.value, "launches": l_.value, "chunks": c.value, "dma_flushes": df.value, "dma_bytes": db.value}

    @staticmethod
    def register(ptr: int, n: int):
        r = _lib.load().nx_host_register(C.c_void_p(ptr), n)
        if r != 0:
            raise RuntimeError(f"nx_host_register: {_lib.status_string(r)}")

    @staticmethod
    def unregister(ptr: int):
        _lib.load().nx_host_unregister(C.c_void_p(ptr))
