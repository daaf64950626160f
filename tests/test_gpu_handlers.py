"""GPU tests of the handler layer — the reference's own handler-level tests restated:
SnappyFrameEncoderTest / SnappyFrameDecoderTest KATs, AbstractIntegrationTest round trips
(EmbeddedChannel identity), FastLzIntegrationTest's random small writes, LZF round trips, and
frame-level byte parity with the oracle's restatement of the Java encoders."""
import random

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nx():
    import netty_amd
    return netty_amd


def _corpus(oracle, kat):
    rnd1m = oracle.java_random_bytes(42, 1 << 20)
    part = bytearray(oracle.java_random_bytes(7, 10240))
    part[:1024] = b"\x02" * 1024
    comp = bytearray(10240)
    r = oracle.java_random_bytes(9, 10240)
    for i in range(0, 10240, 4):
        comp[i] = r[i]
    return {
        "empty": b"", "one": b"A", "two": b"BA",
        "regular": bytes.fromhex(kat["identity_inputs"]["regular"]),
        "large_random": rnd1m, "part_random": bytes(part), "compressible": bytes(comp),
        "long_blank": bytes(102400), "long_same": bytes([123]) * 102400,
        "sequential": bytes(i & 0xFF for i in range(1024)),
        "issue_1002": bytes.fromhex(kat["identity_inputs"]["issue_1002"]),
        "text": oracle.textgen_chunk(5, 300000),
    }


def _identity(nx, enc, dec, data):
    """AbstractIntegrationTest.testIdentity (AbstractIntegrationTest.java:160-189)."""
    ech = nx.EmbeddedChannel(enc)
    assert ech.write_outbound(data)
    compressed = b""
    while (m := ech.read_outbound()) is not None:
        compressed += m
    dch = nx.EmbeddedChannel(dec)
    dch.write_inbound(compressed)
    assert dec.readable_bytes() == 0  # assertFalse(compressed.isReadable())
    out = b""
    while (m := dch.read_inbound()) is not None:
        out += m
    assert out == data
    return compressed


def test_snappy_frame_encoder_kats(nx, kat):
    for v in kat["snappy_frame_encode"]:
        ch = nx.EmbeddedChannel(nx.SnappyFrameEncoder())
        for m in v["msgs"]:
            ch.write_outbound(bytes.fromhex(m))
        got = b""
        while (m := ch.read_outbound()) is not None:
            got += m
        assert got.hex() == v["out"], v["src"]


def test_snappy_frame_decoder_kats(nx, kat):
    for v in kat["snappy_frame_decode"]:
        ch = nx.EmbeddedChannel(nx.SnappyFrameDecoder(v.get("validate", False)))
        if v.get("error"):
            with pytest.raises(nx.DecompressionException):
                ch.write_inbound(bytes.fromhex(v["in"]))
        else:
            ch.write_inbound(bytes.fromhex(v["in"]))
            got = []
            while (m := ch.read_inbound()) is not None:
                got.append(m.hex())
            assert got == v["msgs"], v["src"]


def test_snappy_decoder_corrupted_is_sticky(nx):
    d = nx.SnappyFrameDecoder()
    ch = nx.EmbeddedChannel(d)
    with pytest.raises(nx.DecompressionException):
        ch.write_inbound(bytes([0x03, 0x01, 0x00, 0x00, 0x00]))
    # SnappyFrameDecoder.java:86-89: once corrupted, all input is skipped
    assert not ch.write_inbound(bytes.fromhex("ff060000734e61507059010900006f982eb96e65747479"))


SID = bytes.fromhex("ff060000734e61507059")


@pytest.mark.parametrize("validate", [False, True])
def test_snappy_decoder_chunk_shorter_than_checksum(nx, validate):
    """A data chunk whose length is below its 4-byte checksum is no DecompressionException in the
    reference: readIntLE / skipBytes run past the chunk and the negative slice length fails inside
    ByteBuf (SnappyFrameDecoder.java:171-178, 194-215), which ByteToMessageDecoder wraps in a
    DecoderException (ByteToMessageDecoder.java:297-300).  Heap-buffer messages."""
    tail = b"\x00" * 8  # bytes after the short chunk, so the 4-byte reads succeed
    # UNCOMPRESSED_DATA of length 2: readRetainedSlice(-2) (with validation the empty CRC differs first)
    with pytest.raises(nx.DecoderException) as ei:
        nx.EmbeddedChannel(nx.SnappyFrameDecoder(validate)).write_inbound(SID + b"\x01\x02\x00\x00ab" + tail)
    if validate:
        assert isinstance(ei.value, nx.DecompressionException)
        assert str(ei.value) == "mismatching checksum: a282ead8 (expected: 6261)"
    else:
        assert not isinstance(ei.value, nx.DecompressionException)
        assert str(ei.value) == "java.lang.IllegalArgumentException: minimumReadableBytes : -2 (expected: >= 0)"
    # COMPRESSED_DATA of length 1: readSlice(-3), or writerIndex below readerIndex when validating
    with pytest.raises(nx.DecoderException) as ei:
        nx.EmbeddedChannel(nx.SnappyFrameDecoder(validate)).write_inbound(SID + b"\x00\x01\x00\x00a" + tail)
    assert not isinstance(ei.value, nx.DecompressionException)
    assert str(ei.value).startswith("java.lang.IndexOutOfBoundsException" if validate else
                                    "java.lang.IllegalArgumentException: minimumReadableBytes : -3")
    # too few bytes after the header for the 4-byte checksum read: IndexOutOfBoundsException
    with pytest.raises(nx.DecoderException) as ei:
        nx.EmbeddedChannel(nx.SnappyFrameDecoder(validate)).write_inbound(SID + b"\x00\x01\x00\x00a")
    assert str(ei.value) == "java.lang.IndexOutOfBoundsException: readerIndex(14) + length(4) exceeds writerIndex(15)"


@pytest.mark.parametrize("jumbo", [False, True])
def test_snappy_identity_and_parity(nx, oracle, kat, jumbo):
    for name, data in _corpus(oracle, kat).items():
        comp = _identity(nx, nx.SnappyFrameEncoder(jumbo=jumbo), nx.SnappyFrameDecoder(), data)
        want, _ = oracle.snappy_frame_encode(data, jumbo=jumbo)
        assert comp == want, name
        # and the validating decoder accepts it
        d = nx.SnappyFrameDecoder(True)
        assert b"".join(d.channel_read(comp)) == data


def test_snappy_seeded_regressions(nx, oracle, kat):
    # SnappyIntegrationTest.java:73-108 (16 MiB java.util.Random(seed).nextBytes)
    for seed in kat["identity_inputs"]["snappy_seeds"]:
        data = oracle.java_random_bytes(seed, 16 << 20)
        comp = _identity(nx, nx.SnappyFrameEncoder(), nx.SnappyFrameDecoder(), data)
        assert comp == oracle.snappy_frame_encode(data)[0]


def test_snappy_streaming_partial_writes(nx, oracle):
    # AbstractDecoderTest/FastLzIntegrationTest style: inbound bytes arrive in random small pieces
    data = oracle.textgen_chunk(21, 200000)
    comp = oracle.snappy_frame_encode(data)[0]
    rng = random.Random(3)
    for validate in (False, True):
        d = nx.SnappyFrameDecoder(validate)
        out, p = b"", 0
        while p < len(comp):
            k = rng.randint(1, 4000)
            out += b"".join(d.channel_read(comp[p:p + k]))
            p += k
        assert out == data and d.readable_bytes() == 0


def test_snappy_decoder_skippable_split(nx):
    # RESERVED_SKIPPABLE whose body arrives in pieces (numBytesToSkip, SnappyFrameDecoder.java:91-99,137-150)
    stream = bytes.fromhex("ff060000734e61507059") + bytes([0x80, 10, 0, 0]) + b"0123456789" + \
        bytes.fromhex("010900006f982eb96e65747479")
    d = nx.SnappyFrameDecoder(True)
    got = []
    for piece in (stream[:16], stream[16:20], stream[20:]):
        got += d.channel_read(piece)
    assert got == [b"netty"]


@pytest.mark.parametrize("level,checksum", [(0, False), (1, False), (0, True), (1, True)])
def test_fastlz_identity(nx, oracle, kat, level, checksum):
    # FastLzIntegrationTest uses LEVEL_AUTO (FastLzFrameEncoder(boolean)), which is level 1 for every
    # <= 65535-byte chunk (FastLz.java:99-103)
    for name, data in _corpus(oracle, kat).items():
        comp = _identity(nx, nx.FastLzFrameEncoder(level, checksum), nx.FastLzFrameDecoder(checksum), data)
        assert comp == oracle.fastlz_frame_encode(data, level=level, checksum=checksum), name


def _oracle_fastlz_frames_decode(oracle, fr):
    p, out = 0, b""
    while p < len(fr):
        opt = fr[p + 3]
        p += 4 + (4 if opt & 0x10 else 0)
        clen = int.from_bytes(fr[p:p + 2], "big")
        p += 2
        olen = int.from_bytes(fr[p:p + 2], "big") if opt & 1 else clen
        p += 2 if opt & 1 else 0
        out += oracle.fastlz_decompress(fr[p:p + clen], olen)[1] if opt & 1 else fr[p:p + clen]
        p += clen
    return out


@pytest.mark.parametrize("checksum", [False, True])
def test_fastlz_level2_parity_including_readu16_corruption(nx, oracle, kat, checksum):
    """LEVEL_2 through FastLzFrameEncoder: for chunk k >= 1 of a large message readU16's
    `offset + 1 >= readableBytes()` test (FastLz.java:552-557) degenerates, and the level-2 run
    check then emits wrong runs — the reference corrupts such messages.  The GPU path must
    reproduce the reference bytes, corruption included."""
    for name, data in _corpus(oracle, kat).items():
        want = oracle.fastlz_frame_encode(data, level=2, checksum=checksum)
        got = nx.FastLzFrameEncoder(2, checksum).encode(data)
        assert got == want, name
        dec = b"".join(nx.FastLzFrameDecoder(False).channel_read(got))
        assert dec == _oracle_fastlz_frames_decode(oracle, want), name
    big = oracle.textgen_chunk(5, 300000)
    assert _oracle_fastlz_frames_decode(oracle, oracle.fastlz_frame_encode(big, level=2)) != big  # the quirk is real


def test_fastlz_reader_index_quirk_parity(nx, oracle):
    # FastLz.readU16 uses readableBytes() of the message (FastLz.java:552-557): encode the same bytes
    # at different reader indices and with multi-chunk messages; bytes must match the restatement.
    data = oracle.textgen_chunk(8, 140000)
    for r0 in (0, 1, 1000):
        prefix = bytes(r0)
        for level in (1, 2):
            got = nx.FastLzFrameEncoder(level).encode(b"", reader_index=r0, buffer=prefix + data)
            assert got == oracle.fastlz_frame_encode(data, level=level, r0=r0), (r0, level)


def test_fastlz_random_small_writes(nx, oracle):
    # FastLzIntegrationTest.java:64-113: encoder input and decoder input split into random pieces
    rng = random.Random(11)
    data = oracle.textgen_chunk(2, 50000)
    enc = nx.FastLzFrameEncoder(0, True)
    comp = b""
    p = 0
    while p < len(data):
        k = rng.randint(1, 99)
        comp += enc.encode(data[p:p + k])
        p += k
    dec = nx.FastLzFrameDecoder(True)
    out, p = b"", 0
    while p < len(comp):
        k = rng.randint(1, 99)
        out += b"".join(dec.channel_read(comp[p:p + k]))
        p += k
    assert out == data


def test_fastlz_decoder_errors(nx, oracle):
    with pytest.raises(nx.DecompressionException, match="unexpected block identifier"):
        nx.FastLzFrameDecoder().channel_read(b"XYZ\x00\x00\x01a")
    good = oracle.fastlz_frame_encode(oracle.textgen_chunk(1, 5000), level=1, checksum=True)
    bad = bytearray(good)
    bad[4] ^= 0xFF  # checksum byte
    with pytest.raises(nx.DecompressionException, match="mismatching checksum"):
        nx.FastLzFrameDecoder(True).channel_read(bytes(bad))
    # the checksum is ignored by a decoder built without one (FastLzFrameDecoder.java:171)
    assert b"".join(nx.FastLzFrameDecoder(False).channel_read(bytes(bad))) == oracle.textgen_chunk(1, 5000)


def test_lzf_encoder_messages_through_one_handle(nx, oracle):
    """Several repetitive messages through ONE LzfEncoder (its ChunkEncoder table persists across
    encode() calls, LzfEncoder.java:57,161-163,219): each message's bytes equal the stateful oracle's
    (orc_lzf_encoder_*), and the decoder restores every message."""
    import random
    r = random.Random(23)
    words = [bytes(r.randrange(97, 101) for _ in range(r.randrange(2, 6))) for _ in range(10)]
    base = b" ".join(r.choice(words) for _ in range(3000))
    msgs = [base, base, base[5:], base[:999] + b"!" + base[999:], oracle.textgen_chunk(4, 140000), base * 30]
    enc, st, dec = nx.LzfEncoder(16), oracle.LzfEncoderState(16), nx.LzfDecoder()
    for i, m in enumerate(msgs):
        comp = enc.encode(m)
        assert comp == st.encode(m), i
        assert b"".join(dec.channel_read(comp)) == m, i


@pytest.mark.parametrize("threshold", [16, 1000])
def test_lzf_identity(nx, oracle, kat, threshold):
    for name, data in _corpus(oracle, kat).items():
        comp = _identity(nx, nx.LzfEncoder(threshold), nx.LzfDecoder(), data)
        assert comp == oracle.lzf_frame_encode(data, threshold), name


def test_lzf_decoder_errors(nx):
    with pytest.raises(nx.DecompressionException, match="unexpected block identifier"):
        nx.LzfDecoder().channel_read(b"AB\x00\x00\x01x")
    with pytest.raises(nx.DecompressionException, match="unknown type of chunk"):
        nx.LzfDecoder().channel_read(b"ZV\x07\x00\x01x")
    with pytest.raises(nx.DecompressionException):
        nx.LzfDecoder().channel_read(b"ZV\x01\x00\x02\x00\x05" + bytes([0x20, 0x05]))


# ---- LZ4 frame handlers (Lz4FrameEncoder / Lz4FrameDecoder over the GPU block + XXH32 kernels) ----
def _lz4_encode_all(enc, data, step=None):
    out = b""
    step = step or max(len(data), 1)
    for i in range(0, len(data), step):
        out += enc.encode(data[i:i + step])
    return out + enc.finish_encode()


@pytest.mark.parametrize("validate", [False, True])
def test_lz4_identity_and_parity(nx, oracle, kat, validate):
    """Lz4FrameIntegrationTest (AbstractIntegrationTest.testIdentity) over the shared corpus; the
    stream equals the oracle's Lz4FrameEncoder restatement byte for byte."""
    for name, data in _corpus(oracle, kat).items():
        enc, dec = nx.Lz4FrameEncoder(), nx.Lz4FrameDecoder(validate)
        comp = _lz4_encode_all(enc, data)
        assert comp == oracle.lz4_frame_encode(data), name
        dch = nx.EmbeddedChannel(dec)
        dch.write_inbound(comp)
        assert dec.readable_bytes() == 0
        out = b""
        while (m := dch.read_inbound()) is not None:
            out += m
        assert out == data, name


def test_lz4_decoder_test_vector_and_errors(nx):
    """Lz4FrameDecoderTest.java:33-147 with the reference's own stream and corrupted bytes."""
    from tests.test_oracle_kat import LZ4_DECODER_TEST_DATA as D
    assert nx.Lz4FrameDecoder(True).channel_read(D) == [b"Netty"]
    assert nx.Lz4FrameEncoder().encode(b"Netty") == b""  # buffered until flush / close
    e = nx.Lz4FrameEncoder()
    e.encode(b"Netty")
    assert e.finish_encode() == D
    for idx, val, msg in [(1, 0x00, "unexpected block identifier"), (12, 0xFF, "invalid compressedLength"),
                          (16, 0xFF, "invalid decompressedLength"), (13, 0x01, "mismatch"),
                          (8, 0x36, "unexpected blockType"), (17, 0x01, "mismatching checksum"),
                          (44, 0x01, "checksum error")]:
        d = bytearray(D)
        d[idx] = val
        with pytest.raises(nx.DecompressionException, match=msg):
            nx.Lz4FrameDecoder(True).channel_read(bytes(d))
    # without validateChecksums the flipped checksum is not noticed (Lz4FrameDecoder() default)
    d = bytearray(D)
    d[17] = 0x01
    assert nx.Lz4FrameDecoder().channel_read(bytes(d)) == [b"Netty"]


def test_lz4_streaming_partial_writes(nx, oracle):
    """Small writes into the encoder's block buffer and byte-dribbled reads give the same stream and data."""
    data = oracle.textgen_chunk(8, 200000) + oracle.java_random_bytes(4, 30000)
    comp = _lz4_encode_all(nx.Lz4FrameEncoder(), data, step=7777)
    assert comp == oracle.lz4_frame_encode(data)
    dec = nx.Lz4FrameDecoder(True)
    out = b""
    for i in range(0, len(comp), 5003):
        out += b"".join(dec.channel_read(comp[i:i + 5003]))
    assert out == data and dec.readable_bytes() == 0
    # after the end block the decoder is FINISHED and discards what follows
    assert dec.channel_read(b"garbage") == [] and dec.readable_bytes() == 0


def test_lz4_block_size_and_flush(nx, oracle):
    data = oracle.textgen_chunk(12, 10000)
    enc = nx.Lz4FrameEncoder(4096)
    comp = enc.encode(data[:5000]) + enc.flush() + enc.encode(data[5000:]) + enc.finish_encode()
    level = oracle.lz4_compression_level(4096)
    want = (oracle.lz4_frame_block(data[:4096], level) + oracle.lz4_frame_block(data[4096:5000], level)
            + oracle.lz4_frame_block(data[5000:9096], level) + oracle.lz4_frame_block(data[9096:], level)
            + oracle.lz4_frame_end(level))
    assert comp == want
    assert b"".join(nx.Lz4FrameDecoder(True).channel_read(comp)) == data


@pytest.mark.parametrize("block_size", [64, 4096, 1 << 16])
def test_lz4_encode_after_close(nx, block_size):
    """after close(), write()'s allocateBuffer(allowEmptyReturn = true) returns EMPTY_BUFFER
    when the message's blocks need fewer than blockSize bytes (Lz4FrameEncoder.java:216-218), and
    encode() then throws IllegalStateException (:233-239); a message whose blocks need at least
    blockSize bytes gets a buffer and passes through unchanged.  Both through the synchronous handle
    and as batcher jobs, and an empty message passes either way."""
    # smallest n with n + n / 255 + 16 + 21 >= blockSize (maxCompressedLength + HEADER_LENGTH)
    n_min = next(n for n in range(block_size + 1) if n + n // 255 + 37 >= block_size)
    small, big = b"s" * max(1, n_min - 1), bytes(range(256)) * (n_min // 256 + 1)
    big = big[:max(n_min, 1)]
    for path in ("sync", "batcher"):
        enc = nx.Lz4FrameEncoder(block_size)
        b = nx.Batcher() if path == "batcher" else None

        def run(data, op=0):
            if b is None:
                return enc.encode(data) if op == 0 else enc.encode(data) + enc.finish_encode()
            t = b.submit_encode(enc, data, op=op)
            b.flush()
            b.wait(t)
            return b.result(t)[0]

        run(b"x" * 10, op=2)  # closes the stream
        if block_size > 37:
            with pytest.raises(nx.IllegalStateException, match="encode finished and not enough space to write remaining data"):
                run(small)
        assert run(big) == big
        assert run(b"") == b""
        if b is not None:
            b.close()


def test_lzf_encoder_total_length_argument(nx, oracle):
    """LzfEncoder(totalLength, compressThreshold) (LzfEncoder.java:127-166): totalLength outside
    16..65535 is refused with the reference's message (:147-150); inside it the output is the default
    encoder's (the non-allocating ChunkEncoder sizes its table from max(totalLength, MAX_CHUNK_LEN))."""
    for bad in (15, 65536, -1):
        with pytest.raises(ValueError, match=f"totalLength: {bad} \\(expected: 16-65535\\)"):
            nx.LzfEncoder(total_length=bad)
    msgs = [oracle.textgen_chunk(i, n) for i, n in enumerate((20, 100, 5000, 70000))]
    for tl in (16, 100, 4096, 65535):
        e, ref = nx.LzfEncoder(total_length=tl), nx.LzfEncoder()
        for m in msgs:
            assert e.encode(m) == ref.encode(m) == oracle.lzf_frame_encode(m)
