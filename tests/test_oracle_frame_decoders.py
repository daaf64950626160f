"""The oracle's frame-decoder restatements (oracle/frame_decoders.py) on CPU: the reference's own
decoder tests (SnappyFrameDecoderTest, LzfDecoderTest, Lz4FrameDecoderTest), the ByteBuf failures of
short chunks, sticky corruption, the validating-mode leftover re-parse, and round trips of every
framing through random read splits.  The GPU handles and the batcher are checked against these in
tests/test_gpu_frame_fuzz.py."""
import random
import zlib

import pytest

from oracle import frame_decoders as F

SID = bytes.fromhex("ff060000734e61507059")


def test_snappy_frame_decoder_kats(kat):
    """SnappyFrameDecoderTest.java:50-199 through the restated decode() loop."""
    for v in kat["snappy_frame_decode"]:
        d = F.SnappyFrameDecoder(v.get("validate", False))
        if v.get("error"):
            with pytest.raises(F.DecompressionException):
                d.channel_read(bytes.fromhex(v["in"]))
        else:
            assert [m.hex() for m in d.channel_read(bytes.fromhex(v["in"]))] == v["msgs"], v["src"]


def test_snappy_decoder_corrupted_is_sticky():
    d = F.SnappyFrameDecoder()
    with pytest.raises(F.DecompressionException):
        d.channel_read(bytes([0x03, 0x01, 0x00, 0x00, 0x00]))
    assert d.channel_read(bytes.fromhex("ff060000734e61507059010900006f982eb96e65747479")) == []


@pytest.mark.parametrize("validate", [False, True])
def test_snappy_decoder_chunk_shorter_than_checksum(validate):
    """The same expectations as tests/test_gpu_handlers.py's test of the GPU handle."""
    tail = b"\x00" * 8
    with pytest.raises(F.DecoderException) as ei:
        F.SnappyFrameDecoder(validate).channel_read(SID + b"\x01\x02\x00\x00ab" + tail)
    if validate:
        assert isinstance(ei.value, F.DecompressionException)
        assert str(ei.value) == "mismatching checksum: a282ead8 (expected: 6261)"
    else:
        assert not isinstance(ei.value, F.DecompressionException)
        assert str(ei.value) == "java.lang.IllegalArgumentException: minimumReadableBytes : -2 (expected: >= 0)"
    with pytest.raises(F.DecoderException) as ei:
        F.SnappyFrameDecoder(validate).channel_read(SID + b"\x00\x01\x00\x00a" + tail)
    assert not isinstance(ei.value, F.DecompressionException)
    assert str(ei.value).startswith("java.lang.IndexOutOfBoundsException" if validate else
                                    "java.lang.IllegalArgumentException: minimumReadableBytes : -3")
    with pytest.raises(F.DecoderException) as ei:
        F.SnappyFrameDecoder(validate).channel_read(SID + b"\x00\x01\x00\x00a")
    assert str(ei.value) == "java.lang.IndexOutOfBoundsException: readerIndex(14) + length(4) exceeds writerIndex(15)"


def test_snappy_decoder_negative_literal_length(oracle):
    """A code-63 literal whose Java int length + 1 is negative: out.writeBytes(in, length) fails in
    ensureWritable's argument check (IllegalArgumentException, wrapped as DecoderException)."""
    body = b"\x05" + bytes([63 << 2]) + (0xFFFFFFF0).to_bytes(4, "little") + b"xyz"
    crc = oracle.snappy_checksum(b"")
    chunk = b"\x00" + (len(body) + 4).to_bytes(3, "little") + crc.to_bytes(4, "little") + body
    for validate in (False, True):
        with pytest.raises(F.DecoderException) as ei:
            F.SnappyFrameDecoder(validate).channel_read(SID + chunk)
        assert not isinstance(ei.value, F.DecompressionException)
        assert str(ei.value) == "java.lang.IllegalArgumentException: minWritableBytes : -15 (expected: >= 0)"


def test_snappy_validating_leftover_is_reparsed(oracle):
    """SnappyFrameDecoder.java:205-212: a validating decoder reads the chunk through `in` itself, so a
    compressed chunk whose block ends early (preamble 0) leaves the rest to be parsed as the next chunk
    header; the non-validating decoder slices the whole chunk."""
    inner = b"\x01\x09\x00\x00" + oracle.snappy_checksum(b"hello").to_bytes(4, "little") + b"hello"  # an UNCOMPRESSED chunk
    payload = b"\x00" + inner  # preamble 0: decode() returns at once, consuming 1 byte
    crc = oracle.snappy_checksum(b"")
    chunk = b"\x00" + (len(payload) + 4).to_bytes(3, "little") + crc.to_bytes(4, "little") + payload
    assert F.SnappyFrameDecoder(True).channel_read(SID + chunk) == [b"", b"hello"]
    assert F.SnappyFrameDecoder(False).channel_read(SID + chunk) == [b""]


def test_snappy_skippable_across_reads(oracle):
    """RESERVED_SKIPPABLE longer than the bytes at hand (SnappyFrameDecoder.java:137-151, 91-99)."""
    data = oracle.textgen_chunk(4, 5000)
    fr, _ = oracle.snappy_frame_encode(data)
    skip = b"\x80" + (300).to_bytes(3, "little") + bytes(300)
    s = fr[:10] + skip + fr[10:]
    for cut in (11, 14, 100, 313, 314, 320):
        msgs, err = F.run(F.SnappyFrameDecoder(True), [s[:cut], s[cut:]])
        assert err is None and b"".join(msgs) == data, cut


def test_lzf_decoder_tests():
    """LzfDecoderTest.java:39-68."""
    with pytest.raises(F.DecompressionException, match="unexpected block identifier"):
        F.LzfDecoder().channel_read(b"\x12\x34\x00\x00\x00")
    with pytest.raises(F.DecompressionException, match="unknown type of chunk"):
        F.LzfDecoder().channel_read(b"ZV\xff\x00\x00\x00\x00")
    d = F.LzfDecoder()
    with pytest.raises(F.DecompressionException):
        d.channel_read(b"ZV\x05\x00\x00")
    assert d.channel_read(b"ZV\x00\x00\x01a") == []  # CORRUPTED skips (:229-231)


def test_lz4_frame_decoder_tests(oracle):
    """Lz4FrameDecoderTest.java:50-147 through the restated decoder (validating)."""
    from test_oracle_kat import LZ4_DECODER_TEST_DATA as D
    assert F.Lz4FrameDecoder(True).channel_read(D) == [b"Netty"]
    cases = [(1, 0x00, "unexpected block identifier"), (12, 0xFF, "invalid compressedLength"),
             (16, 0xFF, "invalid decompressedLength"), (13, 0x01, "stream corrupted: compressedLength"),
             (8, 0x36, "unexpected blockType"), (44, 0x01, "stream corrupted: checksum error"),
             (17, 0x01, "stream corrupted: mismatching checksum")]
    for idx, val, msg in cases:
        d = bytearray(D)
        d[idx] = val
        with pytest.raises(F.DecompressionException) as ei:
            F.Lz4FrameDecoder(True).channel_read(bytes(d))
        assert str(ei.value).startswith(msg), (idx, str(ei.value))
    # the end block finishes the stream: later bytes are skipped (:250-254)
    dec = F.Lz4FrameDecoder(True)
    assert dec.channel_read(D + b"junk after the end") == [b"Netty"]
    assert dec.channel_read(b"more") == []


def test_fastlz_decoder_errors(oracle):
    """FastLzFrameDecoder.java:121-124 (magic), :160-164 (length mismatch), :171-180 (checksum)."""
    with pytest.raises(F.DecompressionException, match="unexpected block identifier"):
        F.FastLzFrameDecoder().channel_read(b"FLY\x00\x00\x00")
    data = oracle.textgen_chunk(8, 3000)
    fr = oracle.fastlz_frame_encode(data, level=1, checksum=True)
    assert F.FastLzFrameDecoder(True).channel_read(fr) == [data]
    bad = bytearray(fr)
    bad[5] ^= 1  # the Adler32
    with pytest.raises(F.DecompressionException, match="mismatching checksum"):
        F.FastLzFrameDecoder(True).channel_read(bytes(bad))
    assert F.FastLzFrameDecoder(False).channel_read(bytes(bad)) == [data]
    bad = bytearray(fr)
    bad[11] ^= 0x40  # originalLength
    with pytest.raises(F.DecompressionException, match=r"originalLength\(\d+\) and actual length"):
        F.FastLzFrameDecoder(False).channel_read(bytes(bad))


def _split(rng, s, n):
    cuts = sorted(rng.randrange(0, len(s) + 1) for _ in range(n - 1))
    return [s[a:c] for a, c in zip([0] + cuts, cuts + [len(s)])]


@pytest.mark.parametrize("codec", ["snappy", "snappy_jumbo", "fastlz1", "fastlz2", "lzf", "lz4"])
def test_round_trips_over_read_splits(oracle, codec):
    """Oracle encoder → oracle decoder, every read split: the messages concatenate to the input."""
    rng = random.Random(zlib.crc32(codec.encode()))
    for k in range(6):
        data = oracle.textgen_chunk(k, rng.choice((1, 100, 5000, 70000))) + oracle.java_random_bytes(k, rng.randint(0, 3000))
        if codec.startswith("snappy"):
            s, _ = oracle.snappy_frame_encode(data, jumbo=codec.endswith("jumbo"))
            dec = F.SnappyFrameDecoder(True)
        elif codec.startswith("fastlz"):
            if codec == "fastlz2":  # level 2 corrupts messages of more than one chunk (readU16 quirk)
                data = data[:65535]
            s = oracle.fastlz_frame_encode(data, level=int(codec[-1]), checksum=bool(k & 1))
            dec = F.FastLzFrameDecoder(True)
        elif codec == "lzf":
            s = oracle.lzf_frame_encode(data)
            dec = F.LzfDecoder()
        else:
            s = oracle.lz4_frame_encode(data)
            dec = F.Lz4FrameDecoder(True)
        msgs, err = F.run(dec, _split(rng, s, rng.randint(1, 6)))
        assert err is None and b"".join(msgs) == data, (codec, k)
