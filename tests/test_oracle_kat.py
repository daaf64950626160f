"""Pins the CPU oracle (oracle/netty_oracle.c) to the reference's own known-answer vectors
(tests/golden/kat.json, transcribed from codec-compression/src/test/... with file:line tags) and to
the reference's round-trip/edge-case corpora (AbstractIntegrationTest.java:77-158)."""
import pytest

ST = {"OFFSET_ZERO": -2, "OFFSET_NEGATIVE": -3, "OFFSET_BEYOND": -4, "PREAMBLE_TOO_LONG": -1, "OVERFLOW": -5}


def test_crc32c_kats(kat, oracle):
    for v in kat["crc32c"]:
        assert oracle.crc32c(bytes.fromhex(v["in"])) == v["crc"], v["src"]
    for v in kat["masked_checksum"]:
        assert oracle.snappy_checksum(bytes.fromhex(v["in"])) == v["masked"], v["src"]
    # SnappyTest.java:250-258 compares calculateChecksum with maskChecksum(0xd6cb8b55)
    assert oracle.snappy_checksum(b"netty") == oracle.mask_checksum(0xd6cb8b55)


def test_snappy_encode_kats(kat, oracle):
    for v in kat["snappy_encode"]:
        assert oracle.snappy_encode(bytes.fromhex(v["in"])).hex() == v["out"], v["src"]


def test_snappy_decode_kats(kat, oracle):
    for v in kat["snappy_decode"]:
        st, out, _ = oracle.snappy_decode(bytes.fromhex(v["in"]))
        want = v["status"] if isinstance(v["status"], int) else ST[v["status"]]
        assert st == want, v["src"]
        if st == 0:
            assert out.hex() == v["out"], v["src"]


def test_snappy_literal_length_classes(kat, oracle):
    # SnappyTest.java:298-324: encodeLiteral/decodeLiteral for each length-code class (60..63)
    for n in kat["snappy_literal_lengths"]["lengths"]:
        if n <= 20:
            continue
        # a literal-only block: preamble + one literal of n zero bytes (what encodeLiteral emits)
        nb = (n - 1).bit_length()
        nbytes = 1 + (nb - 1) // 8 if n > 60 else 0
        tag = bytes([(59 + nbytes) << 2]) + (n - 1).to_bytes(nbytes, "little") if n > 60 else bytes([(n - 1) << 2])
        pre = bytearray()
        v = n
        while v >= 0x80:
            pre.append((v & 0x7F) | 0x80)
            v >>= 7
        pre.append(v)
        st, out, _ = oracle.snappy_decode(bytes(pre) + tag + bytes(n), out_cap=1 << 26)
        assert st == 0 and out == bytes(n)


def test_snappy_frame_encode_kats(kat, oracle):
    for v in kat["snappy_frame_encode"]:
        started = False
        got = b""
        for m in v["msgs"]:
            out, started = oracle.snappy_frame_encode(bytes.fromhex(m), started=started)
            got += out
        assert got.hex() == v["out"], v["src"]


def test_java_random(kat, oracle):
    v = kat["java_random"]
    assert oracle.java_random_bytes(v["seed"], 4).hex() == v["first4"]


def _identity_corpus(oracle):
    rnd1m = oracle.java_random_bytes(42, 1 << 20)
    part = bytearray(oracle.java_random_bytes(7, 10240))
    part[:1024] = b"\x02" * 1024
    comp = bytearray(10240)
    r = oracle.java_random_bytes(9, 10240)
    for i in range(10240):
        comp[i] = r[i] if i % 4 == 0 else 0
    return {
        "empty": b"", "one": b"A", "two": b"BA",
        "regular": b"Netty is a NIO client server framework which enables quick and easy development of network "
                   b"applications such as protocol servers and clients.",
        "large_random": rnd1m, "part_random": bytes(part), "compressible": bytes(comp),
        "long_blank": bytes(102400), "long_same": bytes([123]) * 102400, "sequential": bytes(i & 0xFF for i in range(1024)),
    }


def test_snappy_roundtrip_corpus(oracle, kat):
    corpus = _identity_corpus(oracle)
    corpus["issue_1002"] = bytes.fromhex(kat["identity_inputs"]["issue_1002"])
    for name, data in corpus.items():
        for L in {min(len(data), 65536), min(len(data), 32767)}:
            blk = data[:L]
            enc = oracle.snappy_encode(blk)
            st, out, cons = oracle.snappy_decode(enc, out_cap=65536)
            assert st == 0 and out == blk and cons == len(enc), name


def test_snappy_seeded_regressions(oracle, kat):
    # SnappyIntegrationTest.java:73-108: 16 MiB java.util.Random(seed).nextBytes, framed round trip
    for seed in kat["identity_inputs"]["snappy_seeds"]:
        data = oracle.java_random_bytes(seed, 1 << 20)  # first 1 MiB of the 16 MiB stream
        for jumbo in (False, True):
            frames, _ = oracle.snappy_frame_encode(data, jumbo=jumbo)
            assert frames[:10] == bytes.fromhex("ff060000734e61507059")
            # walk frames and decode each chunk
            p, got = 10, bytearray()
            while p < len(frames):
                t, ln = frames[p], int.from_bytes(frames[p + 1:p + 4], "little")
                crc = int.from_bytes(frames[p + 4:p + 8], "little")
                payload = frames[p + 8:p + 4 + ln]
                if t == 0:
                    st, out, _ = oracle.snappy_decode(payload, 65536)
                    assert st == 0
                else:
                    out = payload
                assert oracle.snappy_checksum(out) == crc
                got += out
                p += 4 + ln
            assert bytes(got) == data


def test_snappy_truncation_and_errors(oracle):
    enc = oracle.snappy_encode(oracle.textgen_chunk(3, 4096))
    full = oracle.snappy_decode(enc, 65536)[1]
    for cut in (1, 2, 3, 10, len(enc) // 2, len(enc) - 1):
        st, out, cons = oracle.snappy_decode(enc[:cut], 65536)
        assert st == 0 and full.startswith(out) and cons <= cut  # silent partial (Snappy.java:352-354)
    # output overflow against the frame decoder's 65536 max capacity
    blk = bytes(70000)
    enc2 = oracle.snappy_encode(blk)
    assert oracle.snappy_decode(enc2, 65536)[0] == -5
    # code-63 literal length 0x7FFFFFFF → negative Java int → error; 0xFFFFFFFF → zero-length literal
    assert oracle.snappy_decode(bytes([0x05, 63 << 2, 0xFF, 0xFF, 0xFF, 0x7F]))[0] == -6
    st, out, _ = oracle.snappy_decode(bytes([0x05, 63 << 2, 0xFF, 0xFF, 0xFF, 0xFF, 0x10]) + b"netty")
    assert st == 0 and out == b"netty"
    # COPY_4 with bit 31 set → OFFSET_NEGATIVE
    assert oracle.snappy_decode(bytes([0x0a, 0x10]) + b"netty" + bytes([0x13, 0, 0, 0, 0x80]))[0] == -3


def test_fastlz_roundtrip_and_quirk(oracle):
    import random
    rng = random.Random(5)
    for level in (1, 2):
        for n in (4, 5, 31, 32, 33, 100, 4096, 65535):
            for kind in ("text", "rand", "zero", "runs"):
                if kind == "text":
                    data = oracle.textgen_chunk(n, n)
                elif kind == "rand":
                    data = bytes(rng.getrandbits(8) for _ in range(n))
                elif kind == "zero":
                    data = bytes(n)
                else:
                    data = bytes((i // 7) & 3 for i in range(n))
                c = oracle.fastlz_compress(data, level)
                r, out = oracle.fastlz_decompress(c, len(data))
                assert r == len(data) and out == data, (level, n, kind)
    # readU16 quirk at LEVEL_2: a degenerate limit corrupts a "qqqr" run
    data = b"abcdefghijklmnop" + b"qqqr" + b"stuvwxyz0123456789"
    good = oracle.fastlz_compress(data, 2, u16_limit=len(data))
    assert oracle.fastlz_decompress(good, len(data))[1] == data
    bad = oracle.fastlz_compress(data, 2, u16_limit=0)
    assert oracle.fastlz_decompress(bad, len(data))[1] != data


def test_fastlz_frame_autolevel(oracle):
    data = oracle.textgen_chunk(11, 70000)
    fr = oracle.fastlz_frame_encode(data, level=0, checksum=True)
    assert fr[:3] == b"FLZ" and fr[3] == 0x11
    assert int.from_bytes(fr[4:8], "big") == oracle.adler32(data[:65535])
    import zlib
    assert oracle.adler32(data) == zlib.adler32(data)


def test_lzf_roundtrip(oracle):
    for n in (16, 17, 100, 4096, 65535):
        for data in (oracle.textgen_chunk(n + 1, n), bytes(n), bytes((i * 7) & 0xFF for i in range(n))):
            blk = oracle.lzf_encode_chunk(data)
            assert blk[:2] == b"ZV"
            if blk[2] == 1:
                clen, ulen = int.from_bytes(blk[3:5], "big"), int.from_bytes(blk[5:7], "big")
                st, out = oracle.lzf_decode_chunk(blk[7:7 + clen], ulen)
                assert st == 0 and out == data
            else:
                assert blk[5:] == data
    # corrupt: back-reference before the output start
    assert oracle.lzf_decode_chunk(bytes([0x20, 0x05]), 3)[0] == -30


class _LzfEncoderPy:
    """Second, independent restatement of compress-lzf 1.0.3 (ChunkEncoder.tryCompress /
    appendEncodedChunk, LZFEncoder.appendEncoded) as one LzfEncoder drives it (Java int arithmetic
    spelled out; the table persists across messages, LzfEncoder.java:57,161-163,219) to cross-check the
    C oracle's transcription (parity unpinned vs the library itself, which is not available offline)."""

    def __init__(self, threshold=16):
        self.ht = [0] * 16384
        self.threshold = threshold

    @staticmethod
    def _i32(x):
        x &= 0xFFFFFFFF
        return x - (1 << 32) if x >= 1 << 31 else x

    def _try_compress(self, inp, pos0, n):
        i32, ht = self._i32, self.ht

        def jhash(h):  # ((h * 57321) >> 9) & _hashModulo, _hashModulo = 16383
            return (i32(h * 57321) >> 9) & 16383

        def first(p):  # (in[p] << 8) + (in[p + 1] & 0xFF), in[] signed
            b = inp[p] - 256 if inp[p] >= 128 else inp[p]
            return i32((b << 8) + inp[p + 1])

        out = bytearray(2 * n + 64)
        ip, op, lit, in_end = pos0, 1, 0, pos0 + n - 4
        seen = first(ip)
        while ip < in_end:
            p2 = inp[ip + 2]
            seen = i32((seen << 8) + p2)
            h = jhash(seen)
            ref = ht[h]
            ht[h] = ip
            off = ip - ref
            if (ref >= ip or ref < pos0 or off > 8192 or inp[ref + 2] != p2 or inp[ref + 1] != (seen >> 8) & 255
                    or inp[ref] != (seen >> 16) & 255):
                out[op] = inp[ip]
                op, ip, lit = op + 1, ip + 1, lit + 1
                if lit == 32:
                    out[op - 33] = 31
                    lit, op = 0, op + 1
                continue
            max_len = min(264, in_end - ip + 2)
            if lit == 0:
                op -= 1
            else:
                out[op - lit - 1] = lit - 1
                lit = 0
            ln = 3
            while ln < max_len and inp[ref + ln] == inp[ip + ln]:
                ln += 1
            ln, off = ln - 2, off - 1
            if ln < 7:
                out[op] = ((off >> 8) + (ln << 5)) & 255
                op += 1
            else:
                out[op], out[op + 1] = ((off >> 8) + (7 << 5)) & 255, ln - 7
                op += 2
            out[op] = off & 255
            op += 2
            ip += ln
            seen = i32((first(ip) << 8) + inp[ip + 2])
            ht[jhash(seen)] = ip
            ip += 1
            seen = i32((seen << 8) + inp[ip + 2])
            ht[jhash(seen)] = ip
            ip += 1
        while ip < pos0 + n:  # handleTail
            out[op] = inp[ip]
            op, ip, lit = op + 1, ip + 1, lit + 1
            if lit == 32:
                out[op - lit - 1] = lit - 1
                lit, op = 0, op + 1
        if lit:
            out[op - lit - 1] = lit - 1
        else:
            op -= 1
        return bytes(out[:op])

    def encode(self, inp):
        res, p = bytearray(), 0
        while True:
            n = min(65535, len(inp) - p)
            chunk = inp[p:p + n]
            body = self._try_compress(inp, p, n) if len(inp) >= self.threshold and n >= 16 else None
            if body is not None and len(body) + 7 < n + 5:
                res += b"ZV\x01" + len(body).to_bytes(2, "big") + n.to_bytes(2, "big") + body
            else:
                res += b"ZV\x00" + n.to_bytes(2, "big") + chunk
            p += n
            if p >= len(inp):
                return bytes(res)


def test_lzf_encoder_restatements_agree(oracle):
    import random
    r = random.Random(7)
    cases = [oracle.textgen_chunk(3, 6000), bytes(3000), bytes(r.randrange(4) for _ in range(4000)),
             bytes(r.randrange(256) for _ in range(999)), b"ab" * 700 + bytes(range(256)) * 3,
             bytes(r.randrange(3) | 0x80 for _ in range(2000)), bytes(16), b"abc" + b"xyz" * 30 + b"abcd" * 40]
    for c in cases:
        assert oracle.lzf_compress_body(c) == _LzfEncoderPy()._try_compress(c, 0, len(c))


def test_lzf_encoder_state_across_messages(oracle):
    """One LzfEncoder over many messages: its ChunkEncoder table persists (LzfEncoder.java:57,161-163,
    219), restated by the C oracle (orc_lzf_encoder_*) and the independent Python class above.  Both
    agree message by message, and every message equals a FRESH encoder's bytes: an entry left by an
    earlier message (or chunk) can never pass tryCompress's 3-byte check before this chunk has written
    that slot itself, because the first occurrence of every trigram in a chunk is written to the table
    (a probe, or one of the two inserts after a match; a position skipped inside a match repeats an
    earlier occurrence).  So the batch kernels' per-chunk fresh tables are exact for a long-lived
    encoder too (netty_oracle.c, lzf.hip)."""
    import random
    r = random.Random(11)
    msgs = []
    for trial in range(30):
        words = [bytes(r.randrange(97, 100) for _ in range(r.randrange(2, 6))) for _ in range(8)]
        base = b" ".join(r.choice(words) for _ in range(r.randrange(20, 500)))
        msgs += [base, base, base[7:], base[:100] + b"#" + base[100:]]
    msgs += [oracle.textgen_chunk(9, 70000), oracle.textgen_chunk(9, 65535 + 40), oracle.textgen_chunk(9, 70000)[3:],
             bytes(15), bytes(5000), b"ab" * 9000]
    enc, py = oracle.LzfEncoderState(16), _LzfEncoderPy(16)
    for i, m in enumerate(msgs):
        got = enc.encode(m)
        assert got == py.encode(m), i
        assert got == oracle.lzf_frame_encode(m, 16), i


def test_textgen_deterministic(oracle):
    a = oracle.textgen_chunk(0, 65536)
    assert a == oracle.textgen_chunk(0, 65536) and a != oracle.textgen_chunk(1, 65536)
    r = len(oracle.snappy_encode(a)) / 65536
    assert 0.40 < r < 0.52  # Netty ratio on the text-like chunks ≈ 0.46


def test_snappy_frame_scan_kats(kat, oracle):
    """The frame-scan restatement against SnappyFrameDecoderTest's streams: every expected exception
    is a scan error or (validating decoders) a checksum mismatch; every expected message is a listed
    chunk whose payload decodes to it."""
    for v in kat["snappy_frame_decode"]:
        buf = bytes.fromhex(v["in"])
        ents, consumed, state, status = oracle.snappy_frame_scan(buf)
        msgs, failed = [], status < 0
        for typ, off, ln, crc in ents:
            payload = buf[off:off + ln]
            if typ == 0:
                st, out, _ = oracle.snappy_decode(payload, 65536)
                failed |= st < 0
            else:
                out = payload
            if v.get("validate") and oracle.snappy_checksum(out) != crc:
                failed = True
            msgs.append(out.hex())
        if v.get("error"):
            assert failed, v["src"]
        else:
            assert not failed and status == 0 and consumed == len(buf), v["src"]
            assert msgs == v["msgs"], v["src"]
        assert bool(state & 2) == (status < 0)


def test_snappy_frame_scan_partial_and_skip(oracle):
    framed, _ = oracle.snappy_frame_encode(oracle.textgen_chunk(3, 70000))
    skippable = bytes([0xFE, 10, 0, 0]) + bytes(10)
    buf = framed + skippable + framed[10:]
    full = oracle.snappy_frame_scan(buf)
    per = len(oracle.snappy_frame_scan(framed)[0])
    assert full[3] == 0 and full[1] == len(buf) and len(full[0]) == 2 * per > 2
    for cut in (3, 10, 11, 25, len(framed) - 1, len(framed) + 6):
        e1, c1, s1, r1 = oracle.snappy_frame_scan(buf[:cut])
        assert r1 == 0 and c1 <= cut
        e2, c2, s2, r2 = oracle.snappy_frame_scan(buf[c1:], s1)
        assert r2 == 0 and c1 + c2 == len(buf)
        assert [(t, o + c1, n, c) for t, o, n, c in e2] == [(t, o, n, c) for t, o, n, c in full[0][len(e1):]]
    e, c, s, r = oracle.snappy_frame_scan(buf, cap=1)
    assert r == oracle.SCAN_LIST_FULL and len(e) == 1 and not s & 2


def test_lz4_block_roundtrip_and_errors(oracle):
    """LZ4 block restatement: round trips and the malformed-input cases the GPU decoder must agree on."""
    import random
    rng = random.Random(4)
    for data in [b"", b"a", b"hello", bytes(100), oracle.textgen_chunk(1, 65536), oracle.java_random_bytes(2, 5000),
                 bytes((i % 7) for i in range(70000)), bytes(rng.getrandbits(8) for _ in range(300))]:
        blk = oracle.lz4_compress(data)
        assert oracle.lz4_decompress(blk, len(data)) == (0, data)
    assert oracle.lz4_decompress(b"\x50hello", 5) == (0, b"hello")
    # sequences: literal 'a' then a 4-byte match at offset 1, then the literal tail "bcdef"
    assert oracle.lz4_decompress(b"\x10a\x01\x00\x50bcdef", 10) == (0, b"aaaaabcdef")
    bad = [(b"", 0), (b"\x50hell", 5), (b"\x50hello", 4), (b"\x50hello", 6), (b"\x10a\x00\x00\x50bcdef", 10),
           (b"\x10a\x02\x00\x50bcdef", 10), (b"\x10a\x01", 10), (b"\xf0", 20), (b"\xf0\xff", 300)]
    for blk, n in bad:
        assert oracle.lz4_decompress(blk, n)[0] == -50, (blk, n)


def _lz4_corpus(oracle):
    import random
    rng = random.Random(5)
    corpus = dict(_identity_corpus(oracle))
    corpus.update({"hello": b"hello", "min_len_12": b"abcdabcdabcd", "min_len_13": b"abcdabcdabcda",
                   "period7": bytes((i % 7) for i in range(70000)), "blank_64k": bytes(65536)})
    for k, n in enumerate([17, 100, 4095, 4096, 32767, 65535, 65536, 65546, 65547, 65548, 131072, 300000]):
        corpus[f"text_{n}"] = oracle.textgen_chunk(1000 + k, n)
    for k, n in enumerate([13, 64, 1000, 65536, 70000]):
        corpus[f"random_{n}"] = rng.randbytes(n)
    for k in range(12):
        corpus[f"text_rand_{k}"] = oracle.textgen_chunk(2000 + k, rng.randrange(1, 70000))
    return corpus


def test_lz4_compress_equals_liblz4(oracle):
    """The LZ4 block compressor is liblz4's LZ4_compress_default, the compressor lz4-java's JNI
    fastCompressor() runs for Lz4FrameEncoder (Lz4FrameEncoder.java:125,163,273): byte-for-byte
    equal to pyarrow's bundled liblz4 (Codec('lz4_raw')) on both table types (byU16 below
    65547 bytes, byU32 above), random and text data, and the end-of-block limits."""
    pa = pytest.importorskip("pyarrow")
    z = pa.Codec("lz4_raw")
    for name, data in _lz4_corpus(oracle).items():
        assert oracle.lz4_compress(data) == z.compress(data).to_pybytes(), name
        assert oracle.lz4_decompress(oracle.lz4_compress(data), len(data)) == (0, data), name


def test_lz4hc_compress_equals_liblz4_level9(oracle):
    """Lz4FrameEncoder(highCompressor = true) compresses with lz4-java's highCompressor(), liblz4's
    LZ4_compress_HC at its default level 9 (Lz4FrameEncoder.java:123-125,161-163): the oracle's
    restatement of the hash-chain match finder (256 candidates, pattern analysis) and the lazy
    three-match parse is byte-for-byte equal to pyarrow's bundled liblz4 at compression_level=9 on the
    LZ4 corpus (text, random, runs, short periods, every end-of-block limit) plus repeated 1-, 2-, 3-
    and 4-byte patterns that drive the pattern analysis, and round-trips through the decoder."""
    pa = pytest.importorskip("pyarrow")
    z = pa.Codec("lz4_raw", compression_level=9)
    corpus = _lz4_corpus(oracle)
    corpus.update({"run_a": b"a" * 5000, "period2": b"ab" * 5000, "period3": b"abc" * 4000, "period4": b"abcd" * 4000,
                   "runs_mixed": (b"x" * 300 + b"yz" * 200 + oracle.textgen_chunk(9, 777)) * 20,
                   "period5_200k": bytes((i % 5) for i in range(200000))})
    for name, data in corpus.items():
        hc = oracle.lz4hc_compress(data)
        assert hc == z.compress(data).to_pybytes(), name
        assert oracle.lz4_decompress(hc, len(data)) == (0, data), name


# The liblz4 the LZ4 / LZ4 HC pins above ran against: pyarrow 25.0.0's libarrow carries
# liblz4's LZ4_VERSION_STRING "1.10.0" (liblz4 exports no version call there, so it is read from the
# library's strings).  Lz4FrameEncoder's lz4-java 1.8.0 bundles liblz4 1.9.3: the pins assume the fast
# compressor and HC level 9 kept their output from 1.9.3 to 1.10.0 (1.10's level changes were to HC
# levels 1-2), so parity with lz4-java's own bytes is "parity unpinned" by a 1.9.3 run.
LZ4_PIN_LIBRARY = "liblz4 1.10.0 (pyarrow 25.0.0)"


def test_lz4_pin_library_version_recorded():
    pa = pytest.importorskip("pyarrow")
    import glob
    import os
    import re
    libs = glob.glob(os.path.join(os.path.dirname(pa.__file__), "libarrow.so.*"))
    assert libs
    blob = open(sorted(libs)[0], "rb").read()
    versions = set(re.findall(rb"\x00(1\.(?:9|10|11)\.\d+)\x00", blob))
    want = LZ4_PIN_LIBRARY.split()[1].encode()
    assert want in versions, (versions, "pyarrow's bundled liblz4 changed: re-check the LZ4 pins and LZ4_PIN_LIBRARY")
    assert pa.__version__ in LZ4_PIN_LIBRARY


def test_snappy_blocks_decode_with_libsnappy(oracle, kat):
    """Independent decode cross-check: pyarrow's bundled libsnappy decodes every
    Netty-format block the oracle encodes (Netty's encoder output differs from libsnappy's, so this
    checks the format, not the encoder's choices, which the SnappyTest KATs pin)."""
    pa = pytest.importorskip("pyarrow")
    sn = pa.Codec("snappy")
    corpus = _identity_corpus(oracle)
    corpus["issue_1002"] = bytes.fromhex(kat["identity_inputs"]["issue_1002"])
    for i in range(8):
        corpus[f"text_{i}"] = oracle.textgen_chunk(i, 65536)
    for name, data in corpus.items():
        for L in {min(len(data), 65536), min(len(data), 32767), min(len(data), 65535)}:
            blk = data[:L]
            enc = oracle.snappy_encode(blk)
            assert sn.decompress(enc, decompressed_size=L).to_pybytes() == blk, (name, L)


# ---- LZ4 frame (§8f row 4): Lz4FrameEncoder / Lz4FrameDecoder / Lz4XXHash32 ----
# Lz4FrameDecoderTest.java:33-41: "Netty" as one non-compressed block, then the end block.
LZ4_DECODER_TEST_DATA = bytes([0x4C, 0x5A, 0x34, 0x42, 0x6C, 0x6F, 0x63, 0x6B, 0x16,
                               0x05, 0, 0, 0, 0x05, 0, 0, 0, 0x86, 0xE4, 0x79, 0x0F,
                               0x4E, 0x65, 0x74, 0x74, 0x79,
                               0x4C, 0x5A, 0x34, 0x42, 0x6C, 0x6F, 0x63, 0x6B, 0x16] + [0] * 12)


def test_xxhash32_against_independent_implementation(oracle):
    """The XXH32 restatement equals python-xxhash (an independent implementation of the published
    algorithm lz4-java 1.8.0 implements) on every tail length and several seeds."""
    xxhash = pytest.importorskip("xxhash")
    import random
    rng = random.Random(3)
    for n in list(range(0, 70)) + [255, 256, 1000, 4097, 65536]:
        d = bytes(rng.getrandbits(8) for _ in range(n))
        for seed in (0, 0x9747B28C, 0xFFFFFFFF, 1):
            assert oracle.xxhash32(d, seed) == xxhash.xxh32_intdigest(d, seed), (n, seed)
    assert oracle.xxhash32(b"", 0) == 0x02CC5D05


def test_lz4_frame_encoder_matches_decoder_test_vector(oracle):
    assert oracle.lz4_checksum(b"Netty") == 0x0F79E486
    assert oracle.lz4_compression_level(1 << 16) == 6  # token 0x16 = NON_COMPRESSED | 6
    assert oracle.lz4_frame_encode(b"Netty") == LZ4_DECODER_TEST_DATA


def test_lz4_frame_scan_decoder_test_cases(oracle):
    """Lz4FrameDecoderTest.java:50-147: each corrupted byte maps to its exception."""
    ents, p, st, res = oracle.lz4_frame_scan(LZ4_DECODER_TEST_DATA)
    assert (ents, p, st, res) == ([(0x10, 21, 5, 5, 0x0F79E486)], len(LZ4_DECODER_TEST_DATA), 1, 0)
    E = oracle.LZ4_ERR
    for idx, val, err in [(1, 0x00, "bad_magic"), (12, 0xFF, "compressed_length"), (16, 0xFF, "decompressed_length"),
                          (13, 0x01, "length_mismatch"), (8, 0x36, "block_type"), (44, 0x01, "end_checksum")]:
        d = bytearray(LZ4_DECODER_TEST_DATA)
        d[idx] = val
        ents, p, st, res = oracle.lz4_frame_scan(bytes(d))
        assert res == E[err] and st & 2, (idx, err, res)
    # data[17] = 0x01: "mismatching checksum" is raised by the checksum check on the decoded block
    d = bytearray(LZ4_DECODER_TEST_DATA)
    d[17] = 0x01
    ents, _, _, res = oracle.lz4_frame_scan(bytes(d))
    assert res == 0 and ents[0][4] != oracle.lz4_checksum(b"Netty")


def test_lz4_frame_roundtrip_and_partial(oracle):
    data = oracle.textgen_chunk(9, 200000) + oracle.java_random_bytes(2, 70000)
    f = oracle.lz4_frame_encode(data)
    ents, p, st, res = oracle.lz4_frame_scan(f)
    assert res == 0 and st == 1 and p == len(f)
    out = b""
    for bt, off, cl, dl, chk in ents:
        blk = f[off:off + cl]
        dec = blk if bt == 0x10 else oracle.lz4_decompress(blk, dl)[1]
        assert oracle.lz4_checksum(dec) == chk
        out += dec
    assert out == data
    assert {e[0] for e in ents} == {0x10, 0x20}
    # a cut inside a payload stops at that block's header; resuming from there finishes the walk
    cut = ents[2][1] + 100
    e1, p1, st1, r1 = oracle.lz4_frame_scan(f[:cut])
    assert (len(e1), p1, st1, r1) == (2, ents[2][1] - 21, 0, 0)
    e2, p2, st2, r2 = oracle.lz4_frame_scan(f[p1:], st1, cap=1)
    assert r2 == oracle.SCAN_LIST_FULL and len(e2) == 1
    # after the end block everything readable is discarded (FINISHED)
    assert oracle.lz4_frame_scan(b"junk", 1) == ([], 4, 1, 0)
