"""HTTP content-coding hooks (netty_amd/http.py) against the reference's own
expectations.  Vectors are transcribed from codec-http/src/test/java/io/netty/handler/codec/http/
(file:line at each table)."""
import pytest

from netty_amd import http

# HttpContentCompressorTest.java:106-131 (default options: brotli, zstd, snappy, gzip, deflate)
DEFAULT = [("", None), (",", None), ("identity", None), ("unknown", None), ("*", "br"), ("br", "br"),
           ("br ; q=0.1", "br"), ("unknown, br", "br"), ("br, gzip", "br"), ("gzip, br", "br"),
           ("identity, br", "br"), ("gzip", "gzip"), ("gzip ; q=0.1", "gzip")]
# HttpContentCompressorOptionsTest.java:38-64, 66-91, 93-118 (all five options)
BR = [("", None), ("*", "br"), ("*;q=0.0", None), ("br", "br"), ("compress, br;q=0.5", "br"),
      ("br; q=0.5, identity", "br"), ("br; q=0, deflate", "br")]
ZSTD = [("", None), ("*;q=0.0", None), ("zstd", "zstd"), ("compress, zstd;q=0.5", "zstd"),
        ("zstd; q=0.5, identity", "zstd"), ("zstd; q=0, deflate", "zstd")]
SNAPPY = [("", None), ("*;q=0.0", None), ("snappy", "snappy"), ("compress, snappy;q=0.5", "snappy"),
          ("snappy; q=0.5, identity", "snappy"), ("snappy; q=0, deflate", "snappy")]


@pytest.mark.parametrize("accept,want", DEFAULT + BR + ZSTD + SNAPPY)
def test_determine_encoding_reference_vectors(accept, want):
    assert http.HttpContentCompressor().determine_encoding(accept) == want


def test_determine_encoding_snappy_only_and_q_parsing():
    c = http.HttpContentCompressor(br=False, zstd=False, gzip=False, deflate=False)
    assert c.determine_encoding("*") == "snappy"
    # a higher-q gzip blocks snappy even when gzip is not configured (:342 compares before :344 checks options)
    assert c.determine_encoding("gzip, snappy;q=0.2") is None
    assert c.determine_encoding("gzip;q=0.2, snappy") == "snappy"
    assert c.determine_encoding("snappy;q=abc") is None         # NumberFormatException → q = 0
    assert c.determine_encoding("snappy;q= 0.5f ") == "snappy"  # Float.parseFloat trims, takes the suffix
    c2 = http.HttpContentCompressor()
    assert c2.determine_encoding("gzip;q=0.5, snappy;q=0.5") == "snappy"  # snappyQ >= gzipQ
    assert c2.determine_encoding("gzip;q=0.6, snappy;q=0.5") == "gzip"
    assert c2.determine_encoding("snappy;q=0.1000000001, gzip;q=0.1") == "snappy"  # equal as float32


@pytest.mark.gpu
def test_snappy_content_decoder_and_encoder():
    import os
    import json
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))
    # HttpContentDecoderTest.java:57-60 SNAPPY_HELLO_WORLD body
    v = [x for x in kat["snappy_frame_decode"] if "HttpContentDecoderTest" in x["src"]][0]
    for name in ("snappy", "SNAPPY", "Snappy"):
        ch = http.new_content_decoder(name)
        assert ch is not None
        ch.write_inbound(bytes.fromhex(v["in"]))
        assert ch.read_inbound() == b"hello, world"
    assert http.new_content_decoder("gzip") is None
    enc, ch = http.HttpContentCompressor().new_content_encoder("snappy;q=0.9, gzip;q=0.5")
    assert enc == "snappy"
    body = b"hello, world " * 1000
    ch.write_outbound(body)
    dec = http.new_content_decoder(enc)
    dec.write_inbound(ch.read_outbound())
    got = b""
    while (m := dec.read_inbound()) is not None:
        got += m
    assert got == body


def _drain(handler, want_lasts, limit_s=60.0):
    """poll() until `want_lasts` LastHttpContent messages came out (poll never blocks)."""
    import time
    out, t0 = [], time.time()
    while sum(isinstance(m, http.LastHttpContent) for m in out) < want_lasts:
        out += handler.poll()
        assert time.time() - t0 < limit_s, "batcher jobs did not complete"
    return out


@pytest.mark.gpu
def test_nonblocking_snappy_http_bodies(oracle):
    """The non-blocking HTTP snappy path: per channel, a snappy response of
    several contents, an identity response and a second snappy response, all encoded by ONE batcher
    flush for every channel; each channel's messages come out in order, the framed bodies equal
    SnappyFrameEncoder's bytes (one encoder per response), and the decoder side restores the bodies
    with HttpContentDecoder's header rewriting."""
    import random
    from netty_amd.handlers import Batcher
    rng = random.Random(5)
    b = Batcher()
    chans = []
    for ch in range(6):
        parts = [oracle.textgen_chunk(ch * 10 + k, rng.randrange(0, 90000)) for k in range(3)] + [b""]
        plain = [b"identity body " * (ch + 1)]
        parts2 = [oracle.textgen_chunk(ch * 10 + 7, 5000)]
        enc = http.SnappyHttpBodyEncoder(b)
        enc.write(http.HttpMessage({"content-length": str(sum(map(len, parts)))}), encoding="snappy")
        for p in parts[:-1]:
            enc.write(http.HttpContent(p))
        enc.write(http.LastHttpContent(parts[-1], {"x-trailer": str(ch)}))
        enc.write(http.HttpMessage({"content-length": str(len(plain[0]))}))  # identity: passes through
        enc.write(http.LastHttpContent(plain[0]))
        enc.write(http.HttpMessage({}), encoding="snappy")
        enc.write(http.LastHttpContent(parts2[0]))
        chans.append((enc, parts, plain, parts2))
    b.flush()
    for enc, parts, plain, parts2 in chans:
        out = _drain(enc, 3)
        head = out[0]
        assert head.headers == {"content-encoding": "snappy", "transfer-encoding": "chunked"}
        want, started = [], False
        for p in parts:
            if p:
                want.append(oracle.snappy_frame_encode(p, started=started)[0])
                started = True
        i = 1
        got = []
        while not isinstance(out[i], http.LastHttpContent):
            got.append(out[i].content)
            i += 1
        assert got == want
        assert out[i].trailers == {"x-trailer": str(chans.index((enc, parts, plain, parts2)))}
        assert out[i + 1].headers == {"content-length": str(len(plain[0]))}
        assert out[i + 2] == http.LastHttpContent(plain[0])
        assert out[i + 3].headers["content-encoding"] == "snappy"
        assert out[i + 4].content == oracle.snappy_frame_encode(parts2[0])[0]
        assert isinstance(out[i + 5], http.LastHttpContent) and len(out) == i + 6
        # inbound: the framed body re-chunked at random points, Content-Encoding in another case
        body = b"".join(got)
        cuts = sorted(rng.randrange(0, len(body) + 1) for _ in range(4))
        pieces = [body[a:c] for a, c in zip([0] + cuts, cuts + [len(body)])]
        dec = http.SnappyHttpBodyDecoder(b, validate_checksums=True)
        dec.read(http.HttpMessage({"content-encoding": " Snappy ", "content-length": str(len(body))}))
        for p in pieces[:-1]:
            dec.read(http.HttpContent(p))
        dec.read(http.LastHttpContent(pieces[-1], {"t": "1"}))
        dec.read(http.HttpMessage({"content-length": "3"}))
        dec.read(http.LastHttpContent(b"abc"))
        b.flush()
        din = _drain(dec, 2)
        assert din[0].headers == {"transfer-encoding": "chunked"}
        k = 1
        dec_body = b""
        while not isinstance(din[k], http.LastHttpContent):
            assert din[k].content  # empty chunks are not forwarded (ByteBufForwarder)
            dec_body += din[k].content
            k += 1
        assert dec_body == b"".join(parts)
        assert din[k] == http.LastHttpContent(b"", {"t": "1"})
        assert din[k + 1].headers == {"content-length": "3"} and din[k + 2] == http.LastHttpContent(b"abc")


@pytest.mark.gpu
def test_nonblocking_snappy_http_corrupted_body_then_next_message(oracle):
    """A corrupted snappy body raises its DecompressionException once: the contents
    decoded before the failure come with it, the body's later contents decode to nothing and its
    LastHttpContent still ends the message, and the next message on the same channel comes out."""
    from netty_amd.handlers import Batcher, DecompressionException
    b = Batcher()
    good = oracle.textgen_chunk(3, 40000)
    framed, _ = oracle.snappy_frame_encode(good)
    c2 = 10 + 4 + int.from_bytes(framed[11:14], "little")  # the second chunk's header
    bad = bytearray(framed)
    bad[c2 + 8 + 20] ^= 0xFF  # damage the second chunk's payload
    first = bytes(bad[:c2 - 3])  # the stream identifier and most of the first chunk
    dec = http.SnappyHttpBodyDecoder(b, validate_checksums=True)
    dec.read(http.HttpMessage({"content-encoding": "snappy"}))
    dec.read(http.HttpContent(first))
    dec.read(http.HttpContent(bytes(bad[len(first):])))
    dec.read(http.HttpContent(b"more bytes after the failure"))
    dec.read(http.LastHttpContent(b"", {"t": "x"}))
    dec.read(http.HttpMessage({"content-length": "3"}))
    dec.read(http.LastHttpContent(b"abc"))
    b.flush()
    import time
    got, err, t0 = [], None, time.time()
    while sum(isinstance(m, http.LastHttpContent) for m in got) < 2:
        try:
            got += dec.poll()
        except DecompressionException as e:
            assert err is None, "the failure is raised once"
            err = e
            got += e.messages
        assert time.time() - t0 < 60
    assert err is not None and "checksum" in str(err)
    assert isinstance(got[0], http.HttpMessage)
    body = b"".join(m.content for m in got[1:] if type(m) is http.HttpContent)
    assert good.startswith(body) and len(body) >= 32767  # the first chunk's message came out
    lasts = [m for m in got if isinstance(m, http.LastHttpContent)]
    assert lasts[0].trailers == {"t": "x"} and lasts[1] == http.LastHttpContent(b"abc")
    assert got[-2].headers == {"content-length": "3"}
