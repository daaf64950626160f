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
