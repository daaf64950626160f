"""Seeded fuzzing of the frame decoders over damaged framed streams, against the oracle's restatement
of the reference's decode() loops (oracle/frame_decoders.py):

* SnappyFrameDecoder (SnappyFrameDecoder.java:85-231): the synchronous handle AND the asynchronous
  batcher must deliver the oracle's messages in the oracle's order and fail with the oracle's
  exception (class and message) after the same messages, validating checksums or not, whatever the
  split of the stream into reads and the flush pattern.
* FastLzFrameDecoder (FastLzFrameDecoder.java:113-207), LzfDecoder (LzfDecoder.java:112-241) and
  Lz4FrameDecoder (Lz4FrameDecoder.java:150-261): the synchronous handles and the batcher against the
  oracle in the same way.

Streams carry damaged chunk types, lengths, checksums and payloads, are cut short or carry junk.
"""
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu

N_STREAMS = 400


@pytest.fixture(scope="module")
def nx():
    import netty_amd
    return netty_amd


@pytest.fixture(scope="module")
def F():
    from oracle import frame_decoders
    return frame_decoders


def _payload(oracle, rng, small=False):
    L = rng.choice((0, rng.randint(1, 40), rng.randint(100, 5000), rng.randint(30000, 70000)))
    if small:
        L = min(L, 65535)
    return oracle.textgen_chunk(rng.randrange(1 << 30), L) if rng.random() < 0.7 else oracle.java_random_bytes(rng.randrange(1 << 30), L)


def _stream(oracle, rng, codec="snappy"):
    parts = []
    for k in range(rng.randint(1, 3)):
        msg = _payload(oracle, rng, small=codec == "fastlz2")
        if codec == "snappy":
            fr, _ = oracle.snappy_frame_encode(msg, started=k > 0)
        elif codec.startswith("fastlz"):
            fr = oracle.fastlz_frame_encode(msg, level=int(codec[-1]) if codec[-1] in "12" else 0, checksum=rng.random() < 0.6)
        elif codec == "lzf":
            fr = oracle.lzf_frame_encode(msg)
        else:
            fr = oracle.lz4_frame_encode(msg, close=k == 2 and rng.random() < 0.5)
        parts.append(fr)
    return b"".join(parts)


def _damage(rng, s: bytes, type_bytes=(0x00, 0x01, 0x02, 0x7F, 0x80, 0xFE, 0xFF)) -> bytes:
    b = bytearray(s)
    for _ in range(rng.randint(1, 2)):
        kind = rng.randrange(6)
        if not b:
            break
        if kind == 0:    # a byte anywhere
            b[rng.randrange(len(b))] = rng.getrandbits(8)
        elif kind == 1:  # a chunk header byte (type or length) or the checksum near a chunk start
            p = rng.randrange(min(len(b), 24))
            b[p] = rng.getrandbits(8)
        elif kind == 2:  # the chunk type at a chunk boundary of the first chunks
            p = 10 if len(b) > 10 else 0
            b[p] = rng.choice(type_bytes)
        elif kind == 3:  # cut short
            del b[rng.randrange(len(b)):]
        elif kind == 4:  # remove a few bytes
            a = rng.randrange(len(b))
            del b[a:a + rng.randint(1, 6)]
        else:            # junk appended
            b += bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 30)))
    return bytes(b)


def _split(rng, s, reads):
    cuts = sorted(rng.randrange(0, len(s) + 1) for _ in range(reads - 1))
    return [s[a:c] for a, c in zip([0] + cuts, cuts + [len(s)])]


def _sync_events(nx, dec, parts):
    msgs, err = [], None
    for p in parts:
        if err is not None:
            assert dec.channel_read(p) == []  # a failed decoder stays corrupted
            continue
        try:
            msgs += dec.channel_read(p)
        except nx.DecoderException as e:
            msgs += list(getattr(e, "decoded", []))
            err = (type(e).__name__, str(e))
    return msgs, err


def _check(got, want, what):
    (gm, ge), (wm, we) = got, want
    assert ge == we, (what, ge, we)
    assert len(gm) == len(wm) and gm == wm, (what, len(gm), len(wm))


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("validate", [True, False])
def test_snappy_frame_decoder_batcher_and_sync_equal_oracle_fuzz(nx, oracle, F, validate, seed):
    rng = random.Random(1000 * seed + validate)
    b = nx.Batcher()
    chans = []
    for i in range(N_STREAMS):
        s = _stream(oracle, rng)
        if i % 5:
            s = _damage(rng, s)
        chans.append((nx.SnappyFrameDecoder(validate), _split(rng, s, rng.randint(1, 4)), []))
    max_reads = max(len(p) for _, p, _ in chans)
    for r in range(max_reads):
        for d, parts, tickets in chans:
            if r < len(parts):
                tickets.append(b.submit_decode(d, parts[r]))
        if r % 2:
            b.flush()
    b.flush()
    n_err = 0
    for d, parts, tickets in chans:
        msgs, err = [], None
        for t in tickets:
            b.wait(t)
            try:
                got = b.result(t)
            except nx.DecoderException as e:
                assert err is None, "a second failure on a corrupted decoder"
                got = list(getattr(e, "decoded", []))
                err = (type(e).__name__, str(e))
            msgs += got
        want = F.run(F.SnappyFrameDecoder(validate), parts)
        _check((msgs, err), want, "batcher")
        _check(_sync_events(nx, nx.SnappyFrameDecoder(validate), parts), want, "sync")
        n_err += err is not None
    assert 0 < n_err < len(chans)


_ALT = {
    "fastlz": (lambda nx, v: nx.FastLzFrameDecoder(v), lambda F, v: F.FastLzFrameDecoder(v), (0x46, 0x4C, 0x5A, 0x00, 0x01, 0x10, 0x11)),
    "fastlz2": (lambda nx, v: nx.FastLzFrameDecoder(v), lambda F, v: F.FastLzFrameDecoder(v), (0x46, 0x4C, 0x5A, 0x00, 0x01, 0x10, 0x11)),
    "lzf": (lambda nx, v: nx.LzfDecoder(), lambda F, v: F.LzfDecoder(), (0x5A, 0x56, 0x00, 0x01, 0x02, 0xFF)),
    "lz4": (lambda nx, v: nx.Lz4FrameDecoder(v), lambda F, v: F.Lz4FrameDecoder(v), (0x16, 0x26, 0x1F, 0x36, 0x00, 0xFF)),
}


def _batcher_events(nx, b, chans):
    """Submit every channel's reads round-robin (a flush after every other round), then collect each
    channel's messages and first failure from its tickets."""
    max_reads = max(len(p) for _, p, _ in chans)
    for r in range(max_reads):
        for d, parts, tickets in chans:
            if r < len(parts):
                tickets.append(b.submit_decode(d, parts[r]))
        if r % 2:
            b.flush()
    b.flush()
    out = []
    for d, parts, tickets in chans:
        msgs, err = [], None
        for t in tickets:
            b.wait(t)
            try:
                got = b.result(t)
            except nx.DecoderException as e:
                assert err is None, "a second failure on a corrupted decoder"
                got = list(getattr(e, "decoded", []))
                err = (type(e).__name__, str(e))
            msgs += got
        out.append((msgs, err))
    return out


@pytest.mark.parametrize("codec", sorted(_ALT))
@pytest.mark.parametrize("validate", [True, False])
def test_alt_frame_decoders_sync_and_batcher_equal_oracle_fuzz(nx, oracle, F, codec, validate):
    mk_gpu, mk_orc, types = _ALT[codec]
    rng = random.Random(zlib.crc32(f"{codec}/{validate}".encode()))
    streams = []
    for i in range(150):
        s = _stream(oracle, rng, codec)
        if i % 5:
            s = _damage(rng, s, types)
        streams.append(_split(rng, s, rng.randint(1, 4)))
    wants = [F.run(mk_orc(F, validate), parts) for parts in streams]
    for i, parts in enumerate(streams):
        _check(_sync_events(nx, mk_gpu(nx, validate), parts), wants[i], f"{codec} sync #{i}")
    b = nx.Batcher()
    got = _batcher_events(nx, b, [(mk_gpu(nx, validate), parts, []) for parts in streams])
    for i, (g, w) in enumerate(zip(got, wants)):
        _check(g, w, f"{codec} batcher #{i}")
    n_err = sum(w[1] is not None for w in wants)
    assert 0 < n_err < len(streams)
