"""Seeded fuzzing of SnappyFrameDecoder (SnappyFrameDecoder.java:85-231) over damaged framed streams:
the synchronous handle and the asynchronous batcher must deliver the same messages in the same
order and fail with the same exception (class and message) after the same messages, validating
checksums or not, whatever the split of the stream into reads and the flush pattern.

The synchronous handle is pinned to the oracle's restatement by test_gpu_handlers.py; this test
holds the batcher — header walk at submit, chunk decode at flush, validating-leftover re-walk at
apply (batcher.cpp) — to it on inputs nobody wrote by hand: streams with damaged chunk types,
lengths, checksums and payloads, cut short or carrying junk.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

N_STREAMS = 400


@pytest.fixture(scope="module")
def nx():
    import netty_amd
    return netty_amd


def _stream(oracle, rng):
    parts = []
    for k in range(rng.randint(1, 3)):
        L = rng.choice((0, rng.randint(1, 40), rng.randint(100, 5000), rng.randint(30000, 70000)))
        msg = oracle.textgen_chunk(rng.randrange(1 << 30), L) if rng.random() < 0.7 else oracle.java_random_bytes(rng.randrange(1 << 30), L)
        fr, _ = oracle.snappy_frame_encode(msg, started=k > 0)
        parts.append(fr)
    return b"".join(parts)


def _damage(rng, s: bytes) -> bytes:
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
            b[p] = rng.choice((0x00, 0x01, 0x02, 0x7F, 0x80, 0xFE, 0xFF))
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


def _sync_events(nx, validate, parts):
    d = nx.SnappyFrameDecoder(validate)
    msgs, err = [], None
    for p in parts:
        if err is not None:
            assert d.channel_read(p) == []  # a failed decoder stays corrupted (:86-89)
            continue
        try:
            msgs += d.channel_read(p)
        except nx.DecoderException as e:
            msgs += list(getattr(e, "decoded", []))
            err = (type(e).__name__, str(e))
    return msgs, err


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("validate", [True, False])
def test_snappy_frame_decoder_batcher_equals_sync_fuzz(nx, oracle, validate, seed):
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
        want_msgs, want_err = _sync_events(nx, validate, parts)
        assert err == want_err, (err, want_err)
        assert msgs == want_msgs, (len(msgs), len(want_msgs))
        n_err += err is not None
    assert 0 < n_err < len(chans)
