"""The FastLZ / LZF / LZ4 handlers as batcher jobs (include/netty_amd.h section 3): encoder jobs of many
handles, submitted interleaved and flushed at arbitrary points, produce exactly the bytes the
synchronous handles and the oracle's restatements of the Java encoders produce
(FastLzFrameEncoder.java:111-172, LzfEncoder.java:169-246, Lz4FrameEncoder.java:221-336), and a
batcher-encoded stream decodes through batcher decoder jobs to the input.  Damaged streams through
decoder jobs are in tests/test_gpu_frame_fuzz.py."""
import random

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nx():
    import netty_amd
    return netty_amd


def _msgs(oracle, rng, k):
    out = []
    for _ in range(k):
        L = rng.choice((0, 1, rng.randint(2, 40), rng.randint(100, 5000), rng.randint(20000, 140000)))
        out.append(oracle.textgen_chunk(rng.randrange(1 << 30), L) if rng.random() < 0.7
                   else oracle.java_random_bytes(rng.randrange(1 << 30), L))
    return out


def _run_jobs(b, chans, flush_every=3):
    """chans: list of (submit(msg) -> ticket, messages).  Round-robin submits, flushes every few
    rounds; returns per channel the list of job outputs (each job = one message)."""
    tickets = [[] for _ in chans]
    rounds = max(len(m) for _, m in chans)
    for r in range(rounds):
        for c, (sub, msgs) in enumerate(chans):
            if r < len(msgs):
                tickets[c].append(sub(msgs[r]))
        if r % flush_every == flush_every - 1:
            b.flush()
    b.flush()
    out = []
    for ts in tickets:
        got = []
        for t in ts:
            b.wait(t)
            res = b.result(t)
            assert len(res) == 1
            got.append(res[0])
        out.append(got)
    return out


@pytest.mark.parametrize("level,checksum", [(0, False), (1, True), (2, False), (2, True)])
def test_fastlz_encoder_jobs_equal_sync_and_oracle(nx, oracle, level, checksum):
    rng = random.Random(level * 2 + checksum)
    b = nx.Batcher()
    chans = []
    for c in range(24):
        e = nx.FastLzFrameEncoder(level, checksum)
        chans.append((lambda m, e=e: b.submit_encode(e, m), _msgs(oracle, rng, rng.randint(1, 5))))
    got = _run_jobs(b, chans)
    for (_, msgs), outs in zip(chans, got):
        s = nx.FastLzFrameEncoder(level, checksum)
        for m, o in zip(msgs, outs):
            assert o == s.encode(m) == oracle.fastlz_frame_encode(m, level=level, checksum=checksum)


@pytest.mark.parametrize("threshold", [16, 100, 100000])
def test_lzf_encoder_jobs_equal_sync_and_oracle(nx, oracle, threshold):
    rng = random.Random(threshold)
    b = nx.Batcher()
    chans = []
    for c in range(24):
        e = nx.LzfEncoder(threshold)
        chans.append((lambda m, e=e: b.submit_encode(e, m), _msgs(oracle, rng, rng.randint(1, 5))))
    got = _run_jobs(b, chans)
    for (_, msgs), outs in zip(chans, got):
        s = nx.LzfEncoder(threshold)
        for m, o in zip(msgs, outs):
            assert o == s.encode(m) == oracle.lzf_frame_encode(m, compress_threshold=threshold)


@pytest.mark.parametrize("block_size,high", [(64, False), (4096, False), (1 << 16, False), (4096, True)])
def test_lz4_encoder_jobs_equal_sync(nx, oracle, block_size, high):
    """encode / flush / close interleaved over many handles; the bytes equal the synchronous handle's
    for the same call sequence (its block buffer carried across calls).  high: highCompressor encoders
    (LZ4_compress_HC blocks, launched apart from the fast ones)."""
    rng = random.Random(block_size + high)
    b = nx.Batcher()
    chans, ops = [], []
    for c in range(16):
        e = nx.Lz4FrameEncoder(block_size, high_compressor=high and c % 2 == 0)
        msgs = _msgs(oracle, rng, rng.randint(2, 6))
        op = [rng.choice((0, 0, 0, 1)) for _ in msgs]
        op[-1] = rng.choice((1, 2))
        if rng.random() < 0.3:  # a message after close passes through if its blocks need >= blockSize bytes (:216-239)
            n_min = next(n for n in range(block_size + 1) if n + n // 255 + 37 >= block_size)
            msgs.append((b"after close " * (n_min // 12 + 1))[:max(1, n_min)])
            op.append(0)
            op[-2] = 2
        it = iter(op)
        chans.append((lambda m, e=e, it=it: b.submit_encode(e, m, op=next(it)), msgs))
        ops.append(op)
    got = _run_jobs(b, chans)
    for c, ((_, msgs), op, outs) in enumerate(zip(chans, ops, got)):
        s = nx.Lz4FrameEncoder(block_size, high_compressor=high and c % 2 == 0)
        for m, k, o in zip(msgs, op, outs):
            want = s.encode(m)
            if k == 1:
                want += s.flush()
            elif k == 2:
                want += s.finish_encode()
            assert o == want
        # the whole stream decodes to the input (through the oracle's decoder)
        from oracle import frame_decoders as F
        stream = b"".join(outs)
        closed_at = op.index(2) if 2 in op else None
        want_data = b"".join(msgs[:closed_at + 1] if closed_at is not None else msgs)
        dm, err = F.run(F.Lz4FrameDecoder(True), [stream])
        assert err is None
        if closed_at is not None or op[-1] == 1:
            assert b"".join(dm) == want_data


@pytest.mark.parametrize("codec", ["fastlz", "lzf", "lz4"])
def test_alt_round_trip_through_batcher(nx, oracle, codec):
    """Encoder jobs → framed bytes → decoder jobs (split reads), many channels at once."""
    rng = random.Random(len(codec))
    b = nx.Batcher()
    chans, encs = [], []
    for c in range(20):
        e = {"fastlz": lambda: nx.FastLzFrameEncoder(1, True), "lzf": lambda: nx.LzfEncoder(),
             "lz4": lambda: nx.Lz4FrameEncoder(1 << 16)}[codec]()
        msgs = _msgs(oracle, rng, rng.randint(1, 4))
        chans.append((lambda m, e=e: b.submit_encode(e, m, op=1) if codec == "lz4" else b.submit_encode(e, m), msgs))
    streams = [b"".join(o) for o in _run_jobs(b, chans)]
    decs = [{"fastlz": lambda: nx.FastLzFrameDecoder(True), "lzf": lambda: nx.LzfDecoder(),
             "lz4": lambda: nx.Lz4FrameDecoder(True)}[codec]() for _ in streams]
    tickets = [[] for _ in streams]
    for r in range(4):
        for i, s in enumerate(streams):
            q = len(s) // 4
            part = s[r * q:(r + 1) * q] if r < 3 else s[3 * q:]
            tickets[i].append(b.submit_decode(decs[i], part))
        b.flush()
    for i, ts in enumerate(tickets):
        out = []
        for t in ts:
            b.wait(t)
            out += b.result(t)
        assert b"".join(out) == b"".join(chans[i][1]), i
