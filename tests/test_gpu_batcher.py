"""GPU tests of the asynchronous cross-channel batcher (include/netty_amd.h section 3): many
SnappyFrameEncoder / SnappyFrameDecoder instances (one per simulated channel) submit their
encode()/decode() calls, ONE flush launches them all, and every channel's bytes equal the oracle's
restatement of the Java handlers (SnappyFrameEncoder.java:79-117, SnappyFrameDecoder.java:85-231)."""
import ctypes as C
import random

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nx():
    import netty_amd
    return netty_amd


def _messages(oracle, n=64):
    rng = random.Random(17)
    msgs = []
    for i in range(n):
        k = i % 8
        if k == 0:
            msgs.append(b"")
        elif k == 1:
            msgs.append(oracle.textgen_chunk(i, rng.randrange(1, 19)))          # <= 18 bytes: one unencoded chunk
        elif k == 2:
            msgs.append(oracle.java_random_bytes(i, rng.randrange(20000, 200000)))
        elif k == 3:
            msgs.append(bytes(rng.randrange(1000, 70000)))
        else:
            msgs.append(oracle.textgen_chunk(i, rng.randrange(19, 300000)))
    return msgs


@pytest.mark.parametrize("jumbo", [False, True])
def test_batcher_64_encoders_one_launch(nx, oracle, jumbo):
    msgs = _messages(oracle)
    b = nx.Batcher()
    encs = [nx.SnappyFrameEncoder(jumbo=jumbo) for _ in msgs]
    for rnd in range(2):  # the second round: the stream identifier is not repeated (:84-87)
        tickets = [b.submit_encode(e, m) for e, m in zip(encs, msgs)]
        before = b.stats()
        b.flush()
        after = b.stats()
        assert after["flushes"] == before["flushes"] + 1
        assert after["launches"] - before["launches"] == 3  # CRC32C + Snappy.encode + finish, all channels
        while not all(b.poll(t) for t in tickets):
            pass
        for i, (t, m) in enumerate(zip(tickets, msgs)):
            got = b.result(t)
            want, _ = oracle.snappy_frame_encode(m, jumbo=jumbo, started=rnd == 1 or not m)
            if not m:
                assert got == [b""], i  # nothing written for an unreadable input
                continue
            assert got == [want], (rnd, i, len(m))


def test_batcher_64_decoders_one_launch(nx, oracle):
    msgs = _messages(oracle)
    streams = []
    for m in msgs:
        f, _ = oracle.snappy_frame_encode(m)
        streams.append(f if m else oracle.snappy_frame_encode(b"x")[0])
    want = [m if m else b"x" for m in msgs]
    b = nx.Batcher()
    decs = [nx.SnappyFrameDecoder(i % 2 == 1) for i in range(len(msgs))]
    rng = random.Random(3)
    # each channel's bytes arrive in two reads split at a random point: the first submit leaves the
    # partial chunk in the decoder's cumulation, the second completes it
    cuts = [rng.randrange(0, len(s) + 1) for s in streams]
    t1 = [b.submit_decode(d, s[:c]) for d, s, c in zip(decs, streams, cuts)]
    t2 = [b.submit_decode(d, s[c:]) for d, s, c in zip(decs, streams, cuts)]
    b.flush()
    st = b.stats()
    assert st["flushes"] == 1 and st["launches"] <= 3
    for i in range(len(msgs)):
        b.wait(t2[i])
        got = b"".join(b.result(t1[i]) + b.result(t2[i]))
        assert got == want[i], i
        assert decs[i].readable_bytes() == 0


def test_batcher_decoder_crc_failure_marks_corrupted(nx, oracle):
    data = oracle.textgen_chunk(9, 100000)
    f, _ = oracle.snappy_frame_encode(data)
    bad = bytearray(f)
    bad[10 + 4] ^= 0xFF  # the first chunk's masked CRC
    b = nx.Batcher()
    d = nx.SnappyFrameDecoder(True)
    ok = nx.SnappyFrameDecoder(True)
    t_bad = b.submit_decode(d, bytes(bad))
    t_ok = b.submit_decode(ok, f)
    t_after = b.submit_decode(d, f[10:])  # later input on the failed decoder is skipped (:86-89)
    b.flush()
    b.wait(t_after)
    with pytest.raises(nx.DecompressionException, match="mismatching checksum"):
        b.result(t_bad)
    assert b"".join(b.result(t_ok)) == data
    assert b.result(t_after) == []


def test_batcher_registered_input(nx, oracle):
    """Encoder input in page-locked host memory (nx_host_register, a pooled direct ByteBuf's chunk)
    is DMA'd at flush without the staging copy."""
    data = oracle.textgen_chunk(11, 1 << 20)
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    addr = C.addressof(buf)
    nx.Batcher.register(addr, len(data))
    try:
        b = nx.Batcher()
        e = nx.SnappyFrameEncoder()
        t = b.submit_encode(e, memoryview(buf), registered_ptr=addr)
        b.wait(t)
        assert b.result(t) == [oracle.snappy_frame_encode(data)[0]]
    finally:
        nx.Batcher.unregister(addr)
