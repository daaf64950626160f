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
        # the staged inputs' host->device gather + CRC32C + Snappy.encode + finish, all channels
        assert after["launches"] - before["launches"] == 4
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
    assert st["flushes"] == 1 and st["launches"] <= 4  # gather, decode (parse + expand), CRC32C, finish
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


def test_batcher_registered_cumulations(nx, oracle):
    """Decoder cumulations in registered memory (nx_snappy_frame_decoder_submit_registered: the socket
    read into a pooled direct buffer) are gathered at flush without the staging copy; mixed in one
    batch with copied cumulations and a registered encoder input, every channel's messages are the
    oracle's (compressed and uncompressed chunks, validating and not)."""
    msgs = _messages(oracle, 48)
    streams = []
    for m in msgs:
        f, _ = oracle.snappy_frame_encode(m)
        streams.append(f if m else oracle.snappy_frame_encode(b"y")[0])
    want = [m if m else b"y" for m in msgs]
    blob = b"".join(streams)
    buf = (C.c_uint8 * (len(blob) + 64)).from_buffer_copy(blob + bytes(64))
    addr = C.addressof(buf)
    enc_in = oracle.textgen_chunk(5, 200000)
    ebuf = (C.c_uint8 * len(enc_in)).from_buffer_copy(enc_in)
    eaddr = C.addressof(ebuf)
    nx.Batcher.register(addr, len(blob) + 64)
    nx.Batcher.register(eaddr, len(enc_in))
    try:
        b = nx.Batcher()
        decs = [nx.SnappyFrameDecoder(i % 3 == 0) for i in range(len(msgs))]
        te = b.submit_encode(nx.SnappyFrameEncoder(), memoryview(ebuf), registered_ptr=eaddr)
        tickets, pos = [], 0
        for i, (d, s) in enumerate(zip(decs, streams)):
            if i % 4 == 3:  # a copied cumulation between registered ones
                tickets.append(b.submit_decode(d, s))
            else:
                t, consumed = b.submit_decode_registered(d, addr + pos, len(s))
                assert consumed == len(s)
                tickets.append(t)
            pos += len(s)
        b.flush()
        b.wait(tickets[-1])
        b.wait(te)
        for i, t in enumerate(tickets):
            assert b"".join(b.result(t)) == want[i], i
        assert b.result(te) == [oracle.snappy_frame_encode(enc_in)[0]]
    finally:
        nx.Batcher.unregister(addr)
        nx.Batcher.unregister(eaddr)


def test_batcher_registered_cumulation_outside_registration(nx, oracle):
    f, _ = oracle.snappy_frame_encode(b"hello, world" * 10)
    buf = (C.c_uint8 * len(f)).from_buffer_copy(f)
    b = nx.Batcher()
    with pytest.raises(RuntimeError, match="submit_registered"):
        b.submit_decode_registered(nx.SnappyFrameDecoder(), C.addressof(buf), len(f))


def test_batcher_autoflush_ordered_across_streams(nx, oracle):
    """Auto-flush (nx_batcher_set_flush_bytes): batches launch while later calls are submitted and
    rotate over the batcher's streams, yet results are applied in flush order: a decoder that fails in
    an early batch delivers nothing from its later jobs in later batches (SnappyFrameDecoder.java:86-89,
    227-230), and every other channel's bytes equal the oracle's."""
    msgs = _messages(oracle, 40)
    b = nx.Batcher(flush_bytes=256 * 1024)
    encs = [nx.SnappyFrameEncoder() for _ in msgs]
    et = [b.submit_encode(e, m) for e, m in zip(encs, msgs)]
    assert b.stats()["flushes"] >= 4  # several batches launched during the submits
    data = oracle.textgen_chunk(21, 300000)
    f, _ = oracle.snappy_frame_encode(data)
    bad = bytearray(f)
    bad[10 + 4] ^= 0xFF
    d_bad, d_ok = nx.SnappyFrameDecoder(True), nx.SnappyFrameDecoder(True)
    t_bad = b.submit_decode(d_bad, bytes(bad))
    t_ok = [b.submit_decode(d_ok, f[k:k + 50000]) for k in range(0, len(f), 50000)]
    fill = [b.submit_encode(nx.SnappyFrameEncoder(), oracle.textgen_chunk(30 + i, 200000)) for i in range(4)]
    t_after = b.submit_decode(d_bad, f[10:])  # a later batch, same failed decoder
    b.flush()
    assert b.stats()["flushes"] >= 7
    b.wait(t_after)
    for t in fill:
        b.wait(t)
    for i, (t, m) in enumerate(zip(et, msgs)):
        b.wait(t)
        want, _ = oracle.snappy_frame_encode(m, started=not m)
        assert b.result(t) == ([b""] if not m else [want]), i
    with pytest.raises(nx.DecompressionException, match="mismatching checksum"):
        b.result(t_bad)
    assert b"".join(b"".join(b.result(t)) for t in t_ok) == data
    assert b.result(t_after) == []


def test_batcher_header_error_after_good_job_same_decoder(nx, oracle):
    """A header-level error found at submit (a reserved unskippable chunk, SnappyFrameDecoder.java:151-157)
    fails its own job with the reference message when the batch is applied; the job submitted before it
    on the same decoder still delivers its messages, and the job after it delivers nothing (the decoder
    is corrupted, :86-89).  Same sequence as the synchronous decoder."""
    msg = oracle.textgen_chunk(11, 5000)
    good, _ = oracle.snappy_frame_encode(msg)
    bad = bytes([0x02, 0x01, 0x00, 0x00, 0x00])
    later, _ = oracle.snappy_frame_encode(b"later bytes of the stream", started=True)
    b = nx.Batcher()
    d = nx.SnappyFrameDecoder(True)
    t1 = b.submit_decode(d, good)
    t2 = b.submit_decode(d, bad)
    t3 = b.submit_decode(d, later)
    b.flush()
    b.wait(t3)
    assert b"".join(b.result(t1)) == msg
    with pytest.raises(nx.DecompressionException, match="Found reserved unskippable chunk type: 0x2"):
        b.result(t2)
    assert b.result(t3) == []
    # the synchronous decoder over the same reads
    s = nx.SnappyFrameDecoder(True)
    assert b"".join(s.channel_read(good)) == msg
    with pytest.raises(nx.DecompressionException, match="Found reserved unskippable chunk type: 0x2"):
        s.channel_read(bad)
    assert s.channel_read(later) == []


def test_batcher_rejected_encoder_submit_keeps_stream_identifier(nx, oracle):
    """A submit that fails its checks (input outside any registered range) leaves the encoder as it was:
    the next submit still writes the stream identifier (SnappyFrameEncoder.java:84-87)."""
    data = oracle.textgen_chunk(5, 1000)
    b = nx.Batcher()
    e = nx.SnappyFrameEncoder()
    buf = C.create_string_buffer(data, len(data))  # never registered
    with pytest.raises(RuntimeError):
        b.submit_encode(e, data, registered_ptr=C.addressof(buf))
    t = b.submit_encode(e, data)
    b.flush()
    b.wait(t)
    assert b.result(t) == [oracle.snappy_frame_encode(data)[0]]


# ---- validating-mode leftovers (SnappyFrameDecoder.java:206-212): a compressed chunk that decodes fewer
# bytes than its length leaves the rest in the cumulation, parsed again as the next chunk header
STREAM_ID = b"\xff\x06\x00\x00sNaPpY"
EMPTY_CRC = 0xA282EAD8  # mask(crc32c of no bytes)


def _chunk(kind, payload, crc):
    n = len(payload) + 4
    return bytes([kind, n & 255, (n >> 8) & 255, n >> 16]) + crc.to_bytes(4, "little") + payload


def leftover_streams(oracle):
    """Streams whose compressed chunks hide further chunks in their unread tails, with the messages the
    reference delivers (worked out from Snappy.decode, Snappy.java:315-393)."""
    x = oracle.textgen_chunk(21, 3000)
    y = oracle.textgen_chunk(22, 40)
    z = oracle.textgen_chunk(23, 60000)
    comp = lambda d: _chunk(0, oracle.snappy_encode(d), oracle.snappy_checksum(d))  # noqa: E731
    unc = lambda d: _chunk(1, d, oracle.snappy_checksum(d))  # noqa: E731
    # preamble 0: decode() returns at once (:324-327), one empty message, the rest is the next header
    zero = lambda rest: _chunk(0, b"\x00" + rest, EMPTY_CRC)  # noqa: E731
    # a 60-byte literal tag with fewer bytes behind it: NOT_ENOUGH_INPUT, the reader rewinds to just
    # after the tag (decodeLiteral :454-494); the message is what was decoded before it
    trunc = lambda d, rest: _chunk(0, oracle.snappy_encode(d) + bytes([59 << 2]) + rest, oracle.snappy_checksum(d))  # noqa: E731
    tail = comp(z)
    # (stream, messages when validating, messages without validation: readSlice drops the tail, :215)
    return [
        (STREAM_ID + zero(comp(x)) + tail, [b"", x, z], [b"", z]),
        (STREAM_ID + zero(zero(unc(y))) + comp(y) + tail, [b"", b"", y, y, z], [b"", y, z]),
        (STREAM_ID + trunc(x, unc(y)) + tail, [x, y, z], [x, z]),
        (STREAM_ID + comp(y) + trunc(y, zero(b"")) + zero(b"") + tail, [y, y, b"", b"", z], [y, y, b"", z]),
    ]


def test_sync_decoder_validating_leftover(nx, oracle):
    """The synchronous handle re-parses a leftover as the next chunk header, as the reference does."""
    for stream, want, plain in leftover_streams(oracle):
        d = nx.SnappyFrameDecoder(True)
        assert d.channel_read(stream) == want
        assert d.readable_bytes() == 0
        assert nx.SnappyFrameDecoder(False).channel_read(stream) == plain


@pytest.mark.parametrize("reads", [1, 3, 7])
@pytest.mark.parametrize("flush_every", [0, 1, 2])
def test_batcher_validating_leftover_equals_sync(nx, oracle, reads, flush_every):
    """The batcher re-walks a validating decoder's stream from the leftover at apply() time: over any
    split of the stream into reads and any flush pattern, every channel receives the synchronous
    decoder's messages in the same order (possibly on an earlier ticket)."""
    rng = random.Random(reads * 10 + flush_every)
    streams = leftover_streams(oracle)
    b = nx.Batcher()
    chans = []
    for stream, want, _ in streams * 2:
        cuts = sorted(rng.randrange(0, len(stream) + 1) for _ in range(reads - 1))
        parts = [stream[a:c] for a, c in zip([0] + cuts, cuts + [len(stream)])]
        chans.append((nx.SnappyFrameDecoder(True), parts, want, []))
    for r in range(reads):
        for d, parts, _, tickets in chans:
            tickets.append(b.submit_decode(d, parts[r]))
        if flush_every and r % flush_every == 0:
            b.flush()
    b.flush()
    for d, parts, want, tickets in chans:
        got = []
        for t in tickets:
            b.wait(t)
            got += b.result(t)
        assert got == want
        s = nx.SnappyFrameDecoder(True)
        sync = []
        for p in parts:
            sync += s.channel_read(p)
        assert sync == want


def test_batcher_validating_leftover_then_error(nx, oracle):
    """A header error inside a leftover fails the continuing job with the reference message, after its
    earlier messages; later input on the decoder is skipped (:86-89)."""
    x = oracle.textgen_chunk(31, 500)
    bad = bytes([0x02, 0x01, 0x00, 0x00, 0x00])
    stream = STREAM_ID + _chunk(0, oracle.snappy_encode(x), oracle.snappy_checksum(x)) + _chunk(0, b"\x00" + bad, EMPTY_CRC)
    later = _chunk(1, b"abcd", oracle.snappy_checksum(b"abcd"))
    b = nx.Batcher()
    d = nx.SnappyFrameDecoder(True)
    t1 = b.submit_decode(d, stream)
    t2 = b.submit_decode(d, later)
    b.flush()
    b.wait(t1)
    b.wait(t2)
    with pytest.raises(nx.DecompressionException, match="Found reserved unskippable chunk type: 0x2") as ei:
        b.result(t1)
    assert ei.value.decoded == [x, b""]
    assert b.result(t2) == []
    s = nx.SnappyFrameDecoder(True)
    with pytest.raises(nx.DecompressionException, match="Found reserved unskippable chunk type: 0x2") as ei:
        s.channel_read(stream)
    assert ei.value.decoded == [x, b""]


def test_batcher_decoder_freed_with_jobs_in_flight(nx, oracle):
    """A handler removed while its jobs are queued (nx_snappy_frame_decoder_free before the flush):
    the jobs keep the handle alive and still deliver their messages (validating and not)."""
    data = oracle.textgen_chunk(41, 150000)
    f, _ = oracle.snappy_frame_encode(data)
    b = nx.Batcher()
    tickets = []
    for validate in (False, True):
        d = nx.SnappyFrameDecoder(validate)
        tickets.append(b.submit_decode(d, f[:len(f) // 2]))
        tickets.append(b.submit_decode(d, f[len(f) // 2:]))
        d.close()  # the owner's reference goes; the two jobs hold theirs
    b.flush()
    got = []
    for t in tickets:
        b.wait(t)
        got.append(b"".join(b.result(t)))
    assert got[0] + got[1] == data and got[2] + got[3] == data
    # the batches are reused afterwards (their jobs, and with them the last references, are deleted)
    d2 = nx.SnappyFrameDecoder(True)
    t = b.submit_decode(d2, f)
    b.flush()
    b.wait(t)
    assert b"".join(b.result(t)) == data


def test_batcher_validating_leftover_registered_autoflush(nx, oracle):
    """Leftover re-walks with registered cumulations and auto-flushes across the batcher's four streams:
    each read's cumulation is placed in a registered arena (bytes [0, consumed) stay valid until the job
    completes, the unconsumed tail is resubmitted with the next read, as ByteToMessageDecoder's
    cumulation), many jobs per decoder are in flight at once, small batches launch on their own, and
    every channel still receives the synchronous decoder's messages in order."""
    streams = [(s, w) for s, w, _ in leftover_streams(oracle)] * 3
    rng = random.Random(77)
    arena_size = 8 * sum(len(s) for s, _ in streams) + 4096
    arena = (C.c_uint8 * arena_size)()
    base = C.addressof(arena)
    nx.Batcher.register(base, arena_size)
    try:
        b = nx.Batcher(flush_bytes=48 << 10)
        chans = []
        for s, w in streams:
            cuts = sorted(rng.randrange(0, len(s) + 1) for _ in range(3))
            parts = [s[a:c] for a, c in zip([0] + cuts, cuts + [len(s)])]
            chans.append([nx.SnappyFrameDecoder(True), parts, w, [], bytearray()])
        pos = 0
        for r in range(4):
            for ch in chans:
                d, parts, _, tickets, cum = ch
                cum += parts[r]
                C.memmove(base + pos, bytes(cum), len(cum))
                t, consumed = b.submit_decode_registered(d, base + pos, len(cum))
                tickets.append(t)
                pos += (len(cum) + 15) & ~15
                del cum[:consumed]
        b.flush()
        for d, parts, want, tickets, cum in chans:
            got = []
            for t in tickets:
                b.wait(t)
                got += b.result(t)
            assert got == want
        assert b.stats()["flushes"] > 1
    finally:
        nx.Batcher.unregister(base)


def test_batcher_leftover_with_released_tickets(nx, oracle):
    """Re-walks of two decoders' jobs whose tickets were released before they completed (the caller
    discarded them): their batch may be reused while the continuations are queued; the batcher stays
    consistent and later jobs complete."""
    from netty_amd import _lib
    L = _lib.load()
    stream, _, _ = leftover_streams(oracle)[0]
    b = nx.Batcher()
    decs = [nx.SnappyFrameDecoder(True) for _ in range(2)]
    for d in decs:
        t = b.submit_decode(d, stream)
        assert L.nx_batcher_release(b._h, t) == 0
    b.flush()
    other = nx.SnappyFrameDecoder(True)
    data = oracle.textgen_chunk(99, 20000)
    for _ in range(3):  # each submit applies what completed; the continuations go out at poll/wait
        t = b.submit_decode(other, oracle.snappy_frame_encode(data, started=_ > 0)[0])
        b.wait(t)
        assert b"".join(b.result(t)) == data


def test_batcher_tiny_chunks_claiming_64k_keep_their_neighbours(oracle):
    """the batcher packs decode slots by what a chunk can decode to (64 bytes per 3
    compressed bytes), not by the 65536 its preamble may claim.  Tiny chunks claiming 65536, and
    chunks that decode to exactly their bound, sit between ordinary ones in one flush: every
    message equals the oracle's, so no slot overran into its neighbour."""
    import random
    import netty_amd as nx
    from oracle import frame_decoders as F
    rng = random.Random(77)
    sid = bytes.fromhex("ff060000734e61507059")

    def chunk(payload, crc_of):
        return b"\x00" + (len(payload) + 4).to_bytes(3, "little") + oracle.snappy_checksum(crc_of).to_bytes(4, "little") + payload

    b = nx.Batcher()
    chans = []
    for i in range(300):
        parts = [sid]
        for k in range(rng.randint(1, 4)):
            kind = rng.randrange(3)
            if kind == 0:  # preamble 65536, one 1-byte literal
                v = bytes([rng.randrange(256)])
                parts.append(chunk(b"\x80\x80\x04" + b"\x00" + v, v))
            elif kind == 1:  # at the bound: literal 'a' then copy-2 tags of 64 bytes, offset 1
                n = rng.randint(1, 40)
                body = b"\x00a" + b"\xfe\x01\x00" * n
                raw = b"a" * (1 + 64 * n)
                pre = oracle.snappy_encode(raw)[:3]  # the varint of len(raw)
                plen = 1 + (len(raw) >= 128) + (len(raw) >= 16384)
                parts.append(chunk(pre[:plen] + body, raw))
            else:
                m = oracle.textgen_chunk(rng.randrange(1 << 20), rng.randint(1, 30000))
                parts.append(oracle.snappy_frame_encode(m, started=True)[0])
        stream = b"".join(parts)
        chans.append((nx.SnappyFrameDecoder(True), stream, rng.random() < 0.5))
    tickets = [b.submit_decode(d, s) for d, s, _ in chans]
    b.flush()
    for (d, s, _), t in zip(chans, tickets):
        b.wait(t)
        try:
            got, err = b.result(t), None
        except nx.DecoderException as e:
            got, err = list(e.decoded), (type(e).__name__, str(e))
        want = F.run(F.SnappyFrameDecoder(True), [s])
        assert (got, err) == want


def test_batcher_reserved_arenas_do_not_grow(oracle):
    """with the pinned arenas sized up front (nx_batcher_reserve_arenas) and the
    auto-flush threshold below them, rounds of submits / flushes after a warm-up allocate nothing."""
    import random
    import netty_amd as nx
    rng = random.Random(3)
    b = nx.Batcher()
    b.reserve(1 << 4)  # the decoder's record workspace, up front
    b.reserve_arenas(8, 8 << 20, 40 << 20)
    b.set_flush_bytes(4 << 20)
    streams = []
    for i in range(48):
        data = oracle.textgen_chunk(rng.randrange(1 << 20), rng.randint(20000, 200000))
        streams.append((data, oracle.snappy_frame_encode(data)[0]))

    def one_round():
        decs = [nx.SnappyFrameDecoder(True) for _ in streams]
        tickets = []
        for d, (_, s) in zip(decs, streams):
            q = len(s) // 2
            tickets.append([b.submit_decode(d, s[:q]), b.submit_decode(d, s[q:])])
        b.flush()
        for (data, _), ts in zip(streams, tickets):
            out = []
            for t in ts:
                b.wait(t)
                out += b.result(t)
            assert b"".join(out) == data

    one_round()
    before = b.arena_stats()
    for _ in range(3):
        one_round()
    after = b.arena_stats()
    assert after["allocs"] == before["allocs"], (before, after)


def test_batcher_large_decode_results_by_dma(oracle):
    """A flush whose decoded messages fill most of a large result arena (>= 64 MiB) goes to host
    memory by one DMA copy from a device mirror (nx_batcher_dma_stats) instead of the finish kernel's
    mapped stores; the messages are the same, and a flush of small chunks (whose result reservation
    is mostly headroom) keeps the mapped path."""
    import random
    import netty_amd as nx
    rng = random.Random(11)
    b = nx.Batcher()
    chans = []
    for i in range(8):  # 8 channels x ~9.4 MiB of 64 KiB-chunk streams: ~75 MiB of messages
        data = b"".join(oracle.textgen_chunk(rng.randrange(1 << 20), 65536) for _ in range(150))
        chans.append((nx.SnappyFrameDecoder(i % 2 == 0), data, oracle.snappy_frame_encode(data)[0]))
    tickets = [(b.submit_decode(d, s), data) for d, data, s in chans]
    b.flush()
    for t, data in tickets:
        b.wait(t)
        assert b"".join(b.result(t)) == data
    st = b.stats()
    assert st["dma_flushes"] == 1 and st["dma_bytes"] >= 64 << 20, st
    # small chunks: bound-sized reservations, few bytes written -> mapped stores
    small = [(nx.SnappyFrameDecoder(True), oracle.textgen_chunk(i, 200)) for i in range(300)]
    ts = [(b.submit_decode(d, oracle.snappy_frame_encode(x)[0]), x) for d, x in small]
    b.flush()
    for t, x in ts:
        b.wait(t)
        assert b"".join(b.result(t)) == x
    assert b.stats()["dma_flushes"] == 1


def test_batcher_chunk_longer_than_its_preamble(oracle):
    """A compressed chunk whose preamble declares fewer bytes than its tags produce: the reference
    decodes it anyway (the output buffer grows to 65 536, SnappyFrameDecoder.java:203, Snappy.java:
    328 only ensures the declared size).  The batcher reserves the declared length for the message,
    so this one spills and is copied from its decode slot at apply; the messages equal the
    synchronous decoder's and the oracle's."""
    import netty_amd as nx
    from oracle import frame_decoders as F
    x = oracle.textgen_chunk(77, 3000)
    block = oracle.snappy_encode(x)
    assert block[:2] == bytes([0xB8, 0x17])  # varint(3000)
    lying = bytes([10]) + block[2:]          # declares 10 bytes, decodes to 3000
    good = oracle.textgen_chunk(78, 5000)
    stream = STREAM_ID + _chunk(0, lying, oracle.snappy_checksum(x)) + oracle.snappy_frame_encode(good, started=True)[0]
    for validate in (True, False):
        want = F.run(F.SnappyFrameDecoder(validate), [stream])
        assert want == ([x, good], None)
        b = nx.Batcher()
        d = nx.SnappyFrameDecoder(validate)
        t = b.submit_decode(d, stream)
        b.flush()
        b.wait(t)
        assert b.result(t) == [x, good]
        assert nx.SnappyFrameDecoder(validate).channel_read(stream) == [x, good]


def _lying_chunk(oracle, seed, n):
    """A COMPRESSED_DATA chunk whose preamble declares 10 bytes but whose tags decode to n."""
    x = oracle.textgen_chunk(seed, n)
    block = oracle.snappy_encode(x)
    plen = 1 + (n >= 128) + (n >= 16384)
    return x, _chunk(0, bytes([10]) + block[plen:], oracle.snappy_checksum(x))


def test_batcher_spills_beyond_the_spill_area(oracle):
    """chunks longer than their preamble go to the flush's 1 MiB spill area in k_dec_finish
    (no device copy at apply); more than that in one flush falls back to apply's copy from the decode
    slot.  20 such 64 KiB chunks (1.25 MiB) across channels, between ordinary chunks, in one flush:
    every message equals the oracle's, both paths taken."""
    import netty_amd as nx
    from oracle import frame_decoders as F
    b = nx.Batcher()
    chans = []
    for i in range(20):
        x, lie = _lying_chunk(oracle, 500 + i, 65536)
        good = oracle.textgen_chunk(600 + i, 9000)
        stream = STREAM_ID + lie + oracle.snappy_frame_encode(good, started=True)[0]
        want = F.run(F.SnappyFrameDecoder(True), [stream])
        assert want == ([x, good], None)
        chans.append((nx.SnappyFrameDecoder(True), stream, [x, good]))
    tickets = [b.submit_decode(d, s) for d, s, _ in chans]
    b.flush()
    for (d, s, want), t in zip(chans, tickets):
        b.wait(t)
        assert b.result(t) == want


def test_batcher_spill_in_a_dma_result_flush(oracle):
    """a chunk longer than its preamble inside a flush whose results go to host memory by
    the DMA copy of the stream's device mirror: the spill area is part of the mirror, so the message
    arrives with the others."""
    import random
    import netty_amd as nx
    rng = random.Random(12)
    b = nx.Batcher()
    chans = []
    for i in range(8):  # ~75 MiB of 64 KiB-chunk messages: the DMA result path
        data = b"".join(oracle.textgen_chunk(rng.randrange(1 << 20), 65536) for _ in range(150))
        chans.append((nx.SnappyFrameDecoder(True), oracle.snappy_frame_encode(data)[0], [data]))
    x, lie = _lying_chunk(oracle, 901, 40000)
    chans.append((nx.SnappyFrameDecoder(True), STREAM_ID + lie, [x]))
    tickets = [b.submit_decode(d, s) for d, s, _ in chans]
    b.flush()
    for (d, s, want), t in zip(chans, tickets):
        b.wait(t)
        assert b"".join(b.result(t)) == b"".join(want)
    assert b.stats()["dma_flushes"] == 1
