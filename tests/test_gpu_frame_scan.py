"""GPU parity: the device Snappy frame scan (nx_snappy_frame_scan_batch) against the oracle's
restatement of SnappyFrameDecoder's chunk walk (oracle/pyoracle.py snappy_frame_scan, pinned by
SnappyFrameDecoderTest's streams in tests/test_oracle_kat.py), and scan → decode end to end."""
import random

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ID = b"\xff\x06\x00\x00sNaPpY"


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def B():
    from netty_amd import batch
    return batch


def _uncompressed_chunk(oracle, d):
    return bytes([1]) + (len(d) + 4).to_bytes(3, "little") + oracle.snappy_checksum(d).to_bytes(4, "little") + d


def _error_streams():
    return [
        b"\xff\x05\x00\x00sNaPp",                                  # stream identifier length
        b"\xff\x06\x00\x00snappy",                                 # stream identifier contents
        b"\x00\x05\x00\x00abcde",                                  # COMPRESSED_DATA before identifier
        b"\x01\x05\x00\x00abcde",                                  # UNCOMPRESSED_DATA before identifier
        b"\x80\x01\x00\x00a",                                      # RESERVED_SKIPPABLE before identifier
        ID + b"\x01\x05\x00\x01",                                  # UNCOMPRESSED_DATA of 65541 bytes
        ID + b"\x00\x08\x00\x00" + bytes(4) + b"\x80\x80\x80\x80",  # preamble > 4 bytes
        ID + b"\x00\x08\x00\x00" + bytes(4) + b"\x81\x80\x04\x00",  # preamble 65537
        ID + b"\x00\x02\x00\x00ab",                                # chunk shorter than its checksum
        ID + b"\x02\x00\x00\x00",                                  # reserved unskippable 0x02
        ID + b"\x7f\x00\x00\x00",                                  # reserved unskippable 0x7f
        ID + b"\x00\x05\x00\x00" + bytes(4) + b"\x80",             # preamble cut by the cumulation: 0, ok
        ID + b"\xff\x06\x00\x00sNaPpY" + b"\x00\x00\x00",          # second identifier, 3 bytes left
    ]


def _streams(oracle, kat, n=48, seed=99):
    rng = random.Random(seed)
    out = [(bytes.fromhex(v["in"]), 0) for v in kat["snappy_frame_decode"]]
    out += [(s, 0) for s in _error_streams()]
    for i in range(n):
        started = rng.random() < 0.85
        parts = [ID] if started else []
        for j in range(rng.randint(0, 5)):
            r = rng.random()
            if r < 0.55:
                data = oracle.textgen_chunk(i * 16 + j, rng.randint(0, 150000))
                parts.append(oracle.snappy_frame_encode(data, started=True)[0])
            elif r < 0.7:  # under 18 bytes the frame encoder writes UNCOMPRESSED_DATA (SnappyFrameEncoder.java:90-115)
                parts.append(oracle.snappy_frame_encode(oracle.java_random_bytes(i * 16 + j, rng.randint(1, 17)),
                                                        started=True)[0])
            elif r < 0.85:
                parts.append(_uncompressed_chunk(oracle, oracle.textgen_chunk(i, rng.randint(0, 65536))))
            else:  # padding
                k = rng.randint(0, 3000)
                parts.append(bytes([rng.randint(0x80, 0xFE)]) + k.to_bytes(3, "little") + bytes(k))
        buf = b"".join(parts)
        if rng.random() < 0.5:
            buf = buf[:rng.randint(0, len(buf))]
        state = 0 if started else int(rng.random() < 0.5)
        if rng.random() < 0.1:
            state |= rng.randint(1, 5000) << 8
        if rng.random() < 0.05:
            state |= 2
        out.append((buf, state))
    out.append((b"", 0))
    out.append((b"", 1 | (7 << 8)))
    return out


def _scan(B, dev, streams, cap):
    bufs = [s for s, _ in streams]
    data, off, _ = B.pack(bufs, dev)
    ln = torch.tensor([len(b) for b in bufs], dtype=torch.int64, device=dev)
    state = torch.tensor([st for _, st in streams], dtype=torch.int64, device=dev).to(torch.int32)
    r = B.snappy_frame_scan(data, off, ln, state, cap)
    torch.cuda.synchronize()
    offs = off.cpu().tolist()
    cnt = r["counts"].cpu().tolist()
    do, dl, mc, sd, sq = (r[k].cpu().tolist() for k in ("data_off", "data_len", "masked_crc", "stream", "seq"))
    listed = {}
    for k in list(range(cnt[0])) + list(range(cap - cnt[1], cap)):
        listed.setdefault(sd[k], []).append((sq[k], 0 if k < cnt[0] else 1, do[k] - offs[sd[k]], dl[k], mc[k] & 0xFFFFFFFF))
    per = {i: sorted(v) for i, v in listed.items()}
    return data, r, cnt, per, state.cpu().tolist()


def _check(oracle, streams, r, per, states, caps=None):
    cons, stat = r["consumed"].cpu().tolist(), r["status"].cpu().tolist()
    for i, (buf, st0) in enumerate(streams):
        got = per.get(i, [])
        assert [e[0] for e in got] == list(range(len(got))), i
        cap = caps(i, got) if caps else None
        ents, c, s, res = oracle.snappy_frame_scan(buf, st0, cap)
        assert [e[1:] for e in got] == ents, i
        assert (cons[i], stat[i], states[i] & 0xFFFFFFFF) == (c, res, s), (i, buf[:32])


def test_frame_scan_parity(dev, B, oracle, kat):
    streams = _streams(oracle, kat)
    cap = 8192
    _, r, cnt, per, states = _scan(B, dev, streams, cap)
    assert cnt[0] + cnt[1] == cnt[2] < cap
    _check(oracle, streams, r, per, states)
    codes = set(r["status"].cpu().tolist())
    assert {-1, -41, -42, -43, -44, -45, -46, -47, -48, -49} <= codes


def test_frame_scan_list_full(dev, B, oracle, kat):
    """A full list stops each affected stream before the chunk it could not list; the stream's
    state and consumed position are those of an oracle scan bounded to the chunks it did list."""
    streams = _streams(oracle, kat, n=24, seed=5)
    cap = 7
    _, r, cnt, per, states = _scan(B, dev, streams, cap)
    assert cnt[0] + cnt[1] == cap and cnt[2] > cap
    stat = r["status"].cpu().tolist()
    assert 1 in stat
    _check(oracle, streams, r, per, states, caps=lambda i, got: len(got) if stat[i] == 1 else None)
    # resuming the stopped streams from `consumed` lists exactly the rest
    cons = r["consumed"].cpu().tolist()
    rest = [(streams[i][0][cons[i]:], states[i] & 0xFFFFFFFF) for i in range(len(streams)) if stat[i] == 1]
    _, r2, _, per2, states2 = _scan(B, dev, rest, 8192)
    _check(oracle, rest, r2, per2, states2)


def test_frame_scan_feeds_decode(dev, B, oracle):
    """scan → nx_snappy_decode_batch on the COMPRESSED list (CRC verified) and nx_crc32c_masked_batch
    on the UNCOMPRESSED list reproduce every stream's messages."""
    rng = random.Random(7)
    streams, msgs = [], []
    for i in range(96):
        parts, want = [ID], []
        for j in range(rng.randint(1, 4)):
            r = rng.random()
            if r < 0.6:
                d = oracle.textgen_chunk(5000 + i * 8 + j, rng.randint(1, 200000))
            elif r < 0.8:
                d = oracle.java_random_bytes(i * 8 + j, rng.randint(18, 100000))
            else:
                d = oracle.java_random_bytes(i * 8 + j, rng.randint(1, 17))
            parts.append(oracle.snappy_frame_encode(d, started=True)[0])
            want.append(d)
        streams.append((b"".join(parts), 0))
        msgs.append(b"".join(want))
    cap = 4096
    data, r, cnt, per, states = _scan(B, dev, streams, cap)
    assert set(r["status"].cpu().tolist()) == {0}
    n0, n1 = cnt[0], cnt[1]
    assert n0 > 0 and n1 > 0
    out_off = torch.arange(n0, dtype=torch.int64, device=dev) * 65536
    out = torch.zeros(n0 * 65536 + 16, dtype=torch.uint8, device=dev)
    d = B.snappy_decode(data, r["data_off"][:n0], r["data_len"][:n0], out, out_off, expected_crc=r["masked_crc"][:n0])
    crc_u = B.crc32c_masked(data, r["data_off"][cap - n1:], r["data_len"][cap - n1:])
    torch.cuda.synchronize()
    assert set(d["status"].cpu().tolist()) == {0}
    assert crc_u.cpu().tolist() == r["masked_crc"][cap - n1:].cpu().tolist()
    olen = d["out_len"].cpu().tolist()
    outh = out.cpu().numpy().tobytes()
    datah = data.cpu().numpy().tobytes()
    do, dl, sd, sq = (r[k].cpu().tolist() for k in ("data_off", "data_len", "stream", "seq"))
    pieces = {}
    for k in range(n0):
        pieces.setdefault(sd[k], []).append((sq[k], outh[k * 65536:k * 65536 + olen[k]]))
    for k in range(cap - n1, cap):
        pieces.setdefault(sd[k], []).append((sq[k], datah[do[k]:do[k] + dl[k]]))
    for i, want in enumerate(msgs):
        assert b"".join(p for _, p in sorted(pieces[i])) == want, i


# ---- one long cumulation: the segmented walk (nx_snappy_frame_scan_long) -----------------------------
def _scan_long(B, dev, buf, st0, cap):
    data = torch.frombuffer(bytearray(buf + bytes(16)), dtype=torch.uint8).to(dev)
    state = torch.tensor([st0], dtype=torch.int64, device=dev).to(torch.int32)
    r = B.snappy_frame_scan_long(data, len(buf), state, cap)
    torch.cuda.synchronize()
    cnt = r["counts"].cpu().tolist()
    do, dl, mc, sd, sq = (r[k].cpu().tolist() for k in ("data_off", "data_len", "masked_crc", "stream", "seq"))
    got = sorted((sq[k], 0 if k < cnt[0] else 1, do[k], dl[k], mc[k] & 0xFFFFFFFF)
                 for k in list(range(cnt[0])) + list(range(cap - cnt[1], cap)))
    assert all(sd[k] == 0 for k in list(range(cnt[0])) + list(range(cap - cnt[1], cap)))
    return got, r["consumed"].item(), r["status"].item(), state.item() & 0xFFFFFFFF, cnt


def _check_long(B, dev, oracle, buf, st0=0, cap=1 << 16):
    got, cons, stat, st, cnt = _scan_long(B, dev, buf, st0, cap)
    ents, c, s, res = oracle.snappy_frame_scan(buf, st0, cap)
    assert [e[0] for e in got] == list(range(len(got)))
    assert [e[1:] for e in got] == ents
    assert (cons, stat, st) == (c, res, s)
    return got, cnt


def _long_stream(oracle, mib, seed, extras=()):
    """A SnappyFrameEncoder stream of ~mib MiB (text, random and short chunks), with `extras`
    (position fraction, bytes) spliced in at chunk boundaries."""
    rng = random.Random(seed)
    parts, size = [ID], 10
    cuts = sorted(extras)
    while size < mib << 20:
        if cuts and size >= cuts[0][0] * (mib << 20):
            parts.append(cuts.pop(0)[1])
            size += len(parts[-1])
            continue
        r = rng.random()
        d = (oracle.textgen_chunk(rng.randrange(1 << 20), rng.randint(100000, 400000)) if r < 0.8
             else oracle.java_random_bytes(rng.randrange(1 << 20), rng.randint(1, 200000)))
        parts.append(oracle.snappy_frame_encode(d, started=True)[0])
        size += len(parts[-1])
    return b"".join(parts)


def _skippable(t, k):
    return bytes([t]) + k.to_bytes(3, "little") + bytes(k)


def test_frame_scan_long_parity(dev, B, oracle, kat):
    """The segmented walk of one long cumulation lists exactly the oracle walk's chunks, consumed
    position, status and state: plain streams, skippable / padding chunks (one of 3 MiB spanning
    segments, so guesses land inside it and are corrected), a second stream identifier, an error
    in the middle, a cut at the end, and the incoming states (no identifier yet, corrupted, bytes
    left to skip)."""
    base = _long_stream(oracle, 24, 1)
    _check_long(B, dev, oracle, base)
    _check_long(B, dev, oracle, base[:len(base) - 12345])                  # partial last chunk
    _check_long(B, dev, oracle, base[:(5 << 20) + 7])
    withskip = _long_stream(oracle, 24, 2, extras=[(0.2, _skippable(0x80, 3 << 20)), (0.5, _skippable(0xFE, 100)),
                                                   (0.6, ID), (0.7, _skippable(0xC3, 70000))])
    _check_long(B, dev, oracle, withskip)
    bad = _long_stream(oracle, 16, 3, extras=[(0.55, b"\x02\x10\x00\x00" + bytes(16))])
    got, _ = _check_long(B, dev, oracle, bad)
    assert len(got) > 50
    bad2 = _long_stream(oracle, 16, 4, extras=[(0.4, b"\x00\x08\x00\x00" + bytes(4) + b"\x81\x80\x04\x00")])
    _check_long(B, dev, oracle, bad2)
    noid = base[10:]
    _check_long(B, dev, oracle, noid, 0)                                     # data before the identifier
    _check_long(B, dev, oracle, noid, 1)                                     # a continuation
    _check_long(B, dev, oracle, noid, 2)                                     # corrupted: discarded
    sk = _skippable(0x90, 5000)
    _check_long(B, dev, oracle, sk[1000:] + base[10:], 1 | (4004 << 8))      # skip carried in
    _check_long(B, dev, oracle, base[:3 << 20], 1)
    # every short stream of the lane-walk tests through the segmented path too (one segment)
    for s, st in _streams(oracle, kat, n=24, seed=11):
        _check_long(B, dev, oracle, s, st)


def test_frame_scan_long_list_full(dev, B, oracle):
    """A list that fills up stops the walk before the first chunk it cannot list, as the lane walk:
    at the first chunk, inside a segment, and exactly at a segment's first chunk."""
    buf = _long_stream(oracle, 12, 5)
    all_ents = oracle.snappy_frame_scan(buf, 0, None)[0]
    n = len(all_ents)
    # the index of the first chunk that starts in the second segment
    first_seg1 = next(i for i, e in enumerate(all_ents) if e[1] - 8 >= 1 << 20)
    for cap in (1, 2, 37, first_seg1, first_seg1 + 1, n - 1, n, n + 5):
        got, cnt = _check_long(B, dev, oracle, buf, 0, cap)
        assert len(got) == min(cap, n)
        assert cnt[2] == min(cap, n) + (1 if cap < n else 0)


def test_frame_scan_long_equals_lane_walk(dev, B, oracle):
    """The segmented walk and the lane walk (nx_snappy_frame_scan_batch, n = 1) give the same list."""
    buf = _long_stream(oracle, 20, 6, extras=[(0.3, _skippable(0x81, 2 << 20))])
    got, _, _, _, _ = _scan_long(B, dev, buf, 0, 1 << 16)
    _, r, cnt, per, states = _scan(B, dev, [(buf, 0)], 1 << 16)
    assert [(e[1], e[2], e[3], e[4]) for e in got] == [(e[1], e[2], e[3], e[4]) for e in per[0]]


def test_frame_scan_long_decoy_chains(dev, B, oracle):
    """Guesses that land on chains that are not the stream's: a 2.5 MiB skippable chunk whose payload
    is itself a valid frame stream (segments inside it guess, walk and link up among themselves), and
    uncompressed chunks straddling segment starts whose payloads carry chunk headers from the segment
    start on (each such guess is a plausible 4-hop run, rejected by the stitch's re-walk).  The list,
    consumed position and state equal the oracle's, and the lane walk's."""
    rng = random.Random(21)
    seg = 1 << 20

    def fake(n):
        """a valid frame stream (no identifier) of about n bytes"""
        out = b""
        while len(out) < n:
            d = oracle.textgen_chunk(rng.randrange(1 << 20), rng.randint(3000, 9000))
            out += oracle.snappy_frame_encode(d, started=True)[0]
        return out

    parts = [ID]
    size = len(ID)

    def add(b):
        nonlocal size
        parts.append(b)
        size += len(b)

    # ordinary chunks, then a skippable chunk whose payload is a frame stream spanning segments
    while size < seg + 5000:
        add(oracle.snappy_frame_encode(oracle.textgen_chunk(rng.randrange(1 << 20), 60000), started=True)[0])
    decoy = fake((5 << 20) // 2)
    add(bytes([0x9A]) + len(decoy).to_bytes(3, "little") + decoy)
    # uncompressed chunks whose payload starts d bytes before a segment start and holds chunk headers
    # from there on
    for k in range(4):
        boundary = (size // seg + 1) * seg
        d = 3 + k
        p = boundary - 8 - d
        while p - size < 4 + 70000:  # ordinary chunks up to within one uncompressed chunk of p
            add(oracle.snappy_frame_encode(oracle.textgen_chunk(rng.randrange(1 << 20), 60000), started=True)[0])
            boundary = (size // seg + 1) * seg
            p = boundary - 8 - d
        gap = p - size - 4
        while gap > 0xFFFFFF:
            add(_skippable(0x85, 0xFFFFFF - 8))
            gap = p - size - 4
        add(_skippable(0x85, gap))
        assert size == p
        payload = bytes(range(d)) + fake(50000)[:65536 - d]
        add(bytes([1]) + (len(payload) + 4).to_bytes(3, "little") + oracle.snappy_checksum(payload).to_bytes(4, "little")
            + payload)
    end = size // seg * seg + seg + 100000
    while size < end:
        add(oracle.snappy_frame_encode(oracle.textgen_chunk(rng.randrange(1 << 20), 60000), started=True)[0])
    buf = b"".join(parts)
    got, _ = _check_long(B, dev, oracle, buf)
    _, r, cnt, per, states = _scan(B, dev, [(buf, 0)], 1 << 16)
    assert [(e[1], e[2], e[3], e[4]) for e in got] == [(e[1], e[2], e[3], e[4]) for e in per[0]]
    assert len(got) > 100
