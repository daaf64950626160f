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
