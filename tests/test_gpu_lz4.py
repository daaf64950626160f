"""GPU parity: LZ4 block decode (nx_lz4_decode_batch, §8f row 4) against the oracle's restatement of
the LZ4 block format (oracle/netty_oracle.c orc_lz4_decompress), and LZ4 block encode
(nx_lz4_encode_batch) against the oracle's LZ4_compress_default restatement (pinned against
liblz4 itself): bytes and status."""
import random

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def B():
    from netty_amd import batch
    return batch


def _run(B, dev, blocks, wants, align=16):
    inp, off, ln = B.pack(blocks, dev, align=align)
    out, ooff = B.out_slots([max(w, 1) for w in wants], dev, align=align)
    want = torch.tensor(wants, dtype=torch.int32, device=dev)
    st = B.lz4_decode(inp, off, ln, out, ooff, want)
    torch.cuda.synchronize()
    outh, oo = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    return st.cpu().tolist(), [outh[o:o + w] for o, w in zip(oo, wants)]


def _corpus(oracle):
    rng = random.Random(11)
    data = [b"a", b"hello", bytes(100), bytes(range(256)) * 3]
    for n in (15, 16, 17, 63, 64, 65, 1000, 4096, 40000, 65536):
        data.append(oracle.textgen_chunk(n, n))
        data.append(bytes(rng.getrandbits(8) for _ in range(min(n, 3000))))
    for per in (1, 2, 3, 7, 64, 65, 300):
        data.append(bytes((i % per) * 31 & 0xFF for i in range(20000)))
    data += [oracle.textgen_chunk(500 + i, 65536) for i in range(32)]
    return data


@pytest.mark.parametrize("align", [16, 1])
def test_lz4_decode_parity(dev, B, oracle, align):
    data = _corpus(oracle)
    blocks = [oracle.lz4_compress(d) for d in data]
    st, outs = _run(B, dev, blocks, [len(d) for d in data], align)
    assert st == [0] * len(data)
    for i, d in enumerate(data):
        assert outs[i] == d, i


def test_lz4_decode_malformed(dev, B, oracle):
    cases = [(b"", 0), (b"\x50hell", 5), (b"\x50hello", 4), (b"\x50hello", 6), (b"\x10a\x00\x00\x50bcdef", 10),
             (b"\x10a\x02\x00\x50bcdef", 10), (b"\x10a\x01", 10), (b"\xf0", 20), (b"\xf0\xff", 300),
             (b"\x10a\x01\x00\x50bcdef", 10), (b"\x50hello", 5), (b"\x1fa\x01\x00\xff\x05\x50bcdef", 300),
             (b"\x1fa\x01\x00\xff\x05\x50bcdef", 285)]
    good = oracle.lz4_compress(oracle.textgen_chunk(3, 30000))
    for cut in (1, 2, 100, len(good) // 2, len(good) - 1):
        cases.append((good[:cut], 30000))
    cases.append((good, 29999))
    cases.append((good, 30001))
    st, outs = _run(B, dev, [c for c, _ in cases], [w for _, w in cases])
    for i, (blk, w) in enumerate(cases):
        ost, obytes = oracle.lz4_decompress(blk, w)
        assert st[i] == ost, (i, blk[:16], w)
        if ost == 0:
            assert outs[i] == obytes


def test_lz4_decode_fuzz_corrupted(dev, B, oracle):
    """Seeded corruptions of valid blocks (byte flips, 255-runs in length fields, truncation, extra
    bytes) and wrong expected lengths, against the oracle's orc_lz4_decompress: same status, and the
    same bytes where it succeeds."""
    rng = random.Random(2024)
    base = [oracle.textgen_chunk(900 + i, n) for i, n in enumerate((300, 4096, 20000, 65536))]
    base += [bytes(rng.getrandbits(8) for _ in range(3000)), bytes((i % 5) * 40 for i in range(9000))]
    blocks, wants = [], []
    for k in range(480):
        d = base[k % len(base)]
        z = bytearray(oracle.lz4_compress(d))
        kind = k % 6
        if kind == 0:
            for _ in range(1 + rng.randrange(3)):
                z[rng.randrange(len(z))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            p = rng.randrange(len(z))
            z[p:p + 1 + rng.randrange(6)] = b"\xff" * (1 + rng.randrange(6))
        elif kind == 2:
            z = z[:rng.randrange(len(z) + 1)]
        elif kind == 3:
            z += bytes(rng.getrandbits(8) for _ in range(1 + rng.randrange(8)))
        elif kind == 4:
            z[rng.randrange(len(z))] = rng.getrandbits(8)
        w = len(d) + (rng.randrange(-3, 4) if kind == 5 else 0)
        blocks.append(bytes(z))
        wants.append(max(w, 0))
    st, outs = _run(B, dev, blocks, wants)
    for i, (blk, w) in enumerate(zip(blocks, wants)):
        ost, obytes = oracle.lz4_decompress(blk, w)
        assert st[i] == ost, (i, w)
        if ost == 0:
            assert outs[i] == obytes, i


def test_lz4_record_overflow_falls_back(dev, B, oracle):
    """A block of 20 000 one-literal + 4-byte-match sequences needs 40 000 records (> 16 384 per slot):
    it is decoded by the lane-serial kernel, with the same result."""
    blk = b"".join(bytes([0x10, 65 + (i % 26), 0x01, 0x00]) for i in range(20000)) + b"\x10z"
    want = 20000 * 5 + 1
    ost, obytes = oracle.lz4_decompress(blk, want)
    assert ost == 0
    st, outs = _run(B, dev, [blk, oracle.lz4_compress(b"xyz" * 1000)], [want, 3000])
    assert st == [0, 0] and outs[0] == obytes and outs[1] == b"xyz" * 1000


@pytest.mark.parametrize("align", [16, 1])
def test_lz4_encode_parity_and_roundtrip(dev, B, oracle, align):
    """GPU encoder bytes == the oracle's greedy compressor, and GPU decode restores the input."""
    data = _corpus(oracle) + [b"", b"abc", oracle.java_random_bytes(5, 65536)]
    inp, off, ln = B.pack(data, dev, align=align)
    cap = [B.lz4_max_compressed_length(len(d)) for d in data]
    out, ooff = B.out_slots(cap, dev, align=align)
    olen, st = B.lz4_encode(inp, off, ln, out, ooff)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(data)
    outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
    blocks = [outh[o:o + n] for o, n in zip(oo, ol)]
    for i, d in enumerate(data):
        assert blocks[i] == oracle.lz4_compress(d), i
    st2, outs = _run(B, dev, blocks, [len(d) for d in data], align)
    assert st2 == [0] * len(data) and outs == list(data)


def _hc_corpus(oracle):
    rng = random.Random(13)
    data = [b"", b"a", b"hello", b"abcdabcdabcda", bytes(100), bytes(range(256)) * 3, b"x" * 5000, b"ab" * 3000,
            b"abc" * 2000, b"abcd" * 2000, (b"q" * 300 + b"rs" * 100 + oracle.textgen_chunk(3, 500)) * 6]
    for n in (13, 17, 64, 1000, 4096, 30000, 65536):
        data.append(oracle.textgen_chunk(900 + n, n))
        data.append(bytes(rng.getrandbits(8) for _ in range(min(n, 2000))))
    data += [bytes((i % p) * 29 & 0xFF for i in range(12000)) for p in (1, 2, 3, 5, 64)]
    data.append(oracle.textgen_chunk(77, 150000))  # > 64 KiB: the chain table wraps, 65535-distance limit
    return data


@pytest.mark.parametrize("align", [16, 1])
def test_lz4hc_encode_parity_and_roundtrip(dev, B, oracle, align):
    """Lz4FrameEncoder(highCompressor = true)'s block compressor (LZ4_compress_HC level 9): GPU bytes ==
    the oracle's restatement (itself byte-equal to liblz4 at level 9), and the blocks decode back."""
    data = _hc_corpus(oracle)
    inp, off, ln = B.pack(data, dev, align=align)
    cap = [B.lz4_max_compressed_length(len(d)) for d in data]
    out, ooff = B.out_slots(cap, dev, align=align)
    olen, st = B.lz4_encode(inp, off, ln, out, ooff, high=True)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(data)
    outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
    blocks = [outh[o:o + n] for o, n in zip(oo, ol)]
    for i, d in enumerate(data):
        assert blocks[i] == oracle.lz4hc_compress(d), i
    st2, outs = _run(B, dev, blocks, [len(d) for d in data], align)
    assert st2 == [0] * len(data) and outs == list(data)


def test_lz4hc_repeated_launches_reuse_tables(dev, B, oracle):
    """A lane's tables carry the earlier blocks' entries (no clearing between blocks: each block gets
    a higher index base); 20 launches over the same lanes give the fresh-context bytes every time."""
    data = [oracle.textgen_chunk(40 + i, 20000 + 531 * i) for i in range(6)]
    want = [oracle.lz4hc_compress(d) for d in data]
    inp, off, ln = B.pack(data, dev)
    out, ooff = B.out_slots([B.lz4_max_compressed_length(len(d)) for d in data], dev)
    for r in range(20):
        olen, st = B.lz4_encode(inp, off, ln, out, ooff, high=True)
        torch.cuda.synchronize()
        outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
        assert [outh[o:o + n] for o, n in zip(oo, ol)] == want, r


def test_lz4hc_table_reset_after_many_blocks_per_wave(dev, B, oracle):
    """a wave's HC tables are zeroed once its blocks' index bases would pass 2^32 (~125 blocks
    per wave, kHcMaxStamp); one call of 130 blocks per wave crosses that reset (a second launch after a
    memset) and every block still equals the oracle.  The workspace stays at the one-block-per-wave
    bound (CUs x 2 tables of 256 KiB)."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    waves = cus * 2
    n = waves * 130
    rng = random.Random(99)
    pool = [oracle.textgen_chunk(700 + k, 40 + 13 * k) for k in range(31)] + [b"ab" * (20 + k) for k in range(7)] + \
           [bytes(rng.getrandbits(8) for _ in range(60 + k)) for k in range(5)]
    data = [pool[(i * 7) % len(pool)] for i in range(n)]
    inp, off, ln = B.pack(data, dev)
    out, ooff = B.out_slots([B.lz4_max_compressed_length(len(d)) for d in data], dev)
    olen, st = B.lz4_encode(inp, off, ln, out, ooff, high=True)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    want = [oracle.lz4hc_compress(p) for p in pool]
    outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
    for i in range(n):
        assert outh[oo[i]:oo[i] + ol[i]] == want[(i * 7) % len(pool)], i
    hb, _ = B.workspace_info(B.WS_LZ4HC_ENC)
    assert 0 < hb <= waves * 256 * 1024
