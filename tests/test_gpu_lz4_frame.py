"""GPU parity for the LZ4 frame codec (§8f row 4): nx_xxhash32_batch against the oracle's XXH32
(itself pinned by Lz4FrameDecoderTest.java:33-41 and python-xxhash), nx_lz4_frame_encode_batch
byte-for-byte against the oracle's Lz4FrameEncoder.flushBufferedData restatement, and
nx_lz4_frame_scan_batch + decode + checksum against the oracle's Lz4FrameDecoder walk, including the
reference's own corrupted-stream cases (Lz4FrameDecoderTest.java:50-147)."""
import random

import pytest

from tests.test_oracle_kat import LZ4_DECODER_TEST_DATA

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


def _blocks(oracle):
    rng = random.Random(5)
    data = [b"", b"a", b"Netty", bytes(15), bytes(16), bytes(range(17)), bytes(range(63)), bytes(range(64)) * 2]
    for n in (65, 100, 1000, 4095, 40000, 65536):
        data.append(oracle.textgen_chunk(n, n))
        data.append(bytes(rng.getrandbits(8) for _ in range(min(n, 5000))))
    data.append(oracle.java_random_bytes(7, 65536))
    data += [oracle.textgen_chunk(900 + i, 65536) for i in range(16)]
    return data


@pytest.mark.parametrize("align", [16, 1])
def test_xxhash32_parity(dev, B, oracle, align):
    data = _blocks(oracle)
    inp, off, ln = B.pack(data, dev, align=align)
    for seed in (0, B.LZ4_DEFAULT_SEED):
        h = B.xxhash32(inp, off, ln, seed)
        torch.cuda.synchronize()
        got = [v & 0xFFFFFFFF for v in h.cpu().tolist()]
        assert got == [oracle.xxhash32(d, seed) for d in data]


@pytest.mark.parametrize("align", [16, 1])
def test_lz4_frame_encode_parity(dev, B, oracle, align):
    data = _blocks(oracle)
    inp, off, ln = B.pack(data, dev, align=align)
    out, ooff = B.out_slots([21 + B.lz4_max_compressed_length(len(d)) for d in data], dev, align=align)
    olen, st = B.lz4_frame_encode(inp, off, ln, out, ooff, 6)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(data)
    outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
    for i, d in enumerate(data):
        want = oracle.lz4_frame_block(d, 6) if d else b""
        assert outh[oo[i]:oo[i] + ol[i]] == want, i
    # "Netty" alone is Lz4FrameDecoderTest's first block
    k = data.index(b"Netty")
    assert outh[oo[k]:oo[k] + ol[k]] + oracle.lz4_frame_end(6) == LZ4_DECODER_TEST_DATA


def _streams(oracle):
    s = [LZ4_DECODER_TEST_DATA]
    for idx, val in [(1, 0x00), (12, 0xFF), (16, 0xFF), (13, 0x01), (8, 0x36), (17, 0x01), (44, 0x01)]:
        d = bytearray(LZ4_DECODER_TEST_DATA)
        d[idx] = val
        s.append(bytes(d))
    big = oracle.lz4_frame_encode(oracle.textgen_chunk(77, 300000) + oracle.java_random_bytes(3, 100000))
    s += [big, big[:-21], big[:1000], big[:21], big[:20], b"", big + b"trailing junk", b"LZ4Block\x26" + bytes(12)]
    s += [oracle.lz4_frame_encode(oracle.textgen_chunk(i, 10000 + 997 * i), close=bool(i & 1)) for i in range(40)]
    return s


def _scan_cmp(B, oracle, dev, streams, states, cap):
    inp, off, ln = B.pack(streams, dev, align=16)
    off64, ln64 = off.to(torch.int64), ln.to(torch.int64)
    st = torch.tensor(states, dtype=torch.int32, device=dev)
    r = B.lz4_frame_scan(inp, off64, ln64, st, cap)
    torch.cuda.synchronize()
    base = off.cpu().tolist()
    nc, nu, _ = r["counts"].cpu().tolist()
    lists = {k: r[k].cpu().tolist() for k in ("data_off", "comp_len", "decomp_len", "checksum", "stream", "seq")}
    got = {}
    for k in list(range(nc)) + list(range(cap - nu, cap)):
        s = lists["stream"][k]
        got.setdefault(s, []).append((lists["seq"][k], 0x20 if k < nc else 0x10, lists["data_off"][k] - base[s],
                                      lists["comp_len"][k], lists["decomp_len"][k], lists["checksum"][k] & 0xFFFFFFFF))
    cons, stat, stt = r["consumed"].cpu().tolist(), r["status"].cpu().tolist(), st.cpu().tolist()
    for s, buf in enumerate(streams):
        ents, p, ost, res = oracle.lz4_frame_scan(buf, states[s])
        mine = [e[1:] for e in sorted(got.get(s, []))]
        assert [e[0] for e in sorted(got.get(s, []))] == list(range(len(mine)))
        assert (mine, cons[s], stt[s], stat[s]) == (ents, p, ost, res), s
    return inp, r, nc, nu


def test_lz4_frame_scan_parity(dev, B, oracle):
    streams = _streams(oracle)
    states = [0] * len(streams)
    states[1] = 1  # finished decoder: everything is skipped
    states[2] = 2  # corrupted decoder
    _scan_cmp(B, oracle, dev, streams, states, cap=4096)


def test_lz4_frame_scan_list_full(dev, B, oracle):
    f = oracle.lz4_frame_encode(oracle.textgen_chunk(5, 65536 * 5))
    inp, off, ln = B.pack([f], dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    r = B.lz4_frame_scan(inp, off.to(torch.int64), ln.to(torch.int64), st, 3)
    torch.cuda.synchronize()
    assert r["status"].item() == 1 and r["counts"][:2].sum().item() == 3
    ents, p, _, _ = oracle.lz4_frame_scan(f)
    assert r["consumed"].item() == ents[3][1] - 21


def test_lz4_frame_scan_decode_roundtrip(dev, B, oracle):
    """Device scan → nx_lz4_decode_batch → XXH32 verify restores every stream's bytes; a flipped stored
    checksum (Lz4FrameDecoderTest data[17]) is reported as NX_ERR_LZ4_CHECKSUM_MISMATCH."""
    payloads = [oracle.textgen_chunk(40 + i, 20000 + 4099 * i) + oracle.java_random_bytes(i, 3000 * (i % 3))
                for i in range(24)]
    streams = [oracle.lz4_frame_encode(p) for p in payloads]
    bad = bytearray(LZ4_DECODER_TEST_DATA)
    bad[17] = 0x01
    streams.append(bytes(bad))
    cap = 1024
    inp, r, nc, nu = _scan_cmp(B, oracle, dev, streams, [0] * len(streams), cap)
    d = B.lz4_frame_decode(inp, r, cap)
    torch.cuda.synchronize()
    out, oo, stc = (t.cpu() for t in d["compressed"])
    roff, rlen, stu = (t.cpu().tolist() for t in d["raw"])
    outh, inh = out.numpy().tobytes(), inp.cpu().numpy().tobytes()
    pieces = {}
    lists = {k: r[k].cpu().tolist() for k in ("stream", "seq", "decomp_len")}
    stc, oo = stc.tolist(), oo.tolist()
    for k in range(nc):
        pieces[(lists["stream"][k], lists["seq"][k])] = (stc[k], outh[oo[k]:oo[k] + lists["decomp_len"][k]])
    for j, k in enumerate(range(cap - nu, cap)):
        pieces[(lists["stream"][k], lists["seq"][k])] = (stu[j], inh[roff[j]:roff[j] + rlen[j]])
    for s, p in enumerate(payloads):
        seqs = sorted(q for (t, q) in pieces if t == s)
        assert all(pieces[(s, q)][0] == 0 for q in seqs), s
        assert b"".join(pieces[(s, q)][1] for q in seqs) == p, s
    assert pieces[(len(payloads), 0)][0] == -56


@pytest.mark.parametrize("block_size", [1 << 18, 1 << 20])
def test_lz4_frame_large_blocks(dev, B, oracle, block_size):
    """Streams from an Lz4FrameEncoder with a block size above 64 KiB (compressionLevel 8 / 10):
    blocks of more than 64 KiB output decode through the lane-serial kernel, by the scan path and by
    the Lz4FrameDecoder handler, with checksums validated."""
    import netty_amd as nx
    data = oracle.textgen_chunk(61, 3 * block_size // 2) + bytes(block_size // 3) + oracle.java_random_bytes(8, 5000)
    f = oracle.lz4_frame_encode(data, block_size=block_size)
    assert f[8] & 0x0F == oracle.lz4_compression_level(block_size)
    assert b"".join(nx.Lz4FrameDecoder(True).channel_read(f)) == data
    cap = 64
    inp, r, nc, nu = _scan_cmp(B, oracle, dev, [f], [0], cap)
    d = B.lz4_frame_decode(inp, r, cap)
    torch.cuda.synchronize()
    out, oo, stc = (t.cpu() for t in d["compressed"])
    assert stc.tolist() == [0] * nc and d["raw"][2].cpu().tolist() == [0] * nu
    seq = r["seq"][:nc].cpu().tolist()
    dl = r["decomp_len"][:nc].cpu().tolist()
    outh, oo = out.numpy().tobytes(), oo.tolist()
    got = {seq[k]: outh[oo[k]:oo[k] + dl[k]] for k in range(nc)}
    inh = inp.cpu().numpy().tobytes()
    for k in range(cap - nu, cap):
        o, n = int(r["data_off"][k]), int(r["decomp_len"][k])
        got[int(r["seq"][k])] = inh[o:o + n]
    assert b"".join(got[i] for i in range(len(got))) == data


def test_lz4_encode_large_and_small_blocks_mixed(dev, B, oracle):
    """Blocks over 64 KiB (liblz4's byU32 table, cleared per block) interleaved with small stamped
    blocks in one launch: bytes equal the oracle's compressor (= liblz4) for every block."""
    data = []
    for i in range(6):
        data.append(oracle.textgen_chunk(300 + i, 200000 + 50000 * i))
        data.append(oracle.textgen_chunk(400 + i, 30000))
    data.append(oracle.java_random_bytes(9, 150000))
    inp, off, ln = B.pack(data, dev, align=1)
    out, ooff = B.out_slots([B.lz4_max_compressed_length(len(d)) for d in data], dev, align=1)
    olen, st = B.lz4_encode(inp, off, ln, out, ooff)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(data)
    outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
    for i, d in enumerate(data):
        assert outh[oo[i]:oo[i] + ol[i]] == oracle.lz4_compress(d), i


def test_lz4_encode_one_lane_large_then_small(dev, B, oracle):
    """one lane encoding a large (byU32, raw-index) block and then a stamped small block in
    the same launch.  The launch has cus * 1024 lanes and lane t encodes blocks t, t + lanes, ...;
    with lanes + 3 blocks, lane 1 takes the 1 MiB block at index 1 and then the text block at
    1 + lanes.  Every block must equal liblz4's bytes (the oracle)."""
    lanes = torch.cuda.get_device_properties(dev).multi_processor_count * 1024
    small = [b"abcdefghijklmnopq"] * (lanes + 3)
    small[1] = oracle.textgen_chunk(5, 1 << 20)
    small[1 + lanes] = oracle.textgen_chunk(6, 40000)
    small[2] = oracle.textgen_chunk(7, 1 << 25)              # MAX_BLOCK_SIZE itself
    small[2 + lanes] = oracle.textgen_chunk(8, 65536)
    inp, off, ln = B.pack(small, dev, align=1)
    out, ooff = B.out_slots([B.lz4_max_compressed_length(len(d)) for d in small], dev, align=1)
    olen, st = B.lz4_encode(inp, off, ln, out, ooff)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    oo, ol = ooff.cpu().tolist(), olen.cpu().tolist()
    for i in (0, 1, 2, 1 + lanes, 2 + lanes, lanes + 2):
        got = out[oo[i]:oo[i] + ol[i]].cpu().numpy().tobytes()
        assert got == oracle.lz4_compress(small[i]), i


@pytest.mark.parametrize("block_size", [1 << 17, 1 << 20])
def test_lz4_frame_encoder_large_block_size(dev, oracle, block_size):
    import netty_amd as nx
    data = oracle.textgen_chunk(71, 2 * block_size + 12345) + oracle.java_random_bytes(1, 70000)
    enc = nx.Lz4FrameEncoder(block_size)
    comp = enc.encode(data) + enc.finish_encode()
    assert comp == oracle.lz4_frame_encode(data, block_size=block_size)
    assert b"".join(nx.Lz4FrameDecoder(True).channel_read(comp)) == data


def test_lz4_frame_encode_parity_high_compressor(dev, B, oracle):
    """nx_lz4_frame_encode_batch_ex with highCompressor: header + LZ4_compress_HC block (or raw when not
    smaller), as Lz4FrameEncoder(highCompressor = true).flushBufferedData writes them."""
    data = [b"Netty", oracle.textgen_chunk(3, 65536), oracle.java_random_bytes(4, 5000), bytes(3000), oracle.textgen_chunk(8, 777)]
    inp, off, ln = B.pack(data, dev)
    out, ooff = B.out_slots([21 + B.lz4_max_compressed_length(len(d)) for d in data], dev)
    olen, st = B.lz4_frame_encode(inp, off, ln, out, ooff, 6, high=True)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(data)
    outh, oo, ol = out.cpu().numpy().tobytes(), ooff.cpu().tolist(), olen.cpu().tolist()
    for i, d in enumerate(data):
        assert outh[oo[i]:oo[i] + ol[i]] == oracle.lz4_frame_block(d, 6, high=True), i


@pytest.mark.parametrize("block_size", [4096, 1 << 16])
def test_lz4_frame_encoder_high_compressor(dev, oracle, block_size):
    """Lz4FrameEncoder(highCompressor = true) through the handle: the oracle's frame bytes (HC blocks),
    smaller than the fast compressor's on text, and the stream decodes."""
    import netty_amd as nx
    data = oracle.textgen_chunk(72, 3 * block_size + 999) + oracle.java_random_bytes(2, 3000)
    enc = nx.Lz4FrameEncoder(block_size, high_compressor=True)
    comp = enc.encode(data[:5000]) + enc.encode(data[5000:]) + enc.finish_encode()
    assert comp == oracle.lz4_frame_encode(data, block_size=block_size, high=True)
    assert len(comp) < len(oracle.lz4_frame_encode(data, block_size=block_size))
    assert b"".join(nx.Lz4FrameDecoder(True).channel_read(comp)) == data


def test_lz4_frame_encoder_max_encode_size(dev, oracle):
    """maxEncodeSize (Lz4FrameEncoder.java:150-170, allocateBuffer :190-214): encode and flush refuse
    pending bytes whose worst-case output exceeds it with the reference's EncoderException message,
    changing nothing; finishEncode does not check (:306-315); maxEncodeSize <= 0 is refused (:168)."""
    import netty_amd as nx
    from netty_amd.handlers import EncoderException
    with pytest.raises(ValueError, match="maxEncodeSize : 0"):
        nx.Lz4FrameEncoder(4096, max_encode_size=0)
    bound = lambda n: n + n // 255 + 16 + 21  # compressor.maxCompressedLength + HEADER_LENGTH
    limit = 2 * bound(4096) + 100
    enc = nx.Lz4FrameEncoder(4096, max_encode_size=limit)
    ref = nx.Lz4FrameEncoder(4096)
    data = oracle.textgen_chunk(5, 20000)
    assert enc.encode(data[:3000]) == ref.encode(data[:3000]) == b""  # 3000 pending: one block's bound
    want = bound(4096) * 2 + bound(3000 + 8000 - 8192)
    with pytest.raises(EncoderException) as ei:
        enc.encode(data[3000:11000])  # 11000 pending: three blocks
    assert str(ei.value) == (f"requested encode buffer size ({want} bytes) exceeds the maximum "
                             f"allowable size ({limit} bytes)")
    # the refused call changed nothing: the same calls then give the unlimited encoder's bytes
    assert enc.encode(data[3000:8000]) == ref.encode(data[3000:8000]) != b""
    assert enc.flush() == ref.flush()
    assert enc.finish_encode() == ref.finish_encode()
    tight = nx.Lz4FrameEncoder(4096, max_encode_size=bound(100) - 1)
    with pytest.raises(EncoderException):
        tight.encode(b"x" * 100)  # even a message that only fills the buffer is sized first
    assert tight.encode(b"x" * 50) == b""
