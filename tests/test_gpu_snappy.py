"""GPU parity: Snappy encode/decode/CRC32C batch kernels vs the CPU oracle (bit-exact), through
the C-ABI (netty_amd.batch → libnetty_amd.so)."""
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


def _corpus(oracle, kat):
    rng = random.Random(1234)
    chunks = []
    for n in list(range(0, 41)) + [59, 60, 61, 62, 63, 64, 65, 127, 128, 129, 255, 256, 1000, 4095, 4096, 4097]:
        chunks.append(oracle.textgen_chunk(n + 17, n))
        chunks.append(bytes(rng.getrandbits(8) for _ in range(n)))
    for n in (32767, 65535, 65536):
        chunks.append(oracle.textgen_chunk(n, n))
        chunks.append(oracle.java_random_bytes(n, n))
        chunks.append(bytes(n))
        chunks.append(bytes([123]) * n)
    chunks.append(bytes(i & 0xFF for i in range(1024)))
    chunks.append(bytes.fromhex(kat["identity_inputs"]["issue_1002"]))
    part = bytearray(oracle.java_random_bytes(7, 10240))
    part[:1024] = b"\x02" * 1024
    chunks.append(bytes(part))
    comp = bytearray(10240)
    r = oracle.java_random_bytes(9, 10240)
    for i in range(0, 10240, 4):
        comp[i] = r[i]
    chunks.append(bytes(comp))
    for i in range(64):
        chunks.append(oracle.textgen_chunk(1000 + i, 65536))
    # periodic data with short periods: exercises overlapping copies (offset < length)
    for per in (1, 2, 3, 5, 7, 13, 31, 63, 64, 65):
        chunks.append(bytes((i % per) * 37 & 0xFF for i in range(9000)))
    return chunks


@pytest.mark.parametrize("in_align,out_align", [(16, 16), (16, 4), (1, 1)])
def test_snappy_encode_parity(dev, B, oracle, kat, in_align, out_align):
    """Output slots 16-aligned (16-byte staged stores), 4-aligned (dword stores) and unaligned (bytes)."""
    chunks = _corpus(oracle, kat)
    inp, off, ln = B.pack(chunks, dev, align=in_align)
    cap = [B.snappy_max_compressed_length(len(c)) + (3 if out_align == 1 else 0) for c in chunks]
    out, ooff = B.out_slots(cap, dev, align=out_align)
    olen, st = B.snappy_encode(inp, off, ln, out, ooff)
    torch.cuda.synchronize()
    olen, st, ooff_h, outh = olen.cpu().tolist(), st.cpu().tolist(), ooff.cpu().tolist(), out.cpu().numpy().tobytes()
    for i, c in enumerate(chunks):
        want = oracle.snappy_encode(c)
        got = outh[ooff_h[i]:ooff_h[i] + olen[i]]
        assert st[i] == 0
        assert got == want, (i, len(c))


@pytest.mark.parametrize("variant,align", [("auto", 16), ("pair", 16), ("pair", 1), ("fused", 16), ("fused", 1), ("naive", 16)])
def test_snappy_decode_parity(dev, B, oracle, kat, naive_decode, variant, align):
    chunks = _corpus(oracle, kat)
    enc = [oracle.snappy_encode(c) for c in chunks]
    inp, off, ln = B.pack(enc, dev, align=align)
    out, ooff = B.out_slots([65536] * len(enc), dev)
    crcs = torch.tensor([oracle.snappy_checksum(c) for c in chunks], dtype=torch.int64).to(torch.int32).to(dev)
    r = B.snappy_decode(inp, off, ln, out, ooff, expected_crc=crcs, want_crc=True, consumed=True,
                        variant="auto" if variant == "naive" else variant, fn=naive_decode if variant == "naive" else None)
    torch.cuda.synchronize()
    st, olen, cons = r["status"].cpu().tolist(), r["out_len"].cpu().tolist(), r["consumed"].cpu().tolist()
    crc = [x & 0xFFFFFFFF for x in r["crc"].cpu().tolist()]
    outh, ooff_h = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    for i, c in enumerate(chunks):
        if len(c) > 65536:
            continue
        assert st[i] == 0, (i, st[i])
        assert olen[i] == len(c)
        assert outh[ooff_h[i]:ooff_h[i] + olen[i]] == c, i
        assert cons[i] == len(enc[i])
        assert crc[i] == oracle.snappy_checksum(c)


def _crafted_streams(oracle, kat):
    cases = [bytes.fromhex(v["in"]) for v in kat["snappy_decode"]]
    base = oracle.snappy_encode(oracle.textgen_chunk(77, 3000))
    cases += [base[:k] for k in (0, 1, 2, 3, 4, 5, 17, 100, len(base) // 2, len(base) - 1)]
    rnd = oracle.snappy_encode(oracle.java_random_bytes(5, 3000))
    cases += [rnd[:k] for k in (2, 3, 4, 100, 2999)]
    cases += [
        bytes([0x05, 63 << 2, 0xFF, 0xFF, 0xFF, 0x7F]),  # literal len invalid
        bytes([0x05, 63 << 2, 0xFF, 0xFF, 0xFF, 0xFF, 0x10]) + b"netty",  # zero-length literal
        bytes([0x0a, 0x10]) + b"netty" + bytes([0x13, 0, 0, 0, 0x80]),  # COPY_4 negative offset
        bytes([0x0a, 0x10]) + b"netty" + bytes([0x13, 5, 0, 0, 0]),  # COPY_4 valid
        bytes([0x0a, 0x10]) + b"netty" + bytes([0x13, 5, 0]),  # COPY_4 truncated
        bytes([0x80, 0x80, 0x05, 0x00]),  # preamble > 65536 (overflow at ensureWritable)
        bytes([0x00]), bytes([0x80]), bytes([0x80, 0x80]),  # preamble 0 / incomplete
        bytes([0x05, 0xF0, 0x04]),  # literal code 60 len byte present, data missing
        bytes([0x05, 0xF0]),  # literal code 60 len byte missing
        bytes([0x40, 0x00 | (59 << 2)]) + bytes(60) + bytes([0x01 | (7 << 2), 0x01]) * 20,  # copies overflow-free
        bytes([0x85, 0x04, 0x00, 0x00]) + bytes([0x02 | (63 << 2), 0x01, 0x00]) * 1030,  # 1 literal + copies > 65536 → overflow
    ]
    return cases


@pytest.mark.parametrize("variant", ["auto", "pair", "fused", "naive"])
def test_snappy_decode_edge_cases(dev, B, oracle, kat, naive_decode, variant):
    cases = _crafted_streams(oracle, kat)
    inp, off, ln = B.pack(cases, dev)
    out, ooff = B.out_slots([65536] * len(cases), dev)
    r = B.snappy_decode(inp, off, ln, out, ooff, consumed=True, variant="auto" if variant == "naive" else variant,
                        fn=naive_decode if variant == "naive" else None)
    torch.cuda.synchronize()
    st, olen, cons = r["status"].cpu().tolist(), r["out_len"].cpu().tolist(), r["consumed"].cpu().tolist()
    outh, ooff_h = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    for i, c in enumerate(cases):
        wst, wout, wcons = oracle.snappy_decode(c, 65536)
        assert st[i] == wst, (i, c[:16].hex(), st[i], wst)
        if wst == 0:
            assert outh[ooff_h[i]:ooff_h[i] + olen[i]] == wout, i
            assert cons[i] == wcons, (i, cons[i], wcons)


def _copy_run(n_out, length, offset=1):
    """A raw Snappy block: preamble n_out, literal 'a', then COPY_2 tags of `length` at `offset`."""
    pre, v = bytearray(), n_out
    while v >= 0x80:
        pre.append((v & 0x7F) | 0x80)
        v >>= 7
    pre.append(v)
    tag = bytes([0x02 | ((length - 1) << 2), offset & 0xFF, offset >> 8])
    return bytes(pre) + bytes([0x00]) + b"a" + tag * ((n_out - 1) // length)


def test_snappy_decode_record_overflow_falls_back(dev, B, oracle):
    """Frames with more output-producing tags than a record slot holds (16384) are decoded by the
    single-kernel path inside nx_snappy_decode_batch; results stay bit-exact with the oracle."""
    cases = [_copy_run(65536, 1), _copy_run(16385, 1), _copy_run(16384, 1), _copy_run(16386, 1)[:-1],
             _copy_run(40000, 2)[:-3] + bytes([0x02 | (3 << 2), 0xFF, 0xFF]),  # ends on an offset-beyond error
             oracle.snappy_encode(oracle.textgen_chunk(5, 65536))]
    inp, off, ln = B.pack(cases, dev, align=1)
    out, ooff = B.out_slots([65536] * len(cases), dev)
    r = B.snappy_decode(inp, off, ln, out, ooff, consumed=True, want_crc=True)
    torch.cuda.synchronize()
    st, olen, cons = r["status"].cpu().tolist(), r["out_len"].cpu().tolist(), r["consumed"].cpu().tolist()
    crc = [x & 0xFFFFFFFF for x in r["crc"].cpu().tolist()]
    outh, ooff_h = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    for i, c in enumerate(cases):
        wst, wout, wcons = oracle.snappy_decode(c, 65536)
        assert st[i] == wst, (i, st[i], wst)
        assert olen[i] == len(wout), i
        assert outh[ooff_h[i]:ooff_h[i] + olen[i]] == wout, i
        assert cons[i] == wcons, (i, cons[i], wcons)
        assert crc[i] == oracle.snappy_checksum(wout), i


def test_snappy_decode_detects_crc_corruption(dev, B, oracle):
    chunks = [oracle.textgen_chunk(500 + i, 65536) for i in range(100)]
    enc = [oracle.snappy_encode(c) for c in chunks]
    crcs = [oracle.snappy_checksum(c) for c in chunks]
    bad = {3, 50, 97}  # BASELINE config 3: a corrupted-CRC subset must be detected
    for i in bad:
        crcs[i] ^= 0x1
    inp, off, ln = B.pack(enc, dev)
    out, ooff = B.out_slots([65536] * len(enc), dev)
    exp = torch.tensor(crcs, dtype=torch.int64).to(torch.int32).to(dev)
    r = B.snappy_decode(inp, off, ln, out, ooff, expected_crc=exp)
    st = r["status"].cpu().tolist()
    assert [i for i, s in enumerate(st) if s != 0] == sorted(bad)
    assert all(st[i] == -7 for i in bad)


def test_crc32c_batch(dev, B, oracle):
    rng = random.Random(9)
    chunks = [bytes(rng.getrandbits(8) for _ in range(n)) for n in
              [0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 2047, 4096, 5000]]
    chunks += [oracle.textgen_chunk(i, 65536) for i in range(4)] + [oracle.textgen_chunk(9, 32767)]
    inp, off, ln = B.pack(chunks, dev, align=1)  # unaligned starts
    got = [x & 0xFFFFFFFF for x in B.crc32c_masked(inp, off, ln).cpu().tolist()]
    assert got == [oracle.snappy_checksum(c) for c in chunks]


def test_crc32c_block_edges_every_alignment(dev, B, oracle):
    """The CRC kernel reads a chunk as 8 KiB blocks of 128-byte lane slots aligned to the chunk END
    (leading/trailing zero padding, init folded into bytes 0..3): lengths around the block and slot
    edges (including chunk bytes 0..3 straddling blocks 0/1), at every start address mod 16."""
    rng = random.Random(11)
    lengths = [4, 5, 7, 8, 127, 128, 129, 8187, 8188, 8189, 8190, 8191, 8192, 8193, 8196, 16380, 16385, 16387, 16388,
               24577, 65535, 65536, 65537, 100003]
    buf, offs, lens, want = bytearray(), [], [], []
    for n in lengths:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        for s in range(16):
            pos = (len(buf) + 15) // 16 * 16 + s
            buf.extend(bytes(pos - len(buf)))
            offs.append(pos)
            buf.extend(data)
            lens.append(n)
        want += [oracle.snappy_checksum(data)] * 16
    buf.extend(bytes(32))
    inp = torch.frombuffer(buf, dtype=torch.uint8).to(dev)
    off = torch.tensor(offs, dtype=torch.int64, device=dev)
    ln = torch.tensor(lens, dtype=torch.int32, device=dev)
    got = [x & 0xFFFFFFFF for x in B.crc32c_masked(inp, off, ln).cpu().tolist()]
    assert got == want


def test_textgen_device_matches_host(dev, B, oracle):
    n, L = 37, 65536
    out = torch.empty(n * L, dtype=torch.uint8, device=dev)
    B.textgen(out, 1000, n, L)
    h = out.cpu().numpy().tobytes()
    for k in (0, 1, 17, 36):
        assert h[k * L:(k + 1) * L] == oracle.textgen_chunk(1000 + k, L)


def test_device_roundtrip_many_chunks(dev, B, oracle):
    """Size-independent property at scale: GPU encode → GPU decode is the identity, CRC verifies,
    and a sample of chunks is byte-identical to the oracle's encoding."""
    n, L = 8192, 65536
    src = torch.empty(n * L, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, n, L)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    ln = torch.full((n,), L, dtype=torch.int32, device=dev)
    cap = B.snappy_max_compressed_length(L)
    cap = (cap + 15) // 16 * 16
    enc = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    eoff = torch.arange(n, dtype=torch.int64, device=dev) * cap
    elen, est = B.snappy_encode(src, off, ln, enc, eoff)
    crc = B.crc32c_masked(src, off, ln)
    dec = torch.empty_like(src)
    r = B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=crc)
    torch.cuda.synchronize()
    assert int((est != 0).sum()) == 0 and int((r["status"] != 0).sum()) == 0
    assert torch.equal(r["out_len"], ln)
    assert torch.equal(dec, src)
    elh, ench = elen.cpu().tolist(), None
    for k in (0, 1, 4095, 8191):
        e = enc[k * cap:k * cap + elh[k]].cpu().numpy().tobytes()
        assert e == oracle.snappy_encode(oracle.textgen_chunk(k, L))


def test_pack_batch_gathers_slots():
    """nx_pack_batch: variable-length slots → one contiguous stream (aligned and unaligned)."""
    import torch
    from netty_amd import batch as B
    g = torch.Generator().manual_seed(5)
    n = 300
    lens = torch.randint(0, 3000, (n,), generator=g, dtype=torch.int32)
    lens[:3] = torch.tensor([0, 1, 17], dtype=torch.int32)
    src_off = torch.arange(n, dtype=torch.int64) * 3072 + torch.randint(0, 16, (n,), generator=g)
    src = torch.randint(0, 256, (n * 3072 + 64,), generator=g, dtype=torch.uint8)
    for shift in (0, 3):
        d_src, d_off, d_len = src.cuda(), src_off.cuda(), lens.cuda()
        dst_off = torch.zeros(n, dtype=torch.int64)
        dst_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
        dst_off += shift
        dst = torch.zeros(int(dst_off[-1] + lens[-1]) + 16, dtype=torch.uint8, device="cuda")
        B.gather(d_src, d_off, d_len, dst, dst_off.cuda())
        want = torch.cat([src[int(o):int(o) + int(l)] for o, l in zip(src_off, lens)])
        got = dst.cpu()[shift:shift + want.numel()]
        assert torch.equal(got, want)


@pytest.mark.parametrize("n", [1, 7, 256, 257, 4097, 16384, 16385])
def test_snappy_encode_batch_size_forms(dev, B, oracle, n):
    """nx_snappy_encode_batch picks the LDS form (n <= CUs), the wave-per-chunk form (n <= 16 384) or
    the dense lane-per-chunk form by batch size: each is bit-exact with the oracle, on mixed sizes
    (1 B .. 64 KiB, text and random) and unaligned starts/outputs."""
    rng = random.Random(n)
    idx = sorted({0, n - 1} | {rng.randrange(n) for _ in range(min(n, 40))})
    sizes = [rng.choice([1, 14, 15, 16, 100, 4096, 32767, 65535, 65536]) if i in idx else 64 for i in range(n)]
    chunks = [(oracle.textgen_chunk(i, s) if i % 2 else bytes(rng.getrandbits(8) for _ in range(s))) if i in idx
              else bytes(s) for i, s in enumerate(sizes)]
    inp, off, ln = B.pack(chunks, dev, align=1)
    cap = [B.snappy_max_compressed_length(len(c)) + 1 for c in chunks]
    out, ooff = B.out_slots(cap, dev, align=1)
    olen, st = B.snappy_encode(inp, off, ln, out, ooff)
    assert int((st != 0).sum()) == 0
    ol, oo = olen.cpu().tolist(), ooff.cpu().tolist()
    for i in idx:
        assert out[oo[i]:oo[i] + ol[i]].cpu().numpy().tobytes() == oracle.snappy_encode(chunks[i]), i
    zero = oracle.snappy_encode(bytes(64))
    for i in range(0, n, max(1, n // 50)):
        if i not in idx:
            assert out[oo[i]:oo[i] + ol[i]].cpu().numpy().tobytes() == zero, i


@pytest.mark.parametrize("fill", [300, 16400])
def test_snappy_encode_parity_hbm_forms(dev, B, oracle, kat, fill):
    """The whole parity corpus (short, random, zero, periodic, KAT inputs) through the HBM-table forms
    (wave per chunk above CUs chunks, lane per chunk above 16 384) whose 64-bit entries decide the
    candidate compare and short matches from the table alone: every chunk equals the oracle's bytes."""
    corpus = _corpus(oracle, kat)
    chunks = corpus + [oracle.textgen_chunk(5000 + i, 200) for i in range(fill - len(corpus))]
    inp, off, ln = B.pack(chunks, dev, align=1)
    cap = [B.snappy_max_compressed_length(len(c)) for c in chunks]
    out, ooff = B.out_slots(cap, dev)
    olen, st = B.snappy_encode(inp, off, ln, out, ooff)
    assert int((st != 0).sum()) == 0
    ol, oo, h = olen.cpu().tolist(), ooff.cpu().tolist(), out.cpu().numpy().tobytes()
    for i in list(range(len(corpus))) + [len(chunks) - 1]:
        assert h[oo[i]:oo[i] + ol[i]] == oracle.snappy_encode(chunks[i]), (i, len(chunks[i]))


def test_snappy_encode_stamp_wrap_many_chunks_per_lane(dev, B, oracle):
    """one encoder lane encodes more chunks than there are table stamps (63), so
    the host splits the batch into launches and re-zeroes the stamped table workspace before the
    stamps wrap (snappy_encode.hip nx_snappy_encode_batch).  Lane t encodes chunks t, t + lanes, ...;
    the chunks of the first and last lane in every launch, and a random sample, must equal the
    oracle's bytes."""
    lanes = torch.cuda.get_device_properties(dev).multi_processor_count * 16 * 64
    n, L = lanes * 63 + 7, 160
    src = torch.empty(n * L, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, n, L)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    ln = torch.full((n,), L, dtype=torch.int32, device=dev)
    cap = (B.snappy_max_compressed_length(L) + 15) // 16 * 16
    out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    ooff = torch.arange(n, dtype=torch.int64, device=dev) * cap
    olen, st = B.snappy_encode(src, off, ln, out, ooff)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    rng = random.Random(5)
    pick = sorted({k * lanes + t for k in range(64) for t in (0, lanes - 1)} | {rng.randrange(n) for _ in range(300)})
    pick = [i for i in pick if i < n]
    ol = olen[pick].cpu().tolist()
    for i, m in zip(pick, ol):
        got = out[i * cap:i * cap + m].cpu().numpy().tobytes()
        assert got == oracle.snappy_encode(oracle.textgen_chunk(i, L)), i
    del src, out
