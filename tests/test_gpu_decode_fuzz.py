"""Seeded mutation fuzzing of every GPU block decoder against the oracle on the same inputs.

Valid blocks (text-like and random payloads, 1-9 KiB) are damaged — bytes overwritten, a run of
bytes removed or repeated, the block cut short or extended with junk — and each damaged block is
decoded on the GPU and by the oracle's restatement of the reference decoder:
  * Snappy.decode (Snappy.java:315-393): status, consumed bytes and, when the status is OK, the
    output (including Java's silent NOT_ENOUGH_INPUT stop, :332-337);
  * FastLz.decompress (FastLz.java:409-543): Java's return value (0 on a bad stream) and output;
  * LZF ChunkDecoder (LzfDecoder.java:205, compress-lzf's decodeChunk): status and output;
  * LZ4 block decode as Lz4FrameDecoder drives it (Lz4FrameDecoder.java:203-208): status and output.
Both the record-expander paths and their lane-serial fallbacks see these inputs (a damaged block can
need more records than a slot, read past its end, or stop early), so the test checks that the
parallel paths reproduce the reference's error behaviour, not just its output on valid data.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N_PER_CODEC = 600


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def B():
    from netty_amd import batch
    return batch


def _payloads(oracle, rng, n):
    out = []
    for i in range(n):
        L = rng.randint(1024, 9000)
        out.append(oracle.textgen_chunk(rng.randrange(1 << 30), L) if i % 3 else oracle.java_random_bytes(rng.randrange(1 << 30), L))
    return out


def _damage(rng, blk: bytes) -> bytes:
    b = bytearray(blk)
    kind = rng.randrange(6)
    if not b:
        return bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 16)))
    if kind == 0:  # overwrite 1-3 bytes
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(len(b))] = rng.getrandbits(8)
    elif kind == 1:  # overwrite a byte near the start (headers, preamble, first tags)
        b[rng.randrange(min(len(b), 8))] = rng.getrandbits(8)
    elif kind == 2:  # remove a run
        a = rng.randrange(len(b))
        del b[a:a + rng.randint(1, 12)]
    elif kind == 3:  # repeat a run
        a = rng.randrange(len(b))
        b[a:a] = b[a:a + rng.randint(1, 12)]
    elif kind == 4:  # cut short
        del b[rng.randrange(len(b)):]
    else:  # junk appended
        b += bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 40)))
    return bytes(b)


def test_snappy_decode_fuzz(dev, B, oracle):
    rng = random.Random(101)
    cases = [_damage(rng, oracle.snappy_encode(p)) for p in _payloads(oracle, rng, N_PER_CODEC)]
    for variant in ("auto", "pair", "fused"):
        inp, off, ln = B.pack(cases, dev)
        out, ooff = B.out_slots([65536] * len(cases), dev)
        r = B.snappy_decode(inp, off, ln, out, ooff, consumed=True, variant=variant)
        torch.cuda.synchronize()
        st, olen, cons = r["status"].cpu().tolist(), r["out_len"].cpu().tolist(), r["consumed"].cpu().tolist()
        outh, oo = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
        n_ok = 0
        for i, c in enumerate(cases):
            wst, wout, wcons = oracle.snappy_decode(c, 65536)
            assert st[i] == wst, (variant, i, c[:12].hex(), st[i], wst)
            if wst == 0:
                n_ok += 1
                assert outh[oo[i]:oo[i] + olen[i]] == wout, (variant, i)
                assert cons[i] == wcons, (variant, i, cons[i], wcons)
        assert 0 < n_ok < len(cases)  # both outcomes are exercised


def test_fastlz_decompress_fuzz(dev, B, oracle):
    rng = random.Random(202)
    pay = _payloads(oracle, rng, N_PER_CODEC)
    blocks = [_damage(rng, oracle.fastlz_compress(p, 1 + (i % 2))) for i, p in enumerate(pay)]
    lims = [len(p) + rng.choice((0, 0, 0, -1, 7)) for p in pay]
    inp, off, ln = B.pack(blocks, dev)
    out, ooff = B.out_slots([max(x, 1) for x in lims], dev)
    lim = torch.tensor(lims, dtype=torch.int32, device=dev)
    res = B.fastlz_decompress(inp, off, ln, out, ooff, lim).cpu().tolist()
    h, oo = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    n_ok = 0
    for i, z in enumerate(blocks):
        wr, wout = oracle.fastlz_decompress(z, lims[i])
        assert res[i] == wr, (i, z[:12].hex(), lims[i], res[i], wr)
        if wr > 0:
            n_ok += 1
            assert h[oo[i]:oo[i] + wr] == wout, i
    assert 0 < n_ok < len(blocks)


def test_lzf_decode_fuzz(dev, B, oracle):
    rng = random.Random(303)
    pay = _payloads(oracle, rng, N_PER_CODEC)
    bodies = [_damage(rng, oracle.lzf_compress_body(p)) for p in pay]
    ulens = [len(p) for p in pay]
    inp, off, ln = B.pack(bodies, dev)
    out, ooff = B.out_slots(ulens, dev)
    ul = torch.tensor(ulens, dtype=torch.int32, device=dev)
    st = B.lzf_decode(inp, off, ln, out, ooff, ul).cpu().tolist()
    h, oo = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    n_ok = 0
    for k, body in enumerate(bodies):
        wst, wout = oracle.lzf_decode_chunk(body, ulens[k])
        assert st[k] == wst, (k, body[:12].hex(), st[k], wst)
        if wst == 0:
            n_ok += 1
            assert h[oo[k]:oo[k] + ulens[k]] == wout, k
    assert 0 < n_ok < len(bodies)


def test_lz4_decode_fuzz(dev, B, oracle):
    rng = random.Random(404)
    pay = _payloads(oracle, rng, N_PER_CODEC)
    blocks = [_damage(rng, oracle.lz4_compress(p)) for p in pay]
    wants = [len(p) + rng.choice((0, 0, 0, -1, 5)) for p in pay]
    inp, off, ln = B.pack(blocks, dev)
    out, ooff = B.out_slots([max(w, 1) for w in wants], dev)
    want = torch.tensor(wants, dtype=torch.int32, device=dev)
    st = B.lz4_decode(inp, off, ln, out, ooff, want)
    torch.cuda.synchronize()
    st = st.cpu().tolist()
    h, oo = out.cpu().numpy().tobytes(), ooff.cpu().tolist()
    n_ok = 0
    for i, blk in enumerate(blocks):
        ost, obytes = oracle.lz4_decompress(blk, wants[i])
        assert st[i] == ost, (i, blk[:12].hex(), wants[i], st[i], ost)
        if ost == 0:
            n_ok += 1
            assert h[oo[i]:oo[i] + wants[i]] == obytes, i
    assert 0 < n_ok < len(blocks)
