"""The lane-per-chunk encoders (LZ4 blocks, FastLZ, LZF) run one chunk per wave for batches up to
16 384 chunks and one chunk per lane above (nx_common.hpp lane_grid); both forms, including waves
that take several chunks, must give the oracle's bytes.  Most chunks are small fillers so the large
batches stay cheap; a sample of real chunks (text / random, up to 64 KiB) is checked everywhere."""
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


def _batch(oracle, n, seed, max_len=65535):
    rng = random.Random(seed)
    idx = sorted({0, n - 1} | {rng.randrange(n) for _ in range(min(n, 24))})
    real = set(idx)
    chunks = []
    for i in range(n):
        if i in real:
            L = rng.choice([5, 31, 32, 100, 4096, 40000, max_len])
            chunks.append(oracle.textgen_chunk(seed * 7919 + i, L) if i % 2 == 0 else oracle.java_random_bytes(seed + i, L))
        else:
            chunks.append(b"netty" * 13)
    return chunks, idx


def _check(out, ooff, olen, st, idx, want):
    st_, ol, oo = st.cpu().tolist(), olen.cpu().tolist(), ooff.cpu().tolist()
    assert all(s == 0 for s in st_)
    for i in idx:
        assert out[oo[i]:oo[i] + ol[i]].cpu().numpy().tobytes() == want(i), i


@pytest.mark.parametrize("n", [3, 5000, 16385])
def test_lz4_encode_forms(dev, B, oracle, n):
    chunks, idx = _batch(oracle, n, 41)
    inp, off, ln = B.pack(chunks, dev, align=1)
    out, ooff = B.out_slots([B.lz4_max_compressed_length(len(c)) for c in chunks], dev)
    olen, st = B.lz4_encode(inp, off, ln, out, ooff)
    _check(out, ooff, olen, st, idx + [1], lambda i: oracle.lz4_compress(chunks[i]))


@pytest.mark.parametrize("n", [3, 5000, 16385])
@pytest.mark.parametrize("level", [1, 2])
def test_fastlz_compress_forms(dev, B, oracle, n, level):
    chunks, idx = _batch(oracle, n, 43 + level)
    inp, off, ln = B.pack(chunks, dev, align=1)
    out, ooff = B.out_slots([len(c) + len(c) // 16 + 96 for c in chunks], dev)
    lv = torch.full((n,), level, dtype=torch.int32, device=dev)
    olen, st = B.fastlz_compress(inp, off, ln, out, ooff, level=lv)
    _check(out, ooff, olen, st, idx + [1], lambda i: oracle.fastlz_compress(chunks[i], level, u16_limit=len(chunks[i])))


@pytest.mark.parametrize("n", [3, 5000, 16385])
def test_lzf_encode_forms(dev, B, oracle, n):
    chunks, idx = _batch(oracle, n, 47)
    inp, off, ln = B.pack(chunks, dev, align=1)
    out, ooff = B.out_slots([B.lzf_max_compressed_length(len(c)) for c in chunks], dev)
    olen, st = B.lzf_encode(inp, off, ln, out, ooff)
    _check(out, ooff, olen, st, idx + [1], lambda i: oracle.lzf_encode_chunk(chunks[i]))
