"""Lane outputs staged in LDS and stored as whole 64/128-byte units: the Snappy
encoder's WriterL, and ByteStageT in the LZ4 / FastLZ / LZF encoders and the FastLZ / LZF decoders.

The staged forms run in the dense (lane-per-chunk) launches, so the encoder batches here hold
16 385 chunks (mostly small fillers, ~20 real ones).  Output slots are packed back to back at odd
(or, for Snappy's dword writer, 4-byte but not unit-aligned) offsets with a sentinel byte between
them: every chunk must equal the oracle's bytes and no byte outside [off, off + len) may change (LZF:
the slot capacity, its encoder uses the slot as scratch) —
the first, partial unit and the tail are the cases the staging has to get right."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SENTINEL = 0xA5


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def B():
    from netty_amd import batch
    return batch


def _chunks(oracle, n, seed, max_len):
    rng = random.Random(seed)
    real = sorted({0, 1, n - 1} | {rng.randrange(n) for _ in range(18)})
    chunks = []
    for i in range(n):
        if i in real:
            L = rng.choice([1, 3, 17, 127, 128, 129, 4095, 40000, max_len])
            chunks.append(oracle.textgen_chunk(seed * 31 + i, L) if i % 3 else oracle.java_random_bytes(seed + i, L))
        else:
            chunks.append(bytes([65 + i % 7]) * (5 + i % 29))
    return chunks, real


def _slots(caps, dev, step_align):
    """Back-to-back slots, each followed by one sentinel byte, starts rounded up to step_align."""
    offs, cur = [], 3
    for c in caps:
        cur = (cur + step_align - 1) // step_align * step_align
        offs.append(cur)
        cur += c + 1
    buf = torch.full((cur + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    return buf, torch.tensor(offs, dtype=torch.int64, device=dev)


def _check(buf, ooff, olen, want, extent=None):
    """Chunk bytes equal want(i) for the listed chunks; every byte outside [off, off + extent) is
    untouched (extent = the output length, or the slot capacity for an encoder that may use its
    slot as scratch)."""
    host = buf.cpu().numpy()
    oo = ooff.cpu().numpy().astype(np.int64)
    ol = olen.cpu().numpy().astype(np.int64)
    for i, w in want.items():
        assert host[oo[i]:oo[i] + ol[i]].tobytes() == w, i
    ext = ol if extent is None else np.asarray(extent, dtype=np.int64)
    written = np.zeros(host.shape[0] + 1, dtype=np.int64)
    np.add.at(written, oo, 1)
    np.add.at(written, oo + ext, -1)
    inside = np.cumsum(written)[:-1] > 0
    outside = host[~inside]
    assert (outside == SENTINEL).all(), f"{int((outside != SENTINEL).sum())} bytes written outside the chunks' outputs"


N_DENSE = 16385


def test_snappy_encoder_units_unaligned(dev, B, oracle):
    chunks, real = _chunks(oracle, N_DENSE, 3, 65536)
    inp, off, ln = B.pack(chunks, dev, align=1)
    buf, ooff = _slots([B.snappy_max_compressed_length(len(c)) for c in chunks], dev, 4)
    olen, st = B.snappy_encode(inp, off, ln, buf, ooff)
    assert int((st != 0).sum()) == 0
    _check(buf, ooff, olen, {i: oracle.snappy_encode(chunks[i]) for i in real})


def test_lz4_encoder_units_unaligned(dev, B, oracle):
    chunks, real = _chunks(oracle, N_DENSE, 5, 65535)
    inp, off, ln = B.pack(chunks, dev, align=1)
    buf, ooff = _slots([B.lz4_max_compressed_length(len(c)) for c in chunks], dev, 1)
    olen, st = B.lz4_encode(inp, off, ln, buf, ooff)
    assert int((st != 0).sum()) == 0
    _check(buf, ooff, olen, {i: oracle.lz4_compress(chunks[i]) for i in real})


@pytest.mark.parametrize("level", [1, 2])
def test_fastlz_encoder_units_unaligned(dev, B, oracle, level):
    chunks, real = _chunks(oracle, N_DENSE, 7 + level, 65535)
    inp, off, ln = B.pack(chunks, dev, align=1)
    buf, ooff = _slots([len(c) + len(c) // 16 + 96 for c in chunks], dev, 1)
    lv = torch.full((N_DENSE,), level, dtype=torch.int32, device=dev)
    olen, st = B.fastlz_compress(inp, off, ln, buf, ooff, level=lv)
    assert int((st != 0).sum()) == 0
    _check(buf, ooff, olen, {i: oracle.fastlz_compress(chunks[i], level, u16_limit=len(chunks[i])) for i in real})


def test_lzf_encoder_units_unaligned(dev, B, oracle):
    chunks, real = _chunks(oracle, N_DENSE, 11, 65535)
    inp, off, ln = B.pack(chunks, dev, align=1)
    caps = [B.lzf_max_compressed_length(len(c)) for c in chunks]
    buf, ooff = _slots(caps, dev, 1)
    olen, st = B.lzf_encode(inp, off, ln, buf, ooff)
    assert int((st != 0).sum()) == 0
    # an incompressible chunk's compressed attempt runs past the raw block it falls back to
    # (ChunkEncoder.tryCompress writes into the workspace first): the slot is scratch up to its capacity
    _check(buf, ooff, olen, {i: oracle.lzf_encode_chunk(chunks[i]) for i in real}, extent=caps)


def _decode_inputs(oracle, n, seed):
    rng = random.Random(seed)
    plain = []
    for i in range(n):
        L = rng.choice([32, 100, 129, 1000, 4097, 30000, 65535])
        plain.append(oracle.textgen_chunk(seed * 131 + i, L) if i % 4 else oracle.java_random_bytes(seed + i, L))
    return plain


def test_fastlz_decoder_units_unaligned(dev, B, oracle):
    plain = _decode_inputs(oracle, 600, 13)
    comp = [oracle.fastlz_compress(p, 1, u16_limit=len(p)) for p in plain]
    inp, off, ln = B.pack(comp, dev, align=1)
    buf, ooff = _slots([len(p) for p in plain], dev, 1)
    lim = torch.tensor([len(p) for p in plain], dtype=torch.int32, device=dev)
    res = B.fastlz_decompress(inp, off, ln, buf, ooff, lim)
    assert res.cpu().tolist() == [len(p) for p in plain]
    _check(buf, ooff, lim, dict(enumerate(plain)))


def test_lzf_decoder_units_unaligned(dev, B, oracle):
    plain = _decode_inputs(oracle, 600, 17)
    blocks = [oracle.lzf_encode_chunk(p) for p in plain]
    keep = [i for i, b in enumerate(blocks) if b[2] == 1]  # compressed blocks: the decoder takes their body
    assert len(keep) > 300
    plain = [plain[i] for i in keep]
    bodies = [blocks[i][7:] for i in keep]
    inp, off, ln = B.pack(bodies, dev, align=1)
    buf, ooff = _slots([len(p) for p in plain], dev, 1)
    olen = torch.tensor([len(p) for p in plain], dtype=torch.int32, device=dev)
    st = B.lzf_decode(inp, off, ln, buf, ooff, olen)
    assert int((st != 0).sum()) == 0
    _check(buf, ooff, olen, dict(enumerate(plain)))


def test_encoder_workspace_placement_report(dev, B, oracle):
    """A dense-form encoder workspace of >= 2 GiB is the fastest of several probed placements
    (nx_common.hpp alloc_placed_workspace); nx_snappy_encode_placement reports the probe times and
    the index kept, which must be the fastest."""
    import ctypes
    from netty_amd import _lib
    import gc
    gc.collect()
    B.workspaces_trim()  # the device's workspace (unless a live handle holds one) is placed anew
    s = torch.cuda.Stream(dev)
    chunks = [b"placement" * 7] * N_DENSE
    inp, off, ln = B.pack(chunks, dev, align=1)
    out, ooff = B.out_slots([B.snappy_max_compressed_length(len(c)) for c in chunks], dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        olen, st = B.snappy_encode(inp, off, ln, out, ooff)
    s.synchronize()
    assert int((st != 0).sum()) == 0
    L = _lib.load()
    ms = (ctypes.c_float * 32)()
    n, pick = ctypes.c_int32(0), ctypes.c_int32(-1)
    assert L.nx_snappy_encode_placement(ms, 32, ctypes.byref(n), ctypes.byref(pick)) == 0
    assert 1 <= n.value <= 24 and 0 <= pick.value < n.value  # four draws of up to six
    probe = [ms[k] for k in range(n.value)]
    assert all(p > 0 for p in probe)
    assert probe[pick.value] == min(probe)
