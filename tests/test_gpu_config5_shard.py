"""configs[4] per-rank GPU leg: bench.SnappyRoundTrip on a shard that does not
start at chunk 0, run in several sub-batches, checked against the oracle.

A rank of the 100 GiB job owns chunk indices [first, first + n) and
generates chunk i from the global seed of index i (Snappy copies never leave their chunk,
Snappy.java:647-649, so each chunk's bytes depend on its index only).  A wrong seed offset on a
rank > 0, a sub-batch boundary off by one, or compressed lengths written to the wrong slots would
all pass a rank-0, single-sub-batch test; these tests pin them."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CHUNK = 65536


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


def test_rank3_of_8_shard_sub_batches(dev, oracle):
    import bench
    from netty_amd import shard as S

    total, world, rank = 1600, 8, 3
    first, hi = S.shard_range(total, rank, world)
    n = hi - first
    assert first == 600 and n == 200
    leg = bench.SnappyRoundTrip(torch, dev, first, n, sub=64)  # sub-batches 64, 64, 64, 8
    assert [m for _, m in leg.batches()] == [64, 64, 64, 8]
    leg.step()
    ok, detect = leg.verify(rank)
    torch.cuda.synchronize()
    assert ok and detect
    # the shard's inputs are the global chunks first .. first + n - 1
    for i in (0, 1, 63, 64, 150, n - 1):
        got = leg.src[i * CHUNK:(i + 1) * CHUNK].cpu().numpy().tobytes()
        assert got == oracle.textgen_chunk(first + i, CHUNK), i
    # compressed lengths of every chunk equal the oracle's Snappy.encode of the global chunk
    want_len = [len(oracle.snappy_encode(oracle.textgen_chunk(first + i, CHUNK))) for i in range(n)]
    assert leg.elen.cpu().tolist() == want_len
    assert leg.comp_bytes() == sum(want_len)
    # frame CRCs (masked CRC32C of the uncompressed chunk) land in the chunk's own slot
    crc = [c & 0xFFFFFFFF for c in leg.crc.cpu().tolist()]
    for i in (0, 64, 127, 128, 199):
        assert crc[i] == oracle.snappy_checksum(oracle.textgen_chunk(first + i, CHUNK)), i
    # compressed bytes: the encode buffer holds one sub-batch at a time; re-run each and sample
    for lo, m in leg.batches():
        leg.run_sub(lo, m)
        torch.cuda.synchronize()
        el = leg.elen[lo:lo + m].cpu().tolist()
        for k in sorted({0, m // 2, m - 1}):
            got = leg.enc[k * leg.cap:k * leg.cap + el[k]].cpu().numpy().tobytes()
            assert got == oracle.snappy_encode(oracle.textgen_chunk(first + lo + k, CHUNK)), (lo, k)
        assert torch.equal(leg.dec[:m * CHUNK], leg.src[lo * CHUNK:(lo + m) * CHUNK])
    assert int((leg.dst != 0).sum()) == 0 and int((leg.est != 0).sum()) == 0


def test_run_rank_world1_small_job(dev):
    """bench.run_rank itself on the GPU at world 1 over a small total with a partial last sub-batch:
    one verified JSON line whose shard, lengths and timings are consistent."""
    import bench
    args = bench.parse(["--total-chunks", "300", "--sub-chunks", "128", "--steps", "1", "--warmup", "1",
                        "--weak-chunks", "130", "--no-cpu-baseline", "--no-e2e", "--no-alt", "--no-frame-scan",
                        "--no-probe-ceiling"])
    lines = []
    line, ok = bench.run_rank(args, 0, 1, 0, emit=lines.append)
    assert ok and len(lines) == 1 and line["verified"] is True
    assert line["n_gpus"] == 1 and line["config"]["global_chunks"] == 300
    assert line["shard"]["first_chunk"] == 0 and line["shard"]["chunks"] == 300
    assert line["crc_corruption_subset_detected"] is True
    assert line["weak_1m_per_gpu"]["verified"] is True and line["weak_1m_per_gpu"]["chunks_per_gpu"] == 130
    assert line["value"] > 0 and line["roofline"]["achieved"] > 0
    assert 0.3 < line["compression_ratio"] < 0.6
