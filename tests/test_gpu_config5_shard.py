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
            o = int(leg.eoff[lo + k])
            got = leg.enc[o:o + el[k]].cpu().numpy().tobytes()
            assert got == oracle.snappy_encode(oracle.textgen_chunk(first + lo + k, CHUNK)), (lo, k)
        assert torch.equal(leg.dec[:m * CHUNK], leg.src[lo * CHUNK:(lo + m) * CHUNK])
    assert int((leg.dst != 0).sum()) == 0 and int((leg.est != 0).sum()) == 0


def test_ring_schedule_encode_decode_calls_differ(dev, oracle):
    """Round 6: encode calls and decode calls of different sizes over a ring of encode slots smaller
    than the shard (bench.SnappyRoundTrip as the 100 GiB job runs it: 5 x 327 680 encodes, 262 144-frame
    decodes).  Encodes 96 / 96 / 108, decodes of 64 over a 171-slot ring: the ring wraps, decode calls
    straddle encode calls, the last decode takes the rest."""
    import bench
    first, n = 1000, 300
    leg = bench.SnappyRoundTrip(torch, dev, first, n, dec_sub=64, enc_sizes=[96, 96, 108])
    assert leg.ring == 108 + 63 and leg.ring < n
    assert leg.ops == bench.schedule([96, 96, 108], 64)
    assert [m for k, _, m in leg.ops if k == "dec"] == [64, 64, 64, 64, 44]
    leg.step()
    ok, detect = leg.verify(0)
    assert ok and detect
    leg.step()
    torch.cuda.synchronize()
    # after a step the ring holds the chunks of the last ring-full: their bytes are the oracle's
    el = leg.elen.cpu().tolist()
    for c in (n - leg.ring, n - 100, n - 1):
        o = int(leg.eoff[c])
        assert o == (c % leg.ring) * leg.cap
        got = leg.enc[o:o + el[c]].cpu().numpy().tobytes()
        assert got == oracle.snappy_encode(oracle.textgen_chunk(first + c, CHUNK)), c
    want = [len(oracle.snappy_encode(oracle.textgen_chunk(first + i, CHUNK))) for i in range(n)]
    assert el == want


def test_encode_plan_launch_sizes(dev):
    """nx_snappy_encode_plan: equal full-occupancy launches in steps of half a block per CU (DESIGN.md §6
    launch table).  On a 256-CU MI355X: the 100 GiB job at N = 1/2/4/8 per rank, and the 1 M weak leg."""
    import bench
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    full = cus * 1280  # 20 waves per CU
    assert bench.encode_plan(full) == [full]
    assert bench.encode_plan(100) == [100]
    for n in (1638400, 819200, 409600, 204800, 1048576, 5 * full + 1, 3 * full - 256):
        p = bench.encode_plan(n)
        assert sum(p) == n and max(p) <= full
        assert len(p) == (n + full - 1) // full
        assert max(p) - min(p) <= cus * 128 + cus * 128  # equal up to one step (+ the last launch's rest)
    if cus == 256:
        assert bench.encode_plan(1638400) == [327680] * 5
        assert bench.encode_plan(819200) == [294912, 262144, 262144]
        assert bench.encode_plan(409600) == [196608, 212992]
        assert bench.encode_plan(204800) == [204800]
        assert bench.encode_plan(1048576) == [262144] * 4


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
