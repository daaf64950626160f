"""N>1 path on CPU (gloo, world_size 2): contiguous chunk shards, the per-rank output-size
all-gather that places each shard in the single output stream, max-over-ranks timing and the
all-ranks verification flag — the same netty_amd.shard helpers bench.py runs over RCCL.

Each rank encodes its shard of a small text batch with the CPU oracle (test-only checker) and
the shards, concatenated at the exchanged offsets, must equal the single-process stream."""
import os
import socket

import pytest
import torch.multiprocessing as mp

N_CHUNKS = 7
CHUNK = 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from netty_amd import shard as S
    from oracle import pyoracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = S.shard_range(N_CHUNKS, rank, world)
    blob = b"".join(O.snappy_encode(O.textgen_chunk(i, CHUNK)) for i in range(lo, hi))
    off, total, sizes = S.exchange_offsets(len(blob))
    slowest = S.max_over_ranks(float(rank + 1))
    ok = S.all_true(True)
    bad = S.all_true(rank == 0)  # one rank false -> all false
    with open(os.path.join(outdir, f"r{rank}.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
        f.write(f"{lo} {hi} {off} {total} {','.join(map(str, sizes))} {slowest} {int(ok)} {int(bad)}\n")
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    from netty_amd.shard import shard_range
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_single_process_fallbacks():
    from netty_amd import shard as S
    assert S.exchange_offsets(123) == (0, 123, [123])
    assert S.max_over_ranks(2.5) == 2.5
    assert S.all_true(False) is False


def test_gloo_world2_offsets_and_stream(tmp_path, oracle):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rows = [open(tmp_path / f"r{r}.txt").read().split() for r in range(world)]
    blobs = [open(tmp_path / f"r{r}.bin", "rb").read() for r in range(world)]
    # contiguous shards covering every chunk
    assert [(int(r[0]), int(r[1])) for r in rows] == [(0, 3), (3, 7)]
    sizes = [len(b) for b in blobs]
    for r, row in enumerate(rows):
        assert int(row[2]) == sum(sizes[:r])          # exchanged offset
        assert int(row[3]) == sum(sizes)              # global total
        assert row[4] == ",".join(map(str, sizes))    # all-gathered sizes
        assert float(row[5]) == float(world)          # max over ranks
        assert row[6] == "1" and row[7] == "0"        # all-ranks flag
    # the shards laid out at their offsets are the single-process stream
    whole = b"".join(oracle.snappy_encode(oracle.textgen_chunk(i, CHUNK)) for i in range(N_CHUNKS))
    stream = bytearray(sum(sizes))
    for r in range(world):
        o = int(rows[r][2])
        stream[o:o + sizes[r]] = blobs[r]
    assert bytes(stream) == whole


# ---------------------------------------------------------------- bench.py's own N>1 path over gloo
class _OracleLeg:
    """CPU stand-in for bench.SnappyRoundTrip (test-only: the oracle is the per-rank worker here).
    It records the chunk range it was given and encodes/decodes those chunks on the CPU."""

    def __init__(self, outdir, rank, first, n):
        from oracle import pyoracle as O
        self.O, self.outdir, self.rank, self.first, self.n, self.sub = O, outdir, rank, first, n, n
        self.blob = b""
        self.steps = 0

    def step(self, record=False):
        O = self.O
        parts = [O.snappy_encode(O.textgen_chunk(i, 65536)) for i in range(self.first, self.first + self.n)]
        self.blob = b"".join(parts)
        self.steps += 1
        self.ok = all(O.snappy_decode(p, 65536)[1] == O.textgen_chunk(i, 65536)
                      for i, p in zip(range(self.first, self.first + self.n), parts))

    def verify(self, rank):
        with open(os.path.join(self.outdir, f"b{rank}.bin"), "wb") as f:
            f.write(self.blob)
        with open(os.path.join(self.outdir, f"b{rank}.txt"), "w") as f:
            f.write(f"{self.first} {self.n} {self.steps}\n")
        return self.ok, True

    def comp_bytes(self):
        return len(self.blob)

    def kernel_ms_per_step(self, steps):
        return 1.0, 1.0, 1.0


class _LegFactory:
    def __init__(self, outdir, rank):
        self.outdir, self.rank = outdir, rank

    def __call__(self, first, n):
        return _OracleLeg(self.outdir, self.rank, first, n)


def _bench_rank(rank, world, port, outdir):
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import bench
    args = bench.parse(["--gpus", str(world), "--total-chunks", "7", "--steps", "2", "--warmup", "1"])
    lines = []
    line, ok = bench.run_rank(args, rank, world, rank, backend="gloo", leg_factory=_LegFactory(outdir, rank),
                              emit=lines.append)
    with open(os.path.join(outdir, f"json{rank}.txt"), "w") as f:
        f.write("\n".join(lines))
    assert ok


def test_bench_run_rank_world2_gloo(tmp_path, oracle):
    """bench.py's run_rank at world 2 over gloo: disjoint shards that cover every chunk, stream offsets
    equal to shard.exchange_offsets' (the all-gathered compressed totals), the max-over-ranks timing
    and exactly one JSON line (rank 0) with n_gpus == 2 and strong scaling over the fixed total."""
    import json
    world = 2
    mp.start_processes(_bench_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rec = [open(tmp_path / f"b{r}.txt").read().split() for r in range(world)]
    ranges = [(int(a), int(a) + int(b)) for a, b, _ in rec]
    assert ranges == [(0, 3), (3, 7)]
    assert all(int(s) == 3 for _, _, s in rec)  # warmup 1 + steps 2
    sizes = [len(open(tmp_path / f"b{r}.bin", "rb").read()) for r in range(world)]
    out0 = open(tmp_path / "json0.txt").read().strip().splitlines()
    out1 = open(tmp_path / "json1.txt").read().strip()
    assert len(out0) == 1 and out1 == ""
    line = json.loads(out0[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["verified"] is True
    assert line["config"]["global_chunks"] == 7 and line["compressed_bytes_per_rank"] == sizes
    assert line["shard"] == {"first_chunk": 0, "chunks": 3, "stream_offset": 0, "stream_bytes": sum(sizes)}
    assert line["value"] > 0 and line["steps"] == 2
    whole = b"".join(oracle.snappy_encode(oracle.textgen_chunk(i, 65536)) for i in range(7))
    assert open(tmp_path / "b0.bin", "rb").read() + open(tmp_path / "b1.bin", "rb").read() == whole
