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
