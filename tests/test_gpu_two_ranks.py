"""bench.py's multi-rank job with the real GPU legs: two ranks, both on the one GPU of
the test box, their collectives over gloo on host tensors (RCCL needs one GPU per rank; the 8-GPU
node is the driver's).  Each rank encodes + decodes its own contiguous shard of configs[4]'s chunk
indices; rank 0 reports the merged line: both shards verified, the all-gathered compressed sizes,
the max-over-ranks time."""
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sub", ["96", "0"])  # fixed calls; the library's launch plan (round 6)
def test_two_ranks_one_gpu(oracle, sub):
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench
    import mp_rank
    argv = ["--total-chunks", "301", "--sub-chunks", sub, "--steps", "1", "--warmup", "1", "--weak-chunks", "40",
            "--no-cpu-baseline", "--no-e2e", "--no-alt", "--no-frame-scan", "--no-probe-ceiling"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=mp_rank.run, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = [json.loads(q.get(timeout=240)) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort(key=lambda g: g["rank"])
    assert all(g["ok"] for g in got)
    assert got[0]["emitted"] == 1 and got[1]["emitted"] == 0  # only rank 0 prints the JSON line
    line = got[0]["line"]
    assert line["n_gpus"] == 2 and line["verified"] is True
    assert line["shard"] == {"first_chunk": 0, "chunks": 150, "stream_offset": 0, "stream_bytes": line["shard"]["stream_bytes"]}
    sizes = line["compressed_bytes_per_rank"]
    want = [sum(len(oracle.snappy_encode(oracle.textgen_chunk(i, 65536))) for i in range(lo, hi)) for lo, hi in ((0, 150), (150, 301))]
    assert sizes == want and line["shard"]["stream_bytes"] == sum(want)
    assert line["weak_1m_per_gpu"]["verified"] is True
    assert line["value"] > 0 and line["ms_per_step"] > 0
