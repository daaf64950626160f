"""Rank entry for tests/test_gpu_two_ranks.py (a module of its own so spawned processes can import it)."""
import json
import os


def run(rank: int, world: int, port: int, argv, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": "0", "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import bench
    args = bench.parse(argv)
    lines = []
    line, ok = bench.run_rank(args, rank, world, 0, backend="gloo", emit=lines.append)
    q.put(json.dumps({"rank": rank, "ok": bool(ok), "line": line if rank == 0 else None, "emitted": len(lines)}))
