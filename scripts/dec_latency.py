"""Snappy decode + verify latency by batch size for both decoder forms (round 5):
the parse/expand pair ("auto") and the wave-parallel fused decoder ("fused"), 1 .. 65 536 text
chunks of 64 KiB, best of `reps` HIP-event timings each, outputs checked.  One JSON line per size.

    python scripts/dec_latency.py [reps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netty_amd import batch as B  # noqa: E402

L = 65536


def best_ms(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        t.append(a.elapsed_time(b))
    return min(t)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    sizes = [int(x) for x in os.environ.get("SIZES", "1,16,64,256,1024,2048,4096,8192,16384,65536").split(",")]
    dev = torch.device("cuda:0")
    nmax = max(sizes)
    src = torch.empty(nmax * L, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, nmax, L)
    cap = (B.snappy_max_compressed_length(L) + 15) // 16 * 16
    enc = torch.empty(nmax * cap, dtype=torch.uint8, device=dev)
    dec = torch.empty(nmax * L, dtype=torch.uint8, device=dev)
    for n in sizes:
        off = torch.arange(n, dtype=torch.int64, device=dev) * L
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
        eoff = torch.arange(n, dtype=torch.int64, device=dev) * cap
        elen, est = B.snappy_encode(src, off, ln, enc, eoff)
        crc = B.crc32c_masked(src, off, ln)
        row = {"chunks": n}
        for v in ("auto", "fused"):
            res = {}
            dec[: n * L].zero_()
            ms = best_ms(lambda: res.__setitem__("d", B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=crc, variant=v)), reps)
            ok = int(est.abs().sum()) == 0 and int(res["d"]["status"].abs().sum()) == 0 and torch.equal(dec[: n * L], src[: n * L])
            row[v + "_ms"] = round(ms, 3)
            row[v + "_ok"] = ok
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
