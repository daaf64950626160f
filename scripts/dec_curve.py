"""Snappy decode + CRC32C verify time against frames per call (round 6; experiments only).

N text-like 64 KiB chunks are encoded once; then for every count n of the list, nx_snappy_decode_batch
(the parse/expand pair, `variant`) decodes the first n frames `reps` times (HIP events, best of reps)
and the output is checked against the inputs.

    python scripts/dec_curve.py reps n1 n2 ... [--variant pair|auto]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from netty_amd import batch as B
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    variant = "pair"
    for a in sys.argv[1:]:
        if a.startswith("--variant="):
            variant = a.split("=", 1)[1]
    reps = int(args[0])
    ns = [int(x) for x in args[1:]]
    N, L = max(ns), 65536
    dev = torch.device("cuda:0")
    src = torch.empty(N * L, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, N, L)
    off = torch.arange(N, dtype=torch.int64, device=dev) * L
    ln = torch.full((N,), L, dtype=torch.int32, device=dev)
    cap = (B.snappy_max_compressed_length(L) + 15) // 16 * 16
    enc = torch.empty(N * cap, dtype=torch.uint8, device=dev)
    eoff = torch.arange(N, dtype=torch.int64, device=dev) * cap
    elen, est = B.snappy_encode(src, off, ln, enc, eoff)
    crc = B.crc32c_masked(src, off, ln)
    dec = torch.empty_like(src)
    for n in ns:
        ts = []
        for i in range(reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = B.snappy_decode(enc, eoff[:n], elen[:n], dec, off[:n], expected_crc=crc[:n], variant=variant)
            b.record()
            torch.cuda.synchronize()
            if i:
                ts.append(a.elapsed_time(b))
        ok = bool(torch.equal(dec[:n * L], src[:n * L])) and int((r["status"] != 0).sum()) == 0 and int((est != 0).sum()) == 0
        ms = min(ts)
        print(json.dumps({"frames": n, "variant": variant, "decode_ms": round(ms, 3), "all_ms": [round(t, 2) for t in ts],
                          "us_per_frame": round(ms * 1e3 / n, 4), "gib_s": round(n * L / (ms / 1e3) / 2**30, 1), "verified": ok}),
              flush=True)


if __name__ == "__main__":
    main()
