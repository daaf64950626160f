"""Decode timing for expander A/B runs: N text-like 64 KiB chunks are encoded once, then
Snappy.decode + CRC32C verify is timed (HIP events) over `reps` launches and checked against the
inputs.  The expander is chosen by NX_EXPAND (unset: k_expand; "window": k_window), read once
per process, so run one process per variant.

    python scripts/dec_time.py [chunks] [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from netty_amd import batch as B
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    L = 65536
    dev = torch.device("cuda:0")
    src = torch.empty(n * L, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, n, L)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    ln = torch.full((n,), L, dtype=torch.int32, device=dev)
    cap = (B.snappy_max_compressed_length(L) + 15) // 16 * 16
    enc = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    eoff = torch.arange(n, dtype=torch.int64, device=dev) * cap
    elen, est = B.snappy_encode(src, off, ln, enc, eoff)
    crc = B.crc32c_masked(src, off, ln)
    dec = torch.empty_like(src)
    ts = []
    for i in range(reps + 1):
        dec.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        r = B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=crc)
        b.record()
        torch.cuda.synchronize()
        if i:
            ts.append(a.elapsed_time(b))
    ok = bool(torch.equal(dec, src)) and int((r["status"] != 0).sum()) == 0 and int((est != 0).sum()) == 0
    C = int(elen.to(torch.int64).sum())
    ms = min(ts)
    print(json.dumps({"chunks": n, "decode_ms": round(ms, 3),
                      "all_ms": [round(t, 2) for t in ts], "gib_s": round(n * L / (ms / 1e3) / 2**30, 1),
                      "algo_gbs": round((C + n * L) / (ms / 1e3) / 1e9, 1), "verified": ok}))


if __name__ == "__main__":
    main()
