"""Snappy encode / decode+verify kernel time vs batch size (1 .. 262 144 text chunks of 64 KiB):
the latency a single handler call sees and the batch size the throughput needs.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netty_amd import batch as B  # noqa: E402

L = 65536


def best_ms(fn, reps=3):
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
    dev = torch.device("cuda:0")
    nmax = 262144
    src = torch.empty(nmax * L, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, nmax, L)
    cap = (B.snappy_max_compressed_length(L) + 15) // 16 * 16
    enc = torch.empty(nmax * cap, dtype=torch.uint8, device=dev)
    dec = torch.empty(nmax * L, dtype=torch.uint8, device=dev)
    rows = []
    for n in (1, 16, 64, 256, 1024, 4096, 16384, 65536, 262144):
        off = torch.arange(n, dtype=torch.int64, device=dev) * L
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
        eoff = torch.arange(n, dtype=torch.int64, device=dev) * cap
        res = {}
        e_ms = best_ms(lambda: res.__setitem__("e", B.snappy_encode(src, off, ln, enc, eoff)))
        elen, est = res["e"]
        crc = B.crc32c_masked(src, off, ln)
        d_ms = best_ms(lambda: res.__setitem__("d", B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=crc)))
        ok = int(est.abs().sum()) == 0 and int(res["d"]["status"].abs().sum()) == 0 and torch.equal(dec[:n * L], src[:n * L])
        rows.append({"chunks": n, "encode_ms": round(e_ms, 3), "decode_verify_ms": round(d_ms, 3),
                     "encode_gib_s": round(n * L / e_ms / 1e-3 / 2**30, 3), "decode_gib_s": round(n * L / d_ms / 1e-3 / 2**30, 3),
                     "verified": ok})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"latency_curve": rows}))


if __name__ == "__main__":
    main()
