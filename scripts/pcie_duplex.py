"""Host-link ceiling for the end-to-end legs: pinned host <-> device copy rates alone and at the same
time on two streams (H2D on one, D2H on the other).
If the two directions share one budget, the end-to-end decode (compressed bytes in, ~2.2x as many
decoded bytes out) is bounded by that budget / (1 + compressed/decoded), not by the D2H rate alone.
Usage: python scripts/pcie_duplex.py [MiB per copy] [reps]"""
import json
import sys
import time

import torch


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = mib << 20
    dev = torch.device("cuda:0")
    h_src = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_src.fill_(7)
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.ones(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        best = None
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        return best

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_src, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_dst.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    t_h2d, t_d2h, t_both = timed(h2d), timed(d2h), timed(both)
    gb = n / 1e9
    out = {"bytes_per_copy": n,
           "h2d_gb_s": round(gb / t_h2d, 2), "d2h_gb_s": round(gb / t_d2h, 2),
           "both_gb_s_total": round(2 * gb / t_both, 2), "both_ms": round(t_both * 1e3, 2),
           "sum_of_alone_ms": round((t_h2d + t_d2h) * 1e3, 2), "max_of_alone_ms": round(max(t_h2d, t_d2h) * 1e3, 2)}
    ratio = 0.4568  # configs[4]'s compressed / decoded bytes
    # decode end to end moves `ratio` bytes in per decoded byte out
    out["decode_bound_gib_s_if_shared"] = round(out["both_gb_s_total"] * 1e9 / (1 + ratio) / 2**30, 2)
    out["decode_bound_gib_s_d2h_only"] = round(out["d2h_gb_s"] * 1e9 / 2**30, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
