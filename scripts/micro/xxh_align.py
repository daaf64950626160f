"""XXH32 batch rate on 16-aligned vs misaligned blocks (the frame decoder hashes raw blocks in place
at header + 21).  262 144 blocks of 32 KiB."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from netty_amd import batch as B  # noqa: E402

dev = torch.device("cuda:0")
n, L = 262144, 32768
src = torch.randint(0, 256, (n * L + 64,), dtype=torch.uint8, device=dev)
ln = torch.full((n,), L - 32, dtype=torch.int32, device=dev)
for shift in (0, 1, 5, 21):
    off = torch.arange(n, dtype=torch.int64, device=dev) * L + shift
    B.xxhash32(src, off, ln)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        B.xxhash32(src, off, ln)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    print(f"shift {shift:2d}: {ms:.3f} ms  {n * (L - 32) / ms / 1e6:.1f} GB/s", flush=True)
