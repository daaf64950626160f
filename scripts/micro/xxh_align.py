"""XXH32, masked-CRC32C and Adler32 batch rates on 16-aligned vs misaligned blocks (the frame decoders checksum
raw blocks in place, after their headers).  262 144 blocks of 32 KiB."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from netty_amd import batch as B  # noqa: E402

dev = torch.device("cuda:0")
n, L = 262144, 32768
src = torch.randint(0, 256, (n * L + 64,), dtype=torch.uint8, device=dev)
ln = torch.full((n,), L - 32, dtype=torch.int32, device=dev)
for name, fn in (("xxh32", B.xxhash32), ("crc32c", B.crc32c_masked), ("adler32", B.adler32)):
  for shift in (0, 1, 5, 21, 48):
    off = torch.arange(n, dtype=torch.int64, device=dev) * L + shift
    fn(src, off, ln)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        fn(src, off, ln)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    print(f"{name} shift {shift:2d}: {ms:.3f} ms  {n * (L - 32) / ms / 1e6:.1f} GB/s", flush=True)
