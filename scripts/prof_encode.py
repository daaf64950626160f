"""Encode-only driver: python scripts/prof_encode.py N R"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netty_amd import batch as B
n = int(sys.argv[1]); R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
L = 65536; dev = torch.device("cuda:0")
src = torch.empty(n * L, dtype=torch.uint8, device=dev); B.textgen(src, 0, n, L)
off = torch.arange(n, dtype=torch.int64, device=dev) * L
ln = torch.full((n,), L, dtype=torch.int32, device=dev)
cap = (B.snappy_max_compressed_length(L) + 15) // 16 * 16
enc = torch.empty(n * cap, dtype=torch.uint8, device=dev)
eoff = torch.arange(n, dtype=torch.int64, device=dev) * cap
elen, est = B.snappy_encode(src, off, ln, enc, eoff); torch.cuda.synchronize()
t = []
for _ in range(R):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(); B.snappy_encode(src, off, ln, enc, eoff, out_len=elen, status=est); b.record(); torch.cuda.synchronize()
    t.append(a.elapsed_time(b))
ms = min(t)
print(f"encode n={n} ms={ms:.1f} GiB/s={n*L/ms/1e3/2**30*1e3:.2f} C={int(elen.sum())}", flush=True)
