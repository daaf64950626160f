"""Decode a few oracle-encoded streams on the GPU and compare with the input (debug helper)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import pyoracle as O
from netty_amd import batch as B
O.build()
d0 = b'Netty is a NIO client server framework which enables quick and easy development of network applications such as protocol servers and clients.'
ins = [d0, O.textgen_chunk(3, 65536), O.java_random_bytes(5, 65536), bytes(65536), O.textgen_chunk(4, 1000)]
encs = [O.snappy_encode(x) for x in ins]
dev = torch.device("cuda:0")
data, off, ln = B.pack(encs, dev)
out = torch.zeros(len(ins) * 65536, dtype=torch.uint8, device=dev)
ooff = torch.arange(len(ins), dtype=torch.int64, device=dev) * 65536
r = B.snappy_decode(data, off, ln, out, ooff)
torch.cuda.synchronize()
for i, x in enumerate(ins):
    n = int(r["out_len"][i]); stt = int(r["status"][i])
    got = bytes(out[i * 65536: i * 65536 + n].cpu().numpy())
    bad = next((j for j in range(min(n, len(x))) if got[j] != x[j]), None)
    print(f"mode={os.environ.get('NX_DEC_PARSE','0')} case {i}: len {n}/{len(x)} status {stt} ok={got == x} first_bad={bad}", flush=True)
