"""Encoder debug driver: encode a few shapes on the GPU and report status / first mismatch vs the oracle."""
import sys, os, random
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netty_amd import batch as B
from oracle import pyoracle as O
dev = torch.device("cuda:0")
rng = random.Random(1)
cases = [("text15", O.textgen_chunk(1, 15)), ("text100", O.textgen_chunk(2, 100)), ("text1000", O.textgen_chunk(3, 1000)),
         ("text64k", O.textgen_chunk(4, 65536)), ("rand1000", rng.randbytes(1000)), ("zeros", bytes(65536)),
         ("rand64k", rng.randbytes(65536)), ("period7", bytes((i % 7) * 37 & 255 for i in range(9000)))]
for name, c in cases:
    inp, off, ln = B.pack([c], dev, align=16)
    out, ooff = B.out_slots([B.snappy_max_compressed_length(len(c))], dev, align=16)
    olen, st = B.snappy_encode(inp, off, ln, out, ooff)
    torch.cuda.synchronize()
    s, n = int(st[0]), int(olen[0])
    want = O.snappy_encode(c)
    got = out[:n].cpu().numpy().tobytes() if s == 0 else b""
    first = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), None)
    print(f"{name:10s} status {s} len {n} want {len(want)} equal {got == want} first_diff {first}", flush=True)
