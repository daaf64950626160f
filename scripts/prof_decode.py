"""Decode-only driver for rocprofv3 (PMC / kernel-trace): N text chunks, encode once, decode R times."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netty_amd import batch as B
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
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
for _ in range(R):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    r = B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=crc, variant=os.environ.get("NX_VARIANT", "auto"))
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print("decode ms", [round(t, 3) for t in ts], "GiB/s", round(n * L / min(ts) * 1e3 / 2**30, 2))
print("ok", bool(torch.equal(dec, src)), int((r["status"] != 0).sum()), int(elen.sum()))
