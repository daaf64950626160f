"""LZ4 HC (LZ4_compress_HC level 9) encode throughput by batch size on bench.py's alt-codec mix
(sizes uniform in [4096, 65535], half text-like, half random): one warm-up call, then the best of
two.  Usage: python scripts/hc_scale.py 1024 8192 32768"""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netty_amd import batch as B  # noqa: E402

CH = 65536
sizes = [int(x) for x in sys.argv[1:]] or [1024, 8192]
n = max(sizes)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1234)
src = torch.empty(n * CH, dtype=torch.uint8, device=dev)
B.textgen(src, 0, n, CH)
view = src.view(n, CH)
view[1::2] = torch.randint(0, 256, (len(range(1, n, 2)), CH), dtype=torch.uint8, device=dev, generator=g)
ln = torch.randint(4096, 65536, (n,), dtype=torch.int32, device=dev, generator=g)
off = torch.arange(n, dtype=torch.int64, device=dev) * CH
zcap = (B.lz4_max_compressed_length(CH) + 15) // 16 * 16
zout = torch.empty(n * zcap, dtype=torch.uint8, device=dev)
zoff = torch.arange(n, dtype=torch.int64, device=dev) * zcap
for m in sizes:
    ts = []
    for k in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        zl, zs = B.lz4_encode(src, off[:m], ln[:m], zout, zoff[:m], high=True)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    U = int(ln[:m].to(torch.int64).sum())
    t = min(ts[1:])
    print(json.dumps({"chunks": m, "ms": round(t, 2), "gib_s": round(U / (t / 1e3) / 2**30, 4), "ok": int((zs != 0).sum()) == 0}), flush=True)
