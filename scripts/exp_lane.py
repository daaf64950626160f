"""EXPERIMENT timing: lane-per-frame wide-copy decode vs the parse/expand pair (text frames)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netty_amd import batch as B, _lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
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
dec = torch.empty_like(src)
lib = ctypes.CDLL(_lib.load()._name)
f = lib.nx_snappy_decode_batch_lane_experiment
f.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_uint32, ctypes.c_void_p]
olen = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
def run():
    f(enc.data_ptr(), eoff.data_ptr(), elen.data_ptr(), dec.data_ptr(), off.data_ptr(), olen.data_ptr(), st.data_ptr(), n,
      torch.cuda.current_stream().cuda_stream)
ts = []
for _ in range(3):
    dec.zero_()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(); run(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
print("lane decode ms", [round(t, 3) for t in ts], "ok", bool(torch.equal(dec, src)), int((st != 0).sum()), flush=True)
