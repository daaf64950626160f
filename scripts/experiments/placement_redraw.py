"""Does a second draw of 32 GiB table placements (after freeing all but the best of the first draw)
land elsewhere?  Probes each table with the encoder's request chain (netty_amd/tools/probe_ceiling.hip,
no inserts, 262144 lanes) and prints G probes/s per table, per round."""
import ctypes, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "netty_amd", "libnx_probe_ceiling.so"))
lib.nx_probe_ceiling.restype = ctypes.c_int32
lib.nx_probe_ceiling.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
dev = torch.device("cuda:0")
lanes, steps = 262144, 4096
inp = torch.empty(lanes * 16384, dtype=torch.int32, device=dev)
sink = torch.empty(lanes, dtype=torch.int32, device=dev)

def probe(t):
    ms = ctypes.c_float(0)
    assert lib.nx_probe_ceiling(t.data_ptr(), inp.data_ptr(), sink.data_ptr(), lanes, steps, 258, 0, ctypes.byref(ms),
                                ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
    return round(lanes * steps / (ms.value / 1e3) / 1e9, 2)

keep = []
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    tabs = []
    while torch.cuda.mem_get_info(dev)[0] > lanes * 16384 * 8 + (8 << 30) and len(tabs) < 6:
        tabs.append(torch.zeros(lanes * 16384, dtype=torch.int64, device=dev))
    rates = [probe(t) for t in tabs]
    print("round", rnd, "rates", rates, "kept", [probe(t) for t in keep], flush=True)
    best = max(range(len(rates)), key=lambda i: rates[i])
    keep = [tabs[best]] if not keep or rates[best] > probe(keep[0]) else keep
    del tabs
    torch.cuda.empty_cache()
