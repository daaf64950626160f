"""LZ4 block latency for blocks above 64 KiB: one 1 MiB and one 32 MiB (2^25) text block
encoded/decoded alone (one lane does the block), plus 256 x 1 MiB in one launch, kernel ms by HIP
events; liblz4 (pyarrow lz4_raw, one host thread) on the same bytes beside it.  Prints one JSON line."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from netty_amd import batch  # noqa: E402


def text_block(n_bytes, dev, first=0):
    k = (n_bytes + 65535) // 65536
    buf = torch.empty(k * 65536, dtype=torch.uint8, device=dev)
    batch.textgen(buf, first, k, 65536)
    return buf[:n_bytes].contiguous()


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


def case(size, count, dev):
    src = torch.cat([text_block(size, dev, first=i * 7) for i in range(count)]) if count > 1 else text_block(size, dev)
    in_off = torch.arange(count, dtype=torch.int64, device=dev) * size
    in_len = torch.full((count,), size, dtype=torch.int32, device=dev)
    capb = (batch.lz4_max_compressed_length(size) + 15) // 16 * 16
    out = torch.empty(count * capb, dtype=torch.uint8, device=dev)
    out_off = torch.arange(count, dtype=torch.int64, device=dev) * capb
    res = {}
    enc_ms = timed(lambda: res.__setitem__("e", batch.lz4_encode(src, in_off, in_len, out, out_off)))
    out_len, st = res["e"]
    assert int(st.abs().sum()) == 0
    dec = torch.empty(count * size, dtype=torch.uint8, device=dev)
    dec_ms = timed(lambda: res.__setitem__("d", batch.lz4_decode(out, out_off, out_len, dec, in_off, in_len)))
    assert int(res["d"].abs().sum()) == 0 and torch.equal(dec, src)
    r = {"block_bytes": size, "blocks": count, "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
         "encode_gib_s": round(count * size / enc_ms / 1e-3 / 2**30, 3), "decode_gib_s": round(count * size / dec_ms / 1e-3 / 2**30, 3),
         "ratio": round(float(out_len.sum()) / (count * size), 4)}
    try:
        import pyarrow as pa
        host = src[:size].cpu().numpy().tobytes()
        c = pa.Codec("lz4_raw")
        t0 = time.perf_counter()
        z = c.compress(host)
        t1 = time.perf_counter()
        c.decompress(z, decompressed_size=size)
        t2 = time.perf_counter()
        r["liblz4_1thread_encode_gib_s"] = round(size / (t1 - t0) / 2**30, 3)
        r["liblz4_1thread_decode_gib_s"] = round(size / (t2 - t1) / 2**30, 3)
        r["liblz4_ratio"] = round(len(z.to_pybytes()) / size, 4)
    except ImportError:
        pass
    return r


def main():
    dev = torch.device("cuda:0")
    rows = [case(65536, 1, dev), case(1 << 20, 1, dev), case(1 << 25, 1, dev), case(1 << 20, 256, dev)]
    print(json.dumps({"lz4_large_blocks": rows}))


if __name__ == "__main__":
    main()
