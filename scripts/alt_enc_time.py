"""Alt-codec encoder timing for occupancy A/B runs (round 6): the bench's configs[3] batch (262 144 chunks,
sizes uniform in [4096, 65535], half text-like, half random), FastLZ level 1 / 2, LZF and LZ4 encode, best
of `reps` HIP-event timings each; every chunk is decoded back and compared with its source.

    python scripts/alt_enc_time.py [chunks] [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from netty_amd import batch as B
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    CH = 65536
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    src = torch.empty(n * CH, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, n, CH)
    view = src.view(n, CH)
    view[1::2] = torch.randint(0, 256, (len(range(1, n, 2)), CH), dtype=torch.uint8, device=dev, generator=g)
    ln = torch.randint(4096, 65536, (n,), dtype=torch.int32, device=dev, generator=g)
    off = torch.arange(n, dtype=torch.int64, device=dev) * CH
    U = int(ln.to(torch.int64).sum())
    dec = torch.empty_like(src)
    col = torch.arange(CH, device=dev)

    def same():
        for a in range(0, n, 16384):
            m = col.view(1, -1) < ln[a:a + 16384].view(-1, 1)
            if not torch.equal(dec.view(n, CH)[a:a + 16384][m], src.view(n, CH)[a:a + 16384][m]):
                return False
        return True

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            t = a.elapsed_time(b)
            best = t if best is None else min(best, t)
        return best

    res = {"chunks": n}
    cap = (max(B.fastlz_max_compressed_length(CH), B.lzf_max_compressed_length(CH), B.lz4_max_compressed_length(CH)) + 15) // 16 * 16
    out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    ooff = torch.arange(n, dtype=torch.int64, device=dev) * cap
    box = {}
    for level in (1, 2):
        lv = torch.full((n,), level, dtype=torch.int32, device=dev)
        t = timed(lambda: box.__setitem__("r", B.fastlz_compress(src, off, ln, out, ooff, level=lv)))
        flen, fst = box["r"]
        dec.zero_()
        d = B.fastlz_decompress(out, ooff, flen, dec, off, ln)
        ok = int((fst != 0).sum()) == 0 and bool(torch.equal(d, ln)) and same()
        res[f"fastlz_l{level}"] = {"encode_ms": round(t, 2), "encode_gib_s": round(U / t * 1e3 / 2**30, 2), "verified": ok}
    t = timed(lambda: box.__setitem__("l", B.lzf_encode(src, off, ln, out, ooff)))
    llen, lst = box["l"]
    res["lzf"] = {"encode_ms": round(t, 2), "encode_gib_s": round(U / t * 1e3 / 2**30, 2), "verified": int((lst != 0).sum()) == 0}
    t = timed(lambda: box.__setitem__("z", B.lz4_encode(src, off, ln, out, ooff)))
    zlen, zst = box["z"]
    dec.zero_()
    zd = B.lz4_decode(out, ooff, zlen, dec, off, ln)
    ok = int((zst != 0).sum()) == 0 and int((zd != 0).sum()) == 0 and same()
    res["lz4"] = {"encode_ms": round(t, 2), "encode_gib_s": round(U / t * 1e3 / 2**30, 2), "verified": ok}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
