"""Decode timing of the alt codecs on bench.py's configs[3] mix (262 144 blocks, sizes uniform in
[4096, 65535], half text-like, half random): FastLZ L1 / L2, LZF, LZ4 blocks, best of `reps` HIP-event
timings per decode call, outputs checked on a sample.  For library A/B runs (scripts/build_dec_variant.sh).
Usage: python scripts/alt_dec_time.py [n] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netty_amd import batch as B  # noqa: E402

CH = 65536


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
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

    def best(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return min(ts)

    out = {"chunks": n}
    cap = (B.fastlz_max_compressed_length(CH) + 15) // 16 * 16
    fo = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    foff = torch.arange(n, dtype=torch.int64, device=dev) * cap
    for level in (1, 2):
        lv = torch.full((n,), level, dtype=torch.int32, device=dev)
        fl, fs = B.fastlz_compress(src, off, ln, fo, foff, level=lv)
        dec.zero_()
        t = best(lambda: B.fastlz_decompress(fo, foff, fl, dec, off, ln))
        r = B.fastlz_decompress(fo, foff, fl, dec, off, ln)
        k = 4096
        ok = bool(torch.equal(r, ln)) and all(bool(torch.equal(dec[i * CH:i * CH + int(ln[i])], src[i * CH:i * CH + int(ln[i])]))
                                              for i in range(0, n, n // k))
        out[f"fastlz_l{level}"] = {"ms": round(t, 3), "gib_s": round(U / (t / 1e3) / 2**30, 2), "ok": ok}
    del fo
    # LZF: the compressed ("ZV" type 1) blocks of lzf_encode's chunk stream, body at +7 (bench.py's leg)
    lcap = (B.lzf_max_compressed_length(CH) + 15) // 16 * 16
    lo = torch.empty(n * lcap, dtype=torch.uint8, device=dev)
    loff = torch.arange(n, dtype=torch.int64, device=dev) * lcap
    B.lzf_encode(src, off, ln, lo, loff)
    idx = torch.nonzero(lo[loff + 2] == 1).flatten()
    boff = loff[idx] + 7
    blen = (lo[loff[idx] + 3].to(torch.int32) << 8) | lo[loff[idx] + 4].to(torch.int32)
    uo, ul = off[idx], ln[idx]
    dec.zero_()
    t = best(lambda: B.lzf_decode(lo, boff, blen, dec, uo, ul))
    r = B.lzf_decode(lo, boff, blen, dec, uo, ul)
    sel = idx[::max(1, idx.numel() // 4096)].tolist()
    ok = int((r != 0).sum()) == 0 and all(bool(torch.equal(dec[i * CH:i * CH + int(ln[i])], src[i * CH:i * CH + int(ln[i])])) for i in sel)
    Ul = int(ul.to(torch.int64).sum())
    out["lzf"] = {"ms": round(t, 3), "blocks": int(idx.numel()), "gib_s": round(Ul / (t / 1e3) / 2**30, 2), "ok": ok}
    del lo
    zcap = (B.lz4_max_compressed_length(CH) + 15) // 16 * 16
    zo = torch.empty(n * zcap, dtype=torch.uint8, device=dev)
    zoff = torch.arange(n, dtype=torch.int64, device=dev) * zcap
    zl, zs = B.lz4_encode(src, off, ln, zo, zoff)
    dec.zero_()
    t = best(lambda: B.lz4_decode(zo, zoff, zl, dec, off, ln))
    out["lz4"] = {"ms": round(t, 3), "gib_s": round(U / (t / 1e3) / 2**30, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
