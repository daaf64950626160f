"""Time the single-cumulation frame walk (nx_snappy_frame_scan_long) against the lane walk on one
~1 GiB SnappyFrameEncoder stream of text-like 64 KiB chunks (as bench.py's frame_scan.long_stream),
and check the two lists are equal.  Run under rocprofv3 --kernel-trace --stats for the per-kernel
split.  Usage: python scripts/long_scan_prof.py [chunks] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netty_amd import batch as B  # noqa: E402

CH = 65536


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 35840
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    src = torch.empty(m * CH, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, m, CH)
    off = torch.arange(m, dtype=torch.int64, device=dev) * CH
    ln = torch.full((m,), CH, dtype=torch.int32, device=dev)
    cap = (B.snappy_max_compressed_length(CH) + 15) // 16 * 16
    enc = torch.empty(m * cap, dtype=torch.uint8, device=dev)
    eoff = torch.arange(m, dtype=torch.int64, device=dev) * cap
    elen, est = B.snappy_encode(src, off, ln, enc, eoff)
    crc = B.crc32c_masked(src, off, ln)
    del src
    fs = elen.to(torch.int64) + 8
    hp = torch.cumsum(fs, 0) - fs + 10
    total = int((hp[-1] + fs[-1]).item())
    buf = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
    buf[:10] = torch.tensor(list(b"\xff\x06\x00\x00sNaPpY"), dtype=torch.uint8, device=dev)
    clen = fs - 4
    c32 = crc.to(torch.int64) & 0xFFFFFFFF
    hdr = torch.stack([torch.zeros_like(clen), clen & 255, (clen >> 8) & 255, (clen >> 16) & 255,
                       c32 & 255, (c32 >> 8) & 255, (c32 >> 16) & 255, (c32 >> 24) & 255], 1).to(torch.uint8)
    buf[(hp.view(-1, 1) + torch.arange(8, device=dev)).view(-1)] = hdr.view(-1)
    B.gather(enc, eoff, elen, dst=buf, dst_off=hp + 8)
    del enc
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    lens = torch.tensor([total], dtype=torch.int64, device=dev)

    def best(fn):
        fn()
        torch.cuda.synchronize()
        tt, r = [], None
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.zero_()
            a.record()
            r = fn()
            b.record()
            torch.cuda.synchronize()
            tt.append(a.elapsed_time(b))
        return min(tt), tt, r

    t_lane, _, rl = best(lambda: B.snappy_frame_scan(buf, zero, lens, st, m))
    t_long, all_long, rg = best(lambda: B.snappy_frame_scan_long(buf, total, st, m))
    same = all(bool(torch.equal(rl[k][:m], rg[k][:m])) for k in ("data_off", "data_len", "masked_crc", "seq"))
    ok = same and rg["counts"].tolist() == [m, 0, m] and int(rg["consumed"].item()) == total and int(rg["status"].item()) == 0
    print(json.dumps({"bytes": total, "chunks": m, "lane_walk_ms": round(t_lane, 3), "segmented_walk_ms": round(t_long, 3),
                      "segmented_all_ms": [round(x, 3) for x in all_long], "verified": ok}))
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
