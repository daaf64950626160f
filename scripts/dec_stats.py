"""Per-frame pass / round counters of k_expand from a diagnostic build (scripts/mk_dec_stats.py
adds them; the product library has no such symbol), or with --stamps the per-section shader-clock
cycles of scripts/mk_dec_stamps.py's build.

    python scripts/dec_stats.py [--stamps] [chunks]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from netty_amd import batch as B
    from netty_amd import _lib
    args = [a for a in sys.argv[1:] if a != "--stamps"]
    stamps = "--stamps" in sys.argv
    n = int(args[0]) if args else 16384
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
    lib = C.CDLL(_lib.LIB_PATH)
    buf = (C.c_ulonglong * 16)()
    lib.nx_dec_stats_read(buf)  # reset
    dec = torch.empty_like(src)
    r = B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=crc)
    torch.cuda.synchronize()
    assert lib.nx_dec_stats_read(buf) == 0
    names = ["windows", "passes", "rounds", "map_passes", "far_or_unstaged_passes", "overlap_passes", "-", "pieces"]
    ok = bool(torch.equal(dec, src)) and int((r["status"] != 0).sum()) == 0
    if stamps:
        names = ["map_records", "addresses_far_issue_producer_map", "overlap_addresses", "round0_incl_far_wait",
                 "dependent_rounds", "flush_crc", "passes", "frame_total", "window_setup", "expand_prologue", "window_slide",
                 "finish_crc_result", "windows", "parse_reload", "parse_tags", "parse_total"]
        per = {k: buf[i] / n for i, k in enumerate(names)}
        tot = per["frame_total"]
        pas = names[:6]
        frac = {k: round(per[k] / tot, 4) for k in pas + ["window_setup", "expand_prologue", "window_slide", "finish_crc_result"]}
        frac["unaccounted"] = round(1 - sum(frac.values()), 4)
        print(json.dumps({"chunks": n, "verified": ok, "cycles_per_frame": round(tot), "passes_per_frame": round(per["passes"], 1),
                          "windows_per_frame": round(per["windows"], 1),
                          "cycles_per_pass": {k: round(per[k] / per["passes"], 1) for k in pas},
                          "cycles_per_window": {k: round(per[k] / per["windows"], 1) for k in ("window_setup", "expand_prologue", "window_slide")},
                          "fraction_of_frame": frac,
                          "k_parse_cycles_per_wave": {k: round(buf[13 + i] / (n / 64)) for i, k in enumerate(("reload", "tag_loop", "total"))}}))
        return
    print(json.dumps({"chunks": n, "verified": ok, "per_frame": {k: round(buf[i] / n, 2) for i, k in enumerate(names) if k != "-"}}))


if __name__ == "__main__":
    main()
