"""Summarise variant A/B runs made as `rocprofv3 --kernel-trace --stats -d <dir>/kt_<variant>_<round> -o k
-- python3 scripts/dec_time.py ...` (scripts/r5/s24.sh): per variant, the average duration of each
named kernel over all rounds' launches and dec_time's best decode_ms per round.
Usage: python scripts/kt_summary.py <dir> [kernel-substring ...]"""
import glob
import json
import os
import re
import sqlite3
import sys


def main():
    d = sys.argv[1]
    keys = sys.argv[2:] or ["k_parse(", "k_expand("]
    rows = {}
    for db in sorted(glob.glob(os.path.join(d, "kt_*_*", "k_results.db"))):
        m = re.match(r"kt_(.+)_(\d+)$", os.path.basename(os.path.dirname(db)))
        if not m:
            continue
        v = m.group(1)
        r = rows.setdefault(v, {"durs": {k: [] for k in keys}, "decode_ms": []})
        c = sqlite3.connect(db)
        for name, dur in c.execute("select name, duration from kernels"):
            for k in keys:
                if k in name:
                    r["durs"][k].append(dur / 1e6)
        log = os.path.join(d, f"kt_{v}_{m.group(2)}.log")
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{"):
                    j = json.loads(line)
                    r["decode_ms"].append(j.get("decode_ms") or {k: v["ms"] for k, v in j.items() if isinstance(v, dict)})
    out = []
    for v, r in rows.items():
        e = {"variant": v, "decode_ms": r["decode_ms"]}
        for k, xs in r["durs"].items():
            e[k.rstrip("(") + "_ms"] = round(sum(xs) / len(xs), 3) if xs else None
            e[k.rstrip("(") + "_n"] = len(xs)
        out.append(e)
        print(json.dumps(e))
    return out


if __name__ == "__main__":
    main()
