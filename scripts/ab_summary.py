"""Summarise a decoder A/B session (scripts/r6/s12.sh style): k_parse / k_expand per dispatch from
trace_<variant>_<round>.txt, decode + verify from dec_<variant>_<round>.log, alt decoders from alt_dec.log.
    python scripts/ab_summary.py gpurun_out/r6s13
"""
import json
import re
import sys
from collections import defaultdict


def main(d):
    parse, expand, dec = defaultdict(list), defaultdict(list), defaultdict(list)
    import glob
    import os
    for f in sorted(glob.glob(os.path.join(d, "trace_*_*.txt"))):
        v = os.path.basename(f)[6:-4].rsplit("_", 1)[0]
        for line in open(f):
            m = re.search(r"(k_parse|k_expand)\s.*?([\d.]+) ms", line)
            if m:
                (parse if m.group(1) == "k_parse" else expand)[v].append(float(m.group(2)))
    for f in sorted(glob.glob(os.path.join(d, "dec_*_*.log"))):
        v = os.path.basename(f)[4:-4].rsplit("_", 1)[0]
        for line in open(f):
            if line.startswith("{"):
                dec[v].append(json.loads(line)["decode_ms"])
    alt = defaultdict(lambda: defaultdict(list))
    p = os.path.join(d, "alt_dec.log")
    if os.path.exists(p):
        v = None
        for line in open(p):
            w = line.split()
            if w and not line.startswith("{") and not line.startswith("/"):
                v = w[0]
            i = line.find("{")
            if i >= 0 and v:
                for k, x in json.loads(line[i:]).items():
                    if isinstance(x, dict) and "ms" in x:
                        alt[v][k].append(x["ms"])
    med = lambda a: sorted(a)[len(a) // 2]
    for v in parse:
        print(f"{v:8s} k_parse med {med(parse[v]):6.2f} (min {min(parse[v]):6.2f})  k_expand med {med(expand[v]):6.2f} "
              f"(min {min(expand[v]):6.2f})  decode+verify best-of-4 per run {sorted(dec[v])}  "
              + "  ".join(f"{k} {min(a):.2f}-{max(a):.2f}" for k, a in alt[v].items()))


if __name__ == "__main__":
    main(sys.argv[1])
