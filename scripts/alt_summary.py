"""Summarise a scripts/gpu_alt_prof.sh run: per-kernel median launch time and the alt_codecs rates."""
import csv
import json
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_alt"
agg = defaultdict(list)
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    agg[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n, v in agg.items():
    if any(k in n for k in ("parse", "expand", "encode", "compress")):
        print(f"{n:44s} n={len(v):3d} med={sorted(v)[len(v) // 2]:.3f} ms")
lines = [x for x in open(f"{d}/bench.log") if x.startswith("{")]
a = json.loads(lines[-1])["alt_codecs"]
for k in ("fastlz_l1", "fastlz_l2", "lzf", "lz4"):
    print(k, "encode", a[k]["encode_gib_s"], "decode", a[k]["decode_gib_s"], "verified", a[k]["verified"])
print("lz4_frame", {k: a["lz4_frame"][k] for k in ("xxhash32_gib_s", "encode_gib_s", "scan_decode_verify_gib_s", "verified")})
