"""Summarise scripts/pmc_alt_traffic.sh: HBM bytes per call of each alt-codec leg's encode and decode
(bench.bench_alt_codecs order: fastlz_l1, fastlz_l2, lzf, lz4; each phase = one warm-up call + one
timed call).  Dispatches are walked in order; a leg starts at its encoder's first dispatch and every
nx:: kernel until the next encoder belongs to its decode phase (the parse, the shared expander, the
finish/fallback kernels).  FETCH_SIZE doubled for gfx950 (MI355X_MICROARCH.md), WRITE_SIZE as is;
the summary records bench.alt_source_digest() so bench.py only uses it on the same sources."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

LEGS = ("fastlz_l1", "fastlz_l2", "lzf", "lz4")
ENCODERS = ("nx::flz::k_compress", "nx::lzf::k_encode", "nx::lz4::k_lz4_encode")
SKIP = ("nx::k_ws_probe",)          # the encoder workspace's placement probe (a one-off before an encoder)
STOP = ("nx::lz4f::k_xxhash32",)    # the LZ4 frame leg that follows the four block legs
CALLS = 2  # warm-up + timed


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].strip()


def main():
    root, n = sys.argv[1], int(sys.argv[2])
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = collections.defaultdict(float)
        names = {}
        for f in glob.glob(f"{root}/alt_traffic_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = int(r["Dispatch_Id"])
                rows[k] += float(r["Counter_Value"]) * 1024.0  # KiB -> bytes
                names[k] = short(r["Kernel_Name"])
        leg, phase, prev_enc = -1, None, False
        for k in sorted(rows):
            nm = names[k]
            if not nm.startswith("nx::") or nm in SKIP:
                continue
            if nm in STOP and leg >= 0:
                break
            is_enc = nm in ENCODERS
            if is_enc and not prev_enc:
                leg += 1
            prev_enc = is_enc
            if leg < 0 or leg >= len(LEGS):
                continue
            phase = "encode" if is_enc else "decode"
            d = per.setdefault(LEGS[leg], {}).setdefault(phase, {"kernels": collections.Counter(), "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0})
            d[c] += rows[k]
            if c == "FETCH_SIZE":
                d["kernels"][nm] += 1
    out = {"source": "rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE; scripts/alt_traffic_run.py " + str(n),
           "source_digest": bench.alt_source_digest(), "fetch_correction": 2.0, "chunks": n, "calls_per_phase": CALLS,
           "legs": {}}
    for leg, phases in per.items():
        out["legs"][leg] = {}
        for ph, d in phases.items():
            tot = 2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]
            out["legs"][leg][ph] = {"dispatches": dict(d["kernels"]), "read_bytes_per_call": 2.0 * d["FETCH_SIZE"] / CALLS,
                                    "write_bytes_per_call": d["WRITE_SIZE"] / CALLS, "hbm_bytes_per_call": tot / CALLS}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
