"""Summarise the FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_traffic.sh per kernel (per dispatch,
and per 64 KiB chunk of one pass: bench.py decodes every chunk twice — the timed step and the
corrupted-CRC check — and the decoder launches one parse/expand pair per 262 144 frames).  FETCH_SIZE is doubled as MI355X_MICROARCH.md's HBM section prescribes for
gfx950 (it tallies 128-B read requests at 64 B); WRITE_SIZE is taken as is.  Units: bytes."""
import collections, csv, glob, json, sys
root, chunks = sys.argv[1], int(sys.argv[2])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
grid = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}/traffic_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if not name.startswith("nx::"):
                continue
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"]) * 1024.0  # KiB -> bytes
            disp[(name, c)].add(r["Dispatch_Id"])
out = {"source": f"rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE; bench.py --chunks {chunks} --steps 1 --warmup 0",
       "fetch_correction": 2.0, "chunks": chunks, "kernels": {}}
for name, d in agg.items():
    nd = max(len(disp[(name, "FETCH_SIZE")]), len(disp[(name, "WRITE_SIZE")]), 1)
    per_pass = -(-chunks // 262144) if name.startswith("nx::dec::k_parse") or name.startswith("nx::dec::k_expand") else 1
    passes = max(nd // per_pass, 1)
    fetch, write = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
    out["kernels"][name] = {"dispatches": nd, "passes": passes, "fetch_bytes": fetch, "write_bytes": write,
                            "hbm_bytes_total": 2.0 * fetch + write,
                            "hbm_bytes_per_chunk": (2.0 * fetch + write) / (chunks * passes)}
print(json.dumps(out, indent=1))
