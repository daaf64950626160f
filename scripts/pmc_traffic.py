"""Summarise the FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_traffic.sh per kernel: HBM bytes per
64 KiB chunk.  The passes run bench.py with --total-chunks = --sub-chunks = CHUNKS (round 6: 327 680,
one launch of the dense encoder, whose decode call the library runs as parse/expand pairs of 262 144 +
65 536 frames), so every pass (the timed step, verify's pass and its first-call re-runs) encodes and
decodes all CHUNKS chunks, once per dense-encoder dispatch: a kernel's bytes per chunk = its total
bytes / (CHUNKS x encoder dispatches).  FETCH_SIZE is doubled as MI355X_MICROARCH.md's HBM section
prescribes for gfx950 (it tallies 128-B read requests at 64 B); WRITE_SIZE is taken as is.  The
summary records the digest of the kernel sources it was taken on (bench.source_digest()); bench.py
uses a summary only when that digest matches.  Units: bytes."""
import collections, csv, glob, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

root, chunks = sys.argv[1], int(sys.argv[2])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}/traffic_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if not name.startswith("nx::"):
                continue
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"]) * 1024.0  # KiB -> bytes
            disp[(name, c)].add(r["Dispatch_Id"])
enc = [k for k in agg if k.startswith("nx::enc::k_snappy_encode<true, false>")]
passes = float(max(len(disp[(enc[0], "FETCH_SIZE")]), 1)) if enc else 1.0
out = {"source": f"rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE; bench.py --total-chunks {chunks} "
                 f"--sub-chunks {chunks} --steps 1 --warmup 0 --weak-chunks 0 --no-latency --no-probe-ceiling",
       "source_digest": bench.source_digest(), "fetch_correction": 2.0, "chunks_per_pass": chunks, "passes": passes,
       "kernels": {}}
for name, d in agg.items():
    nd = max(len(disp[(name, "FETCH_SIZE")]), len(disp[(name, "WRITE_SIZE")]), 1)
    fetch, write = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
    per = chunks * passes
    out["kernels"][name] = {"dispatches": nd, "fetch_bytes": fetch, "write_bytes": write,
                            "hbm_bytes_total": 2.0 * fetch + write,
                            "read_bytes_per_chunk": 2.0 * fetch / per,
                            "write_bytes_per_chunk": write / per,
                            "hbm_bytes_per_chunk": (2.0 * fetch + write) / per}
print(json.dumps(out, indent=1))
