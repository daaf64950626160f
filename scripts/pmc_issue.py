"""Summarise scripts/pmc_issue.sh per kernel: wave-instructions per 64 KiB chunk by type, and how much of
the chip's issue capacity the kernel used while it ran.  Normalised as scripts/pmc_traffic.py (every
pass encodes and decodes all CHUNKS chunks once per dense-encoder dispatch).  Cycles: GRBM_GUI_ACTIVE
of each dispatch / 8 (rocprofv3 sums it over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'); SIMD-
cycles = cycles x 1024 SIMDs (256 CUs x 4).  A wave64 VALU instruction holds its SIMD-32 for 2 cycles
(MI355X_MICROARCH.md: 'issues each VALU instruction over 2 cycles'), so valu_busy = 2 VALU / SIMD-cycles;
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles and are used only as ratios of each
other (the wave-state split).  The summary records bench.source_digest()."""
import collections, csv, glob, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

root, chunks = sys.argv[1], int(sys.argv[2])
SIMDS = 1024
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for i in (1, 2):
    for f in glob.glob(f"{root}/issue_{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if not name.startswith("nx::"):
                continue
            c = r["Counter_Name"]
            agg[name][f"{c}@{i}"] += float(r["Counter_Value"])
            disp[(name, i)].add(r["Dispatch_Id"])
enc = [k for k in agg if k.startswith("nx::enc::k_snappy_encode<true, false>")]
passes = float(max(len(disp[(enc[0], 1)]), 1)) if enc else 1.0
out = {"source": f"rocprofv3 --pmc (2 passes: instruction mix; wave-cycle split), bench.py --total-chunks {chunks} "
                 f"--sub-chunks {chunks} --steps 1 --warmup 0", "source_digest": bench.source_digest(),
       "chunks_per_pass": chunks, "passes": passes, "simds": SIMDS, "kernels": {}}
for name, d in agg.items():
    per = chunks * passes
    cyc1 = d.get("GRBM_GUI_ACTIVE@1", 0.0) / 8.0
    ins = {k: d.get(f"SQ_INSTS_{k}@1", 0.0) for k in ("VALU", "SALU", "LDS", "SMEM", "VMEM_RD", "VMEM_WR", "BRANCH")}
    tot = sum(ins.values())
    wc = d.get("SQ_WAVE_CYCLES@2", 0.0)
    k = {"dispatches": len(disp[(name, 1)]), "waves": d.get("SQ_WAVES@1", 0.0), "cycles": cyc1,
         "insts_per_chunk": {t: v / per for t, v in ins.items()},
         "valu_busy": 2.0 * ins["VALU"] / (SIMDS * cyc1) if cyc1 else None,
         "insts_per_simd_cycle": tot / (SIMDS * cyc1) if cyc1 else None}
    if wc:
        k["wave_split"] = {"issuing": d.get("SQ_ACTIVE_INST_ANY@2", 0.0) / wc, "stalled_at_issue": d.get("SQ_WAIT_INST_ANY@2", 0.0) / wc,
                           "waitcnt": d.get("SQ_WAIT_ANY@2", 0.0) / wc, "valu_active": d.get("SQ_ACTIVE_INST_VALU@2", 0.0) / wc}
    out["kernels"][name] = k
print(json.dumps(out, indent=1))
