#!/bin/bash
# HBM traffic of the alt-codec kernels (bench.py alt_codecs: FastLZ L1/L2, LZF, LZ4 blocks): separate
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over scripts/alt_traffic_run.py, summarised per leg and
# phase into gpurun_out/alt_traffic.json (copy it under profiles/<round>/: bench.py attaches it to each
# leg's roofline when its source digest matches).
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
N=${N:-262144}
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/alt_traffic_$c" -o p -- \
      python3 "$ROOT/scripts/alt_traffic_run.py" "$N" > "$ROOT/gpurun_out/alt_traffic_$c.log" 2>&1 || exit 1
done
cd "$ROOT" && python scripts/pmc_alt_traffic.py gpurun_out "$N" > gpurun_out/alt_traffic.json
