#!/bin/bash
# Alternate library builds (netty_amd/build_variants/libnetty_amd_<v>.so) on bench.py's configs[3] leg:
# each run is a rocprofv3 kernel trace; summaries via scripts/alt_summary.py.  VARIANTS="4 8" ROUNDS=2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    cp "netty_amd/build_variants/libnetty_amd_$v.so" netty_amd/libnetty_amd.so || exit 1
    D="$ROOT/gpurun_out/ab_alt/${v}_$r"
    mkdir -p "$D"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$D" -o run -- \
        python "$ROOT/bench.py" --total-chunks 16384 --weak-chunks 0 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
        --no-frame-scan --no-probe-ceiling > "$D/bench.log" 2>&1) || exit 1
    python scripts/alt_summary.py "$D" > "$D/summary.txt" 2>&1
  done
done
