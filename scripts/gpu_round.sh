#!/bin/bash
# One gpurun session: smoke → GPU tests → short bench → rocprofv3 kernel trace.
# Each GPU step has its own time limit; stop at the first crash/timeout (exit >= 2 from pytest,
# or any non-zero from the other steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
CHUNKS=${CHUNKS:-65536}
STAGE=${STAGE:-all}

run() { echo "== $*" >> "$OUT/steps.log"; "$@"; local rc=$?; echo "   rc=$rc" >> "$OUT/steps.log"; return $rc; }

if [[ $STAGE == all || $STAGE == smoke ]]; then
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
fi
if [[ $STAGE == all || $STAGE == test ]]; then
  run timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  if [[ $rc -ge 2 ]]; then exit $rc; fi
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  run timeout -k 10 600 python bench.py --total-chunks "$CHUNKS" --weak-chunks 0 --steps 3 --warmup 1 --cpu-seconds 6 > "$OUT/bench.log" 2>&1 || exit 1
fi
if [[ $STAGE == full ]]; then  # the driver's default bench line (configs[4], 100 GiB at N=1)
  run timeout -k 10 900 python bench.py > "$OUT/bench_full.log" 2>&1 || exit 1
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  export TMPDIR=/tmp
  cd /tmp && run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python "$ROOT/bench.py" --total-chunks "$CHUNKS" --weak-chunks 0 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-alt --no-frame-scan > "$OUT/prof.log" 2>&1 || exit 1
  cd "$ROOT"
fi
if [[ $STAGE == all || $STAGE == pmc ]]; then
  run env CHUNKS="$CHUNKS" bash scripts/pmc_traffic.sh || exit 1
fi
echo done >> "$OUT/steps.log"
