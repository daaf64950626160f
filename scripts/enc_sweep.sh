#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out
for w in 8 16 32; do
  NX_ENC_WAVES=$w timeout -k 10 240 python scripts/prof_encode.py 1048576 2 >> gpurun_out/enc_sweep.log 2>&1 || exit 1
done
export TMPDIR=/tmp; cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/encpmc_$c" -o p -- python "$ROOT/scripts/prof_encode.py" 262144 1 >> "$ROOT/gpurun_out/enc_sweep.log" 2>&1 || exit 1
done
