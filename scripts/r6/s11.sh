#!/bin/bash
# Round 6 session 11: the driver's own bench command on the final sources (20 timed steps after 5
# warm-up steps), timed end to end, as the round-end run will be.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6s11
mkdir -p $O
t0=$(date +%s)
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1; rc=$?
echo "bench $rc wall_s $(( $(date +%s) - t0 ))" >> $O/steps.log
exit $rc
