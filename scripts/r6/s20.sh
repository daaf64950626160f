#!/bin/bash
# Round 6 session 20: the round-end sequence on the final tree, as the driver runs it: the -m gpu suite,
# smoke, and the driver's bench command (20 timed steps after 5 warm-up steps), each timed end to end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6s20
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
t0=$(date +%s)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu $rc wall_s $(( $(date +%s) - t0 ))" >> $O/steps.log; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
t0=$(date +%s)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke $rc wall_s $(( $(date +%s) - t0 ))" >> $O/steps.log; fatal $rc smoke; [ $rc -ne 0 ] && exit $rc
t0=$(date +%s)
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1; rc=$?
echo "bench $rc wall_s $(( $(date +%s) - t0 ))" >> $O/steps.log
exit $rc
