#!/bin/bash
# Round 5 session 14 (evidence, part 2): rocprofv3 kernel trace of the bench workload (262 144 chunks
# per dispatch), the FETCH/WRITE traffic passes behind roofline.traffic, and the alt-codec traffic
# passes behind each alt leg's roofline traffic (all on the final kernel sources).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s14
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- \
    python3 "$ROOT/bench.py" --total-chunks 262144 --weak-chunks 0 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-alt \
    --no-frame-scan --no-latency > "$ROOT/$O/prof.log" 2>&1); rc=$?; echo "prof $rc" >> $O/steps.log; fatal $rc prof
CHUNKS=262144 timeout -k 10 700 bash scripts/pmc_traffic.sh; rc=$?; echo "pmc_traffic $rc" >> $O/steps.log; fatal $rc pmc
mv gpurun_out/pmc_traffic.json gpurun_out/traffic_*.log $O/ 2>/dev/null
for c in FETCH_SIZE WRITE_SIZE; do mv gpurun_out/traffic_$c $O/ 2>/dev/null; done
N=262144 timeout -k 10 700 bash scripts/pmc_alt_traffic.sh; rc=$?; echo "alt_pmc $rc" >> $O/steps.log; fatal $rc alt_pmc
mv gpurun_out/alt_traffic.json gpurun_out/alt_traffic_* $O/ 2>/dev/null
exit 0
