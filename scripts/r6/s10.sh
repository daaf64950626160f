#!/bin/bash
# Round 6 session 10: host-side ASan + UBSan of the round-6 library (SAN=address,undefined scripts/asan/build_asan.sh):
# host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the batcher / handler C++ code through the
# end-to-end tool (scripts/asan/build_asan.sh; device code not instrumented): one flush and 4 MiB
# auto-flushes, then several event-loop threads; then the handler tour (scripts/asan/capi_tour.cpp:
# every codec's handlers, batcher jobs, corrupted streams, handles freed with jobs in flight).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6s10
mkdir -p $O
export ASAN_OPTIONS=protect_shadow_gap=0:detect_leaks=1:verify_asan_link_order=0:halt_on_error=1
# the HIP / HSA runtimes' own allocations at exit are not ours (round 5 s34's first run: every leak
# stack ended in libhsa-runtime64 / libamdhip64)
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export LSAN_OPTIONS=suppressions=$(pwd)/scripts/asan/lsan.supp:print_suppressions=0
timeout -k 10 240 netty_amd/build_asan/e2e_capi_asan 32 32 65535 2 0 4 > $O/asan_one_thread.log 2>&1; rc=$?
echo "one_thread $rc" >> $O/steps.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 240 netty_amd/build_asan/e2e_capi_asan 32 32 65535 2 16 4 4 > $O/asan_four_threads.log 2>&1; rc=$?
echo "four_threads $rc" >> $O/steps.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 netty_amd/build_asan/capi_tour_asan 2 > $O/asan_capi_tour.log 2>&1; rc=$?
echo "capi_tour $rc" >> $O/steps.log
case $rc in 124|134|137|139) exit $rc;; esac
# the two-rank GPU test, now also on the library's launch plan
unset ASAN_OPTIONS UBSAN_OPTIONS LSAN_OPTIONS
timeout -k 10 400 python -u -m pytest tests/test_gpu_two_ranks.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_two_ranks.log 2>&1; rc2=$?
echo "two_ranks $rc2" >> $O/steps.log
exit $(( rc > rc2 ? rc : rc2 ))
