#!/bin/bash
# End-to-end tool under several GPU_MAX_HW_QUEUES values (HIP's hardware queues per process; a
# stream shares its queue with others when the process has more streams than queues): HWQ="4 8 16".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for q in ${HWQ:-4 8 16}; do
    echo -n "Q$q " >> gpurun_out/e2e_hwq.log
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 netty_amd/e2e_capi 256 256 65535 3 0 ${FLUSH:-256} >> gpurun_out/e2e_hwq.log 2>&1 || exit 1
  done
done
