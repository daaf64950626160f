#!/bin/bash
# PMC instruction / cycle counters of the decode kernels for alternate library builds
# (netty_amd/build_variants/libnetty_amd_<v>.so; VARIANTS="a b").
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
N=${N:-65536}
for v in ${VARIANTS}; do
  cp "$ROOT/netty_amd/build_variants/libnetty_amd_$v.so" "$ROOT/netty_amd/libnetty_amd.so" || exit 1
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
              "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$ROOT/gpurun_out/pmc_${v}_$i" -o p -- python "$ROOT/scripts/prof_decode.py" $N 1 > "$ROOT/gpurun_out/pmc_${v}_$i.log" 2>&1) || exit 1
  done
done
