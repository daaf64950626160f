#!/bin/bash
# Build scripts/experiments/bin/dec_pipe_<blk> (scripts/experiments/dec_pipe.cpp): the kernel part of
# snappy_decode.hip compiled with NX_PARSE_BLOCK=$1 in one TU with the harness, linked against
# netty_amd/libnetty_amd.so.  Experiments only.
set -eu
cd "$(dirname "$0")/.."
BLK=${1:-128}
mkdir -p scripts/experiments/bin
python3 - <<'PY'
d = open("netty_amd/csrc/snappy_decode.hip").read()
d = d[:d.index("static_assert(nx::kDecSlotBytes")]
d += "\nconstexpr size_t kExpandLds = nx::dec::kTabBytes + nx::dec::kExpandWaves * nx::dec::kExpandWaveLds;\n"
open("scripts/experiments/bin/pipe_dec.hip", "w").write(d)
PY
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I netty_amd/csrc -DNX_PARSE_BLOCK=$BLK \
    -mllvm -phi-node-folding-threshold=16 -mllvm -two-entry-phi-node-folding-threshold=32 \
    -DDEC_SRC="\"bin/pipe_dec.hip\"" \
    -o scripts/experiments/bin/dec_pipe_$BLK scripts/experiments/dec_pipe.cpp -L netty_amd -lnetty_amd -Wl,-rpath,'$ORIGIN/../../../netty_amd'
echo built scripts/experiments/bin/dec_pipe_$BLK
