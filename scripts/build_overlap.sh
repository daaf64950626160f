#!/bin/bash
# Build scripts/experiments/bin/overlap_<stage> (scripts/experiments/overlap.cpp): the kernel parts of
# snappy_encode.hip (with its output stage at $1 dwords per lane) and snappy_decode.hip in one TU,
# linked against netty_amd/libnetty_amd.so (CRC tables).  Experiments only.
set -eu
cd "$(dirname "$0")/.."
SD=${1:-32}
mkdir -p scripts/experiments/bin
python3 - "$SD" <<'PY'
import re, sys
sd = sys.argv[1]
e = open("netty_amd/csrc/snappy_encode.hip").read()
e = e[:e.index("namespace {\nconstexpr unsigned kEncBlock")]
e = e.replace("constexpr int kStageDw = 32;", f"constexpr int kStageDw = {sd};")
import os
if os.environ.get("ENC_LB"):  # the encoder's minimum blocks per CU (register budget)
    e = e.replace("__launch_bounds__(256, 4) k_snappy_encode", f"__launch_bounds__(256, {os.environ['ENC_LB']}) k_snappy_encode")
assert f"kStageDw = {sd};" in e
open(f"scripts/experiments/bin/ov_enc_{sd}.hip", "w").write(e)
d = open("netty_amd/csrc/snappy_decode.hip").read()
d = d[:d.index("static_assert(nx::kDecSlotBytes")]
d += "\nconstexpr size_t kExpandLds = nx::dec::kTabBytes + nx::dec::kExpandWaves * nx::dec::kExpandWaveLds;\n"
open("scripts/experiments/bin/ov_dec.hip", "w").write(d)
PY
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I netty_amd/csrc \
    -mllvm -phi-node-folding-threshold=16 -mllvm -two-entry-phi-node-folding-threshold=32 \
    -DENC_SRC="\"bin/ov_enc_$SD.hip\"" -DDEC_SRC="\"bin/ov_dec.hip\"" \
    -o scripts/experiments/bin/overlap_$SD${ENC_LB:+_lb$ENC_LB} scripts/experiments/overlap.cpp -L netty_amd -lnetty_amd -Wl,-rpath,'$ORIGIN/../../../netty_amd'
echo built scripts/experiments/bin/overlap_$SD${ENC_LB:+_lb$ENC_LB}
