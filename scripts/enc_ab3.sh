#!/bin/bash
# Build the placement-controlled encoder A/B (scripts/experiments/enc_ab3.cpp) for a pair of kernel
# sources: A = the product's snappy_encode.hip, B = $1 (a modified copy).  Each is amalgamated with
# nx_common.hpp (kernel part only: cut before the host entry points) so both builds live in their own
# namespace in one binary.  Output: scripts/experiments/bin/enc_ab3_$2 (MAIN=enc_curve: the
# chunks-per-launch curve harness instead, scripts/experiments/enc_curve.cpp).
set -eu
cd "$(dirname "$0")/.."
B=${1:?variant source}
TAG=${2:?tag}
mkdir -p scripts/experiments/bin
python3 - "$B" "$TAG" <<'EOF'
import re, sys
common = open("netty_amd/csrc/nx_common.hpp").read()
common = common.replace("#pragma once", "")
common = re.sub(r'#include [<"][^>"]+[>"]\n', "", common)
def amalg(src, out):
    s = open(src).read()
    cut = s.index("namespace {\nconstexpr unsigned kEncBlock")
    s = s[:cut]
    s = s.replace('#include "nx_common.hpp"\n', common).replace('#include "workspace.hpp"\n', "")
    s = re.sub(r'#include <[^>]+>\n', "", s)
    open(out, "w").write(s)
amalg("netty_amd/csrc/snappy_encode.hip", "scripts/experiments/bin/encA.hip")
amalg(sys.argv[1], f"scripts/experiments/bin/encB_{sys.argv[2]}.hip")
EOF
cat > scripts/experiments/bin/prelude_$TAG.cpp <<EOF
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <vector>
#include "../../../include/netty_amd_status.h"
#define ENC_A "bin/encA.hip"
#define ENC_B "bin/encB_$TAG.hip"
#include "../${MAIN:-enc_ab3}.cpp"
EOF
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I netty_amd/csrc \
    -o scripts/experiments/bin/${MAIN:-enc_ab3}_$TAG scripts/experiments/bin/prelude_$TAG.cpp
echo built scripts/experiments/bin/${MAIN:-enc_ab3}_$TAG
