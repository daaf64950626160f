#!/bin/bash
# Build netty_amd/build_variants/libnetty_amd_<name>.so: the current library with
# csrc/snappy_decode.hip replaced by another version of it (a file, or a git revision's copy), for
# same-box decoder A/B runs (scripts/ab_dec.sh).  Extra hipcc flags (e.g. -DNX_PARSE_PF=0) after it.
#   scripts/build_dec_variant.sh base ccb28ed          # the round-3 decoder
#   scripts/build_dec_variant.sh nopf HEAD -DNX_PARSE_PF=0
# FILE=batcher.cpp swaps that source instead (any csrc file of the library).
set -eu
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
FILE=${FILE:-snappy_decode.hip}
stem=${FILE%.*}
out=netty_amd/build_variants/$name
mkdir -p "$out"
if [ -f "$src" ]; then cp "$src" "$out/$FILE"; else git show "$src:netty_amd/csrc/$FILE" > "$out/$FILE"; fi
cp netty_amd/csrc/*.hpp "$out/"
make -s -C netty_amd >/dev/null
# (snappy_decode.hip: the Makefile's phi-folding flags come first; flags given here follow them)
[ "$FILE" = snappy_decode.hip ] && set -- -mllvm -phi-node-folding-threshold=16 -mllvm -two-entry-phi-node-folding-threshold=32 "$@"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics "$@" \
    -I netty_amd/csrc -x hip -c "$out/$FILE" -o "$out/$stem.o"
objs=$(ls netty_amd/build/*.o | grep -v "/$stem.o\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "netty_amd/build_variants/libnetty_amd_$name.so" $objs "$out/$stem.o"
echo "netty_amd/build_variants/libnetty_amd_$name.so"
