#!/bin/bash
# Build netty_amd/build_variants/libnetty_amd_<name>.so: the whole current library compiled with extra
# hipcc flags (build options such as -DNX_FLZ_WPCU=16), for same-box A/B runs that copy a variant over
# netty_amd/libnetty_amd.so on the GPU box (scripts/r6/*.sh).
#   scripts/build_lib_variant.sh flz16 -DNX_FLZ_WPCU=16 -DNX_LZF_WPCU=16
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
out=netty_amd/build_variants/$name
mkdir -p "$out"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics"
objs=""
for src in netty_amd/csrc/*.hip netty_amd/csrc/*.cpp; do
  stem=$(basename "${src%.*}")
  extra=""
  [ "$stem" = snappy_decode ] && extra="-mllvm -phi-node-folding-threshold=16 -mllvm -two-entry-phi-node-folding-threshold=32"
  /opt/rocm/bin/hipcc $F $extra "$@" -I netty_amd/csrc -x hip -c "$src" -o "$out/$stem.o" &
  objs="$objs $out/$stem.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "netty_amd/build_variants/libnetty_amd_$name.so" $objs
echo "netty_amd/build_variants/libnetty_amd_$name.so"
