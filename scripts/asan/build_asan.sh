#!/bin/bash
# Host-code AddressSanitizer build of the library's C++ side driven by the end-to-end tool
# (netty_amd/tools/e2e_capi.cpp): every csrc file compiled with ASan on the HOST side only (device
# code is untouched; GPU sanitizers are not available on this pool), linked statically into one
# executable, netty_amd/build_asan/e2e_capi_asan, and the handler tour scripts/asan/capi_tour.cpp as
# netty_amd/build_asan/capi_tour_asan.  Run them on a GPU box with small sizes (scripts/r5/s34.sh):
#   ASAN_OPTIONS=protect_shadow_gap=0:detect_leaks=1 netty_amd/build_asan/e2e_capi_asan 16 16 65535 1 0 4
set -eu
cd "$(dirname "$0")/../.."
H=/opt/rocm/bin/hipcc
SAN=${SAN:-address}  # SAN=address,undefined adds UBSan (host side too)
F="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics -Xarch_host -fsanitize=$SAN -Xarch_host -fno-omit-frame-pointer"
O=netty_amd/build_asan
mkdir -p $O
objs=""
for f in netty_amd/csrc/*.hip netty_amd/csrc/*.cpp; do
  b=$(basename "${f%.*}")
  extra=""
  [ "$b" = snappy_decode ] && extra="-mllvm -phi-node-folding-threshold=16 -mllvm -two-entry-phi-node-folding-threshold=32"
  $H $F $extra -x hip -c "$f" -o "$O/$b.o" &
  objs="$objs $O/$b.o"
done
wait
$H $F -x hip -c netty_amd/tools/e2e_capi.cpp -o $O/e2e_capi.o
$H --offload-arch=gfx950 -Xarch_host -fsanitize=$SAN -o $O/e2e_capi_asan $O/e2e_capi.o $objs
$H $F -x hip -c scripts/asan/capi_tour.cpp -o $O/capi_tour.o
$H --offload-arch=gfx950 -Xarch_host -fsanitize=$SAN -o $O/capi_tour_asan $O/capi_tour.o $objs
echo $O/e2e_capi_asan $O/capi_tour_asan
