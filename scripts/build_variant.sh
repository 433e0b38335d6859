#!/bin/bash
# Build libswbank with extra compile flags into lib/libswbank_NAME.so (A/B of kernel variants on
# one box with SWBANK_LIB=...):   scripts/build_variant.sh NAME "-DSWK_PROF_AHEAD=0 ..."
# (every in-tree .so travels with each gpurun push: delete the variant when its A/B is done)
set -eu
set -o pipefail
NAME=$1; FLAGS=${2:-}
cd "$(dirname "$0")/../smith-waterman-fpga-module_amd"
B=build/var_$NAME; mkdir -p $B lib
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -munsafe-fp-atomics -I../include -Icsrc $FLAGS"
rm -f $B/*.o
pids=""
for u in ktile kwave kaux; do $H -c csrc/swbank_$u.hip -o $B/$u.o & pids="$pids $!"; done
for u in bank launch feeder stream multi; do $H -c csrc/swbank_$u.hip -o $B/$u.o & pids="$pids $!"; done
cc -O2 -fPIC -Wall -Wextra -std=c11 -I../include -Icsrc -c csrc/swbank_host.c -o $B/h.o
for p in $pids; do wait $p; done  # (set -e: a failed compile ends the script)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libswbank_$NAME.so $B/h.o \
  $B/bank.o $B/launch.o $B/feeder.o $B/stream.o $B/multi.o $B/ktile.o $B/kwave.o $B/kaux.o
echo "lib/libswbank_$NAME.so"
