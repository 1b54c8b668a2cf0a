#!/bin/bash
# Build ab/libdpathsim_<name>.so with a variant of the hot kernel: dps_cct1.hip
# from the working copy (or from commit $SRC, or the file $SRCFILE) compiled with extra flags ($2...),
# linked with the other objects of the regular build (run `make` first).
set -eu
cd "$(dirname "$0")/../distributed-pathsim_amd/csrc"
name=$1; shift
mkdir -p ../../ab
src=dps_cct1.hip
if [ -n "${SRCFILE:-}" ]; then
  src=build/_cct1_src_$name.hip
  cp "$SRCFILE" $src
elif [ -n "${SRC:-}" ]; then
  src=build/_cct1_src_$name.hip   # in csrc/build: its includes resolve to csrc/
  git show "$SRC:distributed-pathsim_amd/csrc/dps_cct1.hip" > $src
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -I.. -Wall -Wno-unused-function \
  -Wno-pass-failed -munsafe-fp-atomics "$@" -c $src -o /tmp/cct1_$name.o
objs=$(ls build/*.o | grep -v dps_cct1)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/libdpathsim_$name.so /tmp/cct1_$name.o $objs \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built ab/libdpathsim_$name.so
