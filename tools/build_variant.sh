#!/bin/bash
# Build ab/libdpathsim_<name>.so: a dps_cct.hip source ($SRC, default the
# working copy; e.g. SRC=HEAD takes the last commit's) compiled with extra
# flags ($2...), linked with the other objects of the regular build (run
# `make` first).
set -eu
cd "$(dirname "$0")/../distributed-pathsim_amd/csrc"
name=$1; shift
mkdir -p ../../ab
src=dps_cct.hip
if [ -n "${SRC:-}" ]; then
  src=/tmp/cct_src_$name.hip
  git show "$SRC:distributed-pathsim_amd/csrc/dps_cct.hip" > $src
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -Wall -Wno-unused-function \
  -munsafe-fp-atomics "$@" -c $src -o /tmp/cct_$name.o
objs=$(ls build/*.o | grep -v dps_cct | grep -v dps_topk)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/libdpathsim_$name.so /tmp/cct_$name.o $objs
echo built ab/libdpathsim_$name.so
