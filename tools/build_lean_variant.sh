#!/bin/bash
# Build ab/libdpathsim_<name>.so: dps_cct1.hip compiled with extra flags ($2...)
# and linked with the other objects of the regular build (run `make` first).
set -eu
cd "$(dirname "$0")/../distributed-pathsim_amd/csrc"
name=$1; shift
mkdir -p ../../ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -Wall -Wno-unused-function \
  -Wno-pass-failed -munsafe-fp-atomics "$@" -c dps_cct1.hip -o /tmp/cct1_$name.o
objs=$(ls build/*.o | grep -v dps_cct1)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/libdpathsim_$name.so /tmp/cct1_$name.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built ab/libdpathsim_$name.so
