#!/bin/bash
# Build abb/libdpathsim_<name>.so: the regular objects with one source file
# ($1 relative to csrc) recompiled with extra flags ($3...).
set -eu
cd "$(dirname "$0")/../distributed-pathsim_amd/csrc"
name=$1; src=$2; shift 2
mkdir -p ../../abb
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -I.. -Wall -Wno-unused-function \
  -Wno-pass-failed -munsafe-fp-atomics "$@" -c $src -o /tmp/var_$name.o
objs=$(ls build/*.o | grep -v "/${src}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abb/libdpathsim_$name.so /tmp/var_$name.o $objs \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built abb/libdpathsim_$name.so
