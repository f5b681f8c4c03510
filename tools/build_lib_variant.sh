#!/bin/bash
# Build the whole library with extra -D flags into nonlinear-solvers_amd/lib_<name>/
# (objects in build_<name>/), for same-box A/B runs (tools/gpu.sh ab).
#   bash tools/build_lib_variant.sh NAME "-DFOO=0"
set -e
cd "$(dirname "$0")/.."
name=$1
flags=$2
make -j8 BUILD=nonlinear-solvers_amd/build_$name LIBDIR=nonlinear-solvers_amd/lib_$name \
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Inonlinear-solvers_amd/csrc -Wall $flags" \
  nonlinear-solvers_amd/lib_$name/libnls_amd.so
