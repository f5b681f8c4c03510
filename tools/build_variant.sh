#!/bin/bash
# Build a variant of libnls_amd.so with extra compile flags into nonlinear-solvers_amd/lib_v/.
# usage: bash tools/build_variant.sh "-DNLS_QA_RB1_FROM=99"
set -e
make -j8 -s BUILD=nonlinear-solvers_amd/build_${2:-v} LIBDIR=nonlinear-solvers_amd/lib_${2:-v} \
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Inonlinear-solvers_amd/csrc -Wall $1" \
  nonlinear-solvers_amd/lib_${2:-v}/libnls_amd.so
