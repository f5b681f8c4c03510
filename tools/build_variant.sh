#!/bin/bash
# Build a variant of libnls_amd.so with extra -D flags on the k_p2d translation units
# (nls_pass2a.hip: the G2 operator; nls_kernels.hip: the isotropic passes), linked with
# the default build's other objects, into nonlinear-solvers_amd/lib_<name>/.
# usage: tools/build_variant.sh NAME "-DFOO=1 -DBAR=2" [a|k|ak]
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2; which=${3:-a}
B=nonlinear-solvers_amd/build; V=nonlinear-solvers_amd/build_$name; L=nonlinear-solvers_amd/lib_$name
mkdir -p $V $L
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Inonlinear-solvers_amd/csrc -Wall"
objs=""
for o in nls_kernels nls_pass2g nls_pass2a nls_api nls_stencil_iso2 nls_stencil_iso3 nls_stencil_ani2 nls_stencil_ani3; do
  objs="$objs $B/$o.o"
done
if [[ $which == *a* ]]; then
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -c nonlinear-solvers_amd/csrc/nls_pass2a.hip -o $V/nls_pass2a.o
  objs=${objs/$B\/nls_pass2a.o/$V/nls_pass2a.o}
fi
if [[ $which == *k* ]]; then
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -c nonlinear-solvers_amd/csrc/nls_kernels.hip -o $V/nls_kernels.o
  objs=${objs/$B\/nls_kernels.o/$V/nls_kernels.o}
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 $objs -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o $L/libnls_amd.so
echo built $L/libnls_amd.so
