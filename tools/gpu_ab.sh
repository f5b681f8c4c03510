# A/B of a lib_v variant by per-pass timing at 512^3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/var_base$r.log 2>&1 || exit 1
  NLS_AMD_LIB=$GRAFT_REPO_ROOT/nonlinear-solvers_amd/lib_v/libnls_amd.so timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/var_var$r.log 2>&1 || exit 1
done
grep -H "J= 2\|J= 4\|per step" gpurun_out/var_*.log
