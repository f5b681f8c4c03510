# the full GPU suite + smoke on the default build, then the x-halo fast-body A/B (lib_vhfast)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/lib_vhfast/libnls_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pass4.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/suite_p4_vhfast.txt 2>&1 || { tail -30 $O/suite_p4_vhfast.txt; exit 1; }
tail -1 $O/suite_p4_vhfast.txt
for rep in 1 2; do for v in lib_vhfast lib; do
  echo "== $v rep$rep" >> $O/p4hfast_probe.txt
  NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so timeout -k 10 300 python -u tools/p2_probe.py 512 16 4 >> $O/p4hfast_probe.txt 2>&1 || { tail -20 $O/p4hfast_probe.txt; exit 1; }
done; done
grep -E "==|J= 0|update" $O/p4hfast_probe.txt
timeout -k 10 300 python bench.py > $O/bench_nlse3d_512.json 2> $O/bench.err || exit 1
cat $O/bench_nlse3d_512.json
