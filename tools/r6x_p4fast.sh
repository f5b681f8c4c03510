# k_p4r interior-plane fast body: parity tests on the default build, per-pass probe of lib
# (fast) against lib_vnofast (every step checked), two interleaved rounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pass4.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/suite_p4.txt 2>&1 || { tail -30 $O/suite_p4.txt; exit 1; }
tail -2 $O/suite_p4.txt
for rep in 1 2; do for v in lib lib_vnofast; do
  echo "== $v rep$rep" >> $O/p4fast_probe.txt
  NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so timeout -k 10 300 python -u tools/p2_probe.py 512 16 4 >> $O/p4fast_probe.txt 2>&1 || { tail -20 $O/p4fast_probe.txt; exit 1; }
done; done
grep -E "==|J= 0|update" $O/p4fast_probe.txt
