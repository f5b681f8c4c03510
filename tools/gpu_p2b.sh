cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pass2.py > gpurun_out/t_p2.log 2>&1 || { tail -30 gpurun_out/t_p2.log; exit 1; }
tail -2 gpurun_out/t_p2.log
for rep in 1 2; do for v in "NLS_P2_KZ=256" "NLS_P2_KZ=128"; do
  echo "== $v" ; env NLS_PASS2=1 $v timeout -k 10 120 python tools/p2_probe.py 512 16 4 || exit 1
done; done > gpurun_out/p2probe.log 2>&1
cat gpurun_out/p2probe.log
bash tools/gpu_p2pmc.sh
