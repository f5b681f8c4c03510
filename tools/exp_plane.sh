set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q -m gpu > gpurun_out/pytest_plane.log 2>&1 || { tail -30 gpurun_out/pytest_plane.log; exit 1; }
for v in base m0 m3 base; do
  if [ $v = base ]; then lib=nonlinear-solvers_amd/lib/libnls_amd.so; else lib=nonlinear-solvers_amd/build_$v/libnls_amd.so; fi
  NLS_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/plane_$v.json 2>&1
  NLS_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 --warmup 2 --workload nlse2d_4096 >> gpurun_out/plane_$v.json 2>&1
done
