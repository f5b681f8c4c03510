set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "trajectory or expm" > gpurun_out/pytest_pipe.log 2>&1
for v in base nopipe piperb3 base; do
  if [ $v = base ]; then lib=nonlinear-solvers_amd/lib/libnls_amd.so; else lib=nonlinear-solvers_amd/build_$v/libnls_amd.so; fi
  NLS_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/pipe_$v.json 2>&1
done
