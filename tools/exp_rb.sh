set -e
for v in base rb1 rb2 base; do
  if [ $v = base ]; then lib=nonlinear-solvers_amd/lib/libnls_amd.so; else lib=nonlinear-solvers_amd/build_$v/libnls_amd.so; fi
  NLS_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/rb_$v.json 2>&1
  NLS_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 --workload nlse2d_4096 >> gpurun_out/rb_$v.json 2>&1
done
