# k_p4r (NLS_P4=1) on the GPU: parity tests, per-pass probe of the ring build (lib) and the
# shifting-queue build (lib_vshift), the headline bench with and without the four-vector pass
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pass4.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/suite_p4.txt 2>&1 || { tail -30 $O/suite_p4.txt; exit 1; }
tail -3 $O/suite_p4.txt
for v in lib lib_vshift; do
  echo "== $v" >> $O/p4r_probe.txt
  NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so NLS_P4=1 timeout -k 10 300 python -u tools/p2_probe.py 512 16 4 >> $O/p4r_probe.txt 2>&1 || { tail -20 $O/p4r_probe.txt; exit 1; }
done
cat $O/p4r_probe.txt
NLS_P4=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_p4.json 2> $O/bench_p4.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_p2.json 2> $O/bench_p2.err || exit 1
python -c "import json;[print(f, json.load(open('$O/'+f))['ms_per_step']) for f in ('bench_p4.json','bench_p2.json')]"
