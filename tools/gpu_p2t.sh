cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pass2.py tests/test_gpu_multirank.py tests/test_gpu_stiff.py -k "pass2 or multirank" > gpurun_out/t_p2.log 2>&1 || { tail -30 gpurun_out/t_p2.log; exit 1; }
tail -1 gpurun_out/t_p2.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['step_roofline']['gpu_kernel_ms_per_step'])"
