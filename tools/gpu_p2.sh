# two-vector pass: parity tests, stiff parity, then 512^3 bench default vs NLS_PASS2=1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pass2.py > gpurun_out/t_p2.log 2>&1; rc=$?
tail -5 gpurun_out/t_p2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stiff.py -k "pass2" > gpurun_out/t_p2s.log 2>&1; rc=$?
tail -5 gpurun_out/t_p2s.log
[ $rc -eq 0 ] || exit $rc
NLS_PASS2=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_p2.json 2> gpurun_out/b_p2.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_def.json 2> gpurun_out/b_def.err || exit 1
python - <<'PY'
import json
for f in ("b_p2", "b_def"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["step_roofline"]["gpu_kernel_ms_per_step"])
PY
