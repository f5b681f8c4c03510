# Real (cell-pair) two-vector passes: SG / Gautschi parity, then the SG 8192^2 bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pass2.py tests/test_gpu_gautschi.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_sg.log 2>&1; rc=$?
tail -3 gpurun_out/t_sg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload sg2d_8192 --no-cpu-baseline --steps 6 > gpurun_out/bsg_p2.json 2>&1 || exit 1
NLS_PASS2=0 timeout -k 10 300 python bench.py --workload sg2d_8192 --no-cpu-baseline --steps 6 > gpurun_out/bsg_p1.json 2>&1 || exit 1
for f in gpurun_out/bsg_p2.json gpurun_out/bsg_p1.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',round(d['value'],1),round(d['ms_per_step'],3),d['roofline']['kernel'][:24],round(d['roofline']['avg_launch_ms'],3),round(d['roofline']['frac'],3),{k:round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"; done
