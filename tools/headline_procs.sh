#!/bin/bash
# N fresh processes of the driver's headline command (bench.py --gpus 1 --steps 20 --warmup 5,
# without the CPU baseline), one line each: ms/step, value, the placement kept
#   bash tools/headline_procs.sh TAG N
set -o pipefail
TAG=$1
N=${2:-4}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/proc$i.json" 2> "$OUT/proc$i.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['placement']; \
print(f\"proc{sys.argv[2]} ms/step {d['ms_per_step']:.3f} value {d['value']:.1f} tail {d['roofline']['avg_launch_ms']:.3f} kept {p['chosen']} of {p['candidates']} probe/step {min(p['probe_ms'])/3:.3f}\")" \
    "$OUT/proc$i.json" "$i" | tee -a "$OUT/headline_procs.txt"
done
