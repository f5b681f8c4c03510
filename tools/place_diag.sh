#!/bin/bash
# Placement diagnosis (DESIGN.md section 4 "Placement"): counters per dispatch of the
# placement probe's candidates in ONE process.  Each pass = one rocprofv3 run with one
# counter group + --kernel-trace (no other trace domains), bench.py --steps 2; the probe
# (NLS_PLACE=6 by default) runs every candidate basis through the same 4 steps, so the
# per-dispatch records compare placements of the same code in one process
#   bash tools/place_diag.sh TAG GROUP1 [GROUP2 ...]   (a group: counters joined by '+')
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for grp in "$@"; do
  i=$((i + 1))
  ctrs=$(echo "$grp" | tr '+' ' ')
  echo "[place_diag] $(date +%T) pass $i: $ctrs"
  # shellcheck disable=SC2086
  NLS_PLACE_LOG=1 timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --steps 2 --warmup 0 --prof-steps 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || exit $?
  grep "placement" "$OUT/p$i.log"
done
