#!/bin/bash
# Submit one gpurun call, resubmitting it only while the pool reports that nothing ran
# (no free box / box lost before the command started: status "transient", nothing
# charged).  A command that ran -- whatever its exit status -- is never resubmitted.
#   bash tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1
TMO=$2
CMD=$3
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  st=$(python3 -c "import json; d=json.load(open('gpurun_out/.last_call.json')); print(d.get('status'), d.get('run_s'))" 2>/dev/null)
  echo "[when_free] attempt $attempt rc=$rc status=$st" >> "$LOG.attempts"
  case "$st" in
    "transient 0.0"|"transient None") sleep 150 ;;
    *) exit $rc ;;
  esac
done
exit 3
