#!/bin/bash
# Run "$@" (a GPU step); exit 0 on success or plain test failures (rc 1),
# otherwise propagate -- so that a chain  run_checked.sh A && B  stops after a
# fault, abort, segfault or timeout of A but not after an ordinary failed test.
"$@"
rc=$?
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then exit 0; fi
echo "[run_checked] '$*' exited $rc; stopping" >&2
exit $rc
