#!/bin/bash
set -e
O=gpurun_out/misc; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_all.log 2>&1
