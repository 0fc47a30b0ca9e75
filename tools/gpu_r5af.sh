#!/bin/bash
# round 5: the full GPU suite on the paired split schedule
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5af; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s -k "not slow_nothing" > $O/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "flips|worst|passed|failed|Error" $O/gpu_suite.log | tail -14; exit $rc
