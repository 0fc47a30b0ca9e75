#!/bin/bash
# round 5: smoke and the whole GPU suite at HEAD (after the bench default change)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5final5; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $O/gpu_suite.log | tail -2; exit $rc
