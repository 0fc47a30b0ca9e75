#!/bin/bash
# Round 4: the production-parity and codec suites (dx3 default) + smoke.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/r4c}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_production_parity.py tests/test_gpu_codec.py tests/test_gpu_lanes.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
