#!/bin/bash
# Round-3 evidence, part A: the whole GPU suite and smoke() at the current tree.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/r3final}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
