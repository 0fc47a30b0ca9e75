#!/bin/bash
# Round-4 closing evidence: the whole GPU suite + smoke, the default bench line and its
# rocprofv3 kernel stats (the conv sources are those of profiles/r04/pmc_bench).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/final4}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 1000 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
O=$O bash tools/gpu_r3_final_b.sh
