#!/bin/bash
# VQ argmin (tests, timing, configs 4/5) + the 8x8 staging-slot swap (wino tests, SQ counters).
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
bash tools/gpu_vq.sh || exit 1
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wino.py \
  tests/test_gpu_production_parity.py -k "wino or wx3 or x3 or config45" > $O/wino_tests.log 2>&1 || { tail -30 $O/wino_tests.log; exit 1; }
tail -2 $O/wino_tests.log
OUT=gpurun_out/pmc_x3_swap bash tools/pmc_x3.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_x3_swap > $O/pmc_x3_summary.txt 2>&1 || true
grep -A20 "false, 8>" $O/pmc_x3_summary.txt | grep -E "LDS_BANK|ACTIVE_INST_LDS" 
