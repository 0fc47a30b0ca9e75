#!/bin/bash
# Instruction-cache counters over the wk timing harness (one --pmc pass per binary).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/pmc_wk_ic}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for b in ${BINS:-wk_ablate_0 wk_ablate_127}; do
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
    -d "$O/$b" -o run --output-format csv -- ./tools/native/$b > "$O/$b.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$O" conv3_wk_kernel
