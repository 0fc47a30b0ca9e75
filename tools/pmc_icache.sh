#!/bin/bash
# Instruction-cache counters over the wx3 timing harness (one --pmc pass).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_ic
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
  -d gpurun_out/pmc_ic/run -o run --output-format csv -- ./tools/native/wino_ablate_0 x3 > gpurun_out/pmc_ic/log 2>&1
echo rc=$?
