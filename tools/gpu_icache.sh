#!/bin/bash
# Instruction-cache counters and s_memtime stamps of the wx3 kernel (timing harness).
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ic
timeout -k 10 120 ./tools/native/wino_stamps_0 x3 > gpurun_out/ic/stamps.txt 2>&1 || exit $?
cat gpurun_out/ic/stamps.txt
./tools/pmc_icache.sh
cp gpurun_out/pmc_ic/log gpurun_out/ic/pmc.log
python tools/pmc_summary.py gpurun_out/pmc_ic/run > gpurun_out/ic/summary.txt 2>&1
head -60 gpurun_out/ic/summary.txt
