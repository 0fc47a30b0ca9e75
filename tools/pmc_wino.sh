#!/bin/bash
# PMC passes (counters only, kernel-trace) over the Winograd conv kernel microbench:
# SQ stall breakdown, then FETCH_SIZE and WRITE_SIZE in separate passes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export KB_ONLY=${KB_ONLY:-wino} KB_LEVELS=${KB_LEVELS:-0,2} KB_LAYERS=${KB_LAYERS:-0,11} KB_REPS=${KB_REPS:-3}
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- python3 tools/kbench.py > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run fetch FETCH_SIZE
run write WRITE_SIZE
echo done
