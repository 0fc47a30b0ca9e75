#!/bin/bash
# wk conv: ablation timings (tools/native/wk_ablate_N) next to wx3 (wino_ablate_0 x3), then SQ
# counters of the full kernel (two rocprofv3 --pmc passes, each under its own limit).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/wk_abl}
mkdir -p "$O"
for a in ${ABL:-0 1 2 4 8 16 32 59 63}; do
  timeout -k 10 60 ./tools/native/wk_ablate_$a >> "$O/ablate.log" 2>&1 || exit $?
done
timeout -k 10 60 ./tools/native/wino_ablate_0 x3 >> "$O/ablate.log" 2>&1 || exit $?
cat "$O/ablate.log"
[ "${PMC:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$O/$name" -o run --output-format csv -- ./tools/native/wk_ablate_0 \
    > "$O/$name.log" 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp "$O/$name"/run_counter_collection.csv "$O/$name.csv"
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA
pass sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC
python3 tools/pmc_summary.py "$O" conv3_wk_kernel > "$O/summary.txt"
cat "$O/summary.txt"
