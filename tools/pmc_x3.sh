#!/bin/bash
# SQ counters of the split-f16 Winograd conv (conv3_wino_kernel<3,448,true,...>) on the
# imagenet64 layer shapes (tools/native/wino_ablate_0 x3: L0 c=496, L1 c=504, L2 c=520,
# c=16), one rocprofv3 --pmc pass per counter group (<= 8 SQ counters a pass), each under its
# own time limit.  OUT defaults to gpurun_out/pmc_x3; summarise with tools/pmc_summary.py.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_x3}
EXE=${EXE:-./tools/native/wino_ablate_0}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- "$EXE" x3 \
    > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp "$OUT/$name"/run_counter_collection.csv "$OUT/$name.csv"
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA
pass sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass fetch FETCH_SIZE
pass write WRITE_SIZE
$EXE x3 > "$OUT/timing.log" 2>&1
echo done
