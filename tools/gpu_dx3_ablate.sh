#!/bin/bash
# dx3 ablations (tools/dx3_build_ablate.sh variants) at L0 c=496 / L1 c=504, then SQ counters
# of the base variant.  VARIANTS="0 7 8 ..." must have been built.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for n in ${VARIANTS:-0}; do
  echo "== ablate $n"
  IDF_LIB_PATH=$PWD/tools/ab_lib/dx3_$n/libidfcodec.so KB_ONLY=dx3 KB_LEVELS=0,1 \
    KB_LAYERS=${KB_LAYERS:-6,11} timeout -k 10 120 python -u tools/kbench.py 2>&1 | grep -v amdgpu.ids
  rc=$?; [ $rc -eq 0 ] || exit $rc
done
if [ "${PMC:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  OUT=gpurun_out/pmc_dx3; mkdir -p $OUT
  pass() {
    local name=$1; shift
    KB_ONLY=dx3 KB_LEVELS=0,1 KB_LAYERS=11 KB_REPS=3 timeout -s KILL 120 rocprofv3 --pmc "$@" \
      -d "$OUT/$name" -o run --output-format csv -- python3 tools/kbench.py > "$OUT/$name.log" 2>&1
    local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cp "$OUT/$name"/run_counter_collection.csv "$OUT/$name.csv"
  }
  pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA
  pass sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC
  pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
  python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt | head -60
fi
