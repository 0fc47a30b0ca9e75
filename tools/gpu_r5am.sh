#!/bin/bash
# round 5: SQ counters of the L0 dx3 kernel (kbench, B=128, c=496): where the slab period goes
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5am; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
export KB_B=128 KB_ONLY=dx3 KB_LEVELS=0 KB_LAYERS=11 KB_REPS=5
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run --output-format csv -- python3 tools/kbench.py > $O/p1.log 2>&1 || exit $?
f=$(ls $O/p1/*counter_collection.csv $O/p1/*/*counter_collection.csv 2>/dev/null | head -1); cp "$f" $O/sq1.csv
rm -rf $O/p1; python3 tools/analysis/sq_sum.py $O/sq1.csv
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 tools/kbench.py > $O/p2.log 2>&1 || exit $?
f=$(ls $O/p2/*counter_collection.csv $O/p2/*/*counter_collection.csv 2>/dev/null | head -1); cp "$f" $O/sq2.csv
rm -rf $O/p2
python3 tools/analysis/sq_sum.py $O/sq2.csv
