#!/bin/bash
# Memory-side counters of the L0 c=496 conv layer, wx3 vs dx3 (tools/kbench.py): HBM bytes
# (FETCH_SIZE / WRITE_SIZE, separate passes), the available counter list, then TA/TD/TCP/TCC
# passes named in PASSES (each "name:CTR1,CTR2").
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/pmc_mem; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export KB_ONLY=${KB_ONLY:-wx3,dx3} KB_LEVELS=0 KB_LAYERS=${KB_LAYERS:-11} KB_REPS=3
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 tools/kbench.py > $OUT/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp $OUT/$name/run_counter_collection.csv $OUT/$name.csv
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for p in ${PASSES:-}; do pass ${p%%:*} $(echo ${p#*:} | tr , ' '); done
python3 tools/pmc_summary.py $OUT conv3 > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
