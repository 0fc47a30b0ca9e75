#!/bin/bash
# LDS bank-conflict attribution of the split-f16 Winograd conv: the same three SQ counters on
# wino_ablate builds that drop one LDS user each (0: none, 2: halo reads, 1024: epilogue
# staging reads, 2048: the epilogue's second barrier).  One pass per build, own time limit.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_lds_attr}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for a in ${ABL:-0 2 1024 2048}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d "$OUT/a$a" -o run \
    --output-format csv -- ./tools/native/wino_ablate_$a x3 > "$OUT/a$a.log" 2>&1
  rc=$?; echo "ablate $a rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp "$OUT/a$a"/run_counter_collection.csv "$OUT/a$a.csv"
  python3 tools/pmc_summary.py "$OUT/a$a" > "$OUT/a$a.summary" 2>&1 || true
done
