#!/bin/bash
# Same-box A/B of two vector-epilogue variants (fma row select; ds_write2_b32 staging writes)
# against the committed kernel, alternating.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wab3
for r in 1 2 3; do
  for v in base_0 var_epifma var_epiw2; do
    echo "== wino_${v}"; timeout -k 10 120 ./tools/native/wino_${v} x3 || exit $?
  done
done > gpurun_out/wab3/ab.txt 2>&1
cat gpurun_out/wab3/ab.txt
