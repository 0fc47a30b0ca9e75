#!/bin/bash
# Same-box A/B of the wx3 kernel: wino_base_0 (the committed source, tools/native/ab/) against
# wino_ablate_0 (the working source), alternating.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wab
for r in 1 2 3; do
  for v in base ablate; do
    echo "== wino_${v}_0"; timeout -k 10 120 ./tools/native/wino_${v}_0 x3 || exit $?
  done
done > gpurun_out/wab/ab.txt 2>&1
cat gpurun_out/wab/ab.txt
