#!/bin/bash
# Upper bound of the epilogue's second barrier per n-fragment (timing-only ablation 2048,
# same box, alternating) and the instruction-cache counters of the wx3 kernel.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/epi
for r in 1 2; do
  for v in 0 2048; do
    echo "== wino_ablate_$v"; timeout -k 10 120 ./tools/native/wino_ablate_$v x3 || exit $?
  done
done > gpurun_out/epi/ab.txt 2>&1
cat gpurun_out/epi/ab.txt
bash ./tools/pmc_icache.sh
python tools/pmc_summary.py gpurun_out/pmc_ic/run > gpurun_out/epi/icache.txt 2>&1
cat gpurun_out/epi/icache.txt | head -40
