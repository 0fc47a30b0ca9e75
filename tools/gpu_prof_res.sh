#!/bin/bash
# Kernel stats of the residual configs 4 and 5 (tools/bench_residual.py, 2 steps each).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/prof_res
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$cfg -o run --output-format csv -- \
    python3 tools/bench_residual.py --config $cfg --steps 2 > $O/$cfg.log 2>&1 || exit 1
  f=$(ls $O/$cfg/*kernel_stats.csv $O/$cfg/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/$cfg.csv
  head -12 $O/$cfg.csv | cut -c1-140
done
