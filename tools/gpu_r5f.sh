#!/bin/bash
# round 5: configs 4 / 5 conv kernels, dx3 (default) vs wx3 (IDF_DX3=0), rocprofv3 kernel stats
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5f; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  for m in dx3 wx3; do
    if [ $m = wx3 ]; then export IDF_DX3=0; else unset IDF_DX3; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- \
      python3 -u tools/bench_residual.py --config $c --steps 2 > $O/${c}_$m.json 2> $O/${c}_$m.err || exit 1
    f=$(ls $O/p/*kernel_stats.csv $O/p/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/${c}_$m.csv; rm -rf $O/p
    tail -1 $O/${c}_$m.json | cut -c1-200
  done
done
