#!/bin/bash
# rocprofv3 kernel-trace summaries of the residual configs 4 and 5 (tools/bench_residual.py)
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/res_prof
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/res_prof/$c -o run --output-format csv -- \
    python3 -u tools/bench_residual.py --config $c --steps 2 --warmup 1 > gpurun_out/res_prof/$c.log 2>&1 || exit $?
  cp gpurun_out/res_prof/$c/run_kernel_stats.csv gpurun_out/res_prof/$c.kernel_stats.csv
  tail -1 gpurun_out/res_prof/$c.log | cut -c1-300
  head -12 gpurun_out/res_prof/$c.kernel_stats.csv | cut -c1-140
done
