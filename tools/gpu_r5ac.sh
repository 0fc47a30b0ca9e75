#!/bin/bash
# round 5: CU occupancy of the pipelined bench (kernel trace), and of the serial one
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ac; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for p in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr$p -o run --output-format csv -- python3 -u bench.py --steps 6 --warmup 2 --pipeline $p --no-residual --no-cpu-baseline > $O/bench$p.log 2>&1 || exit $?
  f=$(ls $O/tr$p/*kernel_trace.csv $O/tr$p/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/analysis/cu_util.py "$f" 3 > $O/cu_util_pipeline$p.txt || exit 1
  rm -rf $O/tr$p
  echo "== pipeline $p"; cat $O/cu_util_pipeline$p.txt
done
