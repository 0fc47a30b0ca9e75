#!/bin/bash
# round 5: which HIP calls launch the bench's copyBuffer kernels (kernel + HIP API trace)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5aj; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/tr -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 --no-residual --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
python3 tools/copy_trace.py $O/tr > $O/copies.txt 2>&1; rc=$?
rm -rf $O/tr
cat $O/copies.txt; exit $rc
