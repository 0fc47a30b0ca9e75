#!/bin/bash
# round 5: where the 8x8 dx3 launch spends its time (block timeline build), the 32x32 / 16x16
# launches against round 4's kernel on the same box, and a kernel trace of the 8x8 layers.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5d
export PYTHONDONTWRITEBYTECODE=1
for c in 1 6 11; do
  IDF_LIB_PATH=tools/ab_lib/tl/libidfcodec.so KB_LAYERS=$c timeout -k 10 120 python -u tools/dx3_timeline.py \
    > gpurun_out/r5d/tl_l2_$c.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/r5d/tl_l2_$c.log
done
KB_ONLY=dx3,dx3r4 KB_LEVELS=0,1 KB_LAYERS=0,3,6,9,11 KB_REPS=20 timeout -k 10 300 python -u tools/kbench.py \
  > gpurun_out/r5d/kbench_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5d/kbench_ab.log
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"
KB_ONLY=wx3,dx3 KB_LEVELS=2 KB_LAYERS=0,2,4,6,8,10,11 KB_REPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d gpurun_out/r5d/prof -o run --output-format csv -- python3 -u tools/kbench.py > gpurun_out/r5d/prof.log 2>&1 || exit 1
f=$(ls gpurun_out/r5d/prof/*kernel_trace.csv gpurun_out/r5d/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
cp "$f" gpurun_out/r5d/kernel_trace.csv; rm -rf gpurun_out/r5d/prof
echo done
