#!/bin/bash
# round 5: per-layer time of dx3 vs wx3 at the 8x8 level (B=256 encode, B=128 decode lane) and
# the 32x32 / 16x16 levels (regression check), then a short bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
KB_ONLY=wx3,dx3 KB_LEVELS=2 KB_LAYERS=0,2,4,6,8,10,11 timeout -k 10 200 python -u tools/kbench.py \
  > gpurun_out/r5b_kbench_l2.log 2>&1
rc=$?; echo "kbench L2 rc=$rc"; cat gpurun_out/r5b_kbench_l2.log
[ $rc -ne 0 ] && exit $rc
KB_B=128 KB_ONLY=wx3,dx3 KB_LEVELS=2 KB_LAYERS=0,4,8,11 timeout -k 10 200 python -u tools/kbench.py \
  > gpurun_out/r5b_kbench_l2_b128.log 2>&1
rc=$?; echo "kbench L2 B128 rc=$rc"; cat gpurun_out/r5b_kbench_l2_b128.log
[ $rc -ne 0 ] && exit $rc
KB_ONLY=dx3 KB_LEVELS=0,1 KB_LAYERS=0,6,11 timeout -k 10 200 python -u tools/kbench.py \
  > gpurun_out/r5b_kbench_l01.log 2>&1
rc=$?; echo "kbench L01 rc=$rc"; cat gpurun_out/r5b_kbench_l01.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-residual --cpu-baseline-images-per-proc 2 \
  --cpu-baseline-runs 1 > gpurun_out/r5b_bench.json 2> gpurun_out/r5b_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r5b_bench.err; cut -c1-1500 gpurun_out/r5b_bench.json
exit $rc
