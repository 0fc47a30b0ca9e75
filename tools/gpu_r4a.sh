#!/bin/bash
# Round 4, first GPU pass: dx3 parity + per-layer timing (wx3 vs dx3), then the rANS suite and
# the decode A/B (in-block table producers vs the HEAD prep-kernel decode).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_dx3.py > gpurun_out/dx3_tests.log 2>&1
rc=$?; echo "dx3 tests rc=$rc"; tail -15 gpurun_out/dx3_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
KB_ONLY=wx3,dx3 KB_LEVELS=0,1 KB_LAYERS=0,3,6,9,11 timeout -k 10 300 python -u tools/kbench.py \
  > gpurun_out/dx3_kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/dx3_kbench.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $T tests/test_gpu_rans.py > gpurun_out/rans_tests.log 2>&1
rc=$?; echo "rans tests rc=$rc"; tail -12 gpurun_out/rans_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for b in rans_base_0 rans_bench_0; do
    for n in 3072 6144; do
      echo -n "$b $n: "; timeout -k 10 60 ./tools/native/$b $n || exit $?
    done
  done
done 2>&1 | tee gpurun_out/rans_ab.log
