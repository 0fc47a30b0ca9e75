#!/bin/bash
# wp (two waves per SIMD): parity tests through idf_conv3x3_wq with IDF_WQ_VARIANT=p, then a
# same-box layer A/B against wq and wx3.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/wp
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
IDF_WQ_VARIANT=p timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wq.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  echo "== wp"; IDF_WQ=1 IDF_WQ_VARIANT=p KB_ONLY=wx3 KB_LEVELS=0,1 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
  echo "== wq"; IDF_WQ=1 KB_ONLY=wx3 KB_LEVELS=0,1 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
  echo "== wx3"; IDF_WQ=0 KB_ONLY=wx3 KB_LEVELS=0,1 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
done > $O/ab.log 2>&1
grep -E "==|sampled|c= 496|c= 504|c=  12" $O/ab.log
