#!/bin/bash
# Same-box A/B of wq variants (tree library vs tools/wq_lib/<v>) and wx3, at the kbench layers.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/wq_ab
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wq.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in tree "$@"; do
    echo "== $v"
    if [ $v = tree ]; then L=finalproject-losslessimagecompression_amd/idfcodec/libidfcodec.so; else L=tools/wq_lib/$v/libidfcodec.so; fi
    IDF_LIB_PATH=$L IDF_WQ=1 KB_ONLY=wx3 KB_LEVELS=0,1 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
  done
  echo "== wx3"
  IDF_WQ=0 KB_ONLY=wx3 KB_LEVELS=0,1 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
done > $O/ab.log 2>&1
grep -E "==|sampled|c= 496|c= 504|c=  12" $O/ab.log
