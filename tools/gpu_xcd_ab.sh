#!/bin/bash
# XCD-aware block order of the Winograd kernels: parity subset, then a same-box A/B of the
# bench (tree library = remap on, tools/xcd_lib/off = the dispatcher's order) and kbench.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/xcd
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wx3.py tests/test_gpu_wino.py tests/test_gpu_production_parity.py tests/test_gpu_flow.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
T=finalproject-losslessimagecompression_amd/idfcodec/libidfcodec.so
for r in 1 2 3; do
  for v in on off; do
    if [ $v = on ]; then L=$T; else L=tools/xcd_lib/off/libidfcodec.so; fi
    IDF_LIB_PATH=$L timeout -k 10 180 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b_${v}_$r.json || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('xcd $v', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'frac', d['roofline']['frac'], 'launch', d['roofline']['avg_launch_ms'])"
  done
done | tee $O/summary.txt
