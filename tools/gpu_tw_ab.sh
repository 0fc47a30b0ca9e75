#!/bin/bash
# L0 output tile 32x8 (default) vs 16x16 (IDF_WINO_TW32=16): kbench L0 + bench A/B + parity.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/tw
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for t in 32 16; do
  echo "== twmax $t"; IDF_WINO_TW32=$t KB_ONLY=wx3 KB_LEVELS=0 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
done > $O/kbench.log 2>&1
cat $O/kbench.log
IDF_WINO_TW32=16 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wx3.py tests/test_gpu_production_parity.py tests/test_gpu_flow.py tests/test_gpu_codec.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for t in 32 16; do
    IDF_WINO_TW32=$t timeout -k 10 180 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b_${t}_$r.json || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${t}_$r.json')); print('twmax $t', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'frac', d['roofline']['frac'])"
  done
done | tee $O/summary.txt
