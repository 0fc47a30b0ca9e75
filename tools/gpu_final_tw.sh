#!/bin/bash
# Final check with 16x16 tiles at the 32x32 level: the whole GPU suite + smoke, a same-box
# bench A/B against the 32x8 strips (IDF_WINO_TW32=32), then the default bench line + rocprof.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3s2d
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
O=$O bash tools/gpu_r3_final_a.sh || exit $?
for r in 1 2 3; do
  for t in 16 32; do
    IDF_WINO_TW32=$t timeout -k 10 180 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b_${t}_$r.json || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${t}_$r.json')); print('tw32 $t', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'frac', d['roofline']['frac'])"
  done
done | tee $O/tw_ab.txt
O=$O bash tools/gpu_r3_final_b.sh || exit $?
