#!/bin/bash
# Round 4: same-box bench A/B of the default conv mode (dx3 at the 32x32/16x16 levels) against
# wx3 everywhere (IDF_DX3=0), then the whole GPU suite + smoke.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/r4b}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  for m in 1 0; do
    IDF_DX3=$m timeout -k 10 180 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b_dx3${m}_$r.json || exit $?
    python3 -c "import json; d=json.load(open('$O/b_dx3${m}_$r.json')); print('dx3=$m', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'frac', d['roofline']['frac'], 'launch_ms', d['roofline'].get('avg_launch_ms'))"
  done
done | tee $O/dx3_ab.txt
O=$O bash tools/gpu_r3_final_a.sh || exit $?
