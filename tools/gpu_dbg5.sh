#!/bin/bash
set -u
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dx3.py tests/test_gpu_lanes.py -k "fused" > $O/t.log 2>&1; echo rc=$?; tail -2 $O/t.log
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 120 python -u tools/dbg_cfg4.py $c 2 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['serial'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
O=$O/prof ./tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
grep -E "head_init" $O/prof/kernel_stats.csv | cut -d, -f1-4
