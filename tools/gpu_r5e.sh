#!/bin/bash
# round 5: configs 4/5 blocks on dx3 (teacher-forced), the 8x8 timeline after the one-round-trip
# reduction, the headline bench and the residual configs.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5e; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_production_parity.py -x -v --timeout 300 \
  --timeout-method thread -k "config45 or (teacher_forced and 2-dx3)" -s > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "worst|passed|failed|Error" $O/parity.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -v --timeout 250 --timeout-method thread \
  -k "forward_vs or coupling_flips" -s > $O/flips.log 2>&1
rc=$?; echo "flips rc=$rc"; grep -E "flips|passed|failed|Error" $O/flips.log | tail -6
timeout -k 10 300 python -u tools/flip_probe.py > $O/flip_probe.log 2>&1; echo "probe rc=$?"; grep -v amdgpu.ids $O/flip_probe.log
IDF_LIB_PATH=tools/ab_lib/tl/libidfcodec.so KB_LAYERS=11 timeout -k 10 120 python -u tools/dx3_timeline.py \
  > $O/tl_l2_11.log 2>&1 || exit 1
grep -v amdgpu.ids $O/tl_l2_11.log
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['serial'], d['round_trip_exact_steps'], d['roofline']['frac'])"
for c in resflow-cond-imagenet64 resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 300 python -u tools/bench_residual.py --config $c --steps 3 > $O/res_$c.json 2> $O/res_$c.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_$c.json')); print('$c', d['value'], d['encode_mpx_s'], d['decode_mpx_s'], d['round_trip_exact'], d['roofline']['frac'], d['roofline']['conv_mode'])"
done
