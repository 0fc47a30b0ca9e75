#!/bin/bash
# round 5: branch-free DMA issue -- dx3 parity, L0/L1 layers against round 4's kernel (same box,
# alternating), L0 c=496 slab stamps, then the bench
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5i; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dx3.py -x -q --timeout 120 --timeout-method thread \
  > $O/dx3_tests.log 2>&1
rc=$?; echo "dx3 tests rc=$rc"; tail -3 $O/dx3_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  KB_ONLY=dx3,dx3r4 KB_LEVELS=0,1 KB_LAYERS=0,3,6,9,11 KB_REPS=20 timeout -k 10 300 python -u tools/kbench.py \
    > $O/kbench_ab_$rep.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/kbench_ab_$rep.log | tail -3
done
IDF_LIB_PATH=tools/ab_lib/stamps/libidfcodec.so timeout -k 10 120 python -u tools/dx3_stamps.py > $O/stamps.log 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['serial'], d['round_trip_exact_steps'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
