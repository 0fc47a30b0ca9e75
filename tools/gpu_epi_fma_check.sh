#!/bin/bash
# Epilogue change (fma row select, ds_write2_b32 staging writes): same-box kernel A/B, the GPU
# suite and the bench with the rebuilt library, then the one-GPU N=2 rehearsal.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/epifma
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
bash tools/gpu_wino_ab.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])'
bash tools/gpu_rehearse2.sh > $O/rehearse.txt 2>&1; rc=$?
tail -c 600 $O/rehearse.txt; exit $rc
