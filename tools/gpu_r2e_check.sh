set -u -o pipefail
O=gpurun_out/r2e
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"], d["roofline"]["frac"])'
