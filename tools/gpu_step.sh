# ad-hoc GPU step (edited per experiment): overlapped level encode: parity + bench A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lanes.py tests/test_gpu_codec.py tests/test_gpu_residual.py > gpurun_out/t_enc.log 2>&1; rc=$?; tail -2 gpurun_out/t_enc.log; [ $rc -eq 0 ] || exit $rc
for v in "IDF_ENC_OVERLAP=0" "IDF_ENC_OVERLAP=1" "IDF_ENC_OVERLAP=0" "IDF_ENC_OVERLAP=1"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/b.log 2>&1 || exit $?
  echo "$v: $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"])')"
done
