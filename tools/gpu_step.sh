# ad-hoc GPU step (edited per experiment): bench lanes 1 vs 2, more steps
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for v in "IDF_LANES=1" "IDF_LANES=2" "IDF_LANES=1" "IDF_LANES=2"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/b.log 2>&1 || exit $?
  echo "$v: $(tail -1 gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"])')"
done
