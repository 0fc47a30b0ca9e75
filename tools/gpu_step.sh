# ad-hoc GPU step (edited per experiment): residual configs with decode lanes 1 vs 2
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/resid_lanes.log
for c in resflow-cond-imagenet64 resflows_smallpatch_split resflow-patches-vqvae; do
  for v in 1 2; do
    IDF_LANES=$v timeout -k 10 300 python tools/bench_residual.py --config $c --steps 3 > gpurun_out/r.log 2>&1 || { tail -5 gpurun_out/r.log; exit 1; }
    echo "$c lanes=$v $(tail -1 gpurun_out/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: d[k] for k in d if "ms" in k or "exact" in k})')" | tee -a gpurun_out/resid_lanes.log
  done
done
