#!/bin/bash
# Persistent NF<=2 wx3 blocks: parity tests, then same-box A/B of configs 4/5 (IDF_WX3_PERSIST
# 0/1 on the same library) and of the headline against the baseline library (tools/ab_lib).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/persist_ab
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wx3.py \
  tests/test_gpu_wino.py tests/test_gpu_residual.py tests/test_gpu_production_parity.py -k "not config3_full" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
res() {
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python3 tools/bench_residual.py --config $cfg --steps 3 > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['encode_ms'], d['decode_ms'], d['roofline']['frac'], d['round_trip_exact'])"
}
for rep in 1 2; do
  res c5_off_$rep resflow-patches-vqvae IDF_WX3_PERSIST=0 || exit 1
  res c5_on_$rep resflow-patches-vqvae IDF_WX3_PERSIST=1 || exit 1
  res c4_off_$rep resflows_smallpatch_split IDF_WX3_PERSIST=0 || exit 1
  res c4_on_$rep resflows_smallpatch_split IDF_WX3_PERSIST=1 || exit 1
done
head() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-residual --no-cpu-baseline > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/$name.log') if l.startswith('{')][-1]; print('$name', d['value'], d['encode_ms'], d['decode_ms'], d['roofline']['frac'])"
}
for rep in 1 2; do
  head head_base_$rep IDF_LIB_PATH=$PWD/tools/ab_lib/libidfcodec_base.so || exit 1
  head head_new_$rep || exit 1
done
