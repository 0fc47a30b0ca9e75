#!/bin/bash
# round 5: the full GPU suite (timed, slowest tests listed) and configs 4/5 throughput
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5v; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=25 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -32 $O/suite.log; [ $rc -ne 0 ] && exit $rc
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 300 python -u tools/bench_residual.py --config $c > $O/res_$c.json 2> $O/res_$c.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_$c.json')); r=d.get('roofline', {}); print('$c', d.get('value'), r.get('frac'), r.get('conv_mode'))"
done
