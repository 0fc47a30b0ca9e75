#!/bin/bash
# Round-4 session-3 GPU step: the dx3-prefix tests, then configs 4/5 profiled (kernel stats).
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_production_parity.py -k "prefix or teacher_forced" > $O/prefix_tests.log 2>&1 || { tail -20 $O/prefix_tests.log; exit 1; }
tail -2 $O/prefix_tests.log
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 200 python3 -u tools/bench_residual.py --config $c --steps 5 > $O/b_$c.json 2>$O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  cat $O/b_$c.json | cut -c1-400
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python3 -u tools/bench_residual.py --config $c --steps 3 > $O/p_$c.log 2>&1 || { tail -5 $O/p_$c.log; exit 1; }
done
