#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first crash / timeout (rc not in {0,1}); test assertion failures continue.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name (timeout $to)"; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STAGES=${STAGES:-"tests smoke bench prof"}
for s in $STAGES; do
  case $s in
    tests) step gpu_tests 900 python -m pytest tests -m gpu -q -rf --durations=15 ;;
    fasttests) step gpu_tests 900 python -m pytest tests -m "gpu and not slow" -q -rf --durations=15 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    kbench) step kbench 300 python tools/kbench.py ;;
    bench) step bench 600 python bench.py ;;
    bench_nofold) IDF_FOLD=0 step bench_nofold 600 python bench.py --no-cpu-baseline ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 ;;
  esac
done
echo "=== done"
