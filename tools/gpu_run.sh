#!/bin/bash
# The GPU-box steps of this repo, one parameterised script (run through gpurun):
#   tools/gpu_run.sh OUT STEP [STEP ...]      OUT: a directory under gpurun_out/
# Steps (each under its own time limit; the first failing step ends the run):
#   tests      pytest -m gpu (the whole GPU suite)           -> OUT/gpu_suite.log
#   smoke      __graft_entry__.smoke()                        -> OUT/smoke.log
#   bench      default bench.py (residual configs, CPU baseline) -> OUT/bench.json
#   headline   bench.py without residual configs / CPU baseline  -> OUT/headline.json
#   prof       rocprofv3 --kernel-trace --stats over the headline bench -> OUT/kernel_stats.csv
#   trace      rocprofv3 --kernel-trace over a 4-step headline bench    -> OUT/kernel_trace.csv
#   pmc        tools/pmc_bench.sh (FETCH_SIZE / WRITE_SIZE passes)      -> gpurun_out/pmc_bench
#   rehearse2  the N=2 bench path on one GPU (gloo, both ranks on cuda:0) -> OUT/rehearse2.log
#   repro      the fused-head LDS-ordering reproducer (tools/repro_lds)   -> OUT/repro.log
# BENCH_ARGS adds bench.py arguments to headline / prof / trace.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=$1; shift
mkdir -p "$O"
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
T="timeout -k 10"
for step in "$@"; do
  case $step in
    tests) $T 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
             > "$O/gpu_suite.log" 2>&1 || exit $? ; tail -n 1 "$O/gpu_suite.log" ;;
    smoke) $T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
             || exit $? ; tail -n 1 "$O/smoke.log" ;;
    bench) $T 700 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || exit $? ;;
    headline) $T 400 python -u bench.py --no-residual --no-cpu-baseline ${BENCH_ARGS:-} \
             > "$O/headline.json" 2> "$O/headline.err" || exit $? ;;
    prof) $T 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
            python3 -u bench.py --no-residual --no-cpu-baseline ${BENCH_ARGS:-} > "$O/prof.log" 2>&1 \
            || exit $?
          f=$(ls "$O"/prof/*kernel_stats.csv "$O"/prof/*/*kernel_stats.csv 2>/dev/null | head -1)
          cp "$f" "$O/kernel_stats.csv"; rm -rf "$O/prof" ;;
    trace) $T 400 rocprofv3 --kernel-trace -d "$O/tr" -o run --output-format csv -- \
             python3 -u bench.py --steps 4 --warmup 1 --no-residual --no-cpu-baseline ${BENCH_ARGS:-} \
             > "$O/trace_bench.log" 2>&1 || exit $?
           f=$(ls "$O"/tr/*kernel_trace.csv "$O"/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
           cp "$f" "$O/kernel_trace.csv"; rm -rf "$O/tr" ;;
    pmc) ./tools/pmc_bench.sh || exit $? ;;
    rehearse2) IDF_DIST_BACKEND=gloo IDF_SHARE_GPU=1 IDF_DIST_HOST_GROUP=separate $T 900 \
               python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
               > "$O/rehearse2.log" 2>&1 || exit $? ;;
    repro) $T 200 python -u tools/repro_lds/run_repro.py 20 > "$O/repro.log" 2>&1 || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
