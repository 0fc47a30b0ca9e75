# ad-hoc GPU step (edited per experiment): rANS / codec / lanes parity + a 10-step bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rans.py tests/test_gpu_codec.py tests/test_gpu_lanes.py > gpurun_out/t_rans.log 2>&1; rc=$?; tail -2 gpurun_out/t_rans.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/b.log 2>&1; rc=$?; tail -1 gpurun_out/b.log | cut -c1-400; exit $rc
