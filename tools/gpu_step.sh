# ad-hoc GPU step (edited per experiment): rANS encode timings + rANS/codec parity + bench
set -o pipefail
mkdir -p gpurun_out
cd tools/native && timeout -k 10 60 ./rans_bench_v1 6144 > ../../gpurun_out/rb_v1.log 2>&1 && timeout -k 10 60 ./rans_bench_0 6144 > ../../gpurun_out/rb_new.log 2>&1 && cd ../.. && cat gpurun_out/rb_v1.log gpurun_out/rb_new.log && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rans.py tests/test_gpu_codec.py > gpurun_out/t_rans.log 2>&1; rc=$?; tail -3 gpurun_out/t_rans.log; [ $rc -eq 0 ] && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_enc.log 2>&1 && tail -1 gpurun_out/bench_enc.log | cut -c1-600
