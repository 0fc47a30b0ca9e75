# ad-hoc GPU step (edited per experiment): lanes stagger variants
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python tools/lanes_probe.py > gpurun_out/probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/probe.log | tail -12; exit $rc
