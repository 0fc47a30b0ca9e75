#!/bin/bash
# HBM traffic of the bench's dominant kernel: separate rocprofv3 --pmc passes for FETCH_SIZE
# and WRITE_SIZE (counters only, with --kernel-trace; never combined with trace domains) over
# one bench.py step.  bench.py reads the newest profiles/*/pmc_bench/{fetch,write}.csv.gz for
# roofline.traffic (FETCH_SIZE doubled: the gfx950 correction for 16-B-per-lane streaming
# reads, MI355X_MICROARCH.md "HBM").  Copy gpurun_out/pmc_bench to profiles/<round>/ after.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_bench
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc_bench/$name -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-residual \
    > gpurun_out/pmc_bench/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  # only what bench.pmc_traffic reads (dispatch, kernel, value), gzip-compressed
  python3 - gpurun_out/pmc_bench/$name/run_counter_collection.csv gpurun_out/pmc_bench/$name.csv.gz <<'PY' || exit 1
import csv, gzip, sys
rows = csv.DictReader(open(sys.argv[1]))
with gzip.open(sys.argv[2], "wt", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Value"])
    for r in rows:
        w.writerow([r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Value"]])
PY
  rm -rf gpurun_out/pmc_bench/$name
}
run fetch FETCH_SIZE
run write WRITE_SIZE
# the kernel sources these counters describe: bench.py reports the traffic only while the
# built sources hash the same (bench.conv_source_hash)
python3 -c "import bench; print(bench.conv_source_hash())" > gpurun_out/pmc_bench/source_hash.txt
echo done
