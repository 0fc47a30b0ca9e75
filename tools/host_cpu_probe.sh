#!/bin/bash
# What CPU share does a GPU box give one command?  (affinity, cgroup quota, memory cap)
set -u
echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset} MAX_JOBS=${MAX_JOBS:-unset}"
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/memory.max \
         /sys/fs/cgroup/pids.max /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us; do
  [ -r "$f" ] && echo "$f: $(cat $f)"
done
grep -m1 "model name" /proc/cpuinfo
free -g | head -2
# burn test: 64 busy processes for 3 s each, how much CPU time do they get?
python3 - <<'PY'
import multiprocessing as mp, time, os
def burn(_):
    t0 = time.process_time(); w0 = time.time()
    while time.time() - w0 < 3: pass
    return time.process_time() - t0
for n in (16, 64, 128):
    with mp.get_context("fork").Pool(n) as p:
        w = time.time(); cpu = sum(p.map(burn, range(n))); w = time.time() - w
    print(f"{n} burners: wall {w:.2f}s cpu {cpu:.1f}s -> effective CPUs {cpu / 3:.1f}", flush=True)
PY
