"""The CPU-baseline pool of bench.py: spawned before the GPU is touched,
processes x threads over the usable CPUs, each on its own images; one pass round-trips
exactly with the oracle and reports the split, the affinity / quota and the effective CPUs."""
import os
import sys

from conftest import REPO


def test_cpu_pool_pass_is_exact():
    sys.path.insert(0, REPO)
    import bench
    pool = bench.CpuPool(2, chunk=2, split="2x1")
    try:
        r = bench.cpu_baseline_pool(pool, runs=1)
    finally:
        pool.close()
    assert r["value"] and r["value"] > 0, r
    assert r["cores"] == 2 and r["split"] == "2 processes x 1 threads"
    assert r["affinity_cpus"] == len(os.sched_getaffinity(0))
    assert "exact=True" in r["sample"] and 0 < r["effective_cpus"] <= 2.5


def test_cpu_pool_default_covers_usable_cpus(monkeypatch):
    """Default split: one single-threaded process per usable CPU -- every affine CPU, or the
    cgroup's CPU quota when that is smaller (a GPU box: 16 CPUs of time over 256)."""
    sys.path.insert(0, REPO)
    import bench
    aff, quota, usable = bench.usable_cpus()
    assert aff == sorted(os.sched_getaffinity(0))
    assert usable == (len(aff) if quota is None else max(1, min(len(aff), int(quota + 1e-6))))
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: 16.0)
    assert bench.usable_cpus()[2] == min(16, len(aff))
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: None)
    assert bench.usable_cpus()[2] == len(aff)
