"""Host CPU share for the CPU baselines and the OpenMP checkers.

`nproc` / os.cpu_count() report the whole machine on the GPU box (256), not
the cores this job may use. The share is the affinity mask, capped by the
cgroup CPU quota when one is set (cgroup v2 `cpu.max`, v1 `cfs_quota_us`).
"""
from __future__ import annotations

import math
import os


def _cgroup_quota_cpus():
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        if q > 0 and p > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def cpu_share() -> dict:
    """{"threads": usable cores, "affinity": len(sched_getaffinity), "quota": cgroup CPUs or None,
    "nproc": os.cpu_count()}; threads = affinity, capped by the quota (rounded up)."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_quota_cpus()
    threads = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    return {"threads": threads, "affinity": aff, "quota": quota, "nproc": os.cpu_count()}


def cpu_threads() -> int:
    return cpu_share()["threads"]
