"""Host CPU facts for sizing thread pools and stating baselines honestly.

``os.cpu_count()`` reports every CPU of the machine; a container may be
allowed far fewer (an affinity mask, a cgroup CPU quota).  The CPU baseline
and the checkers use ``usable_cpus()`` threads and report both numbers.
"""
from __future__ import annotations

import os
import platform


def cgroup_quota_cpus():
    """CPUs granted by a cgroup v2 (cpu.max) or v1 (cfs quota) limit, or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            p = int(fh.read())
        if q > 0:
            return max(1, q // p)
    except (OSError, ValueError):
        pass
    return None


def usable_cpus() -> int:
    """CPUs this process may actually run on at once."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_quota_cpus()
    return max(1, min(n, q) if q else n)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def describe() -> dict:
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": cgroup_quota_cpus(),
            "usable": usable_cpus(), "cpu_model": cpu_model()}
