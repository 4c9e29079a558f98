"""CPU budget of this process: the allowed CPU set, capped by the container's CFS quota.

A container limited by quota (cgroup ``cpu.max`` / ``cpu.cfs_quota_us``) rather than by a cpuset
shows every host CPU to ``os.sched_getaffinity``; spreading N busy processes over all of them
burns the quota in a fraction of each CFS period, and then every thread of the group -- the
learner's launch thread included -- sleeps until the next period. Pinning the busy workers to
``budget - reserved`` CPUs keeps the group under its quota (measured: 256 Ape-X actors over 253
visible CPUs on a 16-CPU quota cut the learner from 9.7k to 0.77k SGD steps/s).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional


def cfs_quota_cpus() -> Optional[int]:
    """CPUs' worth of CFS quota (rounded down, >= 1), or None when unlimited / unknown.
    ``DQN_CPU_BUDGET`` overrides."""
    env = os.environ.get('DQN_CPU_BUDGET')
    if env:
        return max(1, int(env))
    try:                                             # cgroup v2
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            return max(1, int(math.floor(int(quota) / int(period))))
        return None
    except (OSError, ValueError):
        pass
    try:                                             # cgroup v1
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
            quota = int(f.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
            period = int(f.read())
        if quota > 0 and period > 0:
            return max(1, quota // period)
    except (OSError, ValueError):
        pass
    return None


def usable_cpus() -> List[int]:
    """The allowed CPU ids, truncated to the quota budget (lowest ids first)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    q = cfs_quota_cpus()
    return cpus[:q] if q is not None and q < len(cpus) else cpus
