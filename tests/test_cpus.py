"""utils/cpus.py: the CPU budget (allowed set capped by the CFS quota) that Ape-X pins its
actor processes to."""
import os

from dist_dqn_amd.utils import cpus


def test_budget_override_caps_usable_cpus(monkeypatch):
    allowed = sorted(os.sched_getaffinity(0))
    monkeypatch.setenv('DQN_CPU_BUDGET', '2')
    assert cpus.cfs_quota_cpus() == 2
    assert cpus.usable_cpus() == allowed[:2]
    monkeypatch.setenv('DQN_CPU_BUDGET', str(len(allowed) + 64))
    assert cpus.usable_cpus() == allowed


def test_quota_reader_handles_this_container(monkeypatch):
    monkeypatch.delenv('DQN_CPU_BUDGET', raising=False)
    q = cpus.cfs_quota_cpus()
    assert q is None or q >= 1
    assert 1 <= len(cpus.usable_cpus()) <= len(os.sched_getaffinity(0))
