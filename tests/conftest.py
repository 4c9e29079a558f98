import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')
    config.addinivalue_line('markers', 'slow: long-running test')


def _needs_fresh_parent(item) -> bool:
    # the 8-rank one-GPU rehearsals need a test process that holds no GPU context yet
    # (tests/test_dist_gpu.py _gpu_free_parent): they run first in a session
    cs = getattr(item, 'callspec', None)
    return ('test_dist_gpu.py::' in item.nodeid and cs is not None
            and int(cs.params.get('world', 0) or 0) >= 8)


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        items[:] = [i for i in items if _needs_fresh_parent(i)] + [i for i in items if not _needs_fresh_parent(i)]
        return
    skip = pytest.mark.skip(reason='no GPU in this environment')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def cpu_config():
    from dist_dqn_amd.config import parse_args
    return parse_args(['--device=cpu', '--seed=0'])
