"""Every built native-extension variant (bf16 _C, fp16 _C_f16, fp32 _C_f32) imports, alone and
all together in one process (module-local pybind types; -Bsymbolic kernel launchers)."""
import importlib
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _built(name):
    pkg = os.path.join(ROOT, 'dist_dqn_amd')
    return any(f.startswith(name + '.') and f.endswith('.so') for f in os.listdir(pkg))


def test_all_variants_import_together():
    names = [n for n in ('_C', '_C_f16', '_C_f32') if _built(n)]
    if not names:
        pytest.skip('native extension not built')
    mods = [importlib.import_module('dist_dqn_amd.' + n) for n in names]
    for m in mods:
        assert hasattr(m, 'qnet_igemm') and hasattr(m, 'optim_pack') and hasattr(m, 'InferServer')


def test_ingest_server_binding_converts_lists():
    """The Ape-X ingest thread's constructor takes Python lists (pybind11 STL casters): a call
    with wrong list sizes must reach the C++ argument check, not fail the type conversion."""
    if not _built('_C'):
        pytest.skip('native extension not built')
    m = importlib.import_module('dist_dqn_amd._C')
    with pytest.raises(RuntimeError, match='argument sizes'):
        m.IngestServer(0, 1, 0, 4, 0.99, [0] * 7, [0] * 4, [0] * 3, [0] * 11, 0)
