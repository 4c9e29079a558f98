"""Every Python source of the package, the scripts and the benchmark byte-compiles (the GPU-only
modules are otherwise first imported on the GPU box)."""
import glob
import os
import py_compile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, 'dist_dqn_amd', '**', '*.py'), recursive=True)
               + glob.glob(os.path.join(ROOT, 'scripts', '*.py')) + [os.path.join(ROOT, 'bench.py'),
                                                                       os.path.join(ROOT, '__graft_entry__.py')])


@pytest.mark.parametrize('path', FILES, ids=lambda p: os.path.relpath(p, ROOT))
def test_compiles(path, tmp_path):
    py_compile.compile(path, cfile=str(tmp_path / 'x.pyc'), doraise=True)
