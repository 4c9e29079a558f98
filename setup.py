"""Build the in-tree native extension ``dist_dqn_amd/_C*.so`` for gfx950.

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

HIP kernels (csrc/kernels/*.hip) include only the HIP headers and compile
fast; torch headers are confined to the two binding translation units.
"""
import glob
import os

from setuptools import setup

os.environ.setdefault('PYTORCH_ROCM_ARCH', 'gfx950')
from torch.utils.cpp_extension import BuildExtension, CUDAExtension  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))


def rel(p):
    return os.path.relpath(p, ROOT)


sources = ([rel(os.path.join(ROOT, 'csrc', 'bindings.cpp')), rel(os.path.join(ROOT, 'csrc', 'net_bindings.cpp'))]
           + sorted(rel(p) for p in glob.glob(os.path.join(ROOT, 'csrc', 'kernels', '*.hip')))
           + sorted(rel(p) for p in glob.glob(os.path.join(ROOT, 'csrc', 'host', '*.cpp'))))

setup(
    name='dist_dqn_amd',
    version='0.1.0',
    packages=['dist_dqn_amd'],
    ext_modules=[CUDAExtension(
        'dist_dqn_amd._C', sources,
        include_dirs=[os.path.join(ROOT, 'csrc')],
        extra_compile_args={
            'cxx': ['-O3', '-std=c++17'],
            'nvcc': ['-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=fast'],
        })],
    cmdclass={'build_ext': BuildExtension.with_options(use_ninja=True)},
)
