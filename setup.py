"""Build the in-tree native extension ``dist_dqn_amd/_C<EXT_SUFFIX>`` for gfx950.

    python setup.py build_ext --inplace        (or: python setup.py)

A direct hipcc build (no hipify pass, no CUDA compatibility layer):
  * csrc/kernels/*.hip   -> hipcc --offload-arch=gfx950 (HIP headers only: fast)
  * csrc/host/*.cpp      -> g++ (C++ host runtime: preprocessing, SPSC rings, CRC32C)
  * csrc/*bindings.cpp   -> hipcc host compile with the torch headers
  * link                 -> hipcc -shared with libtorch / libamdhip64
  * csrc/host/*.cpp also -> dist_dqn_amd/libdqn_host.so (no torch/HIP: loaded by
                            CPU actor processes through ctypes)
Objects go to build/ and are rebuilt when the source or any csrc header is newer.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')
HIPCC = os.path.join(os.environ.get('ROCM_PATH', '/opt/rocm'), 'bin', 'hipcc')
# DQN_DEBUG=1: bounds-checked debug variant (-O1 -g, device DQN_ASSERTs live) built next to
# the release module as dist_dqn_amd/_C_debug*.so; selected at import by DQN_DEBUG_EXT=1
DEBUG = os.environ.get('DQN_DEBUG', '0') == '1'
MOD = '_C_debug' if DEBUG else '_C'
BUILD = os.path.join(ROOT, 'build', 'obj_debug' if DEBUG else 'obj')
OUT = os.path.join(ROOT, 'dist_dqn_amd', MOD + sysconfig.get_config_var('EXT_SUFFIX'))
HOST_OUT = os.path.join(ROOT, 'dist_dqn_amd', 'libdqn_host.so')   # torch-free host runtime (ctypes)


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type='cuda') if 'device_type' in ce.include_paths.__code__.co_varnames \
        else ce.include_paths(cuda=True)
    inc += [sysconfig.get_paths()['include']]
    libdirs = ce.library_paths(device_type='cuda') if 'device_type' in ce.library_paths.__code__.co_varnames \
        else ce.library_paths(cuda=True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ['-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1', '-DTORCH_API_INCLUDE_EXTENSION_H',
            '-DTORCH_EXTENSION_NAME=%s' % MOD, '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi]
    return inc, libdirs, defs


def _newer(src, obj, headers, cmd=None):
    if not os.path.exists(obj):
        return True
    if cmd is not None:                   # a flag change rebuilds too
        stamp = obj + '.cmd'
        line = ' '.join(cmd)
        old = open(stamp).read() if os.path.exists(stamp) else ''
        if old != line:
            with open(stamp, 'w') as f:
                f.write(line)
            return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def build(verbose=False, jobs=None):
    inc, libdirs, defs = _torch_flags()
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(ROOT, 'csrc', '**', '*.h'), recursive=True)
    kern = sorted(glob.glob(os.path.join(ROOT, 'csrc', 'kernels', '*.hip')))
    host = sorted(glob.glob(os.path.join(ROOT, 'csrc', 'host', '*.cpp')))
    binds = sorted(glob.glob(os.path.join(ROOT, 'csrc', '*.cpp')))
    cmds = []
    objs = []
    for src in kern:
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = [HIPCC, '-c', src, '-o', obj, '-O1' if DEBUG else '-O3', '-std=c++17', '-fPIC',
               '--offload-arch=' + ARCH, '-ffp-contract=fast-honor-pragmas', '-I' + os.path.join(ROOT, 'csrc'),
               '-D__HIP_PLATFORM_AMD__=1'] + (['-g', '-DDQN_DEBUG=1'] if DEBUG else [])
        if _newer(src, obj, headers, cmd):
            cmds.append(cmd)
    for src in host:
        obj = os.path.join(BUILD, 'host_' + os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = ['g++', '-c', src, '-o', obj, '-O3', '-std=c++17', '-fPIC', '-Wall']
        if _newer(src, obj, headers, cmd):
            cmds.append(cmd)
    for src in binds:
        obj = os.path.join(BUILD, 'bind_' + os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = [HIPCC, '-c', src, '-o', obj, '-O2', '-std=c++17', '-fPIC', '-I' + os.path.join(ROOT, 'csrc')] + \
              ['-I' + i for i in inc] + defs
        if _newer(src, obj, headers, cmd):
            cmds.append(cmd)

    def run(cmd):
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('compile failed: %s\n%s%s' % (' '.join(cmd), r.stdout, r.stderr))
        return cmd[2] if len(cmd) > 2 else ''

    jobs = jobs or int(os.environ.get('MAX_JOBS', min(16, os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in cf.as_completed([ex.submit(run, c) for c in cmds]):
            f.result()
    host_objs = [o for o in objs if os.path.basename(o).startswith('host_')]
    if not DEBUG and (cmds or not os.path.exists(HOST_OUT)):
        run(['g++', '-shared', '-fPIC', '-o', HOST_OUT] + host_objs + ['-lpthread'])
    if cmds or not os.path.exists(OUT):
        link = [HIPCC, '-shared', '-fPIC', '-o', OUT] + objs + ['-L' + d for d in libdirs] + \
               ['-Wl,-rpath,' + d for d in libdirs] + \
               ['-lc10', '-ltorch', '-ltorch_cpu', '-ltorch_python', '-lamdhip64', '-lc10_hip', '-ltorch_hip']
        run(link)
    return OUT


if __name__ == '__main__':
    args = [a for a in sys.argv[1:] if a not in ('build_ext', '--inplace')]
    print(build(verbose='-v' in args))
