"""Build the in-tree native extensions for gfx950.

    python setup.py build_ext --inplace        (or: python setup.py)

A direct hipcc build (no hipify pass, no CUDA compatibility layer):
  * csrc/kernels/*.hip   -> hipcc --offload-arch=gfx950 (HIP headers only: fast)
  * csrc/host/*.cpp      -> g++ (C++ host runtime: preprocessing, SPSC rings, CRC32C)
  * csrc/*bindings.cpp   -> hipcc host compile with the torch headers
  * link                 -> hipcc -shared with libtorch / libamdhip64
Variants (same sources, one module each):
  * dist_dqn_amd/_C*.so       bf16 MFMA network kernels (default executor)
  * dist_dqn_amd/_C_f16*.so   -DDQN_F16: fp16 MFMA network kernels (--dtype=fp16; csrc/include/dqn_act.h)
  * dist_dqn_amd/_C_f32*.so   -DDQN_F32: fp32 MFMA network kernels (--dtype=fp32, the reference precision)
  * dist_dqn_amd/_C_debug*.so only with DQN_DEBUG=1: -O1 -g, device DQN_ASSERTs (DQN_DEBUG_EXT=1 selects it)
  * dist_dqn_amd/libdqn_host.so  csrc/host/*.cpp without torch/HIP (CPU actor processes, ctypes)
Objects go to build/<variant>/ and are rebuilt when the source, any csrc header or the
compile command changes.
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
SUFFIX = sysconfig.get_config_var('EXT_SUFFIX')
HOST_OUT = os.path.join(ROOT, 'dist_dqn_amd', 'libdqn_host.so')   # torch-free host runtime (ctypes)
# (module name, object dir, extra kernel flags)
VARIANTS = {
    'release': ('_C', 'obj', ['-O3']),
    'f16': ('_C_f16', 'obj_f16', ['-O3', '-DDQN_F16=1']),
    'f32': ('_C_f32', 'obj_f32', ['-O3', '-DDQN_F32=1']),
    'debug': ('_C_debug', 'obj_debug', ['-O1', '-g', '-DDQN_DEBUG=1']),
}


def _torch_flags(mod):
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type='cuda') if 'device_type' in ce.include_paths.__code__.co_varnames \
        else ce.include_paths(cuda=True)
    inc += [sysconfig.get_paths()['include']]
    libdirs = ce.library_paths(device_type='cuda') if 'device_type' in ce.library_paths.__code__.co_varnames \
        else ce.library_paths(cuda=True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ['-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1', '-DTORCH_API_INCLUDE_EXTENSION_H',
            '-DTORCH_EXTENSION_NAME=%s' % mod, '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi]
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


def _plan(variant):
    mod, sub, kflags = VARIANTS[variant]
    inc, libdirs, defs = _torch_flags(mod)
    build = os.path.join(ROOT, 'build', sub)
    os.makedirs(build, exist_ok=True)
    headers = glob.glob(os.path.join(ROOT, 'csrc', '**', '*.h'), recursive=True)
    kern = sorted(glob.glob(os.path.join(ROOT, 'csrc', 'kernels', '*.hip')))
    binds = sorted(glob.glob(os.path.join(ROOT, 'csrc', '*.cpp')))
    cmds, objs = [], []
    vdefs = [f for f in kflags if f.startswith('-D')]
    for src in kern:
        obj = os.path.join(build, os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = [HIPCC, '-c', src, '-o', obj] + kflags + ['-std=c++17', '-fPIC', '--offload-arch=' + ARCH,
                                                       '-ffp-contract=fast-honor-pragmas',
                                                       '-I' + os.path.join(ROOT, 'csrc'), '-D__HIP_PLATFORM_AMD__=1']
        if _newer(src, obj, headers, cmd):
            cmds.append(cmd)
    for src in binds:
        obj = os.path.join(build, 'bind_' + os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = [HIPCC, '-c', src, '-o', obj, '-O2', '-std=c++17', '-fPIC', '-I' + os.path.join(ROOT, 'csrc')] + \
              ['-I' + i for i in inc] + defs + vdefs
        if _newer(src, obj, headers, cmd):
            cmds.append(cmd)
    out = os.path.join(ROOT, 'dist_dqn_amd', mod + SUFFIX)
    # -Bsymbolic: each variant's launchers bind to its own kernels when several are loaded
    link = [HIPCC, '-shared', '-fPIC', '-Wl,-Bsymbolic', '-o', out] + objs + ['-L' + d for d in libdirs] + \
           ['-Wl,-rpath,' + d for d in libdirs] + \
           ['-lc10', '-ltorch', '-ltorch_cpu', '-ltorch_python', '-lamdhip64', '-lc10_hip', '-ltorch_hip']
    return cmds, link, out


def _plan_host():
    build = os.path.join(ROOT, 'build', 'host')
    os.makedirs(build, exist_ok=True)
    headers = glob.glob(os.path.join(ROOT, 'csrc', '**', '*.h'), recursive=True)
    cmds, objs = [], []
    for src in sorted(glob.glob(os.path.join(ROOT, 'csrc', 'host', '*.cpp'))):
        obj = os.path.join(build, os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = ['g++', '-c', src, '-o', obj, '-O3', '-std=c++17', '-fPIC', '-Wall']
        if _newer(src, obj, headers, cmd):
            cmds.append(cmd)
    return cmds, ['g++', '-shared', '-fPIC', '-o', HOST_OUT] + objs + ['-lpthread'], objs


def build(verbose=False, jobs=None, variants=None):
    if variants is None:
        variants = ['debug'] if os.environ.get('DQN_DEBUG', '0') == '1' else ['release', 'f16', 'f32']

    def run(cmd):
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('compile failed: %s\n%s%s' % (' '.join(cmd), r.stdout, r.stderr))
        return cmd[2] if len(cmd) > 2 else ''

    hcmds, hlink, host_objs = _plan_host()
    plans = [_plan(v) for v in variants]
    # the host runtime's objects are linked into every extension module too
    plans = [(c, l[:l.index('-o') + 2] + host_objs + l[l.index('-o') + 2:], o) for c, l, o in plans]
    allc = hcmds + [c for p in plans for c in p[0]]
    jobs = jobs or int(os.environ.get('MAX_JOBS', min(16, os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in cf.as_completed([ex.submit(run, c) for c in allc]):
            f.result()
    if hcmds or not os.path.exists(HOST_OUT):
        run(hlink)
    outs = []
    for cmds, link, out in plans:
        if cmds or hcmds or not os.path.exists(out):
            run(link)
        outs.append(out)
    return outs


if __name__ == '__main__':
    args = [a for a in sys.argv[1:] if a not in ('build_ext', '--inplace')]
    for o in build(verbose='-v' in args):
        print(o)
