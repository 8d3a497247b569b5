'''
Build libato.so for gfx950 in-tree (aircraft_trajectory_optimization_amd/_lib/).

One object per model variant (ato_inst.hip, -DATO_INST=i) plus the C-ABI object, compiled
in parallel with hipcc, and the host-only Hessian structure analysis (ato_hstruct.cpp, g++),
then linked into a shared library. Objects are rebuilt only when
a source or header is newer.
'''
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
OUT = os.path.join(PKG, '_lib')
OBJ = os.path.join(PKG, '_lib', 'obj')
LIB = os.path.join(OUT, 'libato.so')
N_INST = 12
ARCH = os.environ.get('ATO_OFFLOAD_ARCH', 'gfx950')
FLAGS = ['-std=c++20', '-O3', f'--offload-arch={ARCH}', '-fPIC', '-I', os.path.join(REPO, 'include')]


def _deps():
    return glob.glob(os.path.join(CSRC, '*.hpp')) + glob.glob(os.path.join(REPO, 'include', '*.h'))


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


HOST_FLAGS = ['-std=c++20', '-O2', '-fPIC', '-I', os.path.join(REPO, 'include')]


def _compile(job):
    src, obj, extra = job
    if not _stale(obj, [src] + _deps()):
        return obj, 'cached'
    if src.endswith('.cpp'):      # host-only translation unit
        cmd = ['g++', *HOST_FLAGS, *extra, '-c', src, '-o', obj]
    else:
        cmd = ['hipcc', *FLAGS, *extra, '-c', src, '-o', obj]
    res = subprocess.run(cmd, capture_output=True, text=True, check=False)
    if res.returncode != 0:
        raise RuntimeError(f'hipcc failed for {os.path.basename(src)}:\n{res.stderr}')
    return obj, 'built'


def build(verbose=True, jobs=None) -> str:
    ''' compile and link; returns the library path '''
    os.makedirs(OBJ, exist_ok=True)
    work = [(os.path.join(CSRC, 'ato_capi.hip'), os.path.join(OBJ, 'ato_capi.o'), []),
            (os.path.join(CSRC, 'ato_hstruct.cpp'), os.path.join(OBJ, 'ato_hstruct.o'), []),
            (os.path.join(CSRC, 'ato_mesh.hip'), os.path.join(OBJ, 'ato_mesh.o'), []),
            (os.path.join(CSRC, 'ato_kkt.hip'), os.path.join(OBJ, 'ato_kkt.o'), []),
            # no contraction: the interior-point column kernels reproduce the host formulas bit for bit
            (os.path.join(CSRC, 'ato_ipm.hip'), os.path.join(OBJ, 'ato_ipm.o'), ['-ffp-contract=off'])]
    for i in range(N_INST):
        work.append((os.path.join(CSRC, 'ato_inst.hip'), os.path.join(OBJ, f'ato_inst{i}.o'), [f'-DATO_INST={i}']))
    jobs = jobs or min(len(work), max(1, min(8, os.cpu_count() or 4)))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(_compile, work))
    objs = [o for o, _ in results]
    if _stale(LIB, objs) or any(state == 'built' for _, state in results):
        cmd = ['hipcc', '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', LIB, *objs]
        res = subprocess.run(cmd, capture_output=True, text=True, check=False)
        if res.returncode != 0:
            raise RuntimeError(f'link failed:\n{res.stderr}')
    if verbose:
        built = sum(1 for _, s in results if s == 'built')
        print(f'[build_native] {LIB} ({built} objects rebuilt)')
    return LIB


if __name__ == '__main__':
    build()
    sys.exit(0)
