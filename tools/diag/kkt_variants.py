'''
DIAGNOSTIC builds of the KKT kernels (not shipped): compile csrc/ato_kkt.hip with extra
defines and link it with the library's other objects into tools/diag/_lib/libato_<name>.so,
which tools/gpu_check.sh `kktvar` times with tools/bench_kkt.py (ATO_LIB_PATH).

    python tools/diag/kkt_variants.py NAME [-DFLAG ...]      (CPU: build only)
'''
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(ROOT, 'aircraft_trajectory_optimization_amd')


def build(name, flags):
    from aircraft_trajectory_optimization_amd import build_native as bn
    bn.build(verbose=False)
    out = os.path.join(HERE, '_lib')
    os.makedirs(out, exist_ok=True)
    obj = os.path.join(out, f'ato_kkt_{name}.o')
    subprocess.run(['hipcc', *bn.FLAGS, *flags, '-c', os.path.join(PKG, 'csrc', 'ato_kkt.hip'), '-o', obj], check=True)
    objs = [o for o in glob.glob(os.path.join(bn.OBJ, '*.o')) if not o.endswith('ato_kkt.o')] + [obj]
    lib = os.path.join(out, f'libato_{name}.so')
    subprocess.run(['hipcc', '-shared', '-fPIC', f'--offload-arch={bn.ARCH}', '-o', lib, *objs], check=True)
    os.remove(obj)
    print(lib)


if __name__ == '__main__':
    sys.path.insert(0, ROOT)
    build(sys.argv[1], sys.argv[2:])
