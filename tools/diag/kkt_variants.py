'''
DIAGNOSTIC builds of libato.so (not shipped): recompile one translation unit with extra
defines and link it with the library's other objects into tools/diag/_lib/libato_<name>.so,
which tools/gpu_check.sh (`kktvar`, `evalvar`) times through ATO_LIB_PATH.

    python tools/diag/kkt_variants.py NAME [--unit ato_kkt|ato_inst1|...] [--src FILE] [-DFLAG ...]   (CPU)

--src compiles FILE (e.g. an older ato_kkt.hip) in place of the unit's own source.
--patch applies a patch to a copy of the unit's source first: tools/diag/kkt_diag_variants.patch
restores the timing-only ablations (-DATO_KKT_X_NOSEARCH / _NOR / _NOSTORE / _NOUPDATE, results
wrong) and the rejected blocked leaf kernel (-DATO_KKT_X_BLOCKED=1, then ATO_KKT_BLOCKED=1), which
the product source no longer carries.
'''
import argparse
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(ROOT, 'aircraft_trajectory_optimization_amd')


def build(name, unit, flags, src_override=None, patch=None):
    from aircraft_trajectory_optimization_amd import build_native as bn
    bn.build(verbose=False)
    out = os.path.join(HERE, '_lib')
    os.makedirs(out, exist_ok=True)
    obj = os.path.join(out, f'{unit}_{name}.o')
    if unit.startswith('ato_inst'):
        src, extra = os.path.join(PKG, 'csrc', 'ato_inst.hip'), [f'-DATO_INST={unit[len("ato_inst"):]}']
    else:
        src, extra = os.path.join(PKG, 'csrc', unit + '.hip'), []
    if src_override:
        src = os.path.abspath(src_override)
    if patch:
        tmp = os.path.join(HERE, f'_{unit}_{name}.hip')   # two levels below the repo: its relative includes resolve
        with open(src) as f_in, open(tmp, 'w') as f_out:
            f_out.write(f_in.read())
        subprocess.run(['patch', '-s', tmp, os.path.abspath(patch)], check=True)
        src = tmp
        extra = extra + ['-I', os.path.join(PKG, 'csrc')]
    subprocess.run(['hipcc', *bn.FLAGS, *extra, *flags, '-c', src, '-o', obj], check=True)
    objs = [o for o in glob.glob(os.path.join(bn.OBJ, '*.o')) if os.path.basename(o) != unit + '.o'] + [obj]
    lib = os.path.join(out, f'libato_{name}.so')
    subprocess.run(['hipcc', '-shared', '-fPIC', f'--offload-arch={bn.ARCH}', '-o', lib, *objs], check=True)
    os.remove(obj)
    print(lib)


if __name__ == '__main__':
    sys.path.insert(0, ROOT)
    ap = argparse.ArgumentParser()
    ap.add_argument('name')
    ap.add_argument('--unit', default='ato_kkt')
    ap.add_argument('--src', default=None)
    ap.add_argument('--patch', default=None)
    a, rest = ap.parse_known_args()
    build(a.name, a.unit, rest, a.src, a.patch)
