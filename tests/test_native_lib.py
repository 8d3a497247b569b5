'''
The C-ABI library: it must exist, load, export exactly what include/*.h declare, and
its ctypes mirror must match the header's struct layout. No compute calls (no GPU here).
'''
import ctypes
import glob
import os
import re

from aircraft_trajectory_optimization_amd import native

HEADERS = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include',
                                        '*.h')))


def _declared():
    names = set()
    for h in HEADERS:
        txt = open(h, encoding='utf-8').read()
        txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
        names |= set(re.findall(r'\b(ato_[a-z0-9_]+)\s*\(', txt))
    return sorted(names)


def test_library_loads_and_exports_header_symbols():
    lib = native.load()
    declared = _declared()
    assert declared, 'no functions found in include/*.h'
    for name in declared:
        assert hasattr(lib, name), f'{name} declared in include/*.h but not exported'
    assert set(declared) == set(native.EXPORTED_SYMBOLS)
    assert lib.ato_version().decode().startswith('ato 2')


def test_ctypes_struct_layout():
    # ato_gate: 6 int32 + 10 + 3 + 9 + 9 + 1 doubles
    assert ctypes.sizeof(native.AtoGate) == 6 * 4 + (10 + 3 + 9 + 9 + 1) * 8
    # offsets that the header fixes by field order
    assert native.AtoProblemDesc.euler_wraps.offset == 16 * 4
    assert native.AtoProblemDesc.node_geom.offset % 8 == 0


def test_missing_library_fails_loudly(tmp_path):
    import pytest
    with pytest.raises(RuntimeError):
        native.load(str(tmp_path / 'nope.so'))


def test_kkt_plan_desc_layout(tmp_path):
    ''' the ctypes mirror of ato_kkt_plan_desc against the C compiler's layout of the header '''
    import subprocess
    from aircraft_trajectory_optimization_amd.solver.kkt_device import AtoKKTPlanDesc
    names = [f[0] for f in AtoKKTPlanDesc._fields_]
    inc = os.path.dirname(HEADERS[0])
    src = tmp_path / 'layout.c'
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ato_kkt.h"\nint main(void) {\n' +
                   ''.join(f'    printf("%zu\\n", offsetof(ato_kkt_plan_desc, {n}));\n' for n in names) +
                   '    printf("%zu\\n", sizeof(ato_kkt_plan_desc));\n    return 0;\n}\n')
    exe = tmp_path / 'layout'
    subprocess.run(['gcc', '-I', inc, str(src), '-o', str(exe)], check=True)
    out = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert out[:-1] == [getattr(AtoKKTPlanDesc, n).offset for n in names]
    assert out[-1] == ctypes.sizeof(AtoKKTPlanDesc)


def test_ipm_struct_layout(tmp_path):
    ''' the ctypes mirrors of ato_ipm_dims / ato_ipm_bounds against the C compiler's layout '''
    import subprocess
    inc = os.path.dirname(HEADERS[0])
    body = ''
    for ct, cname in ((native.AtoIpmDims, 'ato_ipm_dims'), (native.AtoIpmBounds, 'ato_ipm_bounds')):
        body += ''.join(f'    printf("%zu\\n", offsetof({cname}, {f[0]}));\n' for f in ct._fields_)
        body += f'    printf("%zu\\n", sizeof({cname}));\n'
    src = tmp_path / 'ipm_layout.c'
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ato_ipm.h"\nint main(void) {\n' + body +
                   '    return 0;\n}\n')
    exe = tmp_path / 'ipm_layout'
    subprocess.run(['gcc', '-I', inc, str(src), '-o', str(exe)], check=True)
    out = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = []
    for ct in (native.AtoIpmDims, native.AtoIpmBounds):
        want += [getattr(ct, f[0]).offset for f in ct._fields_] + [ctypes.sizeof(ct)]
    assert out == want
