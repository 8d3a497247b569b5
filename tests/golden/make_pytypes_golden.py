'''
Generate golden vectors from the REFERENCE's drone3d.pytypes (run in the build container,
where /root/reference exists). The reference never travels to the GPU box; only the
JSON this writes (pytypes_golden.json) is committed and used by the tests.

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/make_pytypes_golden.py

Pins (reference file:line):
  OrientationQuaternion.R / Rinv / e1 e2 e3 / qdot   drone3d/pytypes.py:165-258
  Position.xdot                                      drone3d/pytypes.py:66-73
  EulerAngles.R                                      drone3d/pytypes.py:314-334
  DroneConfig / PointConfig defaults                 drone3d/pytypes.py:357-402
'''
import dataclasses
import json
import os

import numpy as np

import drone3d.pytypes as pt   # the reference module (PYTHONPATH=/root/reference)


def main():
    rng = np.random.default_rng(20251015)
    out = {'quaternion': [], 'euler': [], 'configs': {}}
    for i in range(24):
        q = rng.standard_normal(4)
        if i % 2 == 0:
            q = q / np.linalg.norm(q)       # unit and non-unit quaternions
        w = rng.standard_normal(3)
        v = rng.standard_normal(3)
        Q = pt.OrientationQuaternion()
        Q.from_vec(q)
        W = pt.BodyAngularVelocity()
        W.from_vec(w)
        V = pt.BodyLinearVelocity()
        V.from_vec(v)
        out['quaternion'].append({
            'q': q.tolist(), 'w': w.tolist(), 'v': v.tolist(),
            'R': Q.R().tolist(), 'Rinv': Q.Rinv().tolist(),
            'e1': Q.e1().tolist(), 'e2': Q.e2().tolist(), 'e3': Q.e3().tolist(),
            'qdot': Q.qdot(W).to_vec().tolist(),
            'xdot': pt.Position().xdot(Q, V).to_vec().tolist(),
        })
    for _ in range(16):
        abc = rng.uniform(-1.4, 1.4, 3)
        E = pt.EulerAngles()
        E.from_vec(abc)
        out['euler'].append({'abc': abc.tolist(), 'R': E.R().tolist()})
    for cls in (pt.RacerConfig, pt.PointConfig, pt.DroneConfig):
        out['configs'][cls.__name__] = {f.name: getattr(cls(), f.name) for f in dataclasses.fields(cls)}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'pytypes_golden.json')
    with open(path, 'w', encoding='utf-8') as fh:
        json.dump(out, fh, indent=1)
    print('wrote', path)


if __name__ == '__main__':
    main()
