'''
ORACLE (test infrastructure only): vehicle ODEs, restated literally from the reference.

Arrays carry a trailing batch axis and may be complex (complex-step differentiation).
  rotations (ESP / YPR R, M)           drone3d/dynamics/rotations.py:44-102
  drone pose / forces / state          drone3d/dynamics/drone_models.py:47-123
  parametric drone pose                drone3d/dynamics/drone_models.py:249-292
  point mass (global / parametric)     drone3d/dynamics/point_model.py:28-75, :149-213
  DCM attitude (config 5)              NOT in the reference (rotations.py:19-24 has ESP and YPR only):
                                       r = R row-major, R' = R [w]x -- parity unpinned by
                                       construction; pinned by equivalence with the ESP model
                                       (tests/test_dcm_cpu.py)
'''
import numpy as np


def esp_R(q):
    qi, qj, qk, qr = q
    R = np.array([
        [1 - 2 * qj ** 2 - 2 * qk ** 2, 2 * (qi * qj - qk * qr), 2 * (qi * qk + qj * qr)],
        [2 * (qi * qj + qk * qr), 1 - 2 * qi ** 2 - 2 * qk ** 2, 2 * (qj * qk - qi * qr)],
        [2 * (qi * qk - qj * qr), 2 * (qj * qk + qi * qr), 1 - 2 * qi ** 2 - 2 * qj ** 2],
    ])
    return R / (qi ** 2 + qj ** 2 + qk ** 2 + qr ** 2)


def esp_M(q):
    qi, qj, qk, qr = q
    return 0.5 * np.array([[qr, -qk, qj], [qk, qr, -qi], [-qj, qi, qr], [-qi, -qj, -qk]])


def ypr_R(r):
    a, b, c = r
    o, z = np.ones_like(a), np.zeros_like(a)
    Ra = np.array([[np.cos(a), -np.sin(a), z], [np.sin(a), np.cos(a), z], [z, z, o]])
    Rb = np.array([[np.cos(b), z, np.sin(b)], [z, o, z], [-np.sin(b), z, np.cos(b)]])
    Rc = np.array([[o, z, z], [z, np.cos(c), -np.sin(c)], [z, np.sin(c), np.cos(c)]])
    return np.einsum('ijb,jkb->ikb', np.einsum('ijb,jkb->ikb', Ra, Rb), Rc)


def ypr_M(r):
    _, b, c = r
    z, o = np.zeros_like(b), np.ones_like(b)
    return np.array([[z, np.sin(c) / np.cos(b), np.cos(c) / np.cos(b)],
                     [z, np.cos(c), -np.sin(c)],
                     [o, np.sin(c) * np.tan(b), np.cos(c) * np.tan(b)]])


def dcm_R(r):
    ''' the DCM attitude state is R itself (row-major 9-vector) '''
    return np.array([[r[0], r[1], r[2]], [r[3], r[4], r[5]], [r[6], r[7], r[8]]])


def dcm_rdot(r, w):
    ''' R' = R [w]x, row-major '''
    R = dcm_R(r)
    Rd = np.einsum('ijb,jkb->ikb', R, hat(w))
    return Rd.reshape(9, *Rd.shape[2:])


def mv(A, x):
    ''' (3,3,B) or (3,3) times (3,B) '''
    if A.ndim == 2:
        return np.einsum('ij,jb->ib', A, x)
    return np.einsum('ijb,jb->ib', A, x)


def hat(v):
    z = np.zeros_like(v[0])
    return np.array([[z, -v[2], v[1]], [v[2], z, -v[0]], [-v[1], v[0], z]])


def _att(use_quat):
    ''' attitude parameterisation: True / 'esp' quaternion, False / 'ypr' Euler, 'dcm' matrix '''
    if use_quat == 'dcm':
        return 'dcm', 9
    return ('esp', 4) if use_quat in (True, 'esp') else ('ypr', 3)


def drone_zdot(z, u, veh, use_quat, frame, global_r, geo=None):
    '''
    z: (nz, B), u: (4, B). veh: dict of DroneConfig fields. frame: 'global' | 'parametric'.
    geo: dict with Rp (3,3), ks, ky, kn, mag for the parametric frame (fixed node geometry).
    use_quat: True (ESP), False (YPR) or 'dcm'.
    '''
    att, nr = _att(use_quat)
    p, r, vb, wb = z[:3], z[3:3 + nr], z[3 + nr:6 + nr], z[6 + nr:9 + nr]
    Rr = esp_R(r) if att == 'esp' else ypr_R(r) if att == 'ypr' else dcm_R(r)
    kin = (lambda w: mv(esp_M(r), w)) if att == 'esp' else (lambda w: mv(ypr_M(r), w)) if att == 'ypr' \
        else (lambda w: dcm_rdot(r, w))
    if frame == 'global':
        R = Rr
        p_dot = mv(R, vb)
        r_dot = kin(wb)
    else:
        Rp = geo['Rp']
        R_rel = np.einsum('ai,ajb->ijb', Rp, Rr) if global_r else Rr
        vp = mv(R_rel, vb)
        y, n = p[1], p[2]
        s_dot = vp[0] / geo['mag'] / (1 + geo['ky'] * n - geo['kn'] * y)
        y_dot = vp[1] + n * geo['ks'] * s_dot * geo['mag']
        n_dot = vp[2] - y * geo['ks'] * s_dot * geo['mag']
        p_dot = np.array([s_dot, y_dot, n_dot])
        k = np.array([geo['ks'], geo['ky'], geo['kn']])
        wp = k[:, None] * s_dot * geo['mag']
        w_eff = wb if global_r else wb - np.einsum('jib,jb->ib', Rr, wp)
        r_dot = kin(w_eff)
        R = Rr if global_r else np.einsum('ij,jkb->ikb', Rp, Rr)
    Fgb = -veh['m'] * veh['g'] * np.array([R[2, 0], R[2, 1], R[2, 2]])
    Fdb = -np.array([veh['b1'], veh['b2'], veh['b3']])[:, None] * vb
    Kdb = -np.array([veh['bw1'], veh['bw2'], veh['bw3']])[:, None] * wb
    Tb = np.array([0 * u[0], 0 * u[0], u[0] + u[1] + u[2] + u[3]])
    TKb = np.array([(u[0] + u[1] - u[2] - u[3]) * veh['l'],
                    (-u[0] + u[1] + u[2] - u[3]) * veh['l'],
                    (u[0] - u[1] + u[2] - u[3]) * veh['k']])
    Fb = Fdb + Fgb + Tb
    Kb = Kdb + TKb
    Wb = hat(wb)
    Ib = np.array([veh['I1'], veh['I2'], veh['I3']])
    vb_dot = Fb / veh['m'] - mv(Wb, vb)
    wb_dot = (Kb - mv(Wb, Ib[:, None] * wb)) / Ib[:, None]
    return np.concatenate([p_dot, r_dot, vb_dot, wb_dot])


def drone_vg_R(z, use_quat, frame, global_r, geo=None):
    ''' global velocity and global rotation (f_vg, f_R helpers) '''
    att, nr = _att(use_quat)
    r, vb = z[3:3 + nr], z[3 + nr:6 + nr]
    Rr = esp_R(r) if att == 'esp' else ypr_R(r) if att == 'ypr' else dcm_R(r)
    if frame == 'global' or global_r:
        R = Rr
    else:
        R = np.einsum('ij,jkb->ikb', geo['Rp'], Rr)
    return mv(R, vb), R


def point_zdot(z, u, veh, frame, global_r, geo=None):
    ''' point mass; z (6, B), u (3, B) '''
    p, vb = z[:3], z[3:6]
    if frame == 'global':
        R = np.eye(3)
        p_dot = vb
        wb = np.zeros_like(vb)
    else:
        Rp = geo['Rp']
        R_rel = Rp.T if global_r else np.eye(3)
        vp = mv(R_rel, vb)
        y, n = p[1], p[2]
        s_dot = vp[0] / geo['mag'] / (1 + geo['ky'] * n - geo['kn'] * y)
        y_dot = vp[1] + n * geo['ks'] * s_dot * geo['mag']
        n_dot = vp[2] - y * geo['ks'] * s_dot * geo['mag']
        p_dot = np.array([s_dot, y_dot, n_dot])
        k = np.array([geo['ks'], geo['ky'], geo['kn']])
        wp = k[:, None] * s_dot * geo['mag']
        wb = np.zeros_like(vb) if global_r else wp
        R = np.eye(3) if global_r else Rp
    Fgb = -veh['m'] * veh['g'] * np.array([R[2, 0], R[2, 1], R[2, 2]])[:, None] * np.ones_like(vb[0])
    Fdb = -np.array([veh['b1'], veh['b2'], veh['b3']])[:, None] * vb
    Fb = u + Fgb + Fdb
    vb_dot = Fb / veh['m'] - mv(hat(wb), vb)
    return np.concatenate([p_dot, vb_dot])
