'''
ORACLE (test infrastructure only): centreline geometry restated from the reference.

  waypoint closing, s = arange          drone3d/centerlines/spline_centerline.py:232-241, :106-112
  CasADi piecewise polynomial of scipy  drone3d/utils/interp.py:55-84; CasADi pw_const is
    CubicSpline coefficients            ret = val[0] + sum_i (val[i+1]-val[i]) * (t >= tval[i])
  PLANAR r_y fit                        spline_centerline.py:151-176
  cleanly_closed + lateral spline bc    spline_centerline.py:127-148
  Darboux frame and curvatures          spline_centerline.py:266-322
  gate position / orientation snap-fit  drone3d/centerlines/base_centerline.py:314-336
'''
import numpy as np
import scipy.interpolate


def casadi_pw_const(t, tval, val):
    ''' CasADi pw_const as a telescoping sum (the reference's piecewise constants) '''
    ret = val[0]
    for i in range(len(val) - 1):
        ret = ret + (val[i + 1] - val[i]) * (1.0 if t >= tval[i] else 0.0)
    return ret


class RefPwPoly:
    ''' interp.py:55-84 with extrapolate='linear' '''

    def __init__(self, x, y, bc_type):
        sp = scipy.interpolate.CubicSpline(x, y, bc_type=bc_type)
        kc, kx = sp.c, sp.x
        kf = sp(kx[-1])
        self.kx = kx
        self.x0 = [kx[0], *kx]
        self.c0 = [kc[3, 0], *kc[3, :], kf]
        self.c1 = [kc[2, 0], *kc[2, :], sp(kx[-1], 1)]
        self.c2 = [0.0, *kc[1, :], 0.0]
        self.c3 = [0.0, *kc[0, :], 0.0]

    def coeffs(self, t):
        pw = lambda v: casadi_pw_const(t, self.kx, v)  # noqa: E731
        return t - pw(self.x0), pw(self.c0), pw(self.c1), pw(self.c2), pw(self.c3)

    def val(self, t):
        x, c0, c1, c2, c3 = self.coeffs(t)
        return c0 + c1 * x + c2 * x ** 2 + c3 * x ** 3

    def d1(self, t):
        x, _, c1, c2, c3 = self.coeffs(t)
        return c1 + c2 * 2 * x + c3 * 3 * x ** 2

    def d2(self, t):
        x, _, _, c2, c3 = self.coeffs(t)
        return c2 * 2 + c3 * 6 * x


class RefCenterline:
    '''
    Spline centreline with the PLANAR r_y fit (the SplineCenterlineConfig default).
    x: (3, M) waypoints; closed: periodic.
    '''

    def __init__(self, x, closed, gate_shape='circle', gate_ri=1.25, gate_snap_fit=True, gamma=0.9,
                 y_bounds=(-2, 2), n_bounds=(-2, 2)):
        x = np.asarray(x, dtype=float)
        if closed and not (x[:, 0] == x[:, -1]).all():
            x = np.hstack([x, x[:, 0:1]])
        self.x = x
        self.closed = closed
        self.s = np.arange(x.shape[1]) * 1
        self.gate_s = self.s
        self.smin, self.smax = self.s.min(), self.s.max()
        self.gate_shape = gate_shape
        self.gate_ri = gate_ri
        self.gate_snap_fit = gate_snap_fit
        self.gamma = gamma
        self.y_bounds, self.n_bounds = y_bounds, n_bounds
        bc = 'periodic' if closed else 'not-a-knot'
        self.center = scipy.interpolate.CubicSpline(self.s, x.T, bc_type=bc)
        self.xc_pw = [RefPwPoly(self.s, x[i], bc) for i in range(3)]
        # planar lateral fit
        s_fit = np.linspace(self.smin, self.smax, 100)
        es = self.center(s_fit, 1).T
        th = np.arctan2(es[1], es[0])
        for k in range(1, len(th)):
            while th[k] - th[k - 1] > np.pi:
                th[k] -= 2 * np.pi
            while th[k - 1] - th[k] > np.pi:
                th[k] += 2 * np.pi
        th = th + np.pi / 2
        thc = scipy.interpolate.CubicSpline(s_fit, th)
        thc = scipy.interpolate.CubicSpline(self.s, thc(self.s))
        th_fit = thc(s_fit)
        ry = np.array([np.cos(th_fit), np.sin(th_fit), th_fit * 0])
        if closed:
            ry[:, -1] = ry[:, 0]
        ry_grid = ry.T
        if np.linalg.norm(ry_grid[0] - ry_grid[-1]) < 1e-3:
            ry_grid[-1] = ry_grid[0]
            self.cleanly_closed = True
        else:
            self.cleanly_closed = False
        bc = 'periodic' if self.cleanly_closed else 'not-a-knot'
        self.ry_pw = [RefPwPoly(s_fit, ry_grid[:, i], bc) for i in range(3)]

    def param_terms(self, s):
        ''' [xc, xcs, xcss, ry, rys] at scalar s '''
        xc = np.array([p.val(s) for p in self.xc_pw])
        xcs = np.array([p.d1(s) for p in self.xc_pw])
        xcss = np.array([p.d2(s) for p in self.xc_pw])
        ry = np.array([p.val(s) for p in self.ry_pw])
        rys = np.array([p.d1(s) for p in self.ry_pw])
        return xc, xcs, xcss, ry, rys

    def frame(self, s):
        ''' dict with xc, es, ey, en, Rp, ks, ky, kn, mag at scalar s '''
        xc, xcs, xcss, ry, rys = self.param_terms(s)
        mag = np.sqrt(xcs @ xcs)
        es = xcs / mag
        ey = ry - es * (es @ ry)
        ey = ey / np.sqrt(ey @ ey)
        en = np.cross(es, ey)
        one = np.array([[xcs @ es, xcs @ ey], [ry @ es, ry @ ey]])
        kyks = np.linalg.inv(one) @ np.array([xcss @ en, rys @ en]) / mag
        kn = -(np.cross(xcss, xcs) @ en) / mag ** 3
        return {'xc': xc, 'es': es, 'ey': ey, 'en': en, 'Rp': np.stack([es, ey, en], axis=1),
                'ks': kyks[1], 'ky': -kyks[0], 'kn': kn, 'mag': mag}

    def gate_position(self, s):
        return self.frame(s)['xc']

    def gate_orientation(self, s):
        f = self.frame(s)
        es, ey, en = f['es'], f['ey'], f['en']
        if self.gate_snap_fit:
            if abs(es[2]) > 0.9:
                es = np.array([0, 0, 1])
                ey = ey - es * (ey.T @ es)
                ey = ey / np.linalg.norm(ey)
                en = np.cross(es, ey)
            elif abs(en[2]) > 0.9:
                en = np.array([0, 0, 1])
                es = es - en * (es.T @ en)
                es = es / np.linalg.norm(es)
                ey = np.cross(en, es)
        return np.array([es, ey, en]).T
