'''
ORACLE (test infrastructure only): the reference NLP transcription restated in numpy.

Each method cites the reference code it restates (drone3d/raceline/...). g(w) is built
row by row in the reference's order; the Jacobian is obtained by complex-step
differentiation of g, so it does not share any derivation with the product's
hand-written Jacobians.

  decision vector / guesses / bounds   base_raceline.py:670-750, :920-937, :1229-1251,
                                       drone_raceline.py:158-166
  collocation ODE rows                 base_raceline.py:398-434
  interval constraints                 base_raceline.py:436-451, :1114-1130
  continuity                           base_raceline.py:460-490, :1132-1181
  closure                              base_raceline.py:492-514, :1183-1227; drone_raceline.py:47-104
  open-line initial / terminal rows    base_raceline.py:359-361, :516-543; drone_raceline.py:110-148;
                                       point_raceline.py:15-45
  gates                                base_raceline.py:545-595, :891-918, :986-1032
  obstacle spheres                     obstacles/mesh_obstacle.py:219-237
  cost                                 base_raceline.py:601-623
  RK4 transcription (use_rk4)          base_raceline.py:226-230, :322-348, :363-391, :1034-1112;
                                       dynamics_model.py:91-114
'''
import numpy as np

from oracle.ref_collocation import coefficients, intermediate
from oracle import ref_models


def mv_(R, x):
    ''' (3,3[,B]) times (3,B) '''
    return ref_models.mv(R, x)

DRONE_DEFAULTS = dict(m=1.0, g=9.81, b1=0, b2=0, b3=0, collision_radius=0.3, I1=1e-3, I2=1e-3, I3=1.7e-3,
                      l=0.15, k=0.05, T_max=8.1, T_min=0.2, dT_max=20, dT_min=-20, bw1=1e-4, bw2=1e-4,
                      bw3=1e-4, w_max=10, w_min=-10)
POINT_DEFAULTS = dict(m=1.0, g=9.81, b1=0, b2=0, b3=0, collision_radius=0.3, T_max=32.4, T_min=-32.4,
                      dT_max=350, dT_min=-350)


class RefNLP:
    '''
    model: 'drone' | 'point'; frame: 'parametric' | 'global'.
    veh: vehicle parameter dict (defaults per pytypes.py:357-402) plus use_quat, global_r.
    spheres: optional (P, 3) table [dy, dn, available radius] for the obstacle rows.
    '''

    def __init__(self, line, model, frame, N, K, veh=None, closed=True, fix_gate_center=False,
                 R=1e-7, dR=1e-7, h0=1, v0=1, fixed_gates=None, force_regularity=True,
                 quat_flip=False, euler_wraps=0.0, spheres=None, rk4=False, cpc=None):
        self.line, self.model, self.frame = line, model, frame
        base = dict(DRONE_DEFAULTS if model == 'drone' else POINT_DEFAULTS)
        base.update(veh or {})
        self.veh = base
        self.use_quat = bool(base.get('use_quat', False)) if model == 'drone' else False
        # build-side DCM pose (config 5; not in the reference): attitude state R, row-major
        self.use_dcm = bool(base.get('use_dcm', False)) if model == 'drone' else False
        if self.use_dcm:
            self.use_quat = False
        self.att = 'dcm' if self.use_dcm else self.use_quat
        self.global_r = bool(base.get('global_r', False))
        if model == 'drone' and frame == 'global':
            self.global_r = True     # GlobalDroneRaceline._get_model (drone_raceline.py:314-316)
        self.nz = (18 if self.use_dcm else 13 if self.use_quat else 12) if model == 'drone' else 6
        self.nu = 4 if model == 'drone' else 3
        self.nv = self.nz + 2 * self.nu
        self.closed, self.fix_gate_center = closed, fix_gate_center
        self.h0, self.v0 = h0, v0
        self.fixed_gates, self.force_regularity = fixed_gates, force_regularity
        self.quat_flip, self.euler_wraps, self.spheres = quat_flip, euler_wraps, spheres
        # CPC gate progress (build-side, parity unpinned: the reference only displays a CPC
        # trajectory): {'waypoints': (M, 3), 'tol': d_tol}; global frame, no gate rows
        self.cpc = cpc
        self.Rm = np.eye(self.nu) * R if np.isscalar(R) else np.asarray(R)
        self.dRm = np.eye(self.nu) * dR if np.isscalar(dR) else np.asarray(dR)
        # BaseRaceline._setup_checks (base_raceline.py:226-230), run first by the global override
        self.rk4 = bool(rk4)
        if self.rk4:
            self.h0 = h0 = h0 / K
            N = N * K
            K = 0
        # BaseGlobalRaceline._setup_checks (base_raceline.py:873-885)
        if frame == 'global':
            x = np.array(line.x)
            if closed and not (x[:, 0] == x[:, -1]).all():
                x = np.hstack([x, x[:, 0:1]])
            phases = x.shape[1] - 1
            N = int(phases * np.ceil(N / phases))
            self.gate_n_interval = int(N / phases)
        self.N, self.K = N, K
        if self.rk4:
            self.tau, self.B, self.C, self.D = np.zeros(1), np.ones(1), np.zeros((1, 1)), np.ones(1)
        else:
            self.tau, self.B, self.C, self.D = coefficients(K)
        self.nw = N + N * (K + 1) * self.nv
        self.cpc_m = 0 if cpc is None else len(cpc['waypoints'])
        self.cpc_off = self.nw
        self.nw += N * (K + 1) * 3 * self.cpc_m
        self._geo_cache = {}
        self.lbg, self.ubg = None, None
        self.w0, self.lbw, self.ubw = self._decision_vector()
        _, self.lbg, self.ubg = self._build(self.w0[:, None], with_bounds=True)
        self.ng = len(self.lbg)

    # -------------------------------------------------------------- indexing
    def idx(self, n, k):
        return self.N + (n * (self.K + 1) + k) * self.nv

    def get_s(self, n, k):
        ''' base_raceline.py:972-984 '''
        ds = (self.line.smax - self.line.smin) / self.N
        return self.line.smin + ds * (n + self.tau[k])

    def geo(self, s):
        if s not in self._geo_cache:
            self._geo_cache[s] = self.line.frame(s)
        return self._geo_cache[s]

    def f_ode(self, z, u, s):
        if self.model == 'drone':
            return ref_models.drone_zdot(z, u, self.veh, self.att, self.frame, self.global_r,
                                         self.geo(s) if self.frame == 'parametric' else None)
        return ref_models.point_zdot(z, u, self.veh, self.frame, self.global_r,
                                     self.geo(s) if self.frame == 'parametric' else None)

    def rk4_step(self, z, u, h, s):
        ''' one RK4 step with u held and geometry frozen at s (dynamics_model.py:91-114,
        base_raceline.py:1071-1077) '''
        k1 = self.f_ode(z, u, s)
        k2 = self.f_ode(z + h / 2 * k1, u, s)
        k3 = self.f_ode(z + h / 2 * k2, u, s)
        k4 = self.f_ode(z + h * k3, u, s)
        return z + h / 6 * (k1 + k2 * 2 + k3 * 2 + k4)

    def continuity_op(self, z):
        ''' drone_raceline.py:42-45 '''
        if self.model == 'drone' and self.use_quat:
            z = z.copy()
            q = z[3:7]
            z[3:7] = q / np.sqrt(q[0] ** 2 + q[1] ** 2 + q[2] ** 2 + q[3] ** 2)
        if self.model == 'drone' and self.use_dcm:
            # build-side: one Newton-Schulz step towards SO(3), R (3 I - R^T R) / 2
            z = z.copy()
            R = ref_models.dcm_R(z[3:12])
            S = np.einsum('kib,kjb->ijb', R, R)
            P = 1.5 * R - 0.5 * np.einsum('ikb,kjb->ijb', R, S)
            z[3:12] = P.reshape(9, *P.shape[2:])
        return z

    # -------------------------------------------------------------- guesses and bounds
    def _guess_h(self, n):
        if self.h0:
            return self.h0
        if self.frame == 'parametric':
            ds = (self.line.smax - self.line.smin) / self.N
            return ds / self.v0 * self.geo(ds * n)['mag']
        return 1

    def _guess_z(self, n, k):
        z = [0.] * self.nz
        if self.frame == 'parametric':
            z[0] = self.get_s(n, k)
            if not self.global_r:
                z[3] = self.v0
            else:
                v = self.v0 * self.geo(self.get_s(n, k))['es']
                z[3], z[4], z[5] = v
        else:
            gate_no = n / self.gate_n_interval if self.rk4 else (n + k / self.K) / self.gate_n_interval
            xg = self.geo(gate_no)['xc']
            vg = self.geo(gate_no)['es']
            vg = vg / np.linalg.norm(vg) * self.v0
            z[0], z[1], z[2] = xg
            z[3], z[4], z[5] = vg
        if self.model == 'drone':
            if self.use_dcm:      # R of the ESP cold-start quaternion (1, 0, 0, 0)
                z = [*z[:3], 1, 0, 0, 0, -1, 0, 0, 0, -1, *z[3:6], 0, 0, 0]
            elif self.use_quat:
                z = [*z[:3], 1, 0, 0, 0, *z[3:6], 0, 0, 0]
            else:
                z = [*z[:3], 0, 0, 0, *z[3:6], 0, 0, 0]
            if self.frame == 'parametric':
                z[0] = self.get_s(n, k)
        return z

    def _state_bounds(self, s):
        v = self.veh
        inf = np.inf
        if self.model == 'drone':
            if self.use_dcm:
                ru, rl = [inf] * 9, [-inf] * 9
            elif self.use_quat:
                ru, rl = [inf] * 4, [-inf] * 4
            elif self.global_r:
                ru, rl = [inf, np.pi / 2.1, np.pi / 2.1], [-inf, -np.pi / 2.1, -np.pi / 2.1]
            else:
                ru, rl = [np.pi / 2, np.pi / 2.1, np.pi / 2.1], [-np.pi / 2, -np.pi / 2.1, -np.pi / 2.1]
            zu = [inf] * 3 + ru + [inf] * 3 + [v['w_max']] * 3
            zl = [-inf] * 3 + rl + [-inf] * 3 + [v['w_min']] * 3
        else:
            zu, zl = [inf] * 6, [-inf] * 6
        if self.frame == 'parametric':
            zu[0], zu[1], zu[2] = self.line.smax, self.line.y_bounds[1], self.line.n_bounds[1]
            zl[0], zl[1], zl[2] = self.line.smin, self.line.y_bounds[0], self.line.n_bounds[0]
        return zu, zl

    def _decision_vector(self):
        w0, lbw, ubw = [], [], []
        for n in range(self.N):
            h0 = self._guess_h(n)
            w0 += [h0]
            ubw += [h0 * 10]
            lbw += [h0 / 100]
        v = self.veh
        for n in range(self.N):
            for k in range(self.K + 1):
                zu, zl = self._state_bounds(self.get_s(n, k))
                w0 += self._guess_z(n, k) + [0.] * self.nu + [0.] * self.nu
                lbw += zl + [v['T_min']] * self.nu + [v['dT_min']] * self.nu
                ubw += zu + [v['T_max']] * self.nu + [v['dT_max']] * self.nu
        M = self.cpc_m
        for q in range(self.N * (self.K + 1)):
            if M:
                w0 += [1.] * M + [0.] * M + [0.] * M
                lbw += [0.] * 3 * M
                ubw += [1.] * 2 * M + [self.cpc['tol'] ** 2] * M
        return np.array(w0, float), np.array(lbw, float), np.array(ubw, float)

    # -------------------------------------------------------------- g(w)
    def _build(self, w, with_bounds=False):
        N, K, nz, nu = self.N, self.K, self.nz, self.nu
        C, D = self.C, self.D
        H = [w[n] for n in range(N)]
        Z = [[w[self.idx(n, k):self.idx(n, k) + nz] for k in range(K + 1)] for n in range(N)]
        U = [[w[self.idx(n, k) + nz:self.idx(n, k) + nz + nu] for k in range(K + 1)] for n in range(N)]
        dU = [[w[self.idx(n, k) + nz + nu:self.idx(n, k) + nz + 2 * nu] for k in range(K + 1)] for n in range(N)]
        g, lb, ub = [], [], []
        inf = np.inf

        def add(rows, lo, hi):
            rows = list(rows) if isinstance(rows, (list, tuple)) or np.ndim(rows) > 1 else [rows]
            for i, r in enumerate(rows):
                g.append(r)
                lb.append(lo[i] if isinstance(lo, (list, tuple)) else lo)
                ub.append(hi[i] if isinstance(hi, (list, tuple)) else hi)

        param = self.frame == 'parametric'
        # BaseGlobalRaceline._enforce_model: equal step sizes within a phase
        if not param:
            gi = N if self.cpc_m else self.gate_n_interval      # CPC: one total time
            for n in range(0, N, gi):
                for n2 in range(n + 1, n + gi):
                    add(H[n2] - H[n], 0., 0.)
        for n in range(N):
            if self.rk4:
                # _enforce_rk4_interval (base_raceline.py:363-391 global, :1052-1112 parametric)
                if param:
                    add(Z[n][0][0] - self.get_s(n, 0), 0., 0.)
                if n == N - 1:
                    continue
                zn = self.continuity_op(self.rk4_step(Z[n][0], U[n][0], H[n], self.get_s(n, 0)))
                un = U[n][0] + dU[n][0] * H[n] / 2
                if param:
                    add(Z[n + 1][0][1:] - zn[1:], 0., 0.)
                    add(U[n + 1][0] - un, 0., 0.)
                    add(zn[0] - self.get_s(n + 1, 0), 0., 0.)
                else:
                    add(Z[n + 1][0] - zn, 0., 0.)
                    add(U[n + 1][0] - un, 0., 0.)
                if self.model == 'point':
                    u_mag = sum(U[n][0][i] * U[n][0][i] for i in range(nu))
                    add(u_mag / self.veh['T_max'] / self.veh['T_max'], -inf, 1)
                if param and self.force_regularity:
                    gk = self.geo(self.get_s(n, 0))
                    if gk['ky'] ** 2 + gk['kn'] ** 2 > 0.1:
                        add(gk['kn'] * Z[n][0][1] - gk['ky'] * Z[n][0][2], -inf, self.line.gamma)
                continue
            # _enforce_collocation_interval_ode
            for k in range(K + 1):
                poly_ode = 0
                poly_du = 0
                for k2 in range(K + 1):
                    poly_ode = poly_ode + C[k2][k] * Z[n][k2] / H[n]
                    poly_du = poly_du + C[k2][k] * U[n][k2] / H[n]
                if param:
                    add(poly_ode[0], 0, inf)
                if k > 0:
                    func_ode = self.f_ode(Z[n][k], U[n][k], self.get_s(n, k))
                    add(func_ode - poly_ode, 0., 0.)
                add(dU[n][k] - poly_du, 0., 0.)
            # _enforce_collocation_interval_constraints
            if param and self.force_regularity:
                for k in range(K + 1):
                    gk = self.geo(self.get_s(n, k))
                    ky, kn = gk['ky'], gk['kn']
                    if ky ** 2 + kn ** 2 > 0.1:
                        add(kn * Z[n][k][1] - ky * Z[n][k][2], -inf, self.line.gamma)
            if self.model == 'point':
                for k in range(K + 1):
                    u_mag = sum(U[n][k][i] * U[n][k][i] for i in range(nu))   # u.T @ u
                    add(u_mag / self.veh['T_max'] / self.veh['T_max'], -inf, 1)
            # _enforce_collocation_interval_continuity
            if n >= 1:
                ps = 0
                pu = 0
                for k in range(K + 1):
                    ps = ps + Z[n - 1][k] * D[k]
                    pu = pu + U[n - 1][k] * D[k]
                ps = self.continuity_op(ps)
                if param:
                    add(Z[n][0][1:] - ps[1:], 0., 0.)
                else:
                    add(Z[n][0] - ps, 0., 0.)
                add(U[n][0] - pu, 0., 0.)
            if param:
                zN = 0
                for k in range(K + 1):
                    zN = zN + Z[n][k] * D[k]
                add(Z[n][0][0] - self.get_s(n, 0), 0., 0.)
                add(zN[0] - self.get_s(n + 1, 0), 0., 0.)

        def zF():
            if self.rk4:    # base_raceline.py:324-330, :1034-1050
                return self.continuity_op(self.rk4_step(Z[-1][0], U[-1][0], H[-1], self.get_s(N - 1, 0)))
            acc = 0
            for k in range(K + 1):
                acc = acc + Z[-1][k] * D[k]
            return self.continuity_op(acc)

        def uF():
            if self.rk4:    # full step, unlike the interval rows (F10; base_raceline.py:340-341)
                return U[-1][0] + dU[-1][0] * H[-1]
            acc = 0
            for k in range(K + 1):
                acc = acc + U[-1][k] * D[k]
            return acc

        if not self.closed:
            # _enforce_initial_constraints / _enforce_terminal_constraints, at Z[0,0] and _zF()
            for z, u in ((Z[0][0], U[0][0]), (zF(), uF())):
                vg, R = self._vg_R(z)
                add(vg[0] * vg[0] + vg[1] * vg[1] + vg[2] * vg[2], -inf, 0.)    # vg.T @ vg
                if self.model == 'drone':
                    add([R[0, 2], R[1, 2], R[2, 2]], [0., 0., 1.], [0., 0., 1.])  # e3 = R[:, 2]
                    add(z[-3:], 0., 0.)                                          # w_b
                else:
                    Tg = mv_(R, u)                                               # T = R @ Tb
                    add(Tg[0], 0., 0.)
                    add(Tg[1], 0., 0.)
        elif self.model == 'point':
            # base / parametric _enforce_loop_closure
            z0, u0, zf = Z[0][0], U[0][0], zF()
            add(uF() - u0, 0., 0.)
            if not param:
                add(zf - z0, 0., 0.)
            elif self.line.cleanly_closed:
                add(zf[1:] - z0[1:], 0., 0.)
            else:
                raise NotImplementedError('oracle: skew-closed point closure')

        # gates
        if param:
            fixed = self.fixed_gates
            if fixed is None:
                fixed = self.line.gate_s
                if self.line.smin in fixed and self.line.closed and self.closed:
                    fixed = np.array([s for s in fixed if s != self.line.smax])
            for s in fixed:
                s0 = self.get_s(0, 0)
                n = 0
                while not self.get_s(n + 1, 0) > s:
                    n += 1
                    s0 = self.get_s(n, 0)
                if n == N:
                    z_gate = zF()
                else:
                    sf = self.get_s(n + 1, 0)
                    d = (s - s0) / (sf - s0)
                    if self.rk4:
                        z_gate = Z[n][0] + d * (Z[n + 1][0] - Z[n][0])
                    else:
                        Dd = intermediate(K, d)
                        z_gate = 0
                        for k in range(K + 1):
                            z_gate = z_gate + Z[n][k] * Dd[k]
                gs = self.geo(s)
                x_gate = gs['xc'][:, None] + z_gate[1] * gs['ey'][:, None] + z_gate[2] * gs['en'][:, None]
                self._fix_gate(add, x_gate, s, False)
        elif not self.cpc_m:
            for gate_no, n in enumerate(range(0, N, self.gate_n_interval)):
                self._fix_gate(add, Z[n][0][:3], gate_no, True)
            if not self.closed:
                # final gate (base_raceline.py:914-918)
                self._fix_gate(add, zF()[:3], np.array(self.line.x).shape[1] - 1, True)

        if self.spheres is not None:
            for n in range(N):
                for k in range(K + 1):
                    dy, dn, r = self.spheres[n * (K + 1) + k]
                    z = Z[n][k]
                    add((z[1] - dy) ** 2 + (z[2] - dn) ** 2, -inf, max(r, 0) ** 2)

        if self.cpc_m:
            # CPC gate progress (Foehn et al. 2021), node by node in time order: complementarity
            # mu_j (|p - w_j|^2 - nu_j) = 0, order lambda_j <= lambda_{j+1}, progress
            # lambda_{q+1} = lambda_q - mu_q
            M, P = self.cpc_m, N * (K + 1)
            wp = np.asarray(self.cpc['waypoints'], float)
            blk = [w[self.cpc_off + 3 * M * q:self.cpc_off + 3 * M * (q + 1)] for q in range(P)]
            for q in range(P):
                z = Z[q // (K + 1)][q % (K + 1)]
                lam, mu, nu = blk[q][:M], blk[q][M:2 * M], blk[q][2 * M:]
                for j in range(M):
                    d2 = (z[0] - wp[j, 0]) ** 2 + (z[1] - wp[j, 1]) ** 2 + (z[2] - wp[j, 2]) ** 2 - nu[j]
                    add(mu[j] * d2, 0., 0.)
                for j in range(M - 1):
                    add(lam[j] - lam[j + 1], -inf, 0.)
                if q + 1 < P:
                    for j in range(M):
                        add(blk[q + 1][j] - lam[j] + mu[j], 0., 0.)

        if self.model == 'drone' and self.closed:
            # DroneRaceline._enforce_modified_loop_closure (only for closed lines, drone_raceline.py:153)
            z0, u0 = Z[0][0], U[0][0]
            zf, uf = zF(), uF()
            zd = zf - z0
            add(uf - u0, 0., 0.)
            if self.use_dcm:
                add(zd[1:3], 0., 0.)
                add(zd[12:], 0., 0.)
                add(zf[3:12] - z0[3:12], 0., 0.)
            elif self.use_quat:
                add(zd[1:3], 0., 0.)
                add(zd[7:], 0., 0.)
                if self.quat_flip:
                    add(zf[3:7] + z0[3:7], 0., 0.)
                else:
                    add(zf[3:7] - z0[3:7], 0., 0.)
            else:
                add(zd[1:3], 0., 0.)
                add(zd[4:], 0., 0.)
                add(zd[3] - 2 * np.pi * self.euler_wraps, 0., 0.)
            if not param:
                add(zd[0], 0., 0.)
        out = np.array(g)
        if with_bounds:
            return out, np.array(lb, float), np.array(ub, float)
        return out

    def _vg_R(self, z):
        ''' f_vg and f_R of the model (global / global_r attitude; point mass: R = I) '''
        if self.model == 'drone':
            if not (self.frame == 'global' or self.global_r):
                raise NotImplementedError('oracle: open lines with the relative attitude')
            return ref_models.drone_vg_R(z, self.att, self.frame, self.global_r)
        if self.frame == 'parametric' and not self.global_r:
            raise NotImplementedError('oracle: open lines with the relative attitude')
        R = np.eye(3)
        return z[3:6], R

    def _fix_gate(self, add, x_var, s, axial):
        ''' base_raceline.py:545-595 '''
        inf = np.inf
        gate_x = self.geo(s)['xc'][:, None]
        if self.fix_gate_center:
            add(x_var - gate_x, 0., 0.)
            return
        R = self.line.gate_orientation(s)
        d_max = self.line.gate_ri - self.veh['collision_radius']
        if self.line.gate_shape == 'circle':
            e1, e2, e3 = R[:, 0], R[:, 1], R[:, 2]
            dx = x_var - gate_x
            r_sq = (e2 @ dx) ** 2 + (e3 @ dx) ** 2
            add(r_sq, -inf, d_max ** 2)
            if axial:
                add(e1 @ x_var - gate_x[:, 0] @ e1, 0., 0.)
        else:
            delta = R.T @ (x_var - gate_x)
            if axial:
                add(delta, [0., -d_max, -d_max], [0., d_max, d_max])
            else:
                add(delta[1:], -d_max, d_max)

    # -------------------------------------------------------------- public evaluation
    def g(self, w):
        ''' w: (nw,) or (nw, B) -> (ng,) or (ng, B) '''
        w = np.asarray(w)
        single = w.ndim == 1
        out = self._build(w[:, None] if single else w)
        return out[:, 0] if single else out

    def f(self, w):
        ''' cost J (base_raceline.py:601-623) '''
        w = np.asarray(w)
        single = w.ndim == 1
        w2 = w[:, None] if single else w
        J = 0
        for n in range(self.N):
            for k in range(self.K + 1):
                i = self.idx(n, k)
                u = w2[i + self.nz:i + self.nz + self.nu]
                du = w2[i + self.nz + self.nu:i + self.nz + 2 * self.nu]
                L = np.einsum('ib,ij,jb->b', u, self.Rm, u) + np.einsum('ib,ij,jb->b', du, self.dRm, du) + 1
                J = J + L * w2[n] * self.B[k]
        return J[0] if single else J

    def jac_dense(self, w, h=1e-30, chunk=512):
        ''' dense dg/dw (ng, nw) by complex step '''
        w = np.asarray(w, float)
        cols = []
        for c0 in range(0, self.nw, chunk):
            c1 = min(self.nw, c0 + chunk)
            W = np.repeat(w[:, None], c1 - c0, axis=1).astype(complex)
            W[np.arange(c0, c1), np.arange(c1 - c0)] += 1j * h
            cols.append(np.imag(self._build(W)) / h)
        return np.concatenate(cols, axis=1)

    def jvp(self, w, V, h=1e-30):
        ''' dg/dw @ V for V (nw, m) by complex step '''
        W = (np.asarray(w, float)[:, None] + 1j * h * np.asarray(V, float)).astype(complex)
        return np.imag(self._build(W)) / h

    def grad_f(self, w, h=1e-30):
        ''' dense df/dw by complex step '''
        w = np.asarray(w, float)
        W = np.repeat(w[:, None], self.nw, axis=1).astype(complex)
        W[np.arange(self.nw), np.arange(self.nw)] += 1j * h
        return np.imag(self.f(W)) / h

    # -------------------------------------------------------------- Hessian of the Lagrangian (checker)
    def grad_lagrangian(self, w, lam, sigma, h=1e-30, chunk=256):
        ''' sigma grad f + J^T lam by complex step of sigma f + lam^T g (w real) '''
        w = np.asarray(w, float)
        out = np.zeros(self.nw)
        for c0 in range(0, self.nw, chunk):
            c1 = min(self.nw, c0 + chunk)
            W = np.repeat(w[:, None], c1 - c0, axis=1).astype(complex)
            W[np.arange(c0, c1), np.arange(c1 - c0)] += 1j * h
            L = sigma * self.f(W) + np.asarray(lam, float) @ self._build(W)
            out[c0:c1] = np.imag(L) / h
        return out

    def hvp(self, w, lam, sigma, V, eps=1e-5):
        ''' (sigma grad^2 f + sum lam_i grad^2 g_i) V by central differences of the exact
        (complex-step) Lagrangian gradient; truncation error O(eps^2) '''
        V = np.atleast_2d(np.asarray(V, float).T).T
        cols = []
        for j in range(V.shape[1]):
            gp = self.grad_lagrangian(w + eps * V[:, j], lam, sigma)
            gm = self.grad_lagrangian(w - eps * V[:, j], lam, sigma)
            cols.append((gp - gm) / (2 * eps))
        return np.stack(cols, axis=1)
