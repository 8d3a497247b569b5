'''
CPC trajectory data as a RacelineResults (drone3d/utils/cpc_utils.py:14-101), for comparison with
the solved racelines (scripts/race.py:51-54, scripts/fig_8_cpc.py).

The reference interpolates with CasADi pw_lin functions (utils/interp.py:8-15: one extra knot at
t_end + 1 repeating the last value, so values are held after the end and the first segment is
extrapolated before the start); LinearInterpolant restates that piecewise-linear map and its
derivative (the slope of the active segment, segments switching at t >= knot) with numpy.
'''
from typing import Tuple

import numpy as np
from scipy.interpolate import interp1d
from scipy.spatial.distance import cdist

from aircraft_trajectory_optimization_amd.centerlines.base_centerline import BaseCenterline
from aircraft_trajectory_optimization_amd.dynamics.dynamics_model import InterpolatedDynamicsModel
from aircraft_trajectory_optimization_amd.raceline.config import RacelineResults


class LinearInterpolant:
    ''' columns of d (M, n) linearly interpolated over t (M,) (interp.py:8-15 semantics) '''

    def __init__(self, t, d):
        t = np.asarray(t, float)
        d = np.asarray(d, float).reshape(len(t), -1)
        self.knots = np.concatenate([t, [t[-1] + 1.0]])
        self.vals = np.concatenate([d, d[-1:]], axis=0)
        self.slope = np.diff(self.vals, axis=0) / np.diff(self.knots)[:, None]

    def _segment(self, t):
        return int(np.searchsorted(self.knots[1:-1], t, side='right'))

    def __call__(self, t) -> np.ndarray:
        i = self._segment(float(t))
        return (self.vals[i] + self.slope[i] * (float(t) - self.knots[i])).squeeze()

    def derivative(self, t) -> np.ndarray:
        return self.slope[self._segment(float(t))].squeeze()


def package_cpc_data_as_raceline(file: str, line: BaseCenterline, clip: bool = True) \
        -> Tuple[RacelineResults, InterpolatedDynamicsModel]:
    ''' CSV columns t, p (3), q (w, x, y, z), v (3), w (3); clip=True extracts one lap '''
    model = InterpolatedDynamicsModel()
    data = np.genfromtxt(file, delimiter=',')[1:]
    t = data[:, 0]
    x = data[:, 1:4]
    q = data[:, [5, 6, 7, 4]]
    v = data[:, 8:11]
    w = data[:, 11:14]
    if clip:
        x0 = line.p2xc(line.s_min())
        i0 = int(cdist(x, x0[np.newaxis, :]).argmin())
        x_interp = interp1d(t, x.T)
        tp = np.linspace(t[i0 + 10], t.max(), 1000)
        tf = tp[np.array([np.linalg.norm(x[i0] - x_interp(tg)) for tg in tp]).argmin()]
        lap_time = tf - t[i0]
        i1 = np.searchsorted(t, tf) + 1
        t = t[i0:i1] - t[i0]
        x, q, v, w = x[i0:i1], q[i0:i1], v[i0:i1], w[i0:i1]
    else:
        lap_time = t[-1]
    z = np.hstack([x, q])
    u = np.hstack([v, w])
    states = []
    for tk, zk, uk in zip(t, z, u):
        st = model.get_empty_state()
        model.zu2state(st, zk, uk)
        st.t = tk
        states.append(st)
    zi = LinearInterpolant(t, z)
    ui = LinearInterpolant(t, u)
    return RacelineResults(solve_time=-1, ipopt_time=-1, feval_time=-1, feasible=True, states=states,
                           time=lap_time, label='CPC Data', color=[0.5, 0, 0.8, 1], z_interp=zi, u_interp=ui,
                           du_interp=ui.derivative, global_frame=True), model
