'''
Headless replacement of the reference's OpenGL viewer (drone3d/visualization/drone_raceline_fig.py:36):
same constructor, no window. It prints what the viewer's legend shows: label, lap time,
feasibility and the speed range of every raceline. Rendering is out of scope.
'''
from typing import List, Optional

import numpy as np


class DroneRacelineWindow:
    ''' DroneRacelineWindow(line, models=None, results=None, ...) without a display '''

    def __init__(self, line, models=None, results=None, *args, **kwargs):
        self.line = line
        if results is None and len(args) > 0:
            results = args[0]
        if results is not None and not isinstance(results, (list, tuple)):
            results = [results]
        self.results: List = list(results or [])
        for r in self.results:
            print(self.describe(r))

    @staticmethod
    def describe(r) -> str:
        v: Optional[np.ndarray] = None
        if getattr(r, 'states', None):
            v = np.array([np.linalg.norm(s.v.to_vec()) for s in r.states])
        rng = f' speed {v.min():.2f}..{v.max():.2f} m/s' if v is not None else ''
        return f'[headless viewer] {r.label}: lap {r.time:.3f}s feasible={r.feasible}{rng}'
