'''
Headless replacement of the reference's OpenGL viewer (drone3d/visualization/drone_raceline_fig.py:36,
opengl_fig.py:25): the same constructor and the calls the scripts make (ubo, add_object,
update_projection, run, draw, close), no window. It prints what the viewer's legend shows:
label, lap time, feasibility and the speed range of every raceline, and lists added objects.
Rendering is out of scope.
'''
from typing import Dict, List, Optional

import numpy as np


class UBOObject:
    ''' stand-in for the uniform buffer object objects are created against (objects.py:33) '''


class DroneRacelineWindow:
    ''' DroneRacelineWindow(line, models=None, results=None, obstacles=None, fullscreen, run) '''

    def __init__(self, line, models=None, results=None, *args, obstacles: Optional[Dict] = None,
                 run: bool = True, **kwargs):
        # pylint: disable=unused-argument
        self.line = line
        if results is None and len(args) > 0:
            results = args[0]
        if results is not None and not isinstance(results, (list, tuple)):
            results = [results]
        if models is not None and not isinstance(models, (list, tuple)):
            models = [models]
        self.models: List = list(models or [])
        self.results: List = list(results or [])
        self.obstacles: Dict = dict(obstacles or {})
        self.ubo = UBOObject()
        self.objects: Dict[str, object] = {}
        self.should_close = False
        for r in self.results:
            print(self.describe(r))
        for name in self.obstacles:
            print(f'[headless viewer] obstacle: {name}')
        if run:
            self.run()

    @staticmethod
    def describe(r) -> str:
        v: Optional[np.ndarray] = None
        if getattr(r, 'states', None):
            v = np.array([np.linalg.norm(s.v.to_vec()) for s in r.states])
        rng = f' speed {v.min():.2f}..{v.max():.2f} m/s' if v is not None else ''
        return f'[headless viewer] {r.label}: lap {r.time:.3f}s feasible={r.feasible}{rng}'

    def add_object(self, name: str, obj, show: bool = True):
        ''' register a drawable (opengl_fig.py add_object) '''
        self.objects[name] = obj
        print(f'[headless viewer] object: {name} (shown={show})')

    def update_projection(self):
        ''' no projection without a display '''

    def draw(self) -> bool:
        ''' one frame; the headless window closes immediately '''
        self.should_close = True
        return True

    def run(self):
        ''' the event loop: returns at once '''
        self.draw()

    def close(self):
        self.should_close = True
