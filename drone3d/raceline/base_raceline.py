''' drone3d.raceline.base_raceline (reference: drone3d/raceline/base_raceline.py:26-97) '''
from aircraft_trajectory_optimization_amd.raceline.config import GlobalRacelineConfig, \
    ParametricRacelineConfig, RacelineConfig, RacelineResults  # noqa: F401
from aircraft_trajectory_optimization_amd.raceline.solvers import _Raceline as BaseRaceline  # noqa: F401
