'''
ORACLE -- TEST INFRASTRUCTURE ONLY.

A CPU (numpy, fp64) restatement of the reference's raceline NLP transcription, written
independently of the product code, used as the parity checker for the HIP library.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it;
the product package (aircraft_trajectory_optimization_amd) never does.

  ref_geometry.py       spline centreline, Darboux frame, curvatures, gate pose
  ref_collocation.py    Legendre tau, B, C, D
  ref_models.py         drone / point-mass ODEs (complex-step safe)
  ref_transcription.py  g(w), bounds, cost, w0 in reference order; Jacobian by complex step

Pinning (see DESIGN.md "Oracle"): the reference's own path needs CasADi/IPOPT, which are
not installed, so the reference cannot be run here. The oracle is pinned by
  * golden vectors produced by importing the reference's drone3d.pytypes
    (quaternion / Euler rotation and rate formulas, config defaults) -> tests/golden/,
  * the collocation root table values quoted from the reference build (K = 4),
  * the reference's own kinematic-consistency test (tests/test_kinematics.py) restated
    with the oracle's ODE and scipy integration,
  * complex-step differentiation (Jacobians are exact to rounding, not hand-derived).
IPOPT lap-time parity is unpinned (no IPOPT here).
'''
