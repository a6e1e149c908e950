"""Restated constants of the reference (test infrastructure only, see oracle/__init__.py).

Every value cites the reference line it follows; tests/test_oracle_golden.py checks them
against tests/golden/params.json, which tests/golden/make_golden.py produced by importing
the reference's own `src/params.py`.
"""
import math

# DroneData (src/params.py:37-61)
GRAVITY_ACC = 9.81                      # params.py:37
MASS = 0.03277                          # params.py:42 (overrides the URDF mass 0.027)
GRAVITY = GRAVITY_ACC * MASS            # params.py:45
MAX_F = 1.3 * GRAVITY                   # params.py:46
MIN_F = -0.2 * GRAVITY                  # params.py:47
MIN_P_X, MAX_P_X = -1.2, 1.2            # params.py:48-49
MIN_P_Z, MAX_P_Z = -1.2, 1.2            # params.py:50-51
MIN_V_X, MAX_V_X = -1.0, 1.0            # params.py:52-53
MIN_V_Z, MAX_V_Z = -1.0, 1.0            # params.py:54-55
MIN_A_X, MAX_A_X = -5.0, 5.0            # params.py:56-57
MIN_A_Z, MAX_A_Z = -5 + GRAVITY_ACC, 5 + GRAVITY_ACC   # params.py:58-59
MIN_JERK, MAX_JERK = -5.0, 5.0          # params.py:60-61

# URDF-derived values (src/cf2x.urdf via params.py:72-110), used only by the synthetic quad13
L_ARM = 0.0397
KF = 3.16e-10
KM = 7.94e-12
THRUST2WEIGHT = 2.25
J_DIAG = (1.4e-05, 1.4e-05, 2.17e-05)

# ExperimentParameters (src/params.py:113-122)
T = 10                                  # params.py:115
DT = 1 / 50                             # params.py:116
DT_CONV = 1 / 500                       # params.py:117
CTRLS_PER_SAMPLE = int(DT / DT_CONV)    # params.py:118
N_SIM = int(T / DT)                     # params.py:119
N_HORIZON = 30                          # params.py:121
NOISE = 0.01                            # params.py:122

# Stage-cost weights (force_model/ocp.py:38-43, jerk_model/ocp.py:37-42)
W_X_FORCE = (1e2, 1e2, 1e0, 1e0)
W_X_JERK = (1e2, 1e2, 1e0, 1e0, 0.0, 0.0)
W_U = 1e-1
# closed-loop cost weights (force_model/controller.py:40-41, jerk_model/controller.py:40-41)
W_CL = (1e2, 1e2, 1e0, 1e0)

assert CTRLS_PER_SAMPLE == 10 and N_SIM == 500
assert math.isclose(MAX_F, 0.41791581, rel_tol=1e-12)
