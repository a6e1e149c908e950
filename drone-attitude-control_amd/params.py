"""Drone / experiment constants used by the engine's model builders.

Mirrors `src/params.py` of the reference (DroneData :10-110, ExperimentParameters :113-122);
values are checked against tests/golden/params.json (generated from the reference module).
"""
import math


class DroneData:
    """src/params.py:10-70 (only what the hot path and its callers use)."""

    def __init__(self):
        self.GRAVITY_ACC = 9.81                       # :37
        self.MASS = 0.03277                           # :42
        self.GRAVITY = self.GRAVITY_ACC * self.MASS   # :45
        self.max_F = 1.3 * self.GRAVITY               # :46
        self.min_F = -0.2 * self.GRAVITY              # :47
        self.min_p_x, self.max_p_x = -1.2, 1.2        # :48-49
        self.min_p_z, self.max_p_z = -1.2, 1.2        # :50-51
        self.min_v_x, self.max_v_x = -1, 1            # :52-53
        self.min_v_z, self.max_v_z = -1, 1            # :54-55
        self.min_a_x, self.max_a_x = -5, 5            # :56-57
        self.min_a_z = -5 + self.GRAVITY_ACC          # :58
        self.max_a_z = 5 + self.GRAVITY_ACC           # :59
        self.min_jerk, self.max_jerk = -5, 5          # :60-61
        # cf2x.urdf values parsed at :72-110 (used by the synthetic quad13 model)
        self.L = 0.0397
        self.KF = 3.16e-10
        self.KM = 7.94e-12
        self.THRUST2WEIGHT_RATIO = 2.25
        self.J_diag = (1.4e-05, 1.4e-05, 2.17e-05)


class ExperimentParameters:
    """src/params.py:113-122."""

    def __init__(self):
        self.T = 10
        self.dt = 1 / 50
        self.dt_conv = 1 / 500
        self.ctrls_per_sample = int(self.dt / self.dt_conv)
        self.N = int(self.T / self.dt)
        self.N_conv = int(self.T / self.dt_conv)
        self.N_horizon = 30
        self.noise = 0.01


assert math.isclose(DroneData().max_F, 0.41791581, rel_tol=1e-12)
