"""manipulator_mujoco_amd — MI355X-native sampling-MPC rollout engine (UR5e).

Drop-in for the reference's ``cem_planner`` / ``run_cem_planner`` call surface
(alinjar1996/manipulator_mujoco, sampling_based_planner/mjx_planner.py and
mpc_planner.py).  The hot path (basis -> H physics steps -> cost -> best) runs
as hand-written HIP behind the C ABI in ``include/mpcr.h``.
"""

__version__ = "0.1.0"
