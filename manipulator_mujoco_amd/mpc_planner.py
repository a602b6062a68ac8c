"""Headless closed-loop MPC driver (reference: SBP/mpc_planner.py:14-314).

``run_cem_planner`` keeps the reference's keyword arguments, target-switching
logic, printed status line, CSV names and returned dict.  What differs:

* the plant (``cem.data`` + ``mujoco.mj_step`` on CPU in the reference,
  :109-114,179-180) is ``engine.Plant``: the same model stepped on the GPU by
  the rollout kernel (n = 1, H = 1, fp32 state resident on the device);
* the reference's only implemented branch drives a passive OpenGL viewer
  (:146-233) and its headless branch is a stub (:234-236).  Here the loop is
  headless and runs ``max_ticks`` ticks (the viewer loop ran until the window
  closed); ``show_viewer`` is accepted and ignored.
* target bodies are read from the compiled model (``model.body(name).pos /
  .quat``, :124-125,157-158); the reference's writes to ``target_0``'s body
  pose (:165-166,219-220) go to a host-side override table, since they only
  ever change what later ticks read as the target.
"""

from __future__ import annotations

import argparse
import os
import time

import numpy as np

from .engine import Plant
from .planner import cem_planner
from .quat_math import quaternion_distance


class _Bodies:
    """``model.body(name).pos / .quat`` with the reference's writes kept host-side."""

    def __init__(self, model):
        self._names = list(model.names["body"])
        self._pos = {n: np.array(model.body_pos[i], dtype=np.float64) for i, n in enumerate(self._names)}
        self._quat = {n: np.array(model.body_quat[i], dtype=np.float64) for i, n in enumerate(self._names)}

    def pos(self, name):
        return self._pos[name].copy()

    def quat(self, name):
        return self._quat[name].copy()

    def set(self, name, pos, quat):
        self._pos[name] = np.array(pos, dtype=np.float64)
        self._quat[name] = np.array(quat, dtype=np.float64)

    def __contains__(self, name):
        return name in self._pos


def run_cem_planner(num_dof=None, num_batch=None, num_steps=None, maxiter_cem=None, maxiter_projection=None,
                    w_pos=None, w_rot=None, w_col=None, num_elite=None, timestep=None, initial_qpos=None,
                    target_names=None, show_viewer=None, cam_distance=None, show_contact_points=None,
                    position_threshold=None, rotation_threshold=None, save_data=None, data_dir=None,
                    stop_at_final_target=None, *, max_ticks=100, model_path=None, device=None, graph=True,
                    verbose=True, planner_kwargs=None):
    """Run the CEM planner in closed loop for ``max_ticks`` ticks (headless)."""
    if initial_qpos is None:
        initial_qpos = [1.5, -1.8, 1.75, -1.25, -1.6, 0]
    if target_names is None:
        target_names = ["target_0", "target_1", "home"]
    if position_threshold is None:
        position_threshold = 0.04
    if rotation_threshold is None:
        rotation_threshold = 0.3
    if stop_at_final_target is None:
        stop_at_final_target = True
    if save_data:
        os.makedirs(data_dir, exist_ok=True)
    log = print if verbose else (lambda *a, **k: None)

    start_time = time.time()
    cem = cem_planner(num_dof=num_dof, num_batch=num_batch, num_steps=num_steps, maxiter_cem=maxiter_cem,
                      w_pos=w_pos, w_rot=w_rot, w_col=w_col, num_elite=num_elite, timestep=timestep,
                      maxiter_projection=maxiter_projection, model_path=model_path, device=device, graph=graph,
                      verbose=verbose, **({"return_rollouts": False} | (planner_kwargs or {})))
    log(f"Initialized CEM Planner: {round(time.time() - start_time, 2)}s")

    model = cem.model
    data = Plant(model, device=cem.device.index)
    cem.data = data
    bodies = _Bodies(model)

    qpos = data.qpos.copy()
    qpos[np.asarray(model.ctrl_qposadr[:num_dof])] = np.asarray(initial_qpos, dtype=np.float64)
    data.set_state(qpos=qpos)
    data.forward()
    ctrl_q = np.asarray(model.ctrl_qposadr[:num_dof])
    ctrl_v = np.asarray(model.ctrl_dofadr[:num_dof])

    xi_mean = np.zeros(cem.nvar)
    init_position = data.site_xpos_tcp
    init_rotation = data.xquat_hande

    target_pos = bodies.pos(target_names[0])
    target_rot = bodies.quat(target_names[0])
    start_time = time.time()
    _ = cem.compute_cem(xi_mean, data.qpos[ctrl_q], data.qvel[ctrl_v], data.qacc[ctrl_v], target_pos, target_rot)
    log(f"Compute CEM: {round(time.time() - start_time, 2)}s")

    thetadot = np.zeros(num_dof)
    cost_g_list, cost_list, cost_r_list, cost_c_list, thetadot_list, theta_list = [], [], [], [], [], []
    step_ms, eef_dist = [], []
    target_idx = 0
    current_target = target_names[target_idx]
    if show_viewer:
        log("No viewer on this build: running the closed loop headless")

    for _tick in range(int(max_ticks)):
        t0 = time.time()
        if current_target != "home":
            target_pos = bodies.pos(current_target)
            target_rot = bodies.quat(current_target)
        else:
            target_pos = init_position
            target_rot = init_rotation
        if current_target == "target_1" and "target_0" in target_names:
            bodies.set("target_0", data.site_xpos_tcp, data.xquat_hande)

        cost, best_cost_g, best_cost_r, best_cost_c, best_vels, best_traj, xi_mean, _, _ = cem.compute_cem(
            xi_mean, data.qpos[ctrl_q], data.qvel[ctrl_v], data.qacc[ctrl_v], target_pos, target_rot)

        thetadot = np.mean(best_vels[1:num_steps - 2], axis=0)
        data.step(thetadot)

        current_cost_g = np.linalg.norm(data.site_xpos_tcp - target_pos)
        current_cost_r = quaternion_distance(data.xquat_hande, target_rot)
        current_cost = np.round(cost, 2)
        step_ms.append((time.time() - t0) * 1000)
        eef_dist.append(float(current_cost_g))
        log(f'Step Time: {"%.0f" % step_ms[-1]}ms | Cost g: {"%.2f" % (float(current_cost_g))}'
            f' | Cost r: {"%.2f" % (float(current_cost_r))} | Cost c: {"%.2f" % (float(best_cost_c))}'
            f' | Cost: {current_cost}')
        log(f"eef_quat: {data.xquat_hande}")
        log(f"target: {current_target}")

        if current_cost_g < position_threshold and current_cost_r < rotation_threshold:
            if target_idx == len(target_names) - 1:
                if stop_at_final_target:
                    log(f"Reached final target: {current_target}. Stopping motion.")
                    thetadot = np.zeros(num_dof)
                    qvel = data.qvel.copy()
                    qvel[ctrl_v] = thetadot
                    data.set_state(qvel=qvel)
                else:
                    target_idx = 0
                    current_target = target_names[target_idx]
                    log(f"Reached final target. Looping back to first target: {current_target}")
            else:
                target_idx = target_idx + 1
                current_target = target_names[target_idx]
                log(f"Moving to next target: {current_target}")
            if current_target == "home" and "target_0" in target_names:
                bodies.set("target_0", data.site_xpos_tcp, data.xquat_hande)

        cost_g_list.append(best_cost_g)
        cost_r_list.append(best_cost_r)
        cost_c_list.append(best_cost_c)
        thetadot_list.append(thetadot)
        theta_list.append(data.qpos[ctrl_q].copy())
        cost_list.append(current_cost[-1] if isinstance(current_cost, np.ndarray) else current_cost)

    if save_data:
        np.savetxt(f"{data_dir}/costs.csv", cost_list, delimiter=",")
        np.savetxt(f"{data_dir}/thetadot.csv", thetadot_list, delimiter=",")
        np.savetxt(f"{data_dir}/theta.csv", theta_list, delimiter=",")
        np.savetxt(f"{data_dir}/cost_g.csv", cost_g_list, delimiter=",")
        np.savetxt(f"{data_dir}/cost_r.csv", cost_r_list, delimiter=",")
        np.savetxt(f"{data_dir}/cost_c.csv", cost_c_list, delimiter=",")

    return {"cost_g": cost_g_list, "cost_r": cost_r_list, "cost_c": cost_c_list, "cost": cost_list,
            "thetadot": thetadot_list, "theta": theta_list, "step_ms": step_ms, "eef_dist": eef_dist, "target": current_target}


def main(argv=None):  # SBP/mpc_planner.py:256-314
    parser = argparse.ArgumentParser(description="Run CEM planner with configurable parameters (headless)")
    parser.add_argument("--num_dof", type=int, default=6)
    parser.add_argument("--num_batch", type=int, default=1000)
    parser.add_argument("--num_steps", type=int, default=16)
    parser.add_argument("--maxiter_cem", type=int, default=1)
    parser.add_argument("--maxiter_projection", type=int, default=10)
    parser.add_argument("--w_pos", type=float, default=20.0)
    parser.add_argument("--w_rot", type=float, default=3.0)
    parser.add_argument("--w_col", type=float, default=10.0)
    parser.add_argument("--num_elite", type=float, default=0.05)
    parser.add_argument("--timestep", type=float, default=0.05)
    parser.add_argument("--initial_qpos", type=float, nargs="+", default=None)
    parser.add_argument("--no_viewer", action="store_true")
    parser.add_argument("--cam_distance", type=float, default=4)
    parser.add_argument("--no_contact_points", action="store_true")
    parser.add_argument("--position_threshold", type=float, default=0.04)
    parser.add_argument("--rotation_threshold", type=float, default=0.3)
    parser.add_argument("--targets", type=str, nargs="+", default=None)
    parser.add_argument("--save_data", action="store_true")
    parser.add_argument("--data_dir", type=str, default="data")
    parser.add_argument("--continue_after_final", action="store_true")
    parser.add_argument("--max_ticks", type=int, default=100)
    parser.add_argument("--model", type=str, default=None, help="MJCF path or bundled model name")
    parser.add_argument("--no_graph", action="store_true")
    a = parser.parse_args(argv)
    return run_cem_planner(num_dof=a.num_dof, num_batch=a.num_batch, num_steps=a.num_steps,
                           maxiter_cem=a.maxiter_cem, maxiter_projection=a.maxiter_projection, w_pos=a.w_pos,
                           w_rot=a.w_rot, w_col=a.w_col, num_elite=a.num_elite, timestep=a.timestep,
                           initial_qpos=a.initial_qpos, target_names=a.targets, show_viewer=not a.no_viewer,
                           cam_distance=a.cam_distance, show_contact_points=not a.no_contact_points,
                           position_threshold=a.position_threshold, rotation_threshold=a.rotation_threshold,
                           save_data=a.save_data, data_dir=a.data_dir,
                           stop_at_final_target=not a.continue_after_final, max_ticks=a.max_ticks,
                           model_path=a.model, graph=not a.no_graph)


if __name__ == "__main__":
    main()
