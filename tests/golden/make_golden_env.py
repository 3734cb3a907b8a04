"""Golden vectors for the env step's manager semantics, produced by the REFERENCE's own mdp code.

Run in the development container (the reference is mounted read-only at /root/reference; it never
travels to the GPU box):

    python tests/golden/make_golden_env.py

One teacher-forced step of N envs per training stage (0, 1, 2) from a seeded, deliberately eventful
pre-step state (drones near their gates, near the ground, tilted past 90 deg, at the last step of their
episode, with accumulated-gate counts on both sides of the curriculum thresholds).  The step is composed
in the order of ManagerBasedDiffRLEnv.step (extensions/diff.lab/diff/lab/envs/manager_based_diff_rl_env.py:
160-267) from the reference's own code, loaded from its source files with Isaac Lab stand-ins
(tests/golden/il_shim.py):

  action manager (IL, restated: prev <- action <- a)            -> DiffActions.process_actions
      (mdp/diff_action.py:156-206: lag, tanh scale/offset, thrust-estimate error, CTBRController.compute,
       DroneDynamics.step)   [the DroneDynamics step stands in for PhysX, as in the build's default]
  episode_length_buf += 1; terminations: IL time_out (restated), bad_pose / out_of_bound (mdp/termination.py)
      and the contact term (IL illegal_contact over PhysX contact forces: fed the build's lattice count,
      which is "parity unpinned" itself)
  rewards: progress_reward_mine, command_body_rate_penalty, command_rate_penalty, perception_reward,
      success_cross, penalize_bad_pose (mdp/rewards.py:154-253) with the stage's weights
      (racing_ctbr_env.py:281-328), summed f * w * dt in declaration order (IL RewardManager, restated)
  reset of done envs: racing_terrain_levels (IL TerrainImporter.update_env_origins restated) and
      racing_cmd_noise_levels -> RacingCommand.update_noise_level (mdp/curriculums.py, commands.py:385-402);
      IL CommandTerm.reset (metrics to 0, restated) -> RacingCommand._resample_command (commands.py:262-306)
  command compute: RacingCommand._update_metrics + _update_command (commands.py:247-260, 308-350)
  observations: modified_base_lin_vel, base_orientation_r, modified_generated_commands(_gt),
      modified_last_action, cross_obs (mdp/observation.py), group order racing_ctbr_env.py:138-169

Random draws cannot be shared with the reference (torch's stateful generators), so observation noise and
gate-pose noise are off in these vectors (the build's obs_noise / add_gate_noise switches), and the reset
state of a done env (random in both) is not recorded: for done envs only the curriculum (level, noise
level) and the command reset (start gate, zero accumulated gates) are compared.  Every recorded env is
kept away from the discrete thresholds (gate radius 0.35 m, |roll| = pi/2, the stage-0 height bounds, the
collision lattice) by more than the reference/build round-off, by resampling the envs that are not.

The gate table comes from the build's own track generator (seed 42, 8 gates, no obstacles; positions
relative to the env origin, as the reference's terrain.extras["gate_pose"]); it is stored in the fixture
and the tests check the build's table against it.  Env origins: x = y = 0, z = the track's origin height.
"""
from __future__ import annotations

import os
import sys
from types import SimpleNamespace as NS

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import il_shim  # noqa: E402

OUT = os.path.join(HERE, "golden_env.npz")
N = 1024
NT, NL, G = 20, 10, 8
DT = 0.01 * 3  # sim.dt * decimation, a python double as in the reference
MASS0 = 0.6
J0 = [0.0015, 0.002, 0.004]
STAGE_WEIGHTS = {  # racing_ctbr_env.py:281-328: (progress, bodyrate, action_rate, collision, perception, success, bad)
    0: (1.0, -0.02, -0.01, -50.0, 0.1, 10.0, None),
    1: (1.0, -0.1, -0.05, -100.0, 0.1, 20.0, -30.0),
    2: (1.0, -0.1, -0.05, -100.0, 0.1, 20.0, None),
}


class CTBRCfg:
    """CTBRControllerCfg fields for the racing task (racing_ctbr_env.py:127-134 over controller_diff_cfg.py)."""

    arm_length = 0.09
    kappa = 0.016
    motor_tau = 0.0001
    motor_omega = (150, 3000)
    thrustmap = [1.3298253500372892e-06, 0.0038360810526746033, -1.7689986848125325]
    g = 9.81
    use_motor_model = False
    thrust_ctrl_delay = 0.03
    torque_ctrl_delay = (0.03, 0.03, 0.03)
    body_rate_bound = [-6, 6]
    rate_gain_p = [35, 35, 35]
    rate_gain_i = [0.0, 0.0, 0.0]
    rate_gain_d = [0.0005, 0.0005, 0.0003]


def tables():
    from generalizableracing_amd.envs.tracks import build_tracks

    gates, recs, _ = build_tracks(num_types=NT, num_levels=NL, num_gates=G, seed=42, obstacles=False)
    gate_pose = np.zeros((NT, NL, G, 7), np.float32)
    gate_pose[..., :3] = gates[:, :, 0:3].reshape(NT, NL, G, 3)
    gate_pose[..., 3] = 1.0  # orientations are not on the observation path (commands use [:3] only)
    start = recs[:, 2].astype(np.int64).reshape(NT, NL)
    origin_z = recs[:, 1].reshape(NT, NL)
    return gates, recs, gate_pose, start, origin_z


def sample_state(rng, idx, st, gate_pose, origin_z, stage):
    """Fill the pre-step state of envs `idx` (in place in the dict of arrays `st`)."""
    m = len(idx)
    t, lv = st["type"][idx], rng.integers(0, NL, m)
    st["level"][idx] = lv
    gid = rng.integers(0, G, m)
    st["gate_id"][idx] = gid
    gpos = gate_pose[t, lv, gid, :3].astype(np.float64)
    kind = rng.choice(4, m, p=[0.4, 0.3, 0.15, 0.15])
    dirs = rng.normal(size=(m, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    p = gpos + rng.uniform(-4, 4, (m, 3)) * np.array([1, 1, 0.3])
    near = kind == 0
    p[near] = gpos[near] + dirs[near] * rng.uniform(0.05, 0.8, (near.sum(), 1))
    low = kind == 2
    ground = -origin_z[t, lv]
    p[low, 2] = ground[low] + rng.uniform(-0.06, 0.25, low.sum())
    if stage == 0:  # out_of_bound (0, 10) m in the world frame: some below 0 and above 10
        hi = rng.random(m) < 0.05
        p[hi, 2] = 10.0 - origin_z[t, lv][hi] + rng.uniform(-0.3, 0.3, hi.sum())
    roll = rng.uniform(-0.5, 0.5, m)
    tilt = kind == 3
    roll[tilt] = rng.choice([-1, 1], tilt.sum()) * rng.uniform(1.2, 2.0, tilt.sum())
    pitch, yaw = rng.uniform(-0.5, 0.5, m), rng.uniform(-np.pi, np.pi, m)
    q = il_shim.quat_from_euler_xyz(*(torch.tensor(x, dtype=torch.float32) for x in (roll, pitch, yaw))).numpy()
    v = rng.normal(0, 1.5, (m, 3))
    v[near] = (gpos[near] - p[near]) / np.linalg.norm(gpos[near] - p[near], axis=1, keepdims=True) * \
        rng.uniform(0.5, 4.0, (near.sum(), 1))
    st["p"][idx] = p
    st["q"][idx] = q
    st["v"][idx] = v
    st["w"][idx] = rng.normal(0, 1.0, (m, 3))
    st["alpha"][idx] = rng.normal(0, 8.0, (m, 3))
    st["T"][idx] = rng.uniform(2.0, 14.0, m)
    st["tau"][idx] = rng.normal(0, 0.005, (m, 3))
    st["a_prev"][idx] = rng.normal(0, 1.0, (m, 4))
    st["a"][idx] = rng.normal(0, 1.0, (m, 4))
    st["thr_err"][idx] = 1.0 + rng.normal(0, 0.02, m)
    st["m_ctrl"][idx] = MASS0 + rng.uniform(-0.02, 0.02, m)
    st["m_plant"][idx] = MASS0 + rng.uniform(-0.02, 0.02, m)
    st["J"][idx] = np.array(J0) * rng.uniform(0.9, 1.1, (m, 3))
    z = 4.0 + rng.uniform(0, 0.4, m)
    k2 = 0.01 * st["m_ctrl"][idx][:, None] + rng.uniform(0, 0.005, (m, 3))
    k1 = 0.18 * st["m_ctrl"][idx][:, None] + rng.uniform(0, 0.1, (m, 3))
    k2[:, 2] *= z
    k1[:, 2] *= z
    st["k2"][idx], st["k1"][idx] = k2, k1
    st["Kp"][idx] = 35.0 * rng.uniform(0.9, 1.1, (m, 3))
    st["Kd"][idx] = np.array([5e-4, 5e-4, 3e-4]) * rng.uniform(0.9, 1.1, (m, 3))
    st["dT"][idx] = 0.03 * rng.uniform(0.8, 1.3, m)
    st["dtau"][idx] = 0.03 * rng.uniform(0.8, 1.3, (m, 3))
    ep = rng.integers(0, 199, m)
    ep[rng.random(m) < 0.08] = 199  # time-out at this step
    if stage == 2:
        ep[ep == 199] = 266
    st["ep_len"][idx] = ep
    st["acc"][idx] = rng.integers(0, 7, m)
    st["noise_level"][idx] = rng.uniform(0.8, 1.25, m)


class Scene(dict):
    pass


def reference_step(st, stage, gate_pose, start, origin_z, collide, carry=False, noise=None):
    """One step of the reference composition from pre-state `st` (dict of numpy arrays).  carry=True also returns
    what the next step of a free run starts from (make_golden_freerun.py): the controller's filter state and the
    body angular acceleration of the DroneDynamics step (the D-term input the simulator reports next step).
    noise (make_golden_noise.py part G): the gate-pose and observation noise on, with injected draws: noise.gu_pre
    [n, 6] = the noise of the gates each env holds, noise.gu_new / gu_rst = the draws of an update (gate passed) /
    a resample (reset), noise.nz [n, 6] = the observation noise."""
    mdp = il_shim.load_mdp()
    DroneDynamics = mdp["droneDynamics"].DroneDynamics
    DiffActions = mdp["diff_action"].DiffActions
    R, O, Tm, Cu, Cm = mdp["rewards"], mdp["observation"], mdp["termination"], mdp["curriculums"], mdp["commands"]
    CTBRController = sys.modules["diff.lab.controllers"].CTBRController
    f32 = lambda x: torch.tensor(np.asarray(x), dtype=torch.float32)  # noqa: E731
    n = len(st["p"])
    types, levels = torch.tensor(st["type"], dtype=torch.long), torch.tensor(st["level"], dtype=torch.long)
    gp = torch.tensor(gate_pose)
    origins = torch.zeros(n, 3)
    origins[:, 2] = f32(origin_z)[types, levels]
    q = f32(st["q"])
    # the simulator state in the world frame (IL root_state_w); angular velocity / acceleration given in the body
    # frame are handed over in the world frame, as PhysX reports them
    p_w = f32(st["p"]) + origins
    w_w = il_shim.quat_rotate(q, f32(st["w"]))
    alpha_w = il_shim.quat_rotate(q, f32(st["alpha"]))
    data = NS(root_state_w=torch.cat([p_w, q, f32(st["v"]), w_w], 1), body_lin_acc_w=torch.zeros(n, 1, 3),
              body_ang_acc_w=alpha_w[:, None, :])
    robot = NS(data=data)
    terrain = NS(extras={"gate_pose": gp, "next_gate_id": torch.tensor(start)}, terrain_types=types,
                 terrain_levels=levels.clone(), max_terrain_level=NL,
                 cfg=NS(terrain_generator=NS(sub_terrains={"circular": NS(num_gate=G)})))

    def update_env_origins(env_ids, move_up, move_down):  # IL TerrainImporter.update_env_origins (restated)
        terrain.terrain_levels[env_ids] += 1 * move_up - 1 * move_down
        lv = terrain.terrain_levels[env_ids]
        terrain.terrain_levels[env_ids] = torch.where(lv >= terrain.max_terrain_level, -1, torch.clip(lv, 0))
        # (the random level IL draws for lv >= max is marked -1 here: not comparable)

    terrain.update_env_origins = update_env_origins
    scene = Scene(robot=robot)
    scene.terrain, scene.env_origins, scene.device = terrain, origins, "cpu"
    env = NS(num_envs=n, device="cpu", scene=scene, cfg=NS(sim=NS(dt=0.01, gravity=(0.0, 0.0, -9.81)), decimation=3))

    # ---- action manager + DiffActions (the term is built without IL's __init__; fields as __init__ sets them)
    da = DiffActions.__new__(DiffActions)
    da.cfg = NS(sim2real_test=False, max_thrust_weight_ratio=3.0, action_lag=1, random_drag=False)
    da.env, da.robot, da.num_envs, da.device = env, robot, n, "cpu"
    da.dt = env.cfg.sim.dt * env.cfg.decimation
    da.command_type = "CTBRController"
    da.controller_cfg = CTBRCfg()
    da._robot_mass = f32(st["m_ctrl"])
    da._robot_weight = da._robot_mass * abs(env.cfg.sim.gravity[2])
    da._get_scale_factor()
    inertia = torch.tensor(J0).diag().unsqueeze(0).repeat(n, 1, 1)
    ctl = CTBRController(CTBRCfg(), n, "cpu", da._robot_mass, inertia, da.dt)
    ctl.rate_gain_p, ctl.rate_gain_d = f32(st["Kp"]), f32(st["Kd"])
    ctl.thrust_ctrl_delay, ctl.torque_ctrl_delay = f32(st["dT"])[:, None], f32(st["dtau"])
    ctl.gross_thrust, ctl.torque = f32(st["T"])[:, None], f32(st["tau"])
    da.controller = ctl
    plant_J = torch.diag_embed(f32(st["J"]))
    dd = DroneDynamics(n, f32(st["m_plant"]), plant_J, da.dt, 3, random_drag=False, device="cpu")
    dd.drag_coeffs, dd.h_force_drag_coeffs = f32(st["k2"]), f32(st["k1"])
    da.drone_dynamics = dd
    if carry:  # record DroneDynamics.step's input wrench and pre-step body rate (droneDynamics.py:119-135)
        dd_step = dd.step

        def step_rec(tt):
            step_rec.tt, step_rec.wb = tt.clone(), dd.ang_vel_b.clone()
            return dd_step(tt)

        dd.step = step_rec
    da.thr_est_error = f32(st["thr_err"])
    da.action_lag = 1
    a_prev, a = f32(st["a_prev"]), f32(st["a"])
    da.action_buffer = [a_prev.clone()]
    da.force_rotors, da.torque_rotors = torch.zeros(n, 4, 3), torch.zeros(n, 4, 3)
    da.torque_body = torch.zeros(n, 1, 3)
    da._raw_actions = torch.zeros(n, 4)
    # DiffActions.reset_idx -> DroneDynamics.reset_state from the simulator state (env-local frame)
    s0 = da.get_state_from_sim()
    dd.reset_state(torch.cat([s0["pos"], s0["quat"], s0["lin_vel_w"], s0["ang_vel_w"]], 1), torch.arange(n))
    pre = {"p": s0["pos"].clone(), "w": dd.ang_vel_b.clone(), "alpha": s0["ang_acc_b"].clone()}
    am = NS(action=a.clone(), prev_action=a_prev.clone(), get_term=lambda name: da)  # IL ActionManager.process_action
    env.action_manager = am
    da.process_actions(a)
    # ---- the simulator after the step = DroneDynamics' state (world = local + origin)
    p_l, q_n, v_n, wb_n, ww_n = dd.pos, dd.quat, dd.lin_vel_w, dd.ang_vel_b, dd.ang_vel_w
    data.root_state_w = torch.cat([p_l + origins, q_n, v_n, ww_n], 1)
    data.root_pos_w, data.root_quat_w = data.root_state_w[:, :3], q_n
    data.root_lin_vel_w, data.root_ang_vel_w = v_n, ww_n
    data.root_lin_vel_b = data.root_com_lin_vel_b = il_shim.quat_rotate_inverse(q_n, v_n)
    data.root_ang_vel_b = il_shim.quat_rotate_inverse(q_n, ww_n)
    post = {"p": p_l.clone(), "q": q_n.clone(), "v": v_n.clone(), "w": wb_n.clone()}
    env.episode_length_buf = torch.tensor(st["ep_len"], dtype=torch.long) + 1
    max_len = 267 if stage == 2 else 200

    # ---- command term (RacingCommand without IL's __init__; fields as __init__ sets them)
    cmd = Cm.RacingCommand.__new__(Cm.RacingCommand)
    cmd.cfg = NS(consecutive_commands=True, add_noise=noise is not None, make_quat_unique=False, update_threshold=0.35)
    cmd.robot, cmd.env, cmd.num_envs, cmd.device = robot, env, n, "cpu"
    cmd.gate_pose = gp
    cmd.gate_id = torch.tensor(st["gate_id"], dtype=torch.long)
    cmd.next_gate_id = (cmd.gate_id + 1) % G
    pos = gp[types, levels, cmd.gate_id, :3] + origins
    npos = gp[types, levels, cmd.next_gate_id, :3] + origins
    quat = gp[types, levels, cmd.gate_id, 3:]
    cmd.gate_pose_w = torch.cat([pos, quat], 1)
    cmd.gate_pose_gt_w = cmd.gate_pose_w.clone()
    cmd.next_gate_pose_w = torch.cat([npos, quat], 1)
    cmd.next_gate_pose_gt_w = cmd.next_gate_pose_w.clone()
    cmd.metrics = {"accumulate_gates": torch.tensor(st["acc"], dtype=torch.float32), "action_rate": torch.zeros(n),
                   "avg_lin_spd": torch.zeros(n), "avg_ang_spd": torch.zeros(n)}
    nl = f32(st["noise_level"])[:, None]
    for nm in ("pos_x", "pos_y", "pos_z", "roll", "pitch", "yaw"):
        setattr(cmd, f"noise_range_{nm}", torch.tensor([[-0.1, 0.1]]).repeat(n, 1) * nl)
    cmd.noise_level = nl.clone()
    if noise is not None:  # the noisy gates the envs hold from before the step (their (episode, gates passed) draws)
        u = torch.tensor(noise.gu_pre, dtype=torch.float32)
        for k, nm in enumerate(("pos_x", "pos_y", "pos_z")):
            rg = getattr(cmd, f"noise_range_{nm}")
            cmd.gate_pose_w[:, k] += rg[:, 0] + u[:, k] * (rg[:, 1] - rg[:, 0])
            cmd.next_gate_pose_w[:, k] += rg[:, 0] + u[:, 3 + k] * (rg[:, 1] - rg[:, 0])
        gq = il_shim.Queue()
        cm_torch = Cm.torch
        Cm.torch = il_shim.TorchProxy(empty=lambda *size, device=None, **kw: il_shim.ScriptedUniform(
            gq, il_shim.size_of(size)[0]))
    env.command_manager = NS(get_term=lambda name: cmd, _terms={"next_gate_pose": cmd},
                             get_command=lambda name: cmd.command)

    # ---- terminations (IL TerminationManager: OR of the terms; time_outs = the time_out term)
    time_out = env.episode_length_buf >= max_len
    count = torch.tensor([collide(int(types[i] * NL + levels[i]), p_l[i].numpy(), q_n[i].numpy()) for i in range(n)])
    contact = count > 0
    if stage == 0:
        terminated = Tm.out_of_bound(env, bounds=(0.00, 10.0))
    else:
        terminated = contact | Tm.bad_pose(env)
    dones = terminated | time_out

    # ---- rewards (IL RewardManager: value = f * w * dt, summed in declaration order)
    w = STAGE_WEIGHTS[stage]
    f = [R.progress_reward_mine(env, "next_gate_pose"), R.command_body_rate_penalty(env, "force_torque"),
         R.command_rate_penalty(env, "force_torque"),
         (count > 2).float() if stage == 0 else contact.float(),  # collision_penalty_custom / undesired_contacts
         R.perception_reward(env, "next_gate_pose"), R.success_cross(env, "next_gate_pose", threshold=0.35),
         R.penalize_bad_pose(env).float() if w[6] is not None else torch.zeros(n)]
    reward = torch.zeros(n)
    names, step_reward = [], []
    for k, (fk, wk) in enumerate(zip(f, w)):
        if wk is None:
            continue
        value = fk * wk * DT
        reward += value
        names.append(["progress_rewards", "command_bodyrate_penalty", "action_rate", "collision_penalty",
                       "perception_reward", "success_cross", "bad_pose_penalty"][k])
        step_reward.append(value / DT)
    env.reward_manager = NS(_step_reward=torch.stack(step_reward, 1), _term_names=names)

    # ---- reset of the done envs: curriculum, then the command manager's reset
    ids = dones.nonzero(as_tuple=False).squeeze(-1)
    if len(ids):
        Cu.racing_terrain_levels(env, ids, "next_gate_pose", 3, 2)
        if stage == 1:
            Cu.racing_cmd_noise_levels(env, ids, "next_gate_pose", 4, 3, 0.02, 0.03)
        for v in cmd.metrics.values():  # IL CommandTerm.reset
            v[ids] = 0.0
        lv_ok = terrain.terrain_levels[ids] >= 0
        lv_tmp = terrain.terrain_levels.clone()
        lv_tmp[ids[~lv_ok]] = 0  # (the random level is not comparable; any level serves the resample)
        terrain.terrain_levels = lv_tmp
        if noise is not None:
            il_shim.push_gate_noise(gq, noise.gu_rst[ids.numpy()])
        cmd._resample_command(ids)
        terrain.terrain_levels[ids[~lv_ok]] = -1
    reset_gate = cmd.gate_id.clone()
    # ---- command compute: metrics, then gate progress (commands.py:247-260, 308-350)
    cmd._update_metrics()
    if noise is not None:  # the envs _update_command will draw for (commands.py:309-310)
        hit = torch.norm(cmd.gate_pose_gt_w[:, :3] - data.root_state_w[:, :3], dim=-1) < cmd.cfg.update_threshold
        if hit.any():
            il_shim.push_gate_noise(gq, noise.gu_new[hit.numpy()])
    cmd._update_command()
    if noise is not None:
        Cm.torch = cm_torch
        gq.done()
    # ---- observations (noise-free policy group unless `noise`: then the injected observation noise)
    if noise is None:
        pol = torch.cat([O.modified_base_lin_vel(env, add_noise=False), O.base_orientation_r(env, add_noise=False),
                         O.modified_generated_commands(env, "next_gate_pose"),
                         O.modified_last_action(env, "force_torque")], 1)
    else:
        z = torch.tensor(noise.nz, dtype=torch.float32)
        o_torch = O.torch
        O.torch = il_shim.TorchProxy(randn_like=lambda x, **kw: z[:, 0:3].clone(),
                                     randn=lambda *size, device=None, **kw: z[:, 3:6].clone())
        try:
            pol = torch.cat([O.modified_base_lin_vel(env, add_noise=True), O.base_orientation_r(env, add_noise=True),
                             O.modified_generated_commands(env, "next_gate_pose"),
                             O.modified_last_action(env, "force_torque")], 1)
        finally:
            O.torch = o_torch
    cri = torch.cat([O.modified_base_lin_vel(env, add_noise=False), O.base_orientation_r(env, add_noise=False),
                     O.modified_generated_commands_gt(env, "next_gate_pose"),
                     O.modified_last_action(env, "force_torque")], 1)
    aux = O.cross_obs(env, "success_cross")
    out = {"reward": reward, "f": torch.stack(f, 1), "terminated": terminated, "time_out": time_out, "dones": dones,
           "count": count, "post_p": post["p"], "post_q": post["q"], "post_v": post["v"], "post_w": post["w"],
           "gate_id_after": cmd.gate_id, "gate_id_reset": reset_gate,
           "acc_after": cmd.metrics["accumulate_gates"], "level_after": terrain.terrain_levels,
           "noise_level_after": cmd.noise_level[:, 0], "obs_policy": pol, "obs_critic": cri, "obs_aux": aux[:, 0]}
    if carry:
        tq, wb = step_rec.tt[:, 1:4], step_rec.wb
        # alpha as DroneDynamics.step forms it from its own inertia matrices (droneDynamics.py:123)
        jw = (dd.inertia @ wb.unsqueeze(-1)).squeeze(-1)
        out["alpha_b"] = (dd.inertia_inv @ tq.unsqueeze(-1)).squeeze(-1) - \
            (dd.inertia_inv @ torch.linalg.cross(wb, jw).unsqueeze(-1)).squeeze(-1)
        out["ctrl_T"], out["ctrl_tau"] = ctl.gross_thrust[:, 0].clone(), ctl.torque.clone()
    return {k: v.detach().numpy() for k, v in out.items()}, {k: v.detach().numpy() for k, v in pre.items()}


def margins_ok(st, res, gate_pose, origin_z, stage, collide):
    """Envs whose discrete outcomes sit further from every threshold than round-off could move them."""
    n = len(st["p"])
    t, lv = st["type"], st["level"]
    ok = np.ones(n, bool)
    p, q = res["post_p"].astype(np.float64), res["post_q"].astype(np.float64)
    g = gate_pose[t, lv, st["gate_id"], :3]
    d = np.linalg.norm(g - p, axis=1)
    ok &= np.abs(d - 0.35) > 1e-4
    gn = gate_pose[t, lv, (st["gate_id"] + 1) % G, :3]  # after a pass the next gate's distance decides nothing
    cos_roll = 1 - 2 * (q[:, 1] ** 2 + q[:, 2] ** 2)
    ok &= np.abs(cos_roll) > 1e-4
    ok &= np.abs(2 * (q[:, 0] * q[:, 2] - q[:, 3] * q[:, 1])) < 0.9999
    zw = p[:, 2] + origin_z[t, lv]
    ok &= (np.abs(zw) > 1e-4) & (np.abs(zw - 10.0) > 1e-4)
    vb = res["obs_critic"][:, 0:3]
    ok &= np.linalg.norm(vb, axis=1) > 1e-3
    ok &= np.linalg.norm(res["obs_critic"][:, 6:9], axis=1) > 1e-3
    rng = np.random.default_rng(0)
    for i in np.nonzero(ok)[0]:
        k = int(t[i] * NL + lv[i])
        c0 = res["count"][i]
        for _ in range(4):
            dp = rng.uniform(-3e-6, 3e-6, 3)
            dq = res["post_q"][i] + rng.uniform(-3e-7, 3e-7, 4)
            if collide(k, (p[i] + dp).astype(np.float32), dq.astype(np.float32)) != c0:
                ok[i] = False
                break
    del gn
    return ok


def main():
    import oracle
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg

    gates, recs, gate_pose, start, origin_z = tables()
    out = {"gate_pos": gate_pose[..., :3], "start_gate": start.astype(np.int32), "origin_z": origin_z}
    for stage in (0, 1, 2):
        cfg = RacingEnvCfg(scene=SceneCfg(num_envs=N), sim=SimCfg(device="cpu"), stage=stage,
                           terrain=TerrainCfg(obstacles=False)).to_gr_config()
        orc = oracle.Oracle(cfg, gates, recs)
        collide = orc.collision_count
        rng = np.random.default_rng(100 + stage)
        st = {k: np.zeros((N,) + s, np.float64) for k, s in (
            ("p", (3,)), ("q", (4,)), ("v", (3,)), ("w", (3,)), ("alpha", (3,)), ("T", ()), ("tau", (3,)),
            ("a_prev", (4,)), ("a", (4,)), ("thr_err", ()), ("m_ctrl", ()), ("m_plant", ()), ("J", (3,)),
            ("k2", (3,)), ("k1", (3,)), ("Kp", (3,)), ("Kd", (3,)), ("dT", ()), ("dtau", (3,)),
            ("noise_level", ()))}
        for k in ("type", "level", "gate_id", "ep_len", "acc"):
            st[k] = np.zeros(N, np.int64)
        # IL TerrainImporter: terrain_types = floor(arange(N) / (N / num_cols))
        st["type"][:] = torch.div(torch.arange(N), N / NT, rounding_mode="floor").long().numpy()
        todo = np.arange(N)
        for it in range(50):
            sample_state(rng, todo, st, gate_pose, origin_z, stage)
            for k in st:
                if st[k].dtype == np.float64:
                    st[k] = st[k].astype(np.float32).astype(np.float64)
            res, pre = reference_step(st, stage, gate_pose, start, origin_z, collide)
            todo = np.nonzero(~margins_ok(st, res, gate_pose, origin_z, stage, collide))[0]
            if len(todo) == 0:
                break
        assert len(todo) == 0, f"stage {stage}: {len(todo)} envs still near a threshold"
        # the state the reference actually stepped from (local position, body rates, D-term input)
        for k in ("p", "w", "alpha"):
            st[k] = pre[k]
        # the controller's delay filters as the reference evaluates them each step: exp(-dt / delay), fp32
        st["cT"] = torch.exp(-DT / torch.tensor(st["dT"], dtype=torch.float32)).numpy()
        st["ctau"] = torch.exp(-DT / torch.tensor(st["dtau"], dtype=torch.float32)).numpy()
        for k, v in st.items():
            out[f"s{stage}_in_{k}"] = v
        for k, v in res.items():
            out[f"s{stage}_out_{k}"] = v
        d = res["dones"].astype(bool)
        print(f"stage {stage}: {len(todo)} left after {it + 1} rounds; dones {d.sum()}, terminated "
              f"{res['terminated'].sum()}, time_out {res['time_out'].sum()}, contact {(res['count'] > 0).sum()}, "
              f"passes {(res['gate_id_after'] != st['gate_id'])[~d].sum()}, success>0 {(res['obs_aux'] > 0).sum()}")
    conv = {}
    for k, v in out.items():
        v = np.asarray(v)
        if v.dtype == np.float64:
            v = v.astype(np.float32)
        elif v.dtype == np.bool_:
            v = v.astype(np.uint8)
        elif v.dtype == np.int64:
            v = v.astype(np.int32)
        conv[k] = np.ascontiguousarray(v)
    np.savez_compressed(OUT, **conv)
    print(f"wrote {OUT}: {sum(v.nbytes for v in conv.values()) / 1e3:.1f} kB raw, {len(conv)} arrays")


if __name__ == "__main__":
    main()
