"""Golden vectors with the random draws ON, produced by the REFERENCE's own startup-DR, reset, command and observation
code with the BUILD's draws injected in place of torch's.

Run in the development container (the reference is mounted read-only at /root/reference; it never travels to the
GPU box):

    python tests/golden/make_golden_noise.py

torch's stateful generators cannot be reproduced by any re-implementation, so the other fixtures run with the noise
off and hold the draws only to distributions (tests/test_gpu_distributions.py).  What CAN be pinned is the arithmetic
that APPLIES a draw: here every torch.rand / randn / randn_like / uniform_ / sample_uniform call site on the path is fed
the value the build's Philox stream produces for that env, episode and call counter (oracle.draws, the same
gr_rng.h the kernels use), and the reference's own functions compute the result.  Injected call sites:

  part S, startup (gr_init; events.py:30-137, diff_action.py:86):
    randomize_rate_controller_gain_and_thrust_delay  torch.rand -> Kp, (Ki: unused, 0.5), Kd, thrust / torque delays
    randomize_articulation_mass_and_inertia          sample_uniform -> mass add; torch.rand -> inertia scales
                                                     (diagonal entries; the others multiply zeros)
    DiffActions.__init__ thr_est_error               torch.randn (the one line restated: 1 + z * 0.02)
  part R, reset of every env from a varied state (gr_reset; manager_based_diff_rl_env.py:362-410 order):
    racing_terrain_levels -> IL update_env_origins   (restated; a level past the top draws the build's level)
    racing_cmd_noise_levels                          (no draw)
    reset_root_state_racing                          sample_uniform x 2 -> pose (x y z roll pitch yaw), velocity
    DiffActions.reset_idx -> DroneDynamics.reset_idx torch.rand -> z drag, k2, k1; torch.randn -> thrust error
    CommandTerm.reset -> _resample_command           uniform_ x 12 -> gate / next-gate position noise (orientation
                                                     noise draws 0.5: zero angle; gate orientations are not observed)
    observation (policy / critic groups)             randn_like -> velocity noise; randn -> attitude euler noise
  part G, one step with gate passes (gr_step; make_golden_env.reference_step with the noise on):
    _update_command                                  uniform_ -> the new gate / next-gate noise of passing envs
    observation                                      as in part R (counter of the step)
    (the noisy gates an env holds from before the step: gate + the build's noise of its (episode, gates passed))

Outputs are compared within 1e-5 (tests/test_oracle_noise_golden.py on the oracle, tests/test_gpu_noise_golden.py on
the kernel).  Env origins: x = y = 0, z = the track's origin height (as make_golden_env.py).
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
import make_golden_env as GE  # noqa: E402

OUT = os.path.join(HERE, "golden_noise.npz")
N = 512
NT, NL, G = GE.NT, GE.NL, GE.G
DT = GE.DT
f32 = lambda x: torch.tensor(np.asarray(x), dtype=torch.float32)  # noqa: E731


TorchProxy, Queue, _Uniform, _sz, push_gate_noise = (il_shim.TorchProxy, il_shim.Queue, il_shim.ScriptedUniform,
                                                     il_shim.size_of, il_shim.push_gate_noise)


def patch(mod, **over):
    old = mod.torch
    mod.torch = TorchProxy(**over)
    return old


# ------------------------------------------------------------------------------------------------ part S
def reference_startup(dr):
    """Startup DR of N envs from the build's startup draws dr [N, 16] (oracle.draws kind 3)."""
    mdp = il_shim.load_mdp()
    Ev = mdp["events"]
    CTBRController = sys.modules["diff.lab.controllers"].CTBRController
    n = len(dr)
    d = torch.tensor(dr)
    ctl = CTBRController(GE.CTBRCfg(), n, "cpu", torch.full((n,), GE.MASS0),
                         torch.tensor(GE.J0).diag().unsqueeze(0).repeat(n, 1, 1), DT)
    da = NS(controller=ctl)
    q = Queue()
    q.push(d[:, 0:3])                     # Kp
    q.push(torch.full((n, 3), 0.5))       # Ki (unused by the CTBR controller; consumes a draw in the reference)
    q.push(d[:, 3:6])                     # Kd
    q.push(d[:, 6:7])                     # thrust delay
    q.push(d[:, 7:10])                    # torque delays
    scale = torch.full((n, 1, 9), 0.5)    # inertia: diagonal entries 0, 4, 8
    scale[:, 0, 0], scale[:, 0, 4], scale[:, 0, 8] = d[:, 11], d[:, 12], d[:, 13]
    q.push(scale)

    def rand(*size, device=None, **kw):
        return q.take(_sz(size))

    old = patch(Ev, rand=rand)
    asset = Ev.Articulation()  # (the class events.py imported)
    masses = torch.full((n, 1), GE.MASS0)
    inertias = torch.zeros(n, 1, 9)
    inertias[:, 0, 0], inertias[:, 0, 4], inertias[:, 0, 8] = GE.J0
    view = NS(get_masses=lambda: masses.clone(), get_inertias=lambda: inertias.clone(), out={})
    view.set_masses = lambda m, ids: view.out.__setitem__("m", m.clone())
    view.set_inertias = lambda i, ids: view.out.__setitem__("J", i.clone())
    asset.root_physx_view = view
    asset.num_bodies = 1
    asset.data = NS(default_mass=masses.clone(), default_inertia=inertias.clone())
    scene = GE.Scene(robot=asset)
    scene.num_envs = n
    env = NS(scene=scene, device="cpu", num_envs=n, action_manager=NS(get_term=lambda name: da))
    try:
        Ev.randomize_rate_controller_gain_and_thrust_delay(env, None, "force_torque", (0.9, 1.1), (0.8, 1.3))
        il_shim.SAMPLE_HOOK = lambda size: Queue([d[:, 10:11]]).take(size)  # mass add (n, 1 body)
        Ev.randomize_articulation_mass_and_inertia(env, None, il_shim.SceneEntityCfg("robot", body_names="body"),
                                                   (-0.02, 0.02), "add", "uniform", (0.9, 1.1), "scale", "uniform")
    finally:
        il_shim.SAMPLE_HOOK = None
        Ev.torch = old
    q.done()
    J = view.out["J"][:, 0]
    return {
        "Kp": ctl.rate_gain_p, "Kd": ctl.rate_gain_d,
        # the controller's delay filters as CTBRController.compute evaluates them (controller_diff.py:131-139)
        "cT": torch.exp(-ctl.dt / ctl.thrust_ctrl_delay)[:, 0], "ctau": torch.exp(-ctl.dt / ctl.torque_ctrl_delay),
        "m_plant": view.out["m"][:, 0], "J": torch.stack([J[:, 0], J[:, 4], J[:, 8]], 1),
        # diff_action.py:86 thr_est_error = 1 + torch.randn(num_envs) * 0.02
        "thr_err": 1 + d[:, 15] * 0.02,
    }


# ------------------------------------------------------------------------------------------------ shared pieces
def make_cmd(mdp, env, robot, gp, gate_id, origins, types, levels, noise_level, gate_u_pre=None):
    """RacingCommand without IL's __init__ (fields as __init__ sets them), noise on.  gate_u_pre [n, 6]: the noise
    draws of the gates each env holds (gate x y z, next gate x y z), applied as the reference holds them."""
    Cm = mdp["commands"]
    n = len(gate_id)
    cmd = Cm.RacingCommand.__new__(Cm.RacingCommand)
    cmd.cfg = NS(consecutive_commands=True, add_noise=True, make_quat_unique=False, update_threshold=0.35)
    cmd.robot, cmd.env, cmd.num_envs, cmd.device = robot, env, n, "cpu"
    cmd.gate_pose = gp
    cmd.gate_id = torch.tensor(gate_id, dtype=torch.long)
    cmd.next_gate_id = (cmd.gate_id + 1) % G
    pos = gp[types, levels, cmd.gate_id, :3] + origins
    npos = gp[types, levels, cmd.next_gate_id, :3] + origins
    quat = gp[types, levels, cmd.gate_id, 3:]
    cmd.gate_pose_gt_w = torch.cat([pos, quat], 1)
    cmd.next_gate_pose_gt_w = torch.cat([npos, quat], 1)
    cmd.gate_pose_w = cmd.gate_pose_gt_w.clone()
    cmd.next_gate_pose_w = cmd.next_gate_pose_gt_w.clone()
    nl = f32(noise_level)[:, None]
    for nm in ("pos_x", "pos_y", "pos_z", "roll", "pitch", "yaw"):
        setattr(cmd, f"noise_range_{nm}", torch.tensor([[-0.1, 0.1]]).repeat(n, 1) * nl)
    cmd.noise_level = nl.clone()
    if gate_u_pre is not None:  # the position noise these envs drew when their gates were last resampled / updated
        u = f32(gate_u_pre)
        for k, nm in enumerate(("pos_x", "pos_y", "pos_z")):
            rng = getattr(cmd, f"noise_range_{nm}")
            cmd.gate_pose_w[:, k] += rng[:, 0] + u[:, k] * (rng[:, 1] - rng[:, 0])
            cmd.next_gate_pose_w[:, k] += rng[:, 0] + u[:, 3 + k] * (rng[:, 1] - rng[:, 0])
    return cmd


def observe(mdp, env, nz):
    """The policy and critic state groups (racing_ctbr_env.py:138-160) with the observation noise injected: nz [n, 6]
    = velocity noise 0-2 (randn_like), attitude euler noise 3-5 (randn)."""
    O = mdp["observation"]
    z = f32(nz)

    def randn_like(x, **kw):
        assert x.shape == z[:, 0:3].shape
        return z[:, 0:3].clone()

    def randn(*size, device=None, **kw):
        assert _sz(size) == tuple(z[:, 3:6].shape)
        return z[:, 3:6].clone()

    old = patch(O, randn_like=randn_like, randn=randn)
    try:
        pol = torch.cat([O.modified_base_lin_vel(env, add_noise=True), O.base_orientation_r(env, add_noise=True),
                         O.modified_generated_commands(env, "next_gate_pose")], 1)
    finally:
        O.torch = old
    cri = torch.cat([O.modified_base_lin_vel(env, add_noise=False), O.base_orientation_r(env, add_noise=False),
                     O.modified_generated_commands_gt(env, "next_gate_pose")], 1)
    return pol, cri


# ------------------------------------------------------------------------------------------------ part R
def reference_reset(pre, cfg, gate_pose, start, origin_z, cnt):
    """Reset every env (ManagerBasedDiffRLEnv._reset_idx order) from the oracle records `pre`, then the observation
    of call counter `cnt`, with the build's draws injected."""
    import oracle

    mdp = il_shim.load_mdp()
    Ev, Cu, DA = mdp["events"], mdp["curriculums"], mdp["diff_action"]
    DroneDynamics = mdp["droneDynamics"].DroneDynamics
    CTBRController = sys.modules["diff.lab.controllers"].CTBRController
    n = len(pre)
    ids = torch.arange(n)
    types = torch.tensor(pre["type"], dtype=torch.long)
    levels = torch.tensor(pre["level"], dtype=torch.long)
    epoch_new = pre["epoch"].astype(np.int64) + 1
    rd = np.stack([oracle.draws(cfg, i, oracle.DRAW_RESET, int(epoch_new[i])) for i in range(n)])
    nz = np.stack([oracle.draws(cfg, i, oracle.DRAW_OBS, cnt) for i in range(n)])
    gu = np.stack([oracle.draws(cfg, i, oracle.DRAW_GATE, int(epoch_new[i]), 0) for i in range(n)])
    gp = torch.tensor(gate_pose)
    oz = f32(origin_z)

    # ---- the scene before the reset
    data = NS(root_state_w=torch.zeros(n, 13), body_lin_acc_w=torch.zeros(n, 1, 3), body_ang_acc_w=torch.zeros(n, 1, 3),
              default_root_state=torch.tensor([[0.0, 0.0, 0.5, 1.0, 0, 0, 0, 0, 0, 0, 0, 0, 0]]).repeat(n, 1))
    written = {}
    robot = NS(data=data, device="cpu")
    robot.write_root_link_pose_to_sim = lambda pose, env_ids: written.__setitem__("pose", pose.clone())
    robot.write_root_com_velocity_to_sim = lambda vel, env_ids: written.__setitem__("vel", vel.clone())
    terrain = NS(extras={"gate_pose": gp, "next_gate_id": torch.tensor(start)}, terrain_types=types,
                 terrain_levels=levels.clone(), max_terrain_level=NL,
                 cfg=NS(terrain_generator=NS(sub_terrains={"circular": NS(num_gate=G)})))
    origins = torch.zeros(n, 3)
    origins[:, 2] = oz[types, levels]
    scene = GE.Scene(robot=robot)
    scene.terrain, scene.env_origins, scene.device, scene.num_envs = terrain, origins, "cpu", n
    env = NS(num_envs=n, device="cpu", scene=scene, cfg=NS(sim=NS(dt=0.01, gravity=(0.0, 0.0, -9.81)), decimation=3))

    def update_env_origins(env_ids, move_up, move_down):
        """IL TerrainImporter.update_env_origins (restated): a level past the top takes a random level — here the
        build's draw (reset field 19) — and the env origin follows the level."""
        terrain.terrain_levels[env_ids] += 1 * move_up - 1 * move_down
        lv = terrain.terrain_levels[env_ids]
        rnd = torch.floor(f32(rd[:, 19])[env_ids] * NL).long()
        terrain.terrain_levels[env_ids] = torch.where(lv >= terrain.max_terrain_level, rnd, torch.clip(lv, 0))
        scene.env_origins[env_ids, 2] = oz[terrain.terrain_types[env_ids], terrain.terrain_levels[env_ids]]

    terrain.update_env_origins = update_env_origins

    # ---- the terms (constructed without IL's __init__; fields as __init__ sets them)
    cmd = make_cmd(mdp, env, robot, gp, pre["gate_id"], origins, types, levels, pre["noise_level"])
    cmd.metrics = {"accumulate_gates": torch.tensor(pre["acc"], dtype=torch.float32), "action_rate": torch.zeros(n),
                   "avg_lin_spd": torch.zeros(n), "avg_ang_spd": torch.zeros(n)}
    env.command_manager = NS(get_term=lambda name: cmd, _terms={"next_gate_pose": cmd},
                             get_command=lambda name: cmd.command)
    m_ctrl = f32(pre["m_ctrl"])
    da = DA.DiffActions.__new__(DA.DiffActions)
    da.cfg = NS(sim2real_test=False, max_thrust_weight_ratio=3.0, action_lag=1, random_drag=True)
    da.env, da.robot, da.num_envs, da.device = env, robot, n, "cpu"
    da.dt = env.cfg.sim.dt * env.cfg.decimation
    da._robot_mass = m_ctrl
    ctl = CTBRController(GE.CTBRCfg(), n, "cpu", m_ctrl, torch.tensor(GE.J0).diag().unsqueeze(0).repeat(n, 1, 1), da.dt)
    da.controller = ctl
    dd = DroneDynamics(n, m_ctrl, torch.diag_embed(f32(pre["J"])), da.dt, 3, random_drag=True, device="cpu")
    da.drone_dynamics = dd
    da.thr_est_error = torch.ones(n)
    env.action_manager = NS(get_term=lambda name: da)

    # ---- 1. curriculum (stage 1: terrain levels 3 / 2, noise levels 4 / 3, +2 % / -3 %)
    Cu.racing_terrain_levels(env, ids, "next_gate_pose", 3, 2)
    Cu.racing_cmd_noise_levels(env, ids, "next_gate_pose", 4, 3, 0.02, 0.03)
    # ---- 2. reset event: reset_root_state_racing (racing_ctbr_env.py:176-195 ranges)
    q = Queue([f32(rd[:, 0:6]), f32(rd[:, 6:12])])
    il_shim.SAMPLE_HOOK = q.take
    try:
        Ev.reset_root_state_racing(env, ids, {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "z": (-0.5, 0.5), "roll": (-0.2, 0.2),
                                              "pitch": (-0.2, 0.2), "yaw": (-0.7, 0.7)},
                                   {k: (-0.1, 0.1) for k in ("x", "y", "z", "roll", "pitch", "yaw")})
    finally:
        il_shim.SAMPLE_HOOK = None
    q.done()
    data.root_state_w = torch.cat([written["pose"], written["vel"]], 1)
    data.root_pos_w, data.root_quat_w = data.root_state_w[:, :3], data.root_state_w[:, 3:7]
    # ---- 3. action manager: DiffActions.reset_idx (controller, drag DR, dynamics state, thrust-estimate error)
    qr = Queue([f32(rd[:, 12]), f32(rd[:, 13:16]), f32(rd[:, 16:19])])
    qn = Queue([f32(rd[:, 24])])
    old_dd = patch(mdp["droneDynamics"], rand=lambda *size, device=None, **kw: qr.take(_sz(size)))
    old_da = patch(DA, randn=lambda *size, device=None, **kw: qn.take(_sz(size)))
    try:
        da.reset_idx(ids)
    finally:
        mdp["droneDynamics"].torch = old_dd
        DA.torch = old_da
    qr.done()
    qn.done()
    # ---- 4. command manager: metrics to 0 (IL CommandTerm.reset), _resample_command with the gate noise injected
    for v in cmd.metrics.values():
        v[ids] = 0.0
    qg = Queue()
    push_gate_noise(qg, gu)
    Cm = mdp["commands"]
    old_cm = patch(Cm, empty=lambda *size, device=None, **kw: _Uniform(qg, _sz(size)[0]))
    try:
        cmd._resample_command(ids)
    finally:
        Cm.torch = old_cm
    qg.done()
    # ---- 5. observation (the simulator state = the written reset state)
    data.root_lin_vel_w, data.root_ang_vel_w = written["vel"][:, :3], written["vel"][:, 3:]
    data.root_com_lin_vel_b = il_shim.quat_rotate_inverse(data.root_quat_w, data.root_lin_vel_w)
    pol, cri = observe(mdp, env, nz)
    p_local = written["pose"][:, :3] - scene.env_origins
    out = {"p": p_local, "q": written["pose"][:, 3:7], "v": written["vel"][:, :3], "w": dd.ang_vel_b,
           "k2": dd.drag_coeffs, "k1": dd.h_force_drag_coeffs, "thr_err": da.thr_est_error,
           "level": terrain.terrain_levels, "noise_level": cmd.noise_level[:, 0], "gate_id": cmd.gate_id,
           "obs_policy12": pol, "obs_critic12": cri}
    return {k: v.detach().numpy() for k, v in out.items()}


# ------------------------------------------------------------------------------------------------ part G
def reference_step_noisy(st, gate_pose, start, origin_z, collide, cfg, cnt, epoch):
    """One step of make_golden_env.reference_step's composition with the gate and observation noise on: the noisy gates
    each env holds (the draws of its (episode, gates passed)), the update's new noise for passing envs (gates passed +
    1), the resample's for done envs (next episode, 0), the observation noise of counter `cnt`.  Done envs are reset by
    the reference only as far as the command term (their state is not comparable): compared are the envs that do not
    reset."""
    import oracle

    n = len(st["p"])
    acc = st["acc"].astype(np.int64)
    draw = lambda kind, c1, c3: np.stack([oracle.draws(cfg, i, kind, int(c1[i]), int(c3[i]))  # noqa: E731
                                          for i in range(n)])
    ep = np.full(n, epoch, np.int64)
    hooks = NS(gu_pre=draw(oracle.DRAW_GATE, ep, acc), gu_new=draw(oracle.DRAW_GATE, ep, acc + 1),
               gu_rst=draw(oracle.DRAW_GATE, ep + 1, np.zeros(n, np.int64)),
               nz=draw(oracle.DRAW_OBS, np.full(n, cnt, np.int64), np.zeros(n, np.int64)))
    res, _ = GE.reference_step(st, 1, gate_pose, start, origin_z, collide, noise=hooks)
    return res


def main():
    import oracle
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg

    gates, recs, gate_pose, start, origin_z = GE.tables()
    out = {"gate_pos": gate_pose[..., :3], "start_gate": start.astype(np.int32), "origin_z": origin_z}
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=N), sim=SimCfg(device="cpu"), stage=1,
                       terrain=TerrainCfg(obstacles=False)).to_gr_config()
    assert cfg.obs_noise and cfg.add_gate_noise and cfg.dr_startup and cfg.random_drag
    # ---- part S
    dr = np.stack([oracle.draws(cfg, i, oracle.DRAW_STATIC) for i in range(N)])
    for k, v in reference_startup(dr).items():
        out[f"S_{k}"] = v.detach().numpy()
    # ---- part R: a varied pre-state from the oracle (init, reset, 60 random steps), then reset every env
    orc = oracle.Oracle(cfg, gates, recs)
    orc.init()
    orc.reset(None)
    rng = np.random.default_rng(3)
    for _ in range(60):
        orc.step((rng.standard_normal((N, 4)) * 1.2).astype(np.float32))
    pre = orc.envs.copy()
    # a spread of curriculum states: accumulated gates on both sides of every threshold, levels at the top
    pre["acc"] = rng.integers(0, 7, N)
    top = rng.random(N) < 0.15
    pre["level"][top] = NL - 1
    pre["noise_level"] = rng.uniform(0.8, 1.25, N).astype(np.float32)
    cnt = 977
    ref = reference_reset(pre, cfg, gate_pose, start, origin_z, cnt)
    for name in oracle.ENV_DTYPE.names:
        out[f"R_pre_{name}"] = pre[name]
    out["R_cnt"] = np.array([cnt], np.int64)
    out["R_prev_critic"] = orc.obs_critic.copy()
    for k, v in ref.items():
        out[f"R_{k}"] = v
    # ---- part G: golden_env.npz's stage-1 step (1 024 eventful envs near their gates), the noise on
    ge = np.load(os.path.join(HERE, "golden_env.npz"))
    n_g = ge["s1_in_p"].shape[0]
    cfg_g = RacingEnvCfg(scene=SceneCfg(num_envs=n_g), sim=SimCfg(device="cpu"), stage=1,
                         terrain=TerrainCfg(obstacles=False)).to_gr_config()
    st = {k[len("s1_in_"):]: ge[k] for k in ge.files if k.startswith("s1_in_")}
    for k in ("type", "level", "gate_id", "ep_len", "acc"):
        st[k] = st[k].astype(np.int64)
    for k, v in st.items():
        if v.dtype == np.float32:
            st[k] = v.astype(np.float64)
    cnt_g, epoch_g = 4242, 3  # (tests/env_golden.envs_from_fixture: epoch 3)
    collide = oracle.Oracle(cfg_g, gates, recs).collision_count
    res = reference_step_noisy(st, gate_pose, start, origin_z, collide, cfg_g, cnt_g, epoch_g)
    assert np.array_equal(res["dones"], ge["s1_out_dones"].astype(bool))
    out["G_cnt"] = np.array([cnt_g], np.int64)
    out["G_epoch"] = np.array([epoch_g], np.int64)
    out["G_obs_policy"] = res["obs_policy"]
    out["G_gate_id_after"] = res["gate_id_after"]
    live = ~res["dones"].astype(bool)
    print(f"part G: {n_g} envs, {int(live.sum())} live, passes {int((res['gate_id_after'] != st['gate_id'])[live].sum())}")
    print(f"part R: {N} envs, levels moved up {int((ref['level'] > pre['level']).sum())}, down "
          f"{int((ref['level'] < pre['level']).sum())}, past the top {int(top.sum())}")
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
