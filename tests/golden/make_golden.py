"""Generate golden vectors by running the REFERENCE's own pure-torch classes.

Run in the development container (the reference is mounted read-only at
/root/reference there; it never travels to the GPU box):

    python tests/golden/make_golden.py

It imports, from the reference source tree,
  extensions/diff.lab_tasks/.../quadcopter_diff/mdp/dynamics/droneDynamics.py  (DroneDynamics)
  extensions/diff.lab/diff/lab/controllers/controller_diff.py                  (CTBRController)
  extensions/diff.lab/diff/lab/controllers/thrust_controller_diff.py           (ThrustController)
and records inputs/outputs into tests/golden/golden_dynamics.npz.

Isaac Lab is not installed, so `omni.isaac.lab.utils.math` is provided by a
small restatement of the three quaternion helpers the classes call
(quat_mul, quat_rotate, quat_rotate_inverse; Isaac Lab formulas).  The
fixtures therefore pin the reference's own composition (controller law,
filters, drag, explicit Euler order) — not Isaac Lab's helpers, which are
"parity unpinned" (DESIGN.md §Oracle).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REF = os.environ.get("GR_REFERENCE_ROOT", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_dynamics.npz")


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import il_shim  # noqa: E402  (Isaac Lab stand-ins: the three quaternion helpers these classes call)


def load_reference():
    thr, ctl = il_shim.load_controllers()
    dd = il_shim.load(
        "grref_dd",
        os.path.join(REF, "extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/mdp/dynamics/droneDynamics.py"),
    )
    return dd.DroneDynamics, ctl.CTBRController, thr.ThrustController


class CTBRCfg:
    """Plain stand-in for CTBRControllerCfg with the racing task values
    (racing_ctbr_env.py:127-134 over controller_diff_cfg.py:22-54)."""

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


MASS = 0.6  # nominal mass ASSUMPTION (the USD that defines it is not in the reference)
INERTIA = [0.0015, 0.002, 0.004]
DT = 0.01 * 3  # sim.dt * decimation, as DiffActions computes it (diff_action.py:25)


def rand_states(g, n):
    p = torch.randn(n, 3, generator=g) * 2.0
    q = torch.randn(n, 4, generator=g)
    q = q / q.norm(dim=1, keepdim=True)
    v = torch.randn(n, 3, generator=g) * 2.0
    w = torch.randn(n, 3, generator=g) * 1.5
    return p, q, v, w


def main():
    DroneDynamics, CTBRController, ThrustController = load_reference()
    g = torch.Generator().manual_seed(20250815)
    out = {}
    inertia = lambda n: torch.tensor(INERTIA).diag().unsqueeze(0).repeat(n, 1, 1)  # noqa: E731

    # 1) DroneDynamics.step, single step, random_drag off and on
    for rd in (False, True):
        n = 64
        torch.manual_seed(7 + int(rd))
        dd = DroneDynamics(n, torch.full((n,), MASS), inertia(n), DT, 3, random_drag=rd, device="cpu")
        idx = torch.arange(n)
        dd.reset_idx(idx)
        p, q, v, w_w = rand_states(g, n)
        states = torch.cat([p, q, v, w_w], 1)
        dd.reset_state(states, idx)
        w_b_in = dd.ang_vel_b.clone()
        tt = torch.cat([torch.rand(n, 1, generator=g) * 20.0, torch.randn(n, 3, generator=g) * 0.02], 1)
        nxt, acc = dd.step(tt)
        tag = f"dd1_drag{int(rd)}"
        out[tag + "_state_in"] = torch.cat([p, q, v, w_b_in], 1).numpy()
        out[tag + "_tt"] = tt.numpy()
        out[tag + "_drag"] = torch.cat([dd.drag_coeffs, dd.h_force_drag_coeffs], 1).numpy()
        out[tag + "_next"] = nxt.numpy()  # p q v_w w_w
        out[tag + "_acc"] = acc.numpy()
        out[tag + "_wb_out"] = dd.ang_vel_b.numpy()

    # 2) DroneDynamics.step rollout (200 steps, hover-ish thrust + random torques)
    n, T = 16, 200
    torch.manual_seed(11)
    dd = DroneDynamics(n, torch.full((n,), MASS), inertia(n), DT, 3, random_drag=True, device="cpu")
    idx = torch.arange(n)
    dd.reset_idx(idx)
    p, q, v, w_w = rand_states(g, n)
    v = v * 0.2
    w_w = w_w * 0.2
    dd.reset_state(torch.cat([p, q, v, w_w], 1), idx)
    out["ddr_state_in"] = torch.cat([p, q, v, dd.ang_vel_b.clone()], 1).numpy()
    out["ddr_drag"] = torch.cat([dd.drag_coeffs, dd.h_force_drag_coeffs], 1).numpy()
    tts, traj, accs = [], [], []
    for _ in range(T):
        tt = torch.cat([MASS * 9.81 + torch.randn(n, 1, generator=g) * 0.5, torch.randn(n, 3, generator=g) * 0.002], 1)
        nxt, acc = dd.step(tt)
        tts.append(tt)
        traj.append(torch.cat([nxt, dd.ang_vel_b], 1))
        accs.append(acc)
    out["ddr_tt"] = torch.stack(tts).numpy()
    out["ddr_traj"] = torch.stack(traj).numpy()  # [T][n][16] p q v_w w_w w_b
    out["ddr_acc"] = torch.stack(accs).numpy()

    # 3) CTBRController.compute sequences with per-env DR'd gains/delays
    for motor in (False, True):
        cfg = CTBRCfg()
        cfg.use_motor_model = motor
        n, T = 32, 20
        ctl = CTBRController(cfg, n, "cpu", torch.full((n,), MASS), inertia(n), DT)
        s = lambda lo, hi, k: torch.rand(n, k, generator=g) * (hi - lo) + lo  # noqa: E731
        ctl.rate_gain_p = ctl.rate_gain_p * s(0.9, 1.1, 3)
        ctl.rate_gain_d = ctl.rate_gain_d * s(0.9, 1.1, 3)
        ctl.thrust_ctrl_delay = ctl.thrust_ctrl_delay * s(0.8, 1.3, 1)
        ctl.torque_ctrl_delay = ctl.torque_ctrl_delay * s(0.8, 1.3, 3)
        tag = f"ctbr_motor{int(motor)}"
        out[tag + "_kp"] = ctl.rate_gain_p.numpy()
        out[tag + "_kd"] = ctl.rate_gain_d.numpy()
        out[tag + "_dT"] = ctl.thrust_ctrl_delay.numpy()
        out[tag + "_dtau"] = ctl.torque_ctrl_delay.numpy()
        wbs, abs_, cmds, outs, filt = [], [], [], [], []
        for _ in range(T):
            wb = torch.randn(n, 3, generator=g) * 2.0
            ab = torch.randn(n, 3, generator=g) * 20.0
            cmd = torch.cat([torch.rand(n, 1, generator=g) * 30.0 - 5.0, torch.randn(n, 3, generator=g) * 5.0], 1)
            zero3 = torch.zeros(n, 3)
            st = {"pos": zero3, "quat": torch.zeros(n, 4), "lin_vel_w": zero3, "ang_vel_w": zero3, "lin_vel_b": zero3,
                  "ang_vel_b": wb, "lin_acc_w": zero3, "ang_acc_w": zero3, "lin_acc_b": zero3, "ang_acc_b": ab}
            _, tt = ctl.compute(st, cmd)
            wbs.append(wb); abs_.append(ab); cmds.append(cmd); outs.append(tt.clone())
            filt.append(torch.cat([ctl.gross_thrust, ctl.torque], 1).clone())
        out[tag + "_wb"] = torch.stack(wbs).numpy()
        out[tag + "_ab"] = torch.stack(abs_).numpy()
        out[tag + "_cmd"] = torch.stack(cmds).numpy()
        out[tag + "_out"] = torch.stack(outs).numpy()
        out[tag + "_filt"] = torch.stack(filt).numpy()

    # 4) ThrustController.update (motor model)
    n, T = 32, 10
    tc = ThrustController("cpu", n, {"motor_tau": CTBRCfg.motor_tau, "dt": DT, "thrustmap": CTBRCfg.thrustmap,
                                     "arm_length": CTBRCfg.arm_length, "kappa": CTBRCfg.kappa})
    ins, outs = [], []
    for _ in range(T):
        f = torch.rand(n, 4, generator=g) * 20.0
        ins.append(f)
        outs.append(tc.update(f).clone())
    out["thr_in"] = torch.stack(ins).numpy()
    out["thr_out"] = torch.stack(outs).numpy()
    out["thr_B"] = tc.B_allocation.numpy()
    out["thr_Binv"] = tc.B_allocation_inv.numpy()

    # 5) closed loop: raw action -> lag -> tanh/scale/offset * thr_err -> CTBR -> DroneDynamics.step,
    #    DD's own state fed back as the "sim" state
    n, T = 32, 100
    torch.manual_seed(13)
    cfg = CTBRCfg()
    dd = DroneDynamics(n, torch.full((n,), MASS), inertia(n), DT, 3, random_drag=True, device="cpu")
    ctl = CTBRController(cfg, n, "cpu", torch.full((n,), MASS), inertia(n), DT)
    idx = torch.arange(n)
    dd.reset_idx(idx)
    p = torch.zeros(n, 3); p[:, 2] = 1.0
    q = torch.zeros(n, 4); q[:, 0] = 1.0
    dd.reset_state(torch.cat([p, q, torch.zeros(n, 6)], 1), idx)
    thr_err = 1 + torch.randn(n, generator=g) * 0.01
    weight = torch.full((n,), MASS) * 9.81
    scale = torch.hstack([(weight * 3.0 / 2)[:, None], torch.ones(n, 3) * 6])
    offset = torch.hstack([(weight * 3.0 / 2)[:, None], torch.zeros(n, 3)])
    out["cl_drag"] = torch.cat([dd.drag_coeffs, dd.h_force_drag_coeffs], 1).numpy()
    out["cl_thr_err"] = thr_err.numpy()
    lag = torch.zeros(n, 4)
    ab = torch.zeros(n, 3)
    acts, traj, abins, filt = [], [], [], []
    for _ in range(T):
        a = torch.randn(n, 4, generator=g) * 0.3
        raw, lag = lag, a.clone()
        cmd = raw.tanh() * scale + offset
        cmd[:, 0] *= thr_err
        zero3 = torch.zeros(n, 3)
        st = {"pos": dd.pos, "quat": dd.quat, "lin_vel_w": dd.lin_vel_w, "ang_vel_w": dd.ang_vel_w,
              "lin_vel_b": dd.lin_vel_b, "ang_vel_b": dd.ang_vel_b, "lin_acc_w": zero3, "ang_acc_w": zero3,
              "lin_acc_b": zero3, "ang_acc_b": ab}
        w_old = dd.ang_vel_b.clone()
        _, tt = ctl.compute(st, cmd)
        abins.append(ab.clone())
        nxt, _ = dd.step(tt)
        ab = (dd.ang_vel_b - w_old) / DT
        acts.append(a)
        traj.append(torch.cat([nxt[:, :10], dd.ang_vel_b], 1))
        filt.append(torch.cat([ctl.gross_thrust, ctl.torque], 1).clone())
    out["cl_actions"] = torch.stack(acts).numpy()
    out["cl_traj"] = torch.stack(traj).numpy()  # [T][n][13] p q v_w w_b
    out["cl_ab_in"] = torch.stack(abins).numpy()
    out["cl_filt"] = torch.stack(filt).numpy()

    out = {k: np.ascontiguousarray(v.astype(np.float32)) for k, v in out.items()}
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {sum(v.nbytes for v in out.values()) / 1e3:.1f} kB raw, {len(out)} arrays")


if __name__ == "__main__":
    main()
