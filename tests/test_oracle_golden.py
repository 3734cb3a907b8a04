"""CPU oracle vs golden vectors produced by the REFERENCE's own classes
(tests/golden/make_golden.py: DroneDynamics.step, CTBRController.compute,
ThrustController via the motor model, and a closed controller->dynamics loop).

Tolerances: the oracle restates the reference op order in fp32 without FMA;
torch's CPU kernels (bmm, vectorised reductions) round differently in the
last ulp, so single-step results are compared at rtol 1e-6 + atol 1e-6 and
rollouts with a horizon-dependent bound (north star: float state within 1e-5)."""
import math

import numpy as np
import pytest

import oracle
from generalizableracing_amd import _abi

DT = np.float32(0.03)
J = np.array([0.0015, 0.002, 0.004], np.float32)


def cfg(motor=False):
    c = _abi.default_config()
    c.use_motor_model = int(motor)
    return c


def par_rows(n, kp=None, kd=None, cT=None, ctau=None, mass=0.6):
    par = np.zeros((n, 16), np.float32)
    par[:, 0:3] = 35.0 if kp is None else kp
    par[:, 3] = math.exp(-1.0) if cT is None else cT
    par[:, 4:7] = np.array([5e-4, 5e-4, 3e-4], np.float32) if kd is None else kd
    par[:, 7] = mass
    par[:, 8:11] = math.exp(-1.0) if ctau is None else ctau
    par[:, 11] = mass
    par[:, 12:15] = J
    return par


def close(a, b, rtol, atol):
    err = np.abs(a.astype(np.float64) - b) - (atol + rtol * np.abs(b))
    return err.max() <= 0, np.abs(a.astype(np.float64) - b).max()


@pytest.mark.parametrize("rd", [0, 1])
def test_dd_single_step(golden, rd):
    t = f"dd1_drag{rd}"
    s_in, tt, drag = golden[t + "_state_in"], golden[t + "_tt"], golden[t + "_drag"]
    n = s_in.shape[0]
    so, co, xo = oracle.test_dynamics(cfg(), 1, s_in, np.zeros((n, 3)), tt, np.zeros((n, 4)), par_rows(n), drag)
    nxt = golden[t + "_next"]
    for name, got, want in [("p", so[:, :3], nxt[:, :3]), ("q", so[:, 3:7], nxt[:, 3:7]),
                            ("v", so[:, 7:10], nxt[:, 7:10]), ("w_world", xo[:, 6:9], nxt[:, 10:13]),
                            ("w_body", so[:, 10:13], golden[t + "_wb_out"]), ("acc", xo[:, :3], golden[t + "_acc"])]:
        ok, e = close(got, want, 1e-6, 1e-6)
        assert ok, (name, e)


def test_dd_rollout_200(golden):
    s = golden["ddr_state_in"].copy()
    drag = golden["ddr_drag"]
    tts, traj = golden["ddr_tt"], golden["ddr_traj"]
    n = s.shape[0]
    worst = 0.0
    for k in range(tts.shape[0]):
        s, _, xo = oracle.test_dynamics(cfg(), 1, s, np.zeros((n, 3)), tts[k], np.zeros((n, 4)), par_rows(n), drag)
        want = np.concatenate([traj[k][:, :10], traj[k][:, 13:16]], 1)  # p q v_w w_b
        scale = np.maximum(1.0, np.abs(want))
        worst = max(worst, float((np.abs(s - want) / scale).max()))
    assert worst < 1e-5, worst  # 200 explicit-Euler steps, fp32 re-association noise only


@pytest.mark.parametrize("motor", [0, 1])
def test_ctbr_sequence(golden, motor):
    t = f"ctbr_motor{motor}"
    n = golden[t + "_kp"].shape[0]
    cT = np.exp(-DT / golden[t + "_dT"][:, 0].astype(np.float32)).astype(np.float32)
    ctau = np.exp(-DT / golden[t + "_dtau"].astype(np.float32)).astype(np.float32)
    par = par_rows(n, kp=golden[t + "_kp"], kd=golden[t + "_kd"], cT=cT, ctau=ctau)
    filt = np.zeros((n, 4), np.float32)
    s_in = np.zeros((n, 13), np.float32)
    s_in[:, 3] = 1.0
    drag = np.zeros((n, 6), np.float32)
    for k in range(golden[t + "_cmd"].shape[0]):
        s_in[:, 10:13] = golden[t + "_wb"][k]
        so, filt_new, xo = oracle.test_dynamics(cfg(motor), 0, s_in, golden[t + "_ab"][k], golden[t + "_cmd"][k],
                                                filt, par, drag)
        ok, e = close(filt_new, golden[t + "_filt"][k], 2e-6, 2e-6)
        assert ok, ("filter", k, e)
        # the controller's output: [T, tau] (motor 0: the filters, :137-138; motor 1: allocation ->
        # clamp -> ThrustController.update -> B f, :140-144).  B^-1 is torch.inverse's LU in the reference
        # and the closed form here, and T(w) = k2 w^2 + k1 w + k0 cancels near f = 0: 2e-5 of the scale
        ok, e = close(xo[:, 9:13], golden[t + "_out"][k], 2e-5, 2e-5 * np.abs(golden[t + "_out"][k]).max())
        assert ok, ("output", k, e)
        filt = golden[t + "_filt"][k].copy()  # teacher-forced filter state


def test_closed_loop_controller_dynamics(golden):
    """raw action -> lag -> tanh/scale/offset*thr_err -> CTBR -> DroneDynamics.step, 100 steps."""
    acts, traj = golden["cl_actions"], golden["cl_traj"]
    n = acts.shape[1]
    drag = golden["cl_drag"]
    thr = golden["cl_thr_err"].astype(np.float32)
    s0 = np.float32(0.6) * np.float32(9.81) * np.float32(3.0) / np.float32(2.0)
    scale = np.array([s0, 6, 6, 6], np.float32)
    offset = np.array([s0, 0, 0, 0], np.float32)
    s = np.zeros((n, 13), np.float32)
    s[:, 2] = 1.0
    s[:, 3] = 1.0
    filt = np.zeros((n, 4), np.float32)
    lag = np.zeros((n, 4), np.float32)
    ab = np.zeros((n, 3), np.float32)
    worst = 0.0
    for k in range(acts.shape[0]):
        raw, lag = lag, acts[k]
        th = oracle.test_math(1, raw.reshape(-1)).reshape(n, 4)
        cmd = th * scale + offset
        cmd[:, 0] = cmd[:, 0] * thr
        w_old = s[:, 10:13].copy()
        s, filt, _ = oracle.test_dynamics(cfg(), 0, s, ab, cmd, filt, par_rows(n), drag)
        ab = (s[:, 10:13] - w_old) / DT
        want = traj[k]
        scale_w = np.maximum(1.0, np.abs(want))
        worst = max(worst, float((np.abs(s - want) / scale_w).max()))
    assert worst < 1e-5, worst


def test_thrust_controller_update(golden):
    """ThrustController.update on its own (thrust_controller_diff.py:182-186): desired rotor thrusts ->
    Thrust2Omega -> first-order motor lag (c = exp(-dt / 1e-4) = 0 in fp32) -> Omega2Thrust.  The fixture
    starts every sequence from zero motor speed; with c = 0 each call is independent of the last."""
    n = golden["thr_in"].shape[1]
    s = np.zeros((n, 13), np.float32)
    s[:, 3] = 1.0
    for k in range(golden["thr_in"].shape[0]):
        _, _, xo = oracle.test_dynamics(cfg(True), 2, s, np.zeros((n, 3)), golden["thr_in"][k], np.zeros((n, 4)),
                                        par_rows(n), np.zeros((n, 6)))
        ok, e = close(xo[:, 9:13], golden["thr_out"][k], 1e-5, 1e-5)
        assert ok, (k, e)


def test_allocation_matrix(golden):
    """B and B^-1 of the motor model (controller_diff.py:56-69 / thrust_controller_diff.py:44-55): the
    closed-form rows the oracle and kernel use, against the reference's torch.vstack / torch.inverse."""
    l, kap = np.float32(0.09) * np.float32(0.707106769), np.float32(0.016)
    sx, sy, sz = np.array([1, -1, -1, 1]), np.array([-1, -1, 1, 1]), np.array([1, -1, 1, -1])
    B = np.stack([np.ones(4), l * sx, l * sy, kap * sz]).astype(np.float32)
    Bi = np.stack([np.full(4, 0.25), sx / (4 * l), sy / (4 * l), sz / (4 * kap)], 1).astype(np.float32)
    np.testing.assert_allclose(B, golden["thr_B"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(Bi, golden["thr_Binv"], rtol=1e-5, atol=1e-5)

