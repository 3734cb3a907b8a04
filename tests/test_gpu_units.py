"""Device building blocks vs host: portable math and Philox bit-identical,
controller + integrator (gr_test_dynamics) bit-identical to the oracle and
within 1e-5 of the reference's own DroneDynamics / CTBRController vectors."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from generalizableracing_amd import _abi  # noqa: E402

DEV = "cuda:0"


@pytest.fixture(scope="module")
def ctx():
    lib = _abi.load()
    cfg = _abi.default_config()
    cfg.num_envs = 64
    h = C.c_void_p()
    assert lib.gr_create(C.byref(cfg), C.byref(h)) == 0
    yield lib, h, cfg
    lib.gr_destroy(h)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("fn", range(8))
def test_math_bitwise_host_device(ctx, fn):
    lib, h, _ = ctx
    rng = np.random.default_rng(fn)
    x = rng.uniform(-20, 20, 100000).astype(np.float32)
    y = rng.uniform(-5, 5, 100000).astype(np.float32)
    if fn in (2, 6):
        x = np.abs(x) + np.float32(1e-6)
    if fn == 7:
        y = np.where(np.abs(y) < 1e-3, np.float32(1.0), y)
    xd, yd, od = dev(x), dev(y), torch.zeros(x.size, device=DEV)
    assert lib.gr_test_math(h, fn, x.size, xd.data_ptr(), yd.data_ptr(), od.data_ptr(), stream()) == 0
    got = od.cpu().numpy()
    want = oracle.test_math(fn, x, y)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), np.abs(got - want).max()


def test_philox_bitwise(ctx):
    lib, h, cfg = ctx
    n = 4096
    out = torch.zeros(n * 4, dtype=torch.int32, device=DEV)
    assert lib.gr_test_philox(h, n, 7, 11, 13, 17, out.data_ptr(), stream()) == 0
    got = out.cpu().numpy().view(np.uint32).reshape(n, 4)
    assert np.array_equal(got, oracle.test_philox(n, 7, 11, 13, 17, cfg.seed_lo, cfg.seed_hi))


def _run_dyn(lib, h, mode, s, ab, cmd, ci, par, drag):
    n = s.shape[0]
    outs = [torch.zeros(n, k, device=DEV) for k in (13, 4, 13)]
    ins = [dev(np.asarray(a, np.float32)) for a in (s, ab, cmd, ci, par, drag)]
    rc = lib.gr_test_dynamics(h, n, mode, *[t.data_ptr() for t in ins], *[t.data_ptr() for t in outs], stream())
    assert rc == 0
    return [t.cpu().numpy() for t in outs]


def test_dynamics_vs_oracle_and_golden(ctx, golden):
    lib, h, cfg = ctx
    from test_oracle_golden import par_rows  # same parameter rows as the CPU golden test

    for rd in (0, 1):
        t = f"dd1_drag{rd}"
        s, tt, drag = golden[t + "_state_in"], golden[t + "_tt"], golden[t + "_drag"]
        n = s.shape[0]
        args = (s, np.zeros((n, 3)), tt, np.zeros((n, 4)), par_rows(n), drag)
        so, co, xo = _run_dyn(lib, h, 1, *args)
        so2, co2, xo2 = oracle.test_dynamics(cfg, 1, *args)
        assert np.array_equal(so.view(np.uint32), so2.view(np.uint32))
        assert np.array_equal(xo.view(np.uint32), xo2.view(np.uint32))
        nxt = golden[t + "_next"]
        np.testing.assert_allclose(so[:, :10], nxt[:, :10], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(xo[:, 6:9], nxt[:, 10:13], rtol=1e-6, atol=1e-6)
    # 200-step rollout on the device
    s = golden["ddr_state_in"].copy()
    n = s.shape[0]
    for k in range(golden["ddr_tt"].shape[0]):
        s, _, _ = _run_dyn(lib, h, 1, s, np.zeros((n, 3)), golden["ddr_tt"][k], np.zeros((n, 4)), par_rows(n),
                           golden["ddr_drag"])
    want = golden["ddr_traj"][-1]
    want = np.concatenate([want[:, :10], want[:, 13:16]], 1)
    assert (np.abs(s - want) / np.maximum(1, np.abs(want))).max() < 1e-5


@pytest.mark.parametrize("motor", [0, 1])
def test_controller_output_vs_oracle_and_golden(ctx, golden, motor):
    """The controller output [T, tau] (post motor model for motor=1) on the device: bit-identical to the
    oracle, and within the CPU golden test's tolerance of the reference's CTBRController sequence."""
    lib, h, _ = ctx
    from test_oracle_golden import DT, par_rows

    c = _abi.default_config()
    c.num_envs = 64
    c.use_motor_model = motor
    h2 = C.c_void_p()
    assert lib.gr_create(C.byref(c), C.byref(h2)) == 0
    t = f"ctbr_motor{motor}"
    n = golden[t + "_kp"].shape[0]
    cT = np.exp(-DT / golden[t + "_dT"][:, 0].astype(np.float32)).astype(np.float32)
    ctau = np.exp(-DT / golden[t + "_dtau"].astype(np.float32)).astype(np.float32)
    par = par_rows(n, kp=golden[t + "_kp"], kd=golden[t + "_kd"], cT=cT, ctau=ctau)
    s_in = np.zeros((n, 13), np.float32)
    s_in[:, 3] = 1.0
    drag = np.zeros((n, 6), np.float32)
    for k in range(golden[t + "_cmd"].shape[0]):
        s_in[:, 10:13] = golden[t + "_wb"][k]
        filt = np.zeros((n, 4), np.float32) if k == 0 else golden[t + "_filt"][k - 1]
        args = (s_in, golden[t + "_ab"][k], golden[t + "_cmd"][k], filt, par, drag)
        so, co, xo = _run_dyn(lib, h2, 0, *args)
        so2, co2, xo2 = oracle.test_dynamics(c, 0, *args)
        assert np.array_equal(xo.view(np.uint32), xo2.view(np.uint32)), k
        assert np.array_equal(co.view(np.uint32), co2.view(np.uint32)), k
        want = golden[t + "_out"][k]
        assert np.abs(xo[:, 9:13] - want).max() <= 2e-5 * np.abs(want).max() * 2, k
    if motor:
        thr_in = golden["thr_in"][0]
        n2 = thr_in.shape[0]
        s2 = np.zeros((n2, 13), np.float32)
        s2[:, 3] = 1.0
        args = (s2, np.zeros((n2, 3)), thr_in, np.zeros((n2, 4)), par_rows(n2), np.zeros((n2, 6)))
        _, _, xo = _run_dyn(lib, h2, 2, *args)
        _, _, xo2 = oracle.test_dynamics(c, 2, *args)
        assert np.array_equal(xo.view(np.uint32), xo2.view(np.uint32))
        np.testing.assert_allclose(xo[:, 9:13], golden["thr_out"][0], rtol=1e-5, atol=1e-5)
    lib.gr_destroy(h2)



@pytest.mark.gpu
def test_device_status_reports_obstacle_wait_timeout():
    """The bounded obstacle-mask wait of the physics waves: with the partner's signal suppressed
    (gr_test_inject_fault) the step completes, raises GR_STATUS_OBST_WAIT_TIMEOUT in the status word, and
    check_device_status fails loudly; without the fault the word stays clear."""
    from generalizableracing_amd import _abi
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg
    from generalizableracing_amd.envs.racing_env import RacingEnv

    env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=256), sim=SimCfg(device="cuda:0"), stage=1,
                                 terrain=TerrainCfg(obstacles=True)))
    a = torch.zeros(256, 4, device="cuda:0")
    for _ in range(3):
        env.step(a)
    assert env.device_status() == 0
    env._call("gr_test_inject_fault", _abi.GR_FAULT_OBST_NO_SIGNAL)
    env.step(a)
    env._call("gr_test_inject_fault", _abi.GR_FAULT_NONE)
    assert env.device_status(clear=False) & _abi.GR_STATUS_OBST_WAIT_TIMEOUT
    with pytest.raises(RuntimeError, match="obstacle mask"):
        env.check_device_status()
    env.step(a)
    assert env.device_status() == 0
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols", [(1, 1), (1000, 3), (393216, 256), (24577, 4), (70000, 1), (5000, 300),
                                       (3000, 1100)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_column_sum(rows, cols, dtype):
    """gr_column_sum (the PPO update's bias gradients, rsl_rl/linear.py bias_grad) against a float64 sum of
    the same elements; two calls are bit-identical (fixed summation order)."""
    from generalizableracing_amd.rsl_rl.linear import bias_grad

    g = torch.Generator(device="cuda:0").manual_seed(rows + cols)
    x = torch.randn(rows, cols, device="cuda:0", generator=g).to(dtype)
    got = bias_grad(x)
    again = bias_grad(x)
    torch.cuda.synchronize()
    want = x.double().sum(0)
    scale = x.double().abs().sum(0) + 1.0
    assert got.dtype == torch.float32 and got.shape == (cols,)
    assert float(((got.double() - want).abs() / scale).max()) < 1e-6
    assert torch.equal(got, again)


@pytest.mark.parametrize("rows,h,k", [(24576, 256, 4), (24576, 256, 1), (393216, 256, 4), (8193, 64, 8), (1, 4, 3),
                                      (100003, 128, 2)])
def test_leaky_head(rows, h, k):
    """gr_head_forward / gr_head_backward (rsl_rl/linear.py leaky_head: the MLP's last LeakyReLU + output Linear on
    the update's tall batches) against the same op in float64 torch: y, gz to 1e-6 of scale, gw / gb to a few ulps of the
    absolute sums (4e-6); pre-activations exactly 0 take LeakyReLU's negative branch as torch does; repeats bit-identical."""
    from generalizableracing_amd.rsl_rl.linear import leaky_head

    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(rows + 7 * h + k)
    z = torch.randn(rows, h, device=dev, generator=g)
    z[::7, ::5] = 0.0  # the kink
    w = torch.randn(k, h, device=dev, generator=g) * 0.1
    b = torch.randn(k, device=dev, generator=g)
    gy = torch.randn(rows, k, device=dev, generator=g)
    slope = 0.01
    outs = []
    for _ in range(2):
        zz, ww, bb = (t.clone().requires_grad_(True) for t in (z, w, b))
        y = leaky_head(zz, ww, bb, slope)
        y.backward(gy)
        outs.append((y.detach(), zz.grad, ww.grad, bb.grad))
    torch.cuda.synchronize()
    for a, c in zip(*outs):
        assert torch.equal(a, c)
    y, gz, gw, gb = outs[0]
    zd, wd, bd = (t.double().requires_grad_(True) for t in (z, w, b))
    yd = torch.nn.functional.leaky_relu(zd, slope) @ wd.t() + bd
    yd.backward(gy.double())
    a = torch.nn.functional.leaky_relu(z.double(), slope)
    assert float((y.double() - yd.detach()).abs().max()) <= 1e-6 * (1.0 + float((a.abs() @ wd.detach().abs().t()).max()))
    assert float((gz.double() - zd.grad).abs().max()) <= 1e-6 * (1.0 + float(gy.abs().max() * w.abs().sum(0).max()))
    # (fp32 running sums over a wave's rows, then the workgroups' partials in double: a few ulps of the absolute sum)
    assert float((gw.double() - wd.grad).abs().max()) <= 4e-6 * float((gy.double().abs().t() @ a.abs()).max() + 1.0)
    assert float((gb.double() - bd.grad).abs().max()) <= 4e-6 * float(gy.double().abs().sum(0).max() + 1.0)
    # the kink: zero pre-activations take the negative branch (slope * gh), as torch's leaky_relu_backward
    gh = (gy.double() @ w.double())
    zero = z == 0
    torch.testing.assert_close(gz[zero].double(), gh[zero] * slope, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("rows,d,ldx,h", [(24576, 16, 16, 256), (24576, 16, 48, 256), (393216, 16, 48, 256),
                                          (1001, 16, 20, 128), (8193, 32, 36, 64), (5, 4, 4, 8)])
def test_mlp_in_layer(rows, d, ldx, h):
    """gr_mlp_in_forward / gr_mlp_in_backward (the MLP's first Linear + bias + LeakyReLU and its weight / bias
    gradients, rsl_rl/linear.py _LeakyMLPFn) against float64 torch, on strided input rows as the packed mini-batch
    gives them (ldx > d); repeats bit-identical."""
    from generalizableracing_amd import _abi

    lib = _abi.load()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(rows + d + h)
    xs = torch.randn(rows, ldx, device=dev, generator=g)
    x = xs[:, :d]
    w = torch.randn(h, d, device=dev, generator=g) * 0.3
    b = torch.randn(h, device=dev, generator=g) * 0.1
    gh = torch.randn(rows, h, device=dev, generator=g)
    slope = 0.01
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for _ in range(2):
        y = torch.empty(rows, h, device=dev)
        assert lib.gr_mlp_in_forward(x.data_ptr(), rows, d, ldx, w.data_ptr(), b.data_ptr(), h, slope, y.data_ptr(),
                                     st) == 0
        part = torch.empty(lib.gr_mlp_in_partials(rows, d, h), device=dev)
        sums = torch.empty(h * d + h, device=dev)
        assert lib.gr_mlp_in_backward(gh.data_ptr(), y.data_ptr(), x.data_ptr(), rows, d, ldx, h, slope,
                                      part.data_ptr(), sums.data_ptr(), st) == 0
        outs.append((y, sums))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    y, sums = outs[0]
    zd = x.double() @ w.double().t() + b.double()
    yd = torch.nn.functional.leaky_relu(zd, slope)
    assert float((y.double() - yd).abs().max()) <= 1e-6 * (1.0 + float((x.double().abs() @ w.double().abs().t()).max()))
    gz = gh.double() * torch.where(zd > 0, 1.0, slope)
    # (the float derivative is taken on y = lrelu(z): same sign as z except where z rounds across 0)
    gz32 = gh.double() * torch.where(y > 0, 1.0, slope).double()
    gw = gz32.t() @ x.double()
    gb = gz32.sum(0)
    scale_w = float((gz.abs().t() @ x.double().abs()).max()) + 1.0
    assert float((sums[:h * d].view(h, d).double() - gw).abs().max()) <= 4e-6 * scale_w
    assert float((sums[h * d:].double() - gb).abs().max()) <= 4e-6 * (float(gz.abs().sum(0).max()) + 1.0)


@pytest.mark.parametrize("needs_input_grad", [False, True])
def test_mlp_fused_matches_module_path(needs_input_grad):
    """The actor / critic MLP on a tall CUDA batch — fully fused (_LeakyMLPFn: input needs no gradient, as the
    update's observation rows) or with the fused head only (input needs a gradient) — against the same module run
    layer by layer (TallLinear + nn.LeakyReLU): outputs and every parameter gradient within fp32 noise."""
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl import linear

    torch.manual_seed(3)
    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to("cuda:0")
    x0 = torch.randn(3 * linear.SPLIT, 48, device="cuda:0")[:, 8:24]  # a strided view, as the packed mini-batch
    assert linear.mlp_fusable(x0, list(pol.actor)) and linear.mlp_fusable(x0, list(pol.critic))
    res = []
    for fused in (True, False):
        pol.zero_grad()
        x = x0.clone().requires_grad_(True) if needs_input_grad else x0
        if fused:
            out = pol.actor(x).square().sum() + pol.critic(x).square().sum()
        else:
            def run(seq, v):
                for m in seq:
                    v = m(v)
                return v
            out = run(pol.actor, x).square().sum() + run(pol.critic, x).square().sum()
        out.backward()
        gx = x.grad.clone() if needs_input_grad else None
        res.append((float(out), [p.grad.clone() for p in pol.parameters() if p.grad is not None], gx))
    (oa, ga, xa), (ob, gb_, xb) = res
    assert abs(oa - ob) <= 1e-5 * abs(ob)
    assert len(ga) == len(gb_) == len(list(pol.parameters())) - 1  # (std gets no gradient here)
    for a, b in zip(ga, gb_):
        assert float((a - b).norm()) <= 1e-4 * float(b.norm()) + 1e-12
    if needs_input_grad:
        assert float((xa - xb).norm()) <= 1e-4 * float(xb.norm())


@pytest.mark.parametrize("clipped", [True, False])
def test_fused_ppo_losses_match_torch(clipped):
    """fused_loss.ppo_losses (gr_ppo_loss_forward / backward) against PPO's torch ops on the same mini-batch
    (ppo.py:103-169: Gaussian log prob, KL, clipped surrogate, clipped value loss; entropy term on): the losses,
    the KL and every parameter gradient, including ratios at and beyond the clip range."""
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl import fused_loss
    from generalizableracing_amd.rsl_rl.ppo import PPO

    torch.manual_seed(5)
    dev = "cuda:0"
    m = 12288
    pol = ActorCritic(16, 16, 4, [64, 64], [64, 64], "lrelu", init_noise_std=0.7).to(dev)
    alg = PPO(pol, device=dev, clip_param=0.2, entropy_coef=0.01, use_clipped_value_loss=clipped,
              value_loss_coef=0.5)
    obs = torch.randn(m, 16, device=dev)
    cobs = torch.randn(m, 16, device=dev)
    with torch.no_grad():
        mu0 = pol.actor(obs)
        act = mu0 + 0.7 * torch.randn_like(mu0)
        # old log probs spread so that ratios fall inside, at and beyond [0.8, 1.2]
        lp = torch.distributions.Normal(mu0, 0.7).log_prob(act).sum(-1, keepdim=True)
        logp_old = lp + torch.randn(m, 1, device=dev) * 0.3
        v0 = pol.critic(cobs)
        val_old = v0 + torch.randn(m, 1, device=dev) * 0.3
    adv = torch.randn(m, 1, device=dev)
    ret = torch.randn(m, 1, device=dev)
    mu_old = mu0 + 0.05 * torch.randn_like(mu0)
    sig_old = torch.full_like(mu0, 0.65)
    res = []
    for fused in (True, False):
        pol.zero_grad()
        if fused:
            s, v, ent, kl, _, _ = fused_loss.ppo_losses(alg, obs, cobs, act, val_old, adv, ret, logp_old, mu_old,
                                                        sig_old)
            loss = s + alg.value_loss_coef * v - alg.entropy_coef * ent
        else:
            pol.update_distribution(obs)
            lpb = pol.get_actions_log_prob(act)
            vb = pol.evaluate(cobs)
            s, v = alg._ppo_losses(lpb, logp_old, adv, vb, val_old, ret)
            loss = s + alg.value_loss_coef * v - alg.entropy_coef * pol.entropy.mean()
            with torch.no_grad():
                sb = pol.action_std
                kl = torch.sum(torch.log(sb / sig_old + 1.0e-5) + (sig_old ** 2 + (mu_old - pol.action_mean) ** 2)
                               / (2.0 * sb ** 2) - 0.5, axis=-1).mean()
        loss.backward()
        res.append((float(s), float(v), float(kl), [p.grad.clone() for p in pol.parameters()]))
    (sa, va, ka, ga), (sb_, vb_, kb, gb_) = res
    assert abs(sa - sb_) <= 1e-5 * (abs(sb_) + 1e-3), (sa, sb_)
    assert abs(va - vb_) <= 1e-5 * abs(vb_)
    assert abs(ka - kb) <= 1e-5 * (abs(kb) + 1e-3)
    for a, b in zip(ga, gb_):
        assert float((a - b).norm()) <= 1e-4 * float(b.norm()) + 1e-9


@pytest.mark.parametrize("clipped", [True, False])
def test_fused_ppo_losses_keep_nan_like_torch(clipped):
    """torch.max / torch.clamp keep a NaN.  A row with advantage 0 and ratio inf (-0 * inf = NaN in the
    surrogate) makes torch's surrogate NaN; a NaN value makes the value loss NaN.  The fused losses must agree."""
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl import fused_loss
    from generalizableracing_amd.rsl_rl.ppo import PPO

    torch.manual_seed(8)
    dev = "cuda:0"
    m = 1024
    pol = ActorCritic(16, 16, 4, [64, 64], [64, 64], "lrelu", init_noise_std=0.7).to(dev)
    alg = PPO(pol, device=dev, clip_param=0.2, use_clipped_value_loss=clipped)
    obs, cobs = torch.randn(m, 16, device=dev), torch.randn(m, 16, device=dev)
    with torch.no_grad():
        mu0 = pol.actor(obs)
        act = mu0 + 0.7 * torch.randn_like(mu0)
        logp_old = torch.distributions.Normal(mu0, 0.7).log_prob(act).sum(-1, keepdim=True)
        val_old = pol.critic(cobs)
    adv = torch.randn(m, 1, device=dev)
    ret = torch.randn(m, 1, device=dev)
    logp_old[5] = -1e30  # ratio = exp(logp + 1e30) = inf
    adv[5] = 0.0
    ret[9] = float("nan")
    s_f, v_f, _, _, _, _ = fused_loss.ppo_losses(alg, obs, cobs, act, val_old, adv, ret, logp_old, mu0, torch.full_like(mu0, 0.7))
    with torch.no_grad():
        pol.update_distribution(obs)
        s_t, v_t = alg._ppo_losses(pol.get_actions_log_prob(act), logp_old, adv, pol.evaluate(cobs), val_old, ret)
    assert torch.isnan(s_t) and torch.isnan(s_f), (float(s_t), float(s_f))
    assert torch.isnan(v_t) and torch.isnan(v_f), (float(v_t), float(v_f))


def test_fused_combined_loss_matches_separate():
    """fused_loss.ppo_loss (the loss finished on the device: gr_ppo_loss_forward_loss / backward_loss) against
    ppo_losses composed in torch (ppo.py:171-172: surrogate + value_loss_coef * value - entropy_coef * entropy):
    the loss, the means, the accumulators and every parameter gradient bit-identical (the same fp32 ops)."""
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl import fused_loss
    from generalizableracing_amd.rsl_rl.ppo import PPO

    torch.manual_seed(6)
    dev = "cuda:0"
    m = 12288
    pol = ActorCritic(16, 16, 4, [64, 64], [64, 64], "lrelu", init_noise_std=0.7).to(dev)
    alg = PPO(pol, device=dev, clip_param=0.2, entropy_coef=0.01, value_loss_coef=0.5)
    obs, cobs = torch.randn(m, 16, device=dev), torch.randn(m, 16, device=dev)
    with torch.no_grad():
        mu0 = pol.actor(obs)
        act = mu0 + 0.7 * torch.randn_like(mu0)
        logp_old = torch.distributions.Normal(mu0, 0.7).log_prob(act).sum(-1, keepdim=True) \
            + torch.randn(m, 1, device=dev) * 0.3
        val_old = pol.critic(cobs) + torch.randn(m, 1, device=dev) * 0.3
    adv, ret = torch.randn(m, 1, device=dev), torch.randn(m, 1, device=dev)
    mu_old = mu0 + 0.05 * torch.randn_like(mu0)
    sig_old = torch.full_like(mu0, 0.65)
    args = (obs, cobs, act, val_old, adv, ret, logp_old, mu_old, sig_old)
    pol.zero_grad()
    acc = torch.tensor([1.0, 2.0], device=dev)
    kl_out = torch.zeros(1, device=dev)
    loss_a, stats = fused_loss.ppo_loss(alg, *args, acc=acc, kl_out=kl_out)
    loss_a.backward()
    ga = [p.grad.clone() for p in pol.parameters()]
    pol.zero_grad()
    s, v, ent, kl, _, _ = fused_loss.ppo_losses(alg, *args)
    loss_b = s + alg.value_loss_coef * v - alg.entropy_coef * ent
    loss_b.backward()
    gb_ = [p.grad.clone() for p in pol.parameters()]
    assert torch.equal(loss_a, loss_b)
    assert torch.equal(stats, torch.stack([s, v, kl]).detach())
    assert torch.equal(acc, torch.stack([1.0 + s, 2.0 + v]).detach()) and torch.equal(kl_out[0], kl)
    for a, b in zip(ga, gb_):
        assert torch.equal(a, b)


def _actor_critic_shapes():
    # ActorCritic(16, 16, 4) with [256, 256, 256] hidden layers: weights, biases, std (ppo.py:39's parameters)
    sh = []
    for d_in in (16, 16):
        for a, b in ((256, d_in), (256, 256), (256, 256)):
            sh += [(a, b), (a,)]
    sh += [(4, 256), (4,), (1, 256), (1,), (4,)]
    return sh


@pytest.mark.parametrize("max_norm", [1.0, 1.0e3])
def test_flat_adam_matches_torch(max_norm):
    """FlatAdam's clip + step (flat_adam.py, gr_adam_clip / gr_adam_step) vs nn.utils.clip_grad_norm_ +
    torch.optim.Adam (foreach, ppo.py:178-181) over 5 steps with a changing rate; one parameter without a
    gradient (skipped by both, no state).  The clip's norm accumulates in double (torch: fp32 per-tensor norms),
    so the coefficient may differ in the last ulp: 1e-6 relative on the norm and the gradients; the parameters
    within 1e-6 of the rate (a few ulp of one step's size; where a parameter is near zero, that is a large
    relative difference)."""
    from generalizableracing_amd.rsl_rl.flat_adam import FlatAdam

    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = _actor_critic_shapes()
    p0 = [torch.randn(s, generator=g) * 0.1 for s in shapes]
    pa = [p.clone().to(DEV).requires_grad_() for p in p0]
    pb = [p.clone().to(DEV).requires_grad_() for p in p0]
    oa = FlatAdam(pa, lr=1e-3)
    ob = torch.optim.Adam(pb, lr=1e-3)
    skip = 5
    for it in range(5):
        lr = 1e-3 * (1.5 ** it)
        oa.param_groups[0]["lr"] = lr
        for gr_ in ob.param_groups:
            gr_["lr"] = lr
        for i, (a, b) in enumerate(zip(pa, pb)):
            if i == skip:
                a.grad = b.grad = None
                continue
            gg = (torch.randn(a.shape, generator=g) * (0.05 + it)).to(DEV)
            a.grad, b.grad = gg.clone(), gg.clone()
        na = oa.clip_grad_norm_(max_norm)
        nb = torch.nn.utils.clip_grad_norm_(pb, max_norm)
        torch.testing.assert_close(na, nb, rtol=1e-6, atol=0)
        torch.testing.assert_close([a.grad for a in pa if a.grad is not None],
                                   [b.grad for b in pb if b.grad is not None], rtol=2e-6, atol=1e-12)
        vers = [a._version for a in pa]
        oa.step()
        ob.step()
        torch.cuda.synchronize()
        # the stepped parameters' version counters move, as torch's in-place Adam moves them (the fused rollout
        # inference repacks its weights on a version change); the one without a gradient keeps its version
        assert [a._version > v for a, v in zip(pa, vers)] == [i != skip for i in range(len(pa))]
        for a, b in zip(pa, pb):
            torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-6, atol=1e-6 * lr)
    assert pa[skip] not in oa.state or not oa.state[pa[skip]]
    for a, b in zip(pa, pb):
        if b in ob.state:
            sa, sb = oa.state[a], ob.state[b]
            assert float(sa["step"]) == float(sb["step"]) == 5.0
            for k in ("exp_avg", "exp_avg_sq"):  # (near-zero moments: relative to the tensor's scale)
                torch.testing.assert_close(sa[k], sb[k], rtol=2e-6, atol=1e-6 * float(sb[k].abs().max()))
    # torch Adam's state dict loads into FlatAdam and back
    oc = FlatAdam([p.detach().clone().requires_grad_() for p in pb], lr=1e-3)
    oc.load_state_dict(ob.state_dict())
    for p, b in zip(oc.param_groups[0]["params"], pb):
        if b in ob.state:
            torch.testing.assert_close(oc.state[p]["exp_avg_sq"], ob.state[b]["exp_avg_sq"], rtol=0, atol=0)
    od = torch.optim.Adam(pb, lr=1e-3)
    od.load_state_dict(oa.state_dict())
    assert float(od.state[pb[0]]["step"]) == 5.0


def test_flat_adam_graph_capture_reads_rate_tensor():
    """A captured clip + step replays with the rate read from its device tensor at replay: bit-identical to eager
    steps at the same (fp32-rounded) rate."""
    from generalizableracing_amd.rsl_rl.flat_adam import FlatAdam

    g = torch.Generator(device="cpu").manual_seed(4)
    shapes = _actor_critic_shapes()
    p0 = [torch.randn(s, generator=g) * 0.1 for s in shapes]
    pa = [p.clone().to(DEV).requires_grad_() for p in p0]
    pb = [p.clone().to(DEV).requires_grad_() for p in p0]
    grads = [(torch.randn(s, generator=g)).to(DEV) for s in shapes]
    for a, b, gg in zip(pa, pb, grads):
        a.grad, b.grad = gg.clone(), gg.clone()
    lr = torch.tensor(1e-3, device=DEV)
    oa = FlatAdam(pa, lr=lr)
    ob = FlatAdam(pb, lr=float(lr))
    for o in (oa, ob):  # one eager step first (the table is uploaded outside the capture)
        o.clip_grad_norm_(1.0)
        o.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        oa.clip_grad_norm_(1.0)
        oa.step()
    for it in range(3):
        lr.fill_(1e-3 * (it + 1))
        ob.param_groups[0]["lr"] = float(lr)
        for a, b, gg in zip(pa, pb, grads):
            a.grad.copy_(gg * (it + 1))
            b.grad.copy_(gg * (it + 1))
        graph.replay()
        ob.clip_grad_norm_(1.0)
        ob.step()
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.equal(a.detach(), b.detach())


@pytest.mark.parametrize("adaptive", [False, True])
def test_flat_adam_clip_and_step_equals_three_calls(adaptive):
    """gr_adam_clip_step (FlatAdam.clip_and_step: two launches, the graphed update's segment B) is bit-identical to
    gr_adaptive_lr + gr_adam_clip + gr_adam_step over 4 steps, captured and replayed, with the KL below, inside and
    above the rule's band (the rate moves both ways), one parameter without a gradient, and the clip active."""
    from generalizableracing_amd import _abi
    from generalizableracing_amd.rsl_rl.flat_adam import FlatAdam

    g = torch.Generator(device="cpu").manual_seed(5)
    shapes = _actor_critic_shapes()
    p0 = [torch.randn(s, generator=g) * 0.1 for s in shapes]
    pa = [p.clone().to(DEV).requires_grad_() for p in p0]
    pb = [p.clone().to(DEV).requires_grad_() for p in p0]
    grads = [(torch.randn(s, generator=g)).to(DEV) for s in shapes]
    skip = 3
    for i, (a, b, gg) in enumerate(zip(pa, pb, grads)):
        if i != skip:
            a.grad, b.grad = gg.clone(), gg.clone()
    lra, lrb = torch.tensor(1e-3, device=DEV), torch.tensor(1e-3, device=DEV)
    kla, klb = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    oa, ob = FlatAdam(pa, lr=lra), FlatAdam(pb, lr=lrb)
    desired = 0.01
    lib = _abi.load()

    def three():
        if adaptive:
            assert lib.gr_adaptive_lr(klb.data_ptr(), lrb.data_ptr(), C.c_double(desired), C.c_double(1e-5),
                                      C.c_double(1e-2), torch.cuda.current_stream().cuda_stream) == 0
        ob.clip_grad_norm_(0.5)
        ob.step()

    oa.clip_and_step(0.5, kl=kla if adaptive else None, desired_kl=desired)  # (tables uploaded outside the capture)
    three()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        oa.clip_and_step(0.5, kl=kla if adaptive else None, desired_kl=desired)
    for it, kl in enumerate((0.05, 0.001, 0.0, 0.01)):
        kla.fill_(kl)
        klb.fill_(kl)
        for i, (a, b, gg) in enumerate(zip(pa, pb, grads)):
            if i != skip:
                a.grad.copy_(gg * (it + 2))
                b.grad.copy_(gg * (it + 2))
        graph.replay()
        three()
        torch.cuda.synchronize()
        assert torch.equal(lra, lrb), it
        assert torch.equal(oa._norm, ob._norm), it
        for a, b in zip(pa, pb):
            assert torch.equal(a.detach(), b.detach()), it
            if a.grad is not None:
                assert torch.equal(a.grad, b.grad), it
    if adaptive:
        assert float(lra) != 1e-3
    for a, b in zip(pa, pb):
        if b in ob.state:
            for k in ("step", "exp_avg", "exp_avg_sq"):
                assert torch.equal(oa.state[a][k], ob.state[b][k]), k
