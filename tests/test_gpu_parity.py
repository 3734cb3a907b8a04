"""HIP kernel (through the C ABI) vs the CPU oracle — the parity suite proper.

Bar (north star): gate index and done masks bit-exact, float state within
1e-5.  Because kernel and oracle share the elementary functions and are both
built without FMA contraction, the whole state, observations, rewards and
masks are asserted BIT-EXACT here; the 1e-5 tolerance is only used for the
log means (different reduction trees).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from generalizableracing_amd import _abi  # noqa: E402
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402

DEV = "cuda:0"


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def assert_envs_equal(got, want, where=""):
    for name in oracle.ENV_DTYPE.names:
        g, w = bits(got[name]), bits(want[name])
        if not np.array_equal(g, w):
            idx = np.argwhere(g != w)[0]
            raise AssertionError(f"{where}: field {name} differs at {idx}: kernel {got[name][idx[0]]} "
                                 f"oracle {want[name][idx[0]]}")


def kernel_envs(env):
    torch.cuda.synchronize()
    return oracle.planes_to_envs(env.state.cpu().numpy(), env.istate.cpu().numpy())


def make(n, stage=1, integrator="dd_explicit", gates=8, obstacles=True, **ov):
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=stage, integrator=integrator,
                       terrain=TerrainCfg(num_gates=gates, obstacles=obstacles), overrides=ov)
    env = RacingEnv(cfg)
    orc = oracle.from_env(env)
    orc.init()
    return env, orc


def compare_outputs(env, orc, where):
    s = env.obs_buf
    for key, want in (("policy", orc.obs_policy), ("critic", orc.obs_critic)):
        got = s[key].cpu().numpy()
        assert np.array_equal(bits(got), bits(want)), (where, key, np.abs(got - want).max())
    assert np.array_equal(bits(s["auxiliary"].cpu().numpy()[:, 0]), bits(orc.obs_aux)), where


CONFIGS = [
    dict(stage=1),
    dict(stage=1, integrator="semi_implicit"),
    dict(stage=0),
    dict(stage=2),
    dict(stage=1, use_motor_model=1),
    dict(stage=1, gates=32),
    dict(stage=1, obstacles=False),
    dict(stage=1, dr_rotor=1),                               # config C5: per-env rotor constants
    dict(stage=1, dr_rotor=1, use_motor_model=1, gates=32),  # ... through the motor model's allocation
]


@pytest.mark.parametrize("conf", CONFIGS, ids=[str(c) for c in CONFIGS])
def test_env_free_run_bit_exact(conf):
    n, steps = 1000, 120
    conf = dict(conf)
    env, orc = make(n, stage=conf.pop("stage"), integrator=conf.pop("integrator", "dd_explicit"),
                    gates=conf.pop("gates", 8), obstacles=conf.pop("obstacles", True), **conf)
    assert_envs_equal(kernel_envs(env), orc.envs, "init")
    compare_outputs(env, orc, "init")
    env.reset()
    orc.reset(None)
    assert_envs_equal(kernel_envs(env), orc.envs, "reset")
    compare_outputs(env, orc, "reset")
    # random episode lengths (the runner's init_at_random_ep_len) so time-outs happen
    g = torch.Generator().manual_seed(5)
    eplen = torch.randint(0, 200, (n,), generator=g, dtype=torch.int32)
    env.episode_length_buf = eplen.to(DEV)
    orc.envs["ep_len"] = eplen.numpy()
    n_done = 0
    for k in range(steps):
        a = (torch.randn(n, 4, generator=g) * 1.2).numpy().astype(np.float32)
        _, rew, term, tout, extras = env.step(torch.from_numpy(a).to(DEV))
        orc.step(a)
        torch.cuda.synchronize()
        where = f"step {k}"
        assert np.array_equal(bits(rew.cpu().numpy()), bits(orc.reward)), where
        assert np.array_equal(term.cpu().numpy().astype(np.uint8), orc.terminated), where
        assert np.array_equal(tout.cpu().numpy().astype(np.uint8), orc.time_out), where
        dones = env._sets[env._cur]["dones"].cpu().numpy()
        assert np.array_equal(dones, orc.dones), where
        assert_envs_equal(kernel_envs(env), orc.envs, where)
        compare_outputs(env, orc, where)
        log = extras["log"]
        row = np.array([float(log[key]) for key in log])
        want = np.array([orc.log[env._log_keys[key]] for key in log])
        np.testing.assert_allclose(row, want, rtol=2e-5, atol=1e-5, err_msg=where)
        n_done += int(orc.dones.sum())
    assert n_done > 20  # resets were exercised
    # observe(): fresh observation noise, no state change
    env.observe()
    orc.observe()
    compare_outputs(env, orc, "observe")
    # partial reset through a mask
    mask = np.zeros(n, np.uint8)
    mask[::7] = 1
    env.reset(env_ids=np.nonzero(mask)[0])
    orc.reset(mask)
    assert_envs_equal(kernel_envs(env), orc.envs, "masked reset")
    compare_outputs(env, orc, "masked reset")
    # reset over no envs: the reference's _reset_idx([]) logs NaN means and zero termination counts
    _, extras = env.reset(env_ids=np.zeros(0, np.int64))
    log = extras["log"]
    for key in log:
        v = float(log[key])
        if key.startswith(("Episode_Reward/", "Metrics/")):
            assert np.isnan(v), key
        elif key.startswith("Episode_Termination/"):
            assert v == 0.0, key
        else:
            assert np.isfinite(v), key
    env.close()


@pytest.mark.parametrize("n", [1, 63, 257])
def test_ragged_env_counts_bit_exact(n):
    """Env counts that leave most of the last workgroup (and of its waves) empty: a single env, less than one
    wave, one env past a whole workgroup.  Dead lanes must neither store nor disturb the live ones."""
    env, orc = make(n, obstacles=True)
    env.reset()
    orc.reset(None)
    g = torch.Generator().manual_seed(n)
    for k in range(60):
        a = (torch.randn(n, 4, generator=g) * 1.5).numpy().astype(np.float32)
        _, rew, term, tout, _ = env.step(torch.from_numpy(a).to(DEV))
        orc.step(a)
        torch.cuda.synchronize()
        where = f"n {n} step {k}"
        assert np.array_equal(bits(rew.cpu().numpy()), bits(orc.reward)), where
        assert np.array_equal(term.cpu().numpy().astype(np.uint8), orc.terminated), where
        assert np.array_equal(tout.cpu().numpy().astype(np.uint8), orc.time_out), where
        assert_envs_equal(kernel_envs(env), orc.envs, where)
        compare_outputs(env, orc, where)
    env.close()


GRAPH_LEN = 64  # bench.py ACTION_RING: the headline is timed as replays of a 64-step hipGraph


def capture_step_graph(env, actions):
    """The bench's capture (bench.py capture_graph): the host call counter aligned to a multiple of the ring,
    then GRAPH_LEN consecutive env steps on actions[0..GRAPH_LEN) captured in one hipGraph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for k in range(2):
            env.step(actions[k])
    torch.cuda.current_stream().wait_stream(s)
    while env._calls % GRAPH_LEN != 0:
        env.step(actions[env._calls % GRAPH_LEN])
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for k in range(GRAPH_LEN):
            env.step(actions[k])
    torch.cuda.synchronize()
    return graph


# slices of 256 envs at 65 536 envs: type t starts at env ceil(t * 3276.8), workgroups are 256 envs; each slice
# below straddles a workgroup edge and a terrain-type boundary (workgroup 12 holds types 0|1 around env 3277,
# workgroup 24 types 1|2 around 6554, workgroup 179 types 13|14 around 45876) or the last workgroup
FULL_SIZE_SLICES = [3277 - 128, 6554 - 180, 32768 - 128, 45876 - 60, 65536 - 256]


@pytest.mark.parametrize("obstacles", [False, True], ids=["gates_only_C3_headline", "obstacles"])
def test_full_size_teacher_forced_slices(obstacles):
    """65 536 envs (BASELINE C3 size), stepped the way bench.py steps them: replays of a captured 64-step hipGraph.
    Before each replay the slices' state is read; the oracle re-steps each slice 64 times from it (teacher forcing
    over the whole replay) and must match the kernel bit for bit: state, last step's policy row, reward and dones.
    obstacles=False runs the headline instantiation step_kernel<true, false, 8, 1> (LDS track slice staged per
    workgroup over its own terrain-type range); the test asserts that instantiation is the one launched."""
    n, m, replays = 65536, 256, 6
    env, _ = make(n, obstacles=obstacles)
    want_kernel = "step_kernel<false, true, 0, 1>" if obstacles else "step_kernel<true, false, 8, 1>"
    assert env.step_kernel_name() == want_kernel
    env.reset()
    g = torch.Generator().manual_seed(11)
    env.episode_length_buf = torch.randint(0, 200, (n,), generator=g, dtype=torch.int32).to(DEV)
    acts = torch.zeros(GRAPH_LEN, n, 4, device=DEV)
    acts.copy_(torch.randn(GRAPH_LEN, n, 4, generator=g) * 1.2)
    graph = capture_step_graph(env, acts)
    base = env.gr_config
    ot = env.obstacle_table
    gates_h, recs_h = env.track_gates.cpu().numpy(), env.track_records.cpu().numpy()
    seen_types, n_done = set(), 0
    for r in range(replays):
        a = (torch.randn(GRAPH_LEN, n, 4, generator=g) * 1.2)
        acts.copy_(a)  # the graph reads the ring in place
        a = a.numpy()
        torch.cuda.synchronize()
        assert env._calls % GRAPH_LEN == 0 and env._cur == 0
        pre_st = env.state.cpu().numpy()
        pre_ist = env.istate.cpu().numpy()
        prev_crit = env.obs_buf["critic"].cpu().numpy()
        cnt = int(env._counters[0].item())
        graph.replay()
        torch.cuda.synchronize()
        post = kernel_envs(env)
        out = env._sets[env._cur]
        for i0 in FULL_SIZE_SLICES:
            c = _abi.GrConfig.from_buffer_copy(base)
            c.num_envs = m
            c.env_id_offset = i0
            orc = oracle.Oracle(c, gates_h, recs_h, None if ot is None else ot.records, None if ot is None else ot.counts)
            orc.envs[:] = oracle.planes_to_envs(pre_st[:, i0:i0 + m], pre_ist[i0:i0 + m])
            orc.obs_critic[:] = prev_crit[i0:i0 + m]
            orc.counter[0] = cnt
            seen_types.update(orc.envs["type"].tolist())
            for k in range(GRAPH_LEN):
                orc.step(a[k, i0:i0 + m])
                n_done += int(orc.dones.sum())
            where = f"replay {r} slice {i0}"
            assert_envs_equal(post[i0:i0 + m], orc.envs, where)
            assert np.array_equal(bits(out["policy"][i0:i0 + m].cpu().numpy()), bits(orc.obs_policy)), where
            assert np.array_equal(bits(out["critic"][i0:i0 + m].cpu().numpy()), bits(orc.obs_critic)), where
            assert np.array_equal(bits(out["reward"][i0:i0 + m].cpu().numpy()), bits(orc.reward)), where
            assert np.array_equal(out["dones"][i0:i0 + m].cpu().numpy(), orc.dones), where
    del graph
    assert len(seen_types) >= 4, seen_types
    assert n_done > 100  # in-kernel resets were exercised inside the graph
    # invariants on all envs
    e = kernel_envs(env)
    assert np.isfinite(e["p"]).all() and np.isfinite(e["q"]).all() and np.isfinite(e["v"]).all()
    assert np.abs(np.linalg.norm(e["q"].astype(np.float64), axis=1) - 1).max() < 1e-5
    assert (e["level"] >= 0).all() and (e["level"] < 10).all()
    assert (e["gate_id"] >= 0).all() and (e["gate_id"] < 8).all()
    assert (e["ep_len"] >= 0).all() and (e["ep_len"] < 200).all()
    env.close()


def test_obstacle_collisions_teacher_forced():
    """Drones placed in and around the obstacles of their own tracks (walls, orbits, ground obstacles):
    one step must match the oracle (which tests every obstacle, no grid) bit for bit, and many of the
    placed drones must collide."""
    n = 4096
    env, _ = make(n)
    env.reset()
    torch.cuda.synchronize()
    ot = env.obstacle_table
    e = kernel_envs(env)
    rng = np.random.default_rng(9)
    L = env.cfg.terrain.num_rows
    for i in range(n):
        k = int(e["type"][i]) * L + int(e["level"][i])
        j = rng.integers(ot.counts[k])
        rec = ot.records[k, j]
        e["p"][i] = (rec[:3] + rng.uniform(-1, 1, 3) * (rec[17] + 0.08)).astype(np.float32)
        q = rng.normal(size=4)
        e["q"][i] = (q / np.linalg.norm(q)).astype(np.float32)
        e["v"][i] = 0.0
    st, ist = oracle.envs_to_planes(e, env.state.shape[0])
    env.state.copy_(torch.from_numpy(st).to(DEV))
    env.istate.copy_(torch.from_numpy(ist).to(DEV))
    prev_crit = env.obs_buf["critic"].cpu().numpy()
    cnt = int(env._counters[env._calls % 2].item())
    orc = oracle.from_env(env)
    orc.envs[:] = e
    orc.obs_critic[:] = prev_crit
    orc.counter[0] = cnt
    a = np.zeros((n, 4), np.float32)
    _, rew, term, tout, _ = env.step(torch.from_numpy(a).to(DEV))
    orc.step(a)
    torch.cuda.synchronize()
    assert np.array_equal(bits(rew.cpu().numpy()), bits(orc.reward))
    assert np.array_equal(term.cpu().numpy().astype(np.uint8), orc.terminated)
    assert_envs_equal(kernel_envs(env), orc.envs, "obstacle step")
    assert orc.terminated.mean() > 0.2, orc.terminated.mean()
    env.close()


def test_terrain_regeneration_matches_oracle():
    """EventCfg.reset_terrain: after the interval the env regenerates its tracks (new layouts and
    obstacles) and resets every env; the oracle over the new tables agrees bit for bit."""
    n = 512
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=1,
                       terrain=TerrainCfg(regen_interval_s=0.03 * 5))
    env = RacingEnv(cfg)
    env.reset()
    g0 = env.track_gates.clone()
    g = torch.Generator().manual_seed(1)
    for k in range(5):
        _, _, _, _, extras = env.step(torch.randn(n, 4, generator=g).to(DEV))
    assert extras.get("terrain_regenerated") and env.terrain_generation == 1
    assert not torch.equal(g0, env.track_gates)
    orc = oracle.from_env(env)
    torch.cuda.synchronize()
    orc.envs[:] = kernel_envs(env)
    orc.obs_critic[:] = env.obs_buf["critic"].cpu().numpy()
    orc.counter[0] = int(env._counters[env._calls % 2].item())
    assert (orc.envs["ep_len"] == 0).all()
    for k in range(4):  # the 5th step regenerates again
        a = (torch.randn(n, 4, generator=g)).numpy().astype(np.float32)
        _, _, _, _, extras = env.step(torch.from_numpy(a).to(DEV))
        orc.step(a)
        torch.cuda.synchronize()
        assert_envs_equal(kernel_envs(env), orc.envs, f"after regen step {k}")
        assert not extras.get("terrain_regenerated")
    # the regenerating step: the step's reward / dones with the post-reset observations (reference order:
    # interval event, then observation compute), and the previous step's observation tensors untouched
    prev_obs = {k: v for k, v in env.obs_buf.items()}
    prev_copy = {k: v.clone() for k, v in prev_obs.items()}
    a = (torch.randn(n, 4, generator=g)).numpy().astype(np.float32)
    obs, rew, term, tout, extras = env.step(torch.from_numpy(a).to(DEV))
    assert extras.get("terrain_regenerated") and env.terrain_generation == 2
    assert bool((env.episode_length_buf == 0).all())
    orc.step(a)
    want_rew, want_term, want_dones = orc.reward.copy(), orc.terminated.copy(), orc.dones.copy()
    orc2 = oracle.from_env(env)  # the new terrain's tables
    orc2.envs[:] = orc.envs
    orc2.obs_critic[:] = orc.obs_critic
    orc2.obs_aux[:] = orc.obs_aux
    orc2.time_out[:] = orc.time_out
    orc2.counter[0] = orc.counter[0]
    orc2.reset(None)
    orc2.observe()
    torch.cuda.synchronize()
    assert np.array_equal(bits(rew.cpu().numpy()), bits(want_rew))
    assert np.array_equal(term.cpu().numpy().astype(np.uint8), want_term)
    assert np.array_equal(env._sets[env._cur]["dones"].cpu().numpy(), want_dones)
    assert_envs_equal(kernel_envs(env), orc2.envs, "regenerating step")
    compare_outputs(env, orc2, "regenerating step")
    for k, v in prev_obs.items():
        assert torch.equal(v, prev_copy[k]), k
    env.close()


def test_wrapper_across_terrain_regeneration():
    """RslRlVecEnvWrapper over a regenerating step: dones are the step's, the runner's previous
    observation tensor still holds the previous step's rows when process_env_step copies it."""
    n = 256
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=1,
                       terrain=TerrainCfg(regen_interval_s=0.03 * 3))
    venv = RslRlVecEnvWrapper(RacingEnv(cfg))
    obs, _ = venv.get_observations()
    g = torch.Generator().manual_seed(2)
    for k in range(3):
        kept = obs.clone()
        a = torch.randn(n, 4, generator=g).to(DEV)
        obs_next, rew, dones, extras = venv.step(a)
        torch.cuda.synchronize()
        assert torch.equal(obs, kept), k  # the transition's observation tensor is intact
        want = (extras["time_outs"] | venv.env._sets[venv.env._cur]["terminated"]).long()
        assert torch.equal(dones, want), k
        obs = obs_next
    assert extras.get("terrain_regenerated")
    venv.close()


def test_terrain_regeneration_step_graph_captured():
    """The interval step (gr_step + gr_terrain_commit + gr_reset + gr_observe, mdp/events.py:180-204) captured in a
    hipGraph: one replay commits the generation the builder staged and equals the same step run eagerly on a twin
    env bit for bit (state, observations, reward, terminated, dones); both then step on identically on the new
    tracks, which the oracle confirms."""
    n = 4096

    def mk():
        cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=1,
                           terrain=TerrainCfg(regen_interval_s=0.03 * 8))
        env = RacingEnv(cfg)
        env.reset()
        return env

    ea, eb = mk(), mk()
    g = torch.Generator().manual_seed(3)
    acts = [torch.randn(n, 4, generator=g).to(DEV) for _ in range(12)]
    for k in range(7):
        ea.step(acts[k])
        eb.step(acts[k])
    for e in (ea, eb):
        assert e._next_terrain.result()[-1] == 0  # generation 1 staged by the builder
    torch.cuda.synchronize()
    obs_a, rew_a, term_a, _, ex_a = ea.step(acts[7])
    a_buf = acts[7].clone()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        obs_b, rew_b, term_b, _, ex_b = eb.step(a_buf)
    graph.replay()
    torch.cuda.synchronize()
    assert ex_a.get("terrain_regenerated") and ex_b.get("terrain_regenerated")
    assert ea.terrain_generation == eb.terrain_generation == 1
    assert torch.equal(ea.track_gates, eb.track_gates)

    def same(where):
        assert torch.equal(ea.state.view(torch.int32), eb.state.view(torch.int32)), where
        assert torch.equal(ea.istate, eb.istate), where

    same("interval step")
    for k in ("policy", "critic"):
        assert torch.equal(obs_a[k].view(torch.int32), obs_b[k].view(torch.int32)), k
    assert torch.equal(rew_a.view(torch.int32), rew_b.view(torch.int32))
    assert torch.equal(term_a, term_b)
    assert torch.equal(ea._sets[ea._cur]["dones"], eb._sets[eb._cur]["dones"])
    assert bool((eb.episode_length_buf == 0).all())
    del graph
    orc = oracle.from_env(eb)  # the new generation's tables (host copies of what was committed)
    orc.envs[:] = kernel_envs(eb)
    orc.obs_critic[:] = eb.obs_buf["critic"].cpu().numpy()
    orc.counter[0] = int(eb._counters[eb._calls % 2].item())
    for k in range(8, 11):
        ea.step(acts[k])
        eb.step(acts[k])
        orc.step(acts[k].cpu().numpy())
        torch.cuda.synchronize()
        same(f"step {k}")
        assert_envs_equal(kernel_envs(eb), orc.envs, f"after the captured regeneration, step {k}")
    ea.close()
    eb.close()


def test_terrain_reservation_does_not_move_under_a_captured_graph():
    """A generation larger than the reservation reallocates the terrain arrays (gr_terrain_reserve): refused while a
    graph captured over the env may still replay (it would read freed arrays); allowed after forget_captures(), and
    the terrain epoch (gr_terrain_epoch) moves with it."""
    from generalizableracing_amd.envs.tracks import ObstacleTable

    n = 1024
    env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=1,
                                 terrain=TerrainCfg(regen_interval_s=0.03 * 1000)))
    env.reset()
    e0 = env.terrain_epoch
    assert e0 >= 1
    a = torch.zeros(n, 4, device=DEV)
    env.step(a)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        env.step(a)
    graph.replay()
    torch.cuda.synchronize()
    build = env._build_terrain

    def bigger(seed):  # the same generation with twice the obstacle slots per track (counts unchanged)
        gates, recs, obst = build(seed)
        m = obst.max_obstacles
        rec = np.zeros((obst.records.shape[0], 2 * m + 16, obst.records.shape[2]), dtype=np.float32)
        rec[:, :m] = obst.records
        return gates, recs, ObstacleTable(rec, obst.counts, obst.grid_f, obst.grid_i, obst.cells, obst.items)

    env._build_terrain = bigger
    if env._next_terrain is not None:
        env._next_terrain.result()
        env._next_terrain = None
    with pytest.raises(RuntimeError, match="forget_captures"):
        env.regenerate_terrain()
    assert env.terrain_epoch == e0
    del graph
    env.forget_captures()
    env.regenerate_terrain()
    assert env.terrain_epoch == e0 + 1
    env.step(a)
    torch.cuda.synchronize()
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_obs_sink_rows(dtype):
    """gr_bind_obs_sink: step / reset / observe also write the policy and critic rows into the bound tensors,
    bit-equal to torch's round-to-nearest-even cast of the fp32 rows they return (ragged env count, rotor DR,
    resets inside the run); unbinding stops the writes."""
    n = 1000
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=1, overrides=dict(dr_rotor=1))
    venv = RslRlVecEnvWrapper(RacingEnv(cfg))
    sp = torch.full((n, 16), 7.0, device=DEV, dtype=dtype)
    sc = torch.full((n, 16), 7.0, device=DEV, dtype=dtype)
    base_bytes = venv.env.bytes_per_env_step()
    venv.set_obs_sink(sp, sc)
    if dtype == torch.float32:  # the slot IS the output: one write per row, no second (sink) row set
        assert venv.env.bytes_per_env_step() == base_bytes
    else:  # bf16: the rounded rows on top of the fp32 output rows
        assert venv.env.bytes_per_env_step()[1] == base_bytes[1] + 64
    obs, ex = venv.get_observations()
    if dtype == torch.float32:
        assert obs.data_ptr() == sp.data_ptr() and ex["observations"]["critic"].data_ptr() == sc.data_ptr()
    torch.cuda.synchronize()
    assert torch.equal(sp, obs.to(dtype)) and torch.equal(sc, ex["observations"]["critic"].to(dtype))
    g = torch.Generator().manual_seed(4)
    resets = 0
    for k in range(40):
        obs, rew, dones, ex = venv.step((3 * torch.randn(n, 4, generator=g)).to(DEV))
        torch.cuda.synchronize()
        resets += int(dones.sum())
        assert torch.equal(sp, obs.to(dtype)), k
        assert torch.equal(sc, ex["observations"]["critic"].to(dtype)), k
    assert resets > 0
    obs, ex = venv.reset()
    torch.cuda.synchronize()
    assert torch.equal(sp, obs.to(dtype)) and torch.equal(sc, ex["observations"]["critic"].to(dtype))
    venv.set_obs_sink(None)
    keep = sp.clone()
    venv.step(torch.zeros(n, 4, device=DEV))
    torch.cuda.synchronize()
    assert torch.equal(sp, keep)
    with pytest.raises(ValueError):
        venv.set_obs_sink(sp[:, :8].contiguous(), sc[:, :8].contiguous())
    venv.close()


@pytest.mark.gpu
@pytest.mark.parametrize("storage_dtype", ["bfloat16", "float32"])
def test_runner_obs_sink_matches_copy(storage_dtype):
    """OnPolicyRunner with the observation sink (bf16: the step kernel also writes the rounded rows into the storage
    slot; fp32: the storage slot IS the step's observation output, each row written once) trains exactly like the
    copy path: same stored observations, same parameters after two learn() calls."""
    from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg

    runs = []
    for sink in (True, False):
        torch.manual_seed(9)
        cfg = QuadcopterPPORunnerCfg(device=DEV, num_steps_per_env=8)
        cfg.algorithm.storage_obs_dtype = storage_dtype
        cfg.algorithm.obs_sink = sink
        env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=512), sim=SimCfg(device=DEV), stage=1))
        r = OnPolicyRunner(RslRlVecEnvWrapper(env), cfg.to_dict(), log_dir=None, device=DEV)
        assert r.obs_sink is sink
        r.learn(2)
        r.learn(1)
        torch.cuda.synchronize()
        runs.append(r)
    a, b = runs
    T = a.num_steps_per_env
    assert torch.equal(a.alg.storage.observations[1:T], b.alg.storage.observations[1:T])
    assert torch.equal(a.alg.storage.privileged_observations[1:T], b.alg.storage.privileged_observations[1:T])
    for (k, x), (_, y) in zip(a.alg.policy.state_dict().items(), b.alg.policy.state_dict().items()):
        assert torch.equal(x, y), k
    for r in runs:
        r.env.close()
