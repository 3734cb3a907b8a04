"""Golden vectors for the PPO / PPOL2C2 update, produced by the REFERENCE's own algorithm and storage code.

Run in the development container (the reference is mounted read-only at /root/reference; it never
travels to the GPU box):

    python tests/golden/make_golden_ppo.py

Loads standalone/rsl_rl/ext/algorithms/ppo.py, ppo_l2c2.py and storage/rollout_storage.py,
rollout_storage_l2c2.py from the reference tree.  rsl_rl is not installed: `rsl_rl.modules.ActorCritic`
(a type annotation there) is bound to the build's ActorCritic, the policy module both sides step (the MLP +
Normal of upstream rsl_rl, restated in generalizableracing_amd/rsl_rl/actor_critic.py), and
`rsl_rl.utils.split_and_pad_trajectories` (recurrent policies only) to a stub.  So the fixtures pin the
reference's rollout bookkeeping (time-out bootstrap, L2C2's zero-observation skip), GAE and advantage
normalisation, the mini-batch generators, the adaptive-KL learning rate, the clipped surrogate / value
losses, the L2C2 smoothness loss, grad clipping and Adam — over two rollout + update iterations.

Inputs are seeded synthetic rollouts (observations, rewards, dones, time-outs); actions are sampled by the
policy from torch's global generator, reseeded at fixed points so the build can replay the same draws.
For L2C2 the policy's act_inference returns (mean, features) as the vision policy's does
(vision_actor_critic.py:43-144), so `act_inference(...)[0]` is the mean on both sides.
"""
from __future__ import annotations

import copy
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import il_shim  # noqa: E402

OUT = os.path.join(HERE, "golden_ppo.npz")
EXT = os.path.join(il_shim.REF, "standalone/rsl_rl/ext")
N, T, OBS = 64, 24, 16
HP = dict(num_learning_epochs=5, num_mini_batches=4, clip_param=0.2, gamma=0.99, lam=0.95, value_loss_coef=1.0,
          entropy_coef=0.005, learning_rate=5e-4, max_grad_norm=1.0, use_clipped_value_loss=True,
          schedule="adaptive", desired_kl=0.01)


def tuple_policy_class():
    from generalizableracing_amd.rsl_rl import ActorCritic

    class TupleActorCritic(ActorCritic):
        """act_inference -> (mean, features), the vision policy's contract (ppo_l2c2.py:184,189 take [0])."""

        def act_inference(self, observations):
            return self.actor(observations), None

    return TupleActorCritic


def load_reference():
    from generalizableracing_amd.rsl_rl import ActorCritic

    for n in ("rsl_rl", "rsl_rl.modules", "rsl_rl.utils", "standalone", "standalone.rsl_rl", "standalone.rsl_rl.ext"):
        sys.modules.setdefault(n, types.ModuleType(n))
    sys.modules["rsl_rl.modules"].ActorCritic = ActorCritic
    sys.modules["rsl_rl.utils"].split_and_pad_trajectories = il_shim._unsupported
    st = il_shim.synthetic_package("standalone.rsl_rl.ext.storage", os.path.join(EXT, "storage"))
    rs = il_shim.load("standalone.rsl_rl.ext.storage.rollout_storage", os.path.join(EXT, "storage/rollout_storage.py"))
    rs2 = il_shim.load("standalone.rsl_rl.ext.storage.rollout_storage_l2c2",
                       os.path.join(EXT, "storage/rollout_storage_l2c2.py"))
    st.RolloutStorage, st.RolloutStorageL2C2 = rs.RolloutStorage, rs2.RolloutStorageL2C2
    ppo = il_shim.load("grref_ppo", os.path.join(EXT, "algorithms/ppo.py"))
    l2c2 = il_shim.load("grref_ppo_l2c2", os.path.join(EXT, "algorithms/ppo_l2c2.py"))
    return ppo.PPO, l2c2.PPOL2C2


def rollout_inputs(seed, iters=2):
    """Synthetic rollouts: per iteration obs / critic obs [T, N, 16], rewards [T, N], dones [T, N] (long),
    time_outs [T, N] (bool), the last critic obs [N, 16]; step 5 of iteration 1 has an all-zero
    observation batch (L2C2 skips storing it)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for it in range(iters):
        obs = torch.randn(T, N, OBS, generator=g)
        cobs = torch.randn(T, N, OBS, generator=g)
        rew = torch.randn(T, N, generator=g) * 0.1
        dones = (torch.rand(T, N, generator=g) < 0.05).long()
        tout = (torch.rand(T, N, generator=g) < 0.5) & dones.bool()
        last = torch.randn(N, OBS, generator=g)
        if it == 1:
            obs[5] = 0.0
        out.append((obs, cobs, rew, dones, tout, last))
    return out


def make_policy(cls):
    torch.manual_seed(0)
    return cls(OBS, OBS, 4, [64, 64], [64, 64], "lrelu")


def run(alg, data, record, prefix):
    """Two iterations of rollout (act / process_env_step) -> compute_returns -> update; reseeds torch's
    generator at fixed points (the build's test replays the same sequence)."""
    alg.init_storage("rl", N, T, [OBS], [OBS], [4])
    for it, (obs, cobs, rew, dones, tout, last) in enumerate(data):
        torch.manual_seed(100 + it)
        with torch.inference_mode():
            for t in range(T):
                alg.act(obs[t], cobs[t])
                alg.process_env_step(rew[t], dones[t], {"time_outs": tout[t]})
            alg.compute_returns(last)
        st = alg.storage
        for k in ("actions", "values", "actions_log_prob", "mu", "sigma", "rewards", "returns", "advantages"):
            record[f"{prefix}_it{it}_{k}"] = getattr(st, k).clone()
        record[f"{prefix}_it{it}_stored_steps"] = torch.tensor(st.step)
        torch.manual_seed(200 + it)
        losses = alg.update()
        for k, v in losses.items():
            record[f"{prefix}_it{it}_loss_{k}"] = torch.tensor(float(v), dtype=torch.float64)
        record[f"{prefix}_it{it}_lr"] = torch.tensor(float(alg.learning_rate), dtype=torch.float64)
        record[f"{prefix}_it{it}_params"] = torch.cat([p.detach().reshape(-1) for p in alg.policy.parameters()])


def main():
    RefPPO, RefL2C2 = load_reference()
    from generalizableracing_amd.rsl_rl import ActorCritic

    data = rollout_inputs(7)
    rec = {}
    for i, (obs, cobs, rew, dones, tout, last) in enumerate(data):
        for k, v in (("obs", obs), ("cobs", cobs), ("rew", rew), ("dones", dones), ("tout", tout), ("last", last)):
            rec[f"in_it{i}_{k}"] = v
    pol = make_policy(ActorCritic)
    rec["init_params"] = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    run(RefPPO(copy.deepcopy(pol), None, device="cpu", **HP), data, rec, "ppo")
    TAC = tuple_policy_class()
    pol2 = make_policy(TAC)
    run(RefL2C2(pol2, None, device="cpu", value_smoothness_coef=0.1, smoothness_upper_bound=1.0,
                smoothness_lower_bound=0.1, **HP), data, rec, "l2c2")
    out = {}
    for k, v in rec.items():
        a = v.detach().cpu().numpy()
        if a.dtype == np.bool_:
            a = a.astype(np.uint8)
        out[k] = np.ascontiguousarray(a)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {sum(v.nbytes for v in out.values()) / 1e3:.1f} kB raw, {len(out)} arrays; lr "
          f"ppo {float(rec['ppo_it1_lr']):.3e} l2c2 {float(rec['l2c2_it1_lr']):.3e}, stored steps "
          f"{int(rec['l2c2_it1_stored_steps'])}")


if __name__ == "__main__":
    main()
