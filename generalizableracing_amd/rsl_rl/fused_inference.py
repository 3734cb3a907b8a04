"""Fused rollout inference of the MLP ActorCritic on MFMA (libgr.so gr_policy_forward).

Two precisions behind the same call: "bf16" (below: bf16 operands, fp32 accumulation, the C5 option) and
"fp32" (the reference's precision: fp32 operands on v_mfma_f32_16x16x4_f32, each output an fp32 fma
chain; the kernel reads the module's row-major fp32 weights, gr_policy_f32.hip).

Replaces, for the rollout, the calls PPO.act makes on the policy
(standalone/rsl_rl/ext/algorithms/ppo.py:71-85): `policy.act(obs)` (sample Normal(actor(obs), std)),
`policy.evaluate(critic_obs)`, `policy.get_actions_log_prob(actions)`, `action_mean`, `action_std`.
One graph-capturable launch computes both MLPs for every env with bf16 operands and fp32
accumulation, samples the actions (Philox, keyed by env and a device call counter) and sums the log
prob.  The update (PPO.update) keeps the fp32 PyTorch module: `refresh()` repacks its weights after
every update.  BASELINE config C5 ("bf16 obs/rollout buffers, hipGraph-captured step+inference").

Weight packing: every layer runs transposed (Y^T = W X^T) with W as the MFMA A operand of
`v_mfma_f32_16x16x32_bf16`, whose lane l holds A[row l & 15][k = 8 (l >> 4) + j], j = 0..7.  The hidden
activations come straight from the previous layer's accumulator tiles (lane l: rows 4 (l >> 4) + r of
tiles 2s and 2s + 1, column l & 15), so inside a 32-wide k step the kernel's element j of lane l is
hidden unit 32 s + 16 (j >> 2) + 4 (l >> 4) + (j & 3); W2 and W3 are packed in that same k order.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn

from .. import _abi


def _lane_j():
    lane = torch.arange(64).view(64, 1)
    j = torch.arange(8).view(1, 8)
    return lane, j


def pack_w1(w: torch.Tensor) -> torch.Tensor:
    """W1 [H, D] (D <= 32) -> bf16 [H/16, 64, 8]: A[16 t + (l & 15)][8 (l >> 4) + j], zero for k >= D."""
    H, D = w.shape
    lane, j = _lane_j()
    t = torch.arange(H // 16).view(-1, 1, 1)
    rows = 16 * t + (lane & 15).view(1, 64, 1)
    k = (8 * (lane >> 4) + j).view(1, 64, 8).expand(H // 16, 64, 8)
    rows = rows.expand(H // 16, 64, 8)
    vals = w.detach().float()[rows.to(w.device), k.clamp(max=D - 1).to(w.device)]
    vals = torch.where(k.to(w.device) < D, vals, torch.zeros_like(vals))
    return vals.to(torch.bfloat16).contiguous()


def _kperm(s: torch.Tensor, lane: torch.Tensor, j: torch.Tensor) -> torch.Tensor:
    """hidden unit of element j of lane l in k step s (the accumulator-as-operand order)"""
    return 32 * s + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3)


def pack_w2(w: torch.Tensor) -> torch.Tensor:
    """W2 [H, H] -> bf16 [H/16, H/32, 64, 8]."""
    H = w.shape[0]
    lane, j = _lane_j()
    t = torch.arange(H // 16).view(-1, 1, 1, 1)
    s = torch.arange(H // 32).view(1, -1, 1, 1)
    rows = (16 * t + (lane & 15).view(1, 1, 64, 1)).expand(H // 16, H // 32, 64, 8)
    cols = _kperm(s, lane.view(1, 1, 64, 1), j.view(1, 1, 1, 8)).expand(H // 16, H // 32, 64, 8)
    return w.detach().float()[rows.to(w.device), cols.to(w.device)].to(torch.bfloat16).contiguous()


def pack_w3(w: torch.Tensor) -> torch.Tensor:
    """W3 [OUT, H] (OUT <= 16) -> bf16 [H/32, 64, 8], rows >= OUT zero."""
    OUT, H = w.shape
    lane, j = _lane_j()
    s = torch.arange(H // 32).view(-1, 1, 1)
    rows = (lane & 15).view(1, 64, 1).expand(H // 32, 64, 8)
    cols = _kperm(s, lane.view(1, 64, 1), j.view(1, 1, 8)).expand(H // 32, 64, 8)
    vals = w.detach().float()[rows.clamp(max=OUT - 1).to(w.device), cols.to(w.device)]
    vals = torch.where(rows.to(w.device) < OUT, vals, torch.zeros_like(vals))
    return vals.to(torch.bfloat16).contiguous()


def mlp_layers(seq: nn.Sequential):
    """(Linear, act, Linear, act, Linear) -> ([l1, l2, l3], activation code)"""
    mods = list(seq)
    lin = [m for m in mods if isinstance(m, nn.Linear)]
    acts = [m for m in mods if not isinstance(m, nn.Linear)]
    if len(lin) != 3 or len(acts) != 2:
        raise ValueError("fused inference supports MLPs with exactly two hidden layers")
    kinds = {type(a) for a in acts}
    if kinds == {nn.LeakyReLU} and all(abs(a.negative_slope - 0.01) < 1e-12 for a in acts):
        code = _abi.GR_POLICY_ACT_LRELU
    elif kinds == {nn.ELU} and all(a.alpha == 1.0 for a in acts):
        code = _abi.GR_POLICY_ACT_ELU
    else:
        raise ValueError(f"fused inference supports LeakyReLU(0.01) / ELU(1) activations, got {kinds}")
    H = lin[0].out_features
    if H not in (128, 256) or lin[1].in_features != H or lin[1].out_features != H or lin[2].in_features != H:
        raise ValueError("fused inference supports two hidden layers of 128 or 256 units")
    if lin[0].in_features > 32 or lin[0].in_features % 4:
        raise ValueError("fused inference supports up to 32 observations, a multiple of 4")
    return lin, code


class FusedPolicyInference:
    """PPO.act's policy calls for `num_envs` envs in one MFMA launch.  Outputs are persistent device
    tensors (rebind-free, graph-capturable): actions, action_mean [N, A], values [N, 1], log_prob [N],
    action_sigma [N, A].  Used by PPO when the algorithm cfg sets `fused_rollout_inference` (ppo.py)."""

    def __init__(self, policy, num_envs: int, device, seed: int = 0, env_id_offset: int = 0,
                 precision: str = "bf16"):
        self.policy = policy
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be 'bf16' or 'fp32', got {precision!r}")
        self.precision = precision
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("fused policy inference runs on the GPU (HIP); there is no CPU path")
        self._lib = _abi.load()
        a_lin, a_act = mlp_layers(policy.actor)
        c_lin, c_act = mlp_layers(policy.critic)
        if a_act != c_act or a_lin[0].out_features != c_lin[0].out_features:
            raise ValueError("actor and critic must share the hidden width and activation")
        if a_lin[2].out_features > 4 or c_lin[2].out_features != 1:
            raise ValueError("fused inference supports <= 4 actions and a scalar value")
        self.hidden = a_lin[0].out_features
        self.activation = a_act
        self.num_envs = int(num_envs)
        self.num_actions = a_lin[2].out_features
        self.num_obs = (a_lin[0].in_features, c_lin[0].in_features)
        n, dev = self.num_envs, self.device
        self.actions = torch.zeros(n, self.num_actions, device=dev)
        self.action_mean = torch.zeros(n, self.num_actions, device=dev)
        self.values = torch.zeros(n, 1, device=dev)
        self.log_prob = torch.zeros(n, device=dev)
        self.std = torch.zeros(self.num_actions, device=dev)
        self.counters = torch.zeros(2, dtype=torch.int32, device=dev)
        self._calls = 0
        self.seed = int(seed)
        self.env_id_offset = int(env_id_offset)
        self._packed = {}
        self._version = None
        self._plist = None
        self.refresh()

    def _params(self):
        # (collected once per packing: walking the module tree on every act call cost ~20 us of host time per step at
        # 4 096 envs.  Optimizers, load_state_dict and FlatAdam write the parameters in place, which the version
        # tuple sees; a module whose Parameter objects are replaced needs an explicit refresh())
        if self._plist is None:
            ps = list(self.policy.actor.parameters()) + list(self.policy.critic.parameters())
            self._plist = ps + [self.policy.std if self.policy.noise_std_type == "scalar" else self.policy.log_std]
        return self._plist

    def _param_version(self):
        # torch bumps a tensor's version on every in-place write (optimizer.step, load_state_dict, copy_)
        return tuple(p._version for p in self._params())

    @torch.no_grad()
    def refresh(self):
        """Repack the weights (after a PPO update; in place, so captured graphs stay valid)."""
        nets = {"actor": mlp_layers(self.policy.actor)[0], "critic": mlp_layers(self.policy.critic)[0]}
        if self.precision == "fp32":  # the module's own layout: row-major fp32 W [out, in], b [out]
            packs = {name: {k: lin[i].weight.float() if k[0] == "w" else lin[i].bias.float()
                            for i, k in ((0, "w1"), (0, "b1"), (1, "w2"), (1, "b2"), (2, "w3"), (2, "b3"))}
                     for name, lin in nets.items()}
        else:
            packs = {name: self._pack_bf16(lin) for name, lin in nets.items()}
        for name, parts in packs.items():
            for k, v in parts.items():
                key = f"{name}.{k}"
                v = v.detach().to(self.device).contiguous()  # fp32 parameters / bf16 fragments as packed
                if key in self._packed:
                    self._packed[key].copy_(v)
                else:
                    self._packed[key] = v.clone()  # never an alias of the module's parameter
        std = self.policy.std if self.policy.noise_std_type == "scalar" else torch.exp(self.policy.log_std)
        self.std.copy_(std.detach().float())
        self._plist = None  # (re-collected: a repack also follows a replaced parameter)
        self._version = self._param_version()

    def _pack_bf16(self, lin):
        # LeakyReLU: layers 1 and 2 pre-scaled (GR_POLICY_LRELU_PRESCALE, include/gr.h)
        s = _abi.GR_POLICY_LRELU_PRESCALE if self.activation == _abi.GR_POLICY_ACT_LRELU else 1.0
        return {"w1": pack_w1(lin[0].weight * s), "b1": lin[0].bias.detach().float() * s,
                "w2": pack_w2(lin[1].weight * s), "b2": lin[1].bias.detach().float() * s,
                "w3": pack_w3(lin[2].weight), "b3": lin[2].bias.detach().float()}

    def _net(self, name, obs, out, num_obs, num_out):
        p = self._packed
        nt = _abi.GrPolicyNet()
        nt.obs = obs.data_ptr()
        nt.w1, nt.b1 = p[f"{name}.w1"].data_ptr(), p[f"{name}.b1"].data_ptr()
        nt.w2, nt.b2 = p[f"{name}.w2"].data_ptr(), p[f"{name}.b2"].data_ptr()
        nt.w3, nt.b3 = p[f"{name}.w3"].data_ptr(), p[f"{name}.b3"].data_ptr()
        nt.out = out.data_ptr()
        nt.num_obs, nt.num_out = num_obs, num_out
        return nt

    def act(self, obs: torch.Tensor, critic_obs: torch.Tensor | None):
        """-> (actions, values, log_prob, action_mean, action_sigma) for all envs (views of persistent
        buffers, overwritten by the next call).  Weights changed in place since the last packing (a PPO
        update, a checkpoint load) are repacked first; inside a graph capture they must not change.
        critic_obs None: the actor only (sampled actions, mean, log prob; `values` is not written)."""
        n = self.num_envs
        if self._param_version() != self._version:
            self.refresh()
        checks = [(obs, self.num_obs[0])] + ([] if critic_obs is None else [(critic_obs, self.num_obs[1])])
        for x, d in checks:
            if x.shape != (n, d) or x.dtype != torch.float32 or x.device != self.device or not x.is_contiguous():
                raise ValueError(f"expected contiguous fp32 [{n}, {d}] observations on {self.device}, got "
                                 f"{tuple(x.shape)} {x.dtype} {x.device}")
        a = _abi.GrPolicyArgs()
        a.net[0] = self._net("actor", obs, self.action_mean, self.num_obs[0], self.num_actions)
        if critic_obs is not None:
            a.net[1] = self._net("critic", critic_obs, self.values, self.num_obs[1], 1)
        a.std, a.actions, a.log_prob = self.std.data_ptr(), self.actions.data_ptr(), self.log_prob.data_ptr()
        a.counters, a.counter_index = self.counters.data_ptr(), self._calls % 2
        a.num_envs, a.hidden, a.activation, a.env_id_offset = n, self.hidden, self.activation, self.env_id_offset
        a.seed_lo, a.seed_hi = self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF
        a.precision = _abi.GR_POLICY_FP32 if self.precision == "fp32" else _abi.GR_POLICY_BF16
        rc = self._lib.gr_policy_forward(C.byref(a), C.c_void_p(_abi.raw_stream(self.device)))
        if rc != 0:
            raise RuntimeError(f"gr_policy_forward failed (status {rc})")
        self._calls += 1
        return self.actions, self.values, self.log_prob, self.action_mean, self.std.expand(n, self.num_actions)
