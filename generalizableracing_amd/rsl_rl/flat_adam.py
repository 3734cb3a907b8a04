"""The PPO update's gradient-norm clip and Adam step as four device launches (gr_adam_clip / gr_adam_step,
gr_update.hip).

PPO.update (standalone/rsl_rl/ext/algorithms/ppo.py:178-181) runs `nn.utils.clip_grad_norm_(parameters,
max_grad_norm)` then `optimizer.step()` with `torch.optim.Adam(policy.parameters(), lr)` (ppo.py:39).  torch's
foreach implementations of the two are ~55 small launches per mini-batch (per-tensor norms, stacks, lerp,
addcmul, sqrt, div, addcdiv over every parameter list, plus the step-count and bias-correction ops of the
capturable variant): ~0.2 ms of every graphed mini-batch step at 65 536 envs, and most of the step at 4096 envs,
where the update is launch-bound.  Here the parameters are a table of segments (pointers, sizes, one step
counter each; moments in two flat buffers; the table itself in device memory) and the clip is two launches (the
per-block sums of squares, then the norm and the scaling), Adam two (+1 on every stepped segment's counter with its
bias corrections in double, then the element-wise update).

Numerics follow torch's non-capturable foreach Adam (torch/optim/adam.py `_multi_tensor_adam`): m.lerp_(g, 1 -
b1), v.mul_(b2).addcmul_(g, g, 1 - b2), step_size = lr / (1 - b1^t) and sqrt(1 - b2^t) as Python doubles
rounded to fp32, p.addcdiv_(m, sqrt(v) / bc2_sqrt + eps, -step_size); the clip's norm is accumulated in double
in a fixed order (torch: per-tensor fp32 norms, then the norm of those), so the coefficient can differ in the last
ulp.

`FlatAdam` is a torch.optim.Optimizer with Adam's `param_groups` (one group) and a torch-Adam-compatible
`state_dict` / `load_state_dict` ("step" / "exp_avg" / "exp_avg_sq" per parameter, the latter views of the flat
moment buffers).  As in torch, a parameter whose `.grad` is None is skipped (no state, no step count).  `lr` may
be a device tensor: the captured update reads it at replay (ppo.py _GraphedStep).
"""
from __future__ import annotations

import ctypes as C

import torch

MAX_SEGMENTS = 64  # GR_ADAM_MAX_SEGMENTS (include/gr.h)


class GrAdamSegment(C.Structure):
    """Mirror of gr_adam_segment (include/gr.h)."""
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("numel", C.c_int64), ("step_slot", C.c_int32), ("block_start", C.c_int32)]


class GrAdamArgs(C.Structure):
    """Mirror of gr_adam_args (include/gr.h)."""
    _fields_ = [("nseg", C.c_int32), ("nblocks", C.c_int32), ("lr", C.c_double), ("beta1", C.c_double),
                ("beta2", C.c_double), ("eps", C.c_float), ("pad", C.c_int32), ("lr_ptr", C.c_void_p),
                ("step", C.c_void_p), ("coef", C.c_void_p), ("part", C.c_void_p), ("seg", C.c_void_p)]


def _call(name, *args):
    from .. import _abi

    rc = getattr(_abi.load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (status {rc})")


def flat_adam_ok(params) -> bool:
    """CUDA fp32 contiguous parameters, at most MAX_SEGMENTS of them (else torch.optim.Adam)."""
    params = list(params)
    return 0 < len(params) <= MAX_SEGMENTS and all(
        p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in params)


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=0.0, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdam: one parameter group")
        ps = self.param_groups[0]["params"]
        if not flat_adam_ok(ps):
            raise ValueError(f"FlatAdam: 1..{MAX_SEGMENTS} contiguous CUDA fp32 parameters")
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self._m = torch.zeros(n, device=dev, dtype=torch.float32)
        self._v = torch.zeros(n, device=dev, dtype=torch.float32)
        self._steps = torch.zeros(len(ps), device=dev, dtype=torch.float32)
        self._coef = torch.zeros(2 * len(ps), device=dev, dtype=torch.float32)
        self._norm = torch.zeros(1, device=dev, dtype=torch.float32)
        self._slot, off = {}, 0
        for i, p in enumerate(ps):
            self._slot[p] = (i, off)
            off += p.numel()
        self._cache_key, self._cache = None, None
        self._table = self._part = None  # the device segment table and the clip's per-block partial sums

    def _views(self, p):
        i, off = self._slot[p]
        n = p.numel()
        return (self._steps[i], self._m[off:off + n].view_as(p), self._v[off:off + n].view_as(p))

    def _register(self, p):
        if p not in self.state or not self.state[p]:
            st, m, v = self._views(p)
            self.state[p] = {"step": st, "exp_avg": m, "exp_avg_sq": v}

    def _args(self) -> GrAdamArgs | None:
        """The launch arguments over the parameters that have a gradient.  The segment table is checked and
        numbered by gr_adam_prepare and uploaded to the device when the pointers change (never during a graph
        capture: take one eager step first, as with torch's capturable optimizers)."""
        g = self.param_groups[0]
        ps = [p for p in g["params"] if p.grad is not None]
        if not ps:
            return None
        lr = g["lr"]
        key = (tuple(p.grad.data_ptr() for p in ps), tuple(p.data_ptr() for p in ps),
               lr.data_ptr() if torch.is_tensor(lr) else None)
        if key != self._cache_key:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FlatAdam: its parameter table changed during a graph capture (step it eagerly "
                                   "with the captured gradients bound first)")
            table = (GrAdamSegment * len(ps))()
            for s, p in enumerate(ps):
                if not p.grad.is_contiguous() or p.grad.dtype != torch.float32 or p.grad.device != p.device:
                    raise ValueError("FlatAdam: contiguous fp32 gradients on the parameter's device")
                i, moff = self._slot[p]
                t = table[s]
                t.param, t.grad = p.data_ptr(), p.grad.data_ptr()
                t.exp_avg = self._m.data_ptr() + 4 * moff
                t.exp_avg_sq = self._v.data_ptr() + 4 * moff
                t.numel, t.step_slot = p.numel(), i
                self._register(p)
            nblocks = C.c_int32()
            _call("gr_adam_prepare", C.addressof(table), len(ps), C.byref(nblocks))
            dev = self._m.device
            self._table = torch.frombuffer(bytearray(bytes(table)), dtype=torch.uint8).to(dev)
            self._part = torch.empty(nblocks.value, device=dev, dtype=torch.float64)
            a = GrAdamArgs()
            a.nseg, a.nblocks = len(ps), nblocks.value
            a.step, a.coef, a.part = self._steps.data_ptr(), self._coef.data_ptr(), self._part.data_ptr()
            a.seg = self._table.data_ptr()
            a.lr_ptr = lr.data_ptr() if torch.is_tensor(lr) else None
            self._cache_key, self._cache = key, a
        a = self._cache
        b1, b2 = g["betas"]
        a.beta1, a.beta2, a.eps = float(b1), float(b2), float(g["eps"])
        if not torch.is_tensor(lr):
            a.lr = float(lr)
        return a

    def _stream(self):
        from .. import _abi

        return _abi.raw_stream(self._m.device)

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """nn.utils.clip_grad_norm_(params, max_norm) over the parameters with a gradient; returns the norm
        (a device tensor)."""
        a = self._args()
        if a is None:
            return self._norm[0].zero_()
        _call("gr_adam_clip", C.addressof(a), C.c_float(float(max_norm)), self._norm.data_ptr(), self._stream())
        return self._norm[0]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        a = self._args()
        if a is not None:
            _call("gr_adam_step", C.addressof(a), self._stream())
            # the kernel wrote the parameters through raw pointers: bump their version counters as torch's in-place
            # Adam does, so caches keyed on them (the fused rollout inference's packed weights) see the update
            for p in self.param_groups[0]["params"]:
                if p.grad is not None:
                    torch.autograd.graph.increment_version(p)
        return loss

    @torch.no_grad()
    def clip_and_step(self, max_norm: float, kl: torch.Tensor | None = None, desired_kl: float | None = None,
                      lr_min: float = 1e-5, lr_max: float = 1e-2) -> torch.Tensor:
        """[the adaptive rate rule on the device, when kl is given (the rate is then the group's device tensor)] +
        clip_grad_norm_(max_norm) + step(), as gr_adam_clip_step's two launches (the graph-captured update's
        segment B); returns the norm (a device tensor)."""
        a = self._args()
        if a is None:
            return self._norm[0].zero_()
        lr = self.param_groups[0]["lr"]
        if kl is not None and not (torch.is_tensor(lr) and lr.data_ptr() == a.lr_ptr):
            raise ValueError("clip_and_step: the adaptive rule needs the group's rate as a device tensor")
        _call("gr_adam_clip_step", C.addressof(a), C.c_float(float(max_norm)), self._norm.data_ptr(),
              kl.data_ptr() if kl is not None else None, lr.data_ptr() if kl is not None else None,
              C.c_double(float(desired_kl or 0.0)), C.c_double(lr_min), C.c_double(lr_max), self._stream())
        for p in self.param_groups[0]["params"]:
            if p.grad is not None:
                torch.autograd.graph.increment_version(p)
        return self._norm[0]

    def state_dict(self):
        """torch.optim.Adam's non-capturable layout, so the reference runner (on_policy_runner.py:319) can load a
        checkpoint into torch.optim.Adam and step it: `lr` a Python float (the graphed update binds a device tensor
        into the group), `capturable` False, each `step` a CPU fp32 scalar tensor and the moments standalone copies
        (not views of the flat buffers, which torch.save would write whole for every view)."""
        sd = super().state_dict()
        for g in sd["param_groups"]:
            lr = g["lr"]
            g["lr"] = float(lr) if torch.is_tensor(lr) else lr
            g["capturable"] = False
        state = {}
        for idx, st in sd["state"].items():
            state[idx] = {"step": st["step"].detach().to("cpu", torch.float32).clone().reshape(()),
                          "exp_avg": st["exp_avg"].detach().clone(), "exp_avg_sq": st["exp_avg_sq"].detach().clone()}
        sd["state"] = state
        return sd

    def load_state_dict(self, state_dict):
        """torch.optim.Adam's state_dict (or FlatAdam's): group settings and, per parameter with state, the step
        count and moments copied into the flat buffers (the state's tensors stay views of them)."""
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.param_groups[0]["params"]):
            raise ValueError("FlatAdam.load_state_dict: parameter groups do not match")
        g = self.param_groups[0]
        for k in ("betas", "eps"):
            if k in groups[0]:
                g[k] = tuple(groups[0][k]) if k == "betas" else groups[0][k]
        if not torch.is_tensor(g["lr"]):
            lr = groups[0]["lr"]
            g["lr"] = float(lr) if torch.is_tensor(lr) else lr
        self.state.clear()
        self._cache_key = None
        with torch.no_grad():
            self._m.zero_()
            self._v.zero_()
            self._steps.zero_()
            for idx, p in zip(groups[0]["params"], g["params"]):
                s = state_dict["state"].get(idx)
                if not s:
                    continue
                self._register(p)
                mine = self.state[p]
                mine["step"].copy_(torch.as_tensor(s["step"], dtype=torch.float32).reshape(()))
                mine["exp_avg"].copy_(s["exp_avg"])
                mine["exp_avg_sq"].copy_(s["exp_avg_sq"])


def make_adam(params, lr, fused: bool = True):
    """FlatAdam for CUDA fp32 parameters (the C ABI library must load: no silent fallback on a GPU), else
    torch.optim.Adam (CPU runs, other dtypes, fused=False)."""
    params = list(params)
    if fused and flat_adam_ok(params):
        return FlatAdam(params, lr=lr)
    return torch.optim.Adam(params, lr=lr)


def clip_grad_norm_(optimizer, params, max_norm):
    """The clip through the optimizer's table when it is a FlatAdam, else torch's."""
    if isinstance(optimizer, FlatAdam):
        return optimizer.clip_grad_norm_(max_norm)
    return torch.nn.utils.clip_grad_norm_(params, max_norm)
