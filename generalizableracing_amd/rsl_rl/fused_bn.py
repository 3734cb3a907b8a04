"""Training-mode BatchNorm + activation on channels-last rows as one HIP op (libgr.so gr_bn_act_forward /
gr_bn_act_backward, csrc/gr_bn.hip).

The vision stem (rsl_rl/vision_actor_critic.py, reference standalone/rsl_rl/ext/modules/
vision_actor_critic.py:43-144) evaluates Conv -> BatchNorm2d -> LeakyReLU as patch GEMMs on [rows, C]
matrices with millions of rows.  torch runs batch_norm (statistics + transform) and the activation as
separate passes and saves both outputs; here the forward is one statistics pass and one apply pass, the
backward one reduce pass and one element pass, and only the BN input is saved.  The running statistics are
updated exactly as F.batch_norm does (momentum, unbiased variance).  Eval-mode BatchNorm (running
statistics) stays on torch's op.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _abi

_CHANNELS = (4, 8, 16, 32, 64)


def _act_code(act: nn.Module):
    if isinstance(act, nn.LeakyReLU):
        return _abi.GR_POLICY_ACT_LRELU, float(act.negative_slope)
    if isinstance(act, nn.ELU) and float(act.alpha) == 1.0:
        return _abi.GR_POLICY_ACT_ELU, 1.0
    return None


def _stream(x):
    return C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)


class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, act, slope):
        lib = _abi.load()
        m, c = x.shape
        y = torch.empty_like(x)
        stats = torch.empty(4, c, device=x.device, dtype=torch.float32)
        part = torch.empty(int(lib.gr_bn_scratch_doubles(m, c)), device=x.device, dtype=torch.float64)
        w, b = weight.detach().contiguous(), bias.detach().contiguous()
        rc = lib.gr_bn_act_forward(x.data_ptr(), m, c, w.data_ptr(), b.data_ptr(), float(eps), act, float(slope),
                                   y.data_ptr(), stats.data_ptr(), part.data_ptr(), _stream(x))
        if rc != 0:
            raise RuntimeError(f"gr_bn_act_forward failed (status {rc})")
        ctx.save_for_backward(x, w, b, stats)
        ctx.act, ctx.slope = act, slope
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, gy, _gstats):
        lib = _abi.load()
        x, w, b, stats = ctx.saved_tensors
        m, c = x.shape
        gy = gy.contiguous()
        gx = torch.empty_like(x)
        gw = torch.empty(c, device=x.device, dtype=torch.float32)
        gb = torch.empty(c, device=x.device, dtype=torch.float32)
        part = torch.empty(int(lib.gr_bn_scratch_doubles(m, c)), device=x.device, dtype=torch.float64)
        rc = lib.gr_bn_act_backward(x.data_ptr(), gy.data_ptr(), m, c, w.data_ptr(), b.data_ptr(), stats.data_ptr(),
                                    ctx.act, float(ctx.slope), gx.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                                    part.data_ptr(), _stream(x))
        if rc != 0:
            raise RuntimeError(f"gr_bn_act_backward failed (status {rc})")
        return gx, gw, gb, None, None, None


def fused_applicable(bn: nn.BatchNorm2d, act: nn.Module, x: torch.Tensor) -> bool:
    """The HIP op covers training-mode batch statistics of an affine BN on fp32 CUDA rows with C in
    {4, 8, 16, 32, 64}, followed by LeakyReLU or ELU(1)."""
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.is_contiguous() and x.shape[0] >= 2
            and x.shape[1] in _CHANNELS and bn.affine and bn.training and _act_code(act) is not None
            and bn.weight.dtype == torch.float32)


def batch_norm_act(bn: nn.BatchNorm2d, act: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """act(bn(x)) for rows x [M, C] in training mode, running statistics updated as nn.BatchNorm2d does
    (the caller has already counted the batch in num_batches_tracked and passes the momentum it implies)."""
    code, slope = _act_code(act)
    y, stats = _BatchNormAct.apply(x, bn.weight, bn.bias, bn.eps, code, slope)
    if bn.track_running_stats and bn.running_mean is not None:
        momentum = 0.0 if bn.momentum is None else bn.momentum
        if bn.momentum is None and bn.num_batches_tracked is not None:
            momentum = 1.0 / float(bn.num_batches_tracked)
        with torch.no_grad():
            bn.running_mean.mul_(1.0 - momentum).add_(stats[0], alpha=momentum)
            bn.running_var.mul_(1.0 - momentum).add_(stats[3], alpha=momentum)
    return y


def reference_batch_norm_act(bn: nn.BatchNorm2d, act: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """torch's own ops for the same step (tests; eval mode)."""
    return act(F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                            0.0 if bn.momentum is None else bn.momentum, bn.eps))
