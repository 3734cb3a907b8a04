"""nn.Linear for the PPO update's tall mini-batches (tens of thousands to millions of rows).

The weight gradient dW = dY^T X of a Linear reduces over every row of the mini-batch.  As one GEMM,
hipBLASLt tiles only its small [out, in] output, so a handful of workgroups stream all rows: at
65 536 envs (393 216-row mini-batches) the six weight gradients of the 256 x 256 actor + critic took
~4.9 ms of an ~11 ms update step (`profiles/round01_update65536_nn_linear_kernel_stats.csv`).  Here the rows are
split into chunks of SPLIT (a batched GEMM: one workgroup set per chunk) and the partial products are
summed.  Same module tree, parameters and state_dict keys as nn.Linear (the reference's checkpoints
and exporters are unaffected); small batches, inference and TorchScript take F.linear.

`MLP` (the actor / critic Sequential) runs its last LeakyReLU and output Linear as ONE op on those
batches (`leaky_head`: gr_head_forward / gr_head_backward, gr_update.hip): the activation pass, the
small-N head GEMMs and the activation's backward pass each stream a [rows, 256] matrix through HBM
(`profiles/round03_update65536_graphed_kernel_stats.csv`), the fused op reads the pre-activation once
forward and once backward.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

SPLIT = 4096  # rows per chunk (scripts/prof_update.py --split: 2048-4096 best at 65 536 and 4 096 envs)
# set by the graph-captured PPO step (ppo.py _GraphedStep): every Linear takes _TallLinearFn, whose bias
# gradient is gr_column_sum (see bias_grad)
_FORCE_FN = False


def bias_grad(gy: torch.Tensor) -> torch.Tensor:
    """Sum over the rows of gy [M, N] (fp32 out).  On the GPU: gr_column_sum (libgr.so, gr_update.hip), one
    HBM pass in a fixed summation order.  Not PyTorch's gy.sum(0): inside a captured hipGraph its multi-block
    reduction keeps cross-block semaphores in a buffer that, on this ROCm build, is not held by the graph's
    pool (eager allocations between replays reused it and the replays' bias gradients came out wrong,
    scripts/debug_graph_update.py); and as a GEMM with a ones vector hipBLASLt tiles only the N x 1 output
    (1.5 ms at M = 393 216, N = 256, half of the update step)."""
    if gy.device.type != "cuda":
        return gy.float().sum(0)
    from .. import _abi

    lib = _abi.load()
    gy = gy.contiguous()
    m, n = gy.shape
    if gy.dtype == torch.bfloat16:
        dtype = _abi.GR_DTYPE_BF16
    else:
        gy = gy.float()
        dtype = _abi.GR_DTYPE_F32
    part = torch.empty(lib.gr_column_sum_partials(m) * n, device=gy.device, dtype=torch.float32)
    out = torch.empty(n, device=gy.device, dtype=torch.float32)
    rc = lib.gr_column_sum(gy.data_ptr(), dtype, m, n, part.data_ptr(), out.data_ptr(),
                           torch.cuda.current_stream(gy.device).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"gr_column_sum failed (status {rc})")
    return out


def split_k_wgrad(gy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """gy^T x for tall gy [M, N], x [M, K]: split over M into chunks of SPLIT rows, summed."""
    m = x.shape[0]
    s = m // SPLIT
    if s < 2:
        return gy.t() @ x
    gw = torch.bmm(gy[: s * SPLIT].view(s, SPLIT, -1).transpose(1, 2), x[: s * SPLIT].view(s, SPLIT, -1)).sum(0)
    if m > s * SPLIT:
        gw = gw + gy[s * SPLIT:].t() @ x[s * SPLIT:]
    return gw


class _TallLinearFn(torch.autograd.Function):
    # custom_fwd / custom_bwd: under torch.autocast (PPO's opt-in bf16 update) the forward GEMM runs in
    # the autocast dtype and the backward runs under the same autocast state; gradients return in the
    # parameters' dtype
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.wdtype = w.dtype
        return F.linear(x, w, b)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = None
        if ctx.needs_input_grad[0]:
            wg = w.to(gy.dtype)
            gx = gy @ wg
        gw = split_k_wgrad(gy, x.to(gy.dtype)).to(ctx.wdtype) if ctx.needs_input_grad[1] else None
        gb = bias_grad(gy).to(ctx.wdtype) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


class TallLinear(nn.Linear):
    """nn.Linear whose weight gradient is split over the rows for mini-batches of >= 2 * SPLIT rows."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if torch.jit.is_scripting():
            return F.linear(x, self.weight, self.bias)
        return self._forward_eager(x)

    @torch.jit.unused
    def _forward_eager(self, x: torch.Tensor) -> torch.Tensor:
        if x.dim() == 2 and (x.shape[0] >= 2 * SPLIT or _FORCE_FN) \
                and torch.is_grad_enabled() and self.weight.requires_grad:
            return _TallLinearFn.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)


# ------------------------------------------------------------------------------------------ fused head
HEAD_MAX_OUT = 8      # gr_head_*: output features
HEAD_MAX_IN = 256     # gr_head_*: input features (a multiple of 4)


class _LeakyHeadFn(torch.autograd.Function):
    """y = leaky_relu(z, slope) @ w^T + b on the device (gr_head_forward); backward gr_head_backward:
    gz = (gy @ w) * leaky_relu'(z), gw = gy^T leaky_relu(z), gb = sum gy (fixed summation order)."""

    @staticmethod
    def forward(ctx, z, w, b, slope):
        from .. import _abi

        lib = _abi.load()
        z, w, b = z.contiguous(), w.contiguous(), b.contiguous()
        m, h = z.shape
        k = w.shape[0]
        y = torch.empty(m, k, device=z.device, dtype=torch.float32)
        rc = lib.gr_head_forward(z.data_ptr(), m, h, w.data_ptr(), b.data_ptr(), k, float(slope), y.data_ptr(),
                                 torch.cuda.current_stream(z.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"gr_head_forward failed (status {rc})")
        ctx.save_for_backward(z, w)
        ctx.slope = float(slope)
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _abi

        lib = _abi.load()
        z, w = ctx.saved_tensors
        gy = gy.contiguous().float()
        m, h = z.shape
        k = w.shape[0]
        gz = torch.empty_like(z)
        part = torch.empty(lib.gr_head_partials(m, k, h), device=z.device, dtype=torch.float32)
        gw = torch.empty_like(w)
        gb = torch.empty(k, device=z.device, dtype=torch.float32)
        rc = lib.gr_head_backward(z.data_ptr(), gy.data_ptr(), m, h, w.data_ptr(), k, ctx.slope, gz.data_ptr(),
                                  part.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                                  torch.cuda.current_stream(z.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"gr_head_backward failed (status {rc})")
        return gz, gw, gb, None


def leaky_head(z: torch.Tensor, w: torch.Tensor, b: torch.Tensor, slope: float) -> torch.Tensor:
    """leaky_relu(z, slope) @ w^T + b as one device op with its own backward (HIP, gr_update.hip)."""
    return _LeakyHeadFn.apply(z, w, b, slope)


def head_fusable(x: torch.Tensor, act: nn.Module, lin: nn.Module) -> bool:
    """The update's tall fp32 CUDA batches with LeakyReLU -> Linear(<= 256, <= 8) at the end of the MLP."""
    return (isinstance(act, nn.LeakyReLU) and isinstance(lin, nn.Linear) and lin.bias is not None
            and x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and lin.weight.dtype == torch.float32
            and (x.shape[0] >= 2 * SPLIT or _FORCE_FN) and torch.is_grad_enabled() and lin.weight.requires_grad
            and not torch.is_autocast_enabled("cuda")
            and lin.out_features <= HEAD_MAX_OUT and lin.in_features <= HEAD_MAX_IN and lin.in_features % 4 == 0)


class MLP(nn.Sequential):
    """The actor / critic MLP: nn.Sequential with the same children and state_dict keys.  On the update's tall
    CUDA mini-batches its last LeakyReLU + output Linear run fused (leaky_head); everywhere else (rollout,
    inference, CPU, TorchScript) module by module."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if torch.jit.is_scripting():
            for m in self:
                x = m(x)
            return x
        return self._forward_eager(x)

    @torch.jit.unused
    def _forward_eager(self, x: torch.Tensor) -> torch.Tensor:
        mods = list(self)
        if len(mods) >= 2 and head_fusable(x, mods[-2], mods[-1]):
            for m in mods[:-2]:
                x = m(x)
            return leaky_head(x, mods[-1].weight, mods[-1].bias, mods[-2].negative_slope)
        for m in mods:
            x = m(x)
        return x
