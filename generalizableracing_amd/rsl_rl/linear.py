"""nn.Linear for the PPO update's tall mini-batches (tens of thousands to millions of rows).

The weight gradient dW = dY^T X of a Linear reduces over every row of the mini-batch.  As one GEMM,
hipBLASLt tiles only its small [out, in] output, so a handful of workgroups stream all rows: at
65 536 envs (393 216-row mini-batches) the six weight gradients of the 256 x 256 actor + critic took
~4.9 ms of an ~11 ms update step (`profiles/round01_update65536_nn_linear_kernel_stats.csv`).  Here the rows are
split into chunks of SPLIT (a batched GEMM: one workgroup set per chunk) and the partial products are
summed.  Same module tree, parameters and state_dict keys as nn.Linear (the reference's checkpoints
and exporters are unaffected); small batches, inference and TorchScript take F.linear.

`MLP` (the actor / critic Sequential, same children and state_dict keys) runs everything around the hidden
h1 x h2 GEMM in fused HIP ops on those batches (gr_update.hip): the first Linear (K = 16) with its bias and
LeakyReLU (gr_mlp_in_forward) and, backward, its weight / bias gradients straight from the hidden gradient
(gr_mlp_in_backward); the last LeakyReLU with the output Linear (gr_head_forward) and its backward, which also
sums the hidden layer's bias gradient (gr_head_backward).  In torch each activation pass, the small-N head GEMMs
and the bias sums streamed a [rows, 256] matrix through HBM (`profiles/round03_update65536_graphed_kernel_stats.csv`);
DESIGN.md §4f has the before / after.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

SPLIT = 4096  # rows per chunk (scripts/prof_update.py --split: 2048-4096 best at 65 536 and 4 096 envs)
# set by the graph-captured PPO step (ppo.py _GraphedStep): every Linear takes _TallLinearFn, whose bias
# gradient is gr_column_sum (see bias_grad)
_FORCE_FN = False
# {id(parameter): gradient view} while the graph-captured PPO step differentiates into its flat gradient buffer
# (ppo.py _GraphedStep._backward): _FusedMLPsFn's backward then writes a network's six gradients straight into
# their views when they lie back to back in kernel order (gr_mlp_backward's [gW1 | gb1 | gW2 | gb2 | gW3 | gb3]),
# so the step copies none of them
_GRAD_SINK = None


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
                           _abi.raw_stream(gy.device))
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


def tall_wgrad(gy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """gy^T x [N, K] for tall fp32 CUDA gy [M, N] and x [M, K] (x's rows may be strided): gr_patch_wgrad (one MFMA
    pass over the rows, fixed-order partial sums) when it covers (N, K), else split_k_wgrad."""
    m, n = gy.shape
    k = x.shape[1]
    if gy.is_cuda and gy.dtype == torch.float32 and x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1:
        from .. import _abi

        lib = _abi.load()
        floats = int(lib.gr_patch_wgrad_floats(m, n, k))
        if floats > 0:
            gy = gy.contiguous()
            if gy.data_ptr() % 16:  # (gr_patch_wgrad reads gy by 16-B vectors: a contiguous view at an odd storage
                gy = gy.clone()     # offset is re-based, not sent to the fallback or rejected)
            gw = torch.empty(n, k, device=gy.device, dtype=torch.float32)
            part = torch.empty(floats, device=gy.device, dtype=torch.float32)
            rc = lib.gr_patch_wgrad(x.data_ptr(), x.stride(0), gy.data_ptr(), m, n, k, part.data_ptr(), gw.data_ptr(),
                                    _abi.raw_stream(gy.device))
            if rc != 0:
                raise RuntimeError(f"gr_patch_wgrad failed (status {rc})")
            return gw
    return split_k_wgrad(gy, x)


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


# ------------------------------------------------------------------------------------------ fused MLP layers
HEAD_MAX_OUT = 8      # gr_head_*: output features
HEAD_MAX_IN = 256     # gr_head_* / gr_mlp_in_*: hidden features (a multiple of 4)
IN_MAX = 32           # gr_mlp_in_*: input features (a multiple of 4)


def _lib_call(name, *args):
    from .. import _abi

    rc = getattr(_abi.load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (status {rc})")


def _stream(t):
    from .. import _abi

    return _abi.raw_stream(t.device)


def _head_backward(z, gy, w, slope):
    """gr_head_backward -> (gz, gW, gb, column sums of gz)."""
    from .. import _abi

    m, h = z.shape
    k = w.shape[0]
    gz = torch.empty_like(z)
    part = torch.empty(_abi.load().gr_head_partials(m, k, h), device=z.device, dtype=torch.float32)
    sums = torch.empty(k * h + k + h, device=z.device, dtype=torch.float32)
    _lib_call("gr_head_backward", z.data_ptr(), gy.data_ptr(), m, h, w.data_ptr(), k, float(slope), gz.data_ptr(),
              part.data_ptr(), sums.data_ptr(), _stream(z))
    return gz, sums[:k * h].view(k, h), sums[k * h:k * h + k], sums[k * h + k:]


def _head_forward(z, w, b, slope):
    m, h = z.shape
    k = w.shape[0]
    y = torch.empty(m, k, device=z.device, dtype=torch.float32)
    _lib_call("gr_head_forward", z.data_ptr(), m, h, w.data_ptr(), b.data_ptr(), k, float(slope), y.data_ptr(),
              _stream(z))
    return y


class _LeakyHeadFn(torch.autograd.Function):
    """y = leaky_relu(z, slope) @ w^T + b on the device (gr_head_forward); backward gr_head_backward:
    gz = (gy @ w) * leaky_relu'(z), gw = gy^T leaky_relu(z), gb = sum gy (fixed summation order)."""

    @staticmethod
    def forward(ctx, z, w, b, slope):
        z, w, b = z.contiguous(), w.contiguous(), b.contiguous()
        ctx.save_for_backward(z, w)
        ctx.slope = float(slope)
        return _head_forward(z, w, b, slope)

    @staticmethod
    def backward(ctx, gy):
        z, w = ctx.saved_tensors
        gz, gw, gb, _ = _head_backward(z, gy.contiguous().float(), w, ctx.slope)
        return gz, gw, gb, None


def leaky_head(z: torch.Tensor, w: torch.Tensor, b: torch.Tensor, slope: float) -> torch.Tensor:
    """leaky_relu(z, slope) @ w^T + b as one device op with its own backward (HIP, gr_update.hip)."""
    return _LeakyHeadFn.apply(z, w, b, slope)


def _rows_ok(x: torch.Tensor) -> bool:
    """x usable in place by gr_mlp_in_*: unit column stride, row stride a multiple of 4 floats, 16-byte aligned."""
    return x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.stride(0) >= x.shape[1] and x.data_ptr() % 16 == 0


class _LeakyMLPFn(torch.autograd.Function):
    """The whole MLP x -> L1 -> lrelu -> L2 -> lrelu -> L3 for an input that needs no gradient (the update's
    observation rows): gr_mlp_in_forward (L1 + bias + activation), hipBLASLt for the h1 x h2 GEMM,
    gr_head_forward (activation + L3).  Backward: gr_head_backward (gz2, gW3, gb3 and gb2 in one read of z2),
    hipBLASLt for gh1 = gz2 W2, split-K for gW2, gr_mlp_in_backward (gW1, gb1 straight from gh1 and h1: gz1 is
    never stored)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3, slope):
        if not _rows_ok(x):
            x = x.contiguous()
        m, d = x.shape
        h1n = w1.shape[0]
        h1 = torch.empty(m, h1n, device=x.device, dtype=torch.float32)
        _lib_call("gr_mlp_in_forward", x.data_ptr(), m, d, x.stride(0), w1.data_ptr(), b1.data_ptr(), h1n,
                  float(slope), h1.data_ptr(), _stream(x))
        z2 = F.linear(h1, w2, b2)
        y = _head_forward(z2, w3.contiguous(), b3, slope)
        ctx.save_for_backward(x, h1, z2, w2, w3)
        ctx.slope = float(slope)
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _abi

        x, h1, z2, w2, w3 = ctx.saved_tensors
        gz2, gw3, gb3, gb2 = _head_backward(z2, gy.contiguous().float(), w3.contiguous(), ctx.slope)
        gh1 = gz2 @ w2
        gw2 = split_k_wgrad(gz2, h1)
        m, d = x.shape
        h1n = h1.shape[1]
        part = torch.empty(_abi.load().gr_mlp_in_partials(m, d, h1n), device=x.device, dtype=torch.float32)
        sums = torch.empty(h1n * d + h1n, device=x.device, dtype=torch.float32)
        _lib_call("gr_mlp_in_backward", gh1.data_ptr(), h1.data_ptr(), x.data_ptr(), m, d, x.stride(0), h1n,
                  ctx.slope, part.data_ptr(), sums.data_ptr(), _stream(x))
        return None, sums[:h1n * d].view(h1n, d), sums[h1n * d:], gw2, gb2, gw3, gb3, None


def _tall_cuda(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and w.dtype == torch.float32
            and (x.shape[0] >= 2 * SPLIT or _FORCE_FN) and torch.is_grad_enabled() and w.requires_grad
            and not torch.is_autocast_enabled("cuda"))


def head_fusable(x: torch.Tensor, act: nn.Module, lin: nn.Module) -> bool:
    """The update's tall fp32 CUDA batches with LeakyReLU -> Linear(<= 256, <= 8) at the end of the MLP."""
    return (isinstance(act, nn.LeakyReLU) and isinstance(lin, nn.Linear) and lin.bias is not None
            and _tall_cuda(x, lin.weight)
            and lin.out_features <= HEAD_MAX_OUT and lin.in_features <= HEAD_MAX_IN and lin.in_features % 4 == 0)


def mlp_fusable(x: torch.Tensor, mods: list) -> bool:
    """Linear(d <= 32) -> LeakyReLU -> Linear(h1, h2) -> LeakyReLU -> Linear(h2, <= 8), the input needing no
    gradient, on the update's tall batches."""
    if len(mods) != 5 or x.requires_grad:
        return False
    l1, a1, l2, a2, l3 = mods
    return (all(isinstance(m, nn.Linear) and m.bias is not None for m in (l1, l2, l3))
            and isinstance(a1, nn.LeakyReLU) and isinstance(a2, nn.LeakyReLU)
            and a1.negative_slope == a2.negative_slope and head_fusable(x, a2, l3)
            and l1.in_features <= IN_MAX and l1.in_features % 4 == 0 and x.shape[1] == l1.in_features
            and l1.out_features <= HEAD_MAX_IN and l1.out_features % 4 == 0 and l2.in_features == l1.out_features
            and l2.out_features == l3.in_features
            and l1.weight.requires_grad and l2.weight.requires_grad)


class MLP(nn.Sequential):
    """The actor / critic MLP: nn.Sequential with the same children and state_dict keys.  On the update's tall
    CUDA mini-batches everything but the hidden GEMM runs in the fused HIP ops (_LeakyMLPFn; with an input that
    needs a gradient, only the last LeakyReLU + output Linear fuse: leaky_head); everywhere else (rollout,
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
        if mlp_fusable(x, mods):
            l1, a1, l2, _, l3 = mods
            return _LeakyMLPFn.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias,
                                     a1.negative_slope)
        if len(mods) >= 2 and head_fusable(x, mods[-2], mods[-1]):
            for m in mods[:-2]:
                x = m(x)
            return leaky_head(x, mods[-1].weight, mods[-1].bias, mods[-2].negative_slope)
        for m in mods:
            x = m(x)
        return x


# ------------------------------------------------------------------------------ whole-network MFMA kernels (round 4)
class GrMlpNet(C.Structure):
    """Mirror of gr_mlp_net (include/gr.h)."""
    _fields_ = [(n, C.c_void_p) for n in ("x", "w1", "b1", "w2", "b2", "w3", "b3", "h1", "z2", "y", "gy", "gz2",
                                          "grads")] + [("ldx", C.c_int64), ("d", C.c_int32), ("k", C.c_int32),
                                                       ("h1mask", C.c_void_p)]


class GrMlpArgs(C.Structure):
    """Mirror of gr_mlp_args (include/gr.h)."""
    _fields_ = [("net", GrMlpNet * 2), ("rows", C.c_int64), ("nets", C.c_int32), ("hidden", C.c_int32),
                ("slope", C.c_float), ("reserved", C.c_int32), ("partial", C.c_void_p)]


def _mlp_layers(mlp: nn.Module):
    """(l1, l2, l3, slope) of a Linear -> LeakyReLU -> Linear -> LeakyReLU -> Linear stack, else None."""
    mods = list(mlp) if isinstance(mlp, nn.Sequential) else []
    if len(mods) != 5:
        return None
    l1, a1, l2, a2, l3 = mods
    if not (all(isinstance(m, nn.Linear) and m.bias is not None for m in (l1, l2, l3))
            and isinstance(a1, nn.LeakyReLU) and isinstance(a2, nn.LeakyReLU) and a1.negative_slope == a2.negative_slope):
        return None
    return l1, l2, l3, float(a1.negative_slope)


def networks_fusable(nets, xs) -> bool:
    """gr_mlp_forward / _backward cover these networks on these inputs: the update's tall fp32 CUDA batches (inputs
    without gradient, outside autocast) through Linear(d <= 32) -> LeakyReLU -> Linear(H, H) -> LeakyReLU ->
    Linear(H, k <= 4) with H 128 or 256, one slope, 32-bit row offsets."""
    if not torch.is_grad_enabled() or torch.is_autocast_enabled("cuda"):
        return False
    hs, slopes = set(), set()
    for net, x in zip(nets, xs):
        lay = _mlp_layers(net)
        if lay is None:
            return False
        l1, l2, l3, slope = lay
        if not (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and not x.requires_grad
                and (x.shape[0] >= 2 * SPLIT or _FORCE_FN) and x.shape[0] == xs[0].shape[0]):
            return False
        if not (l1.in_features == x.shape[1] and l1.in_features % 4 == 0 and l1.in_features <= 32
                and l1.out_features == l2.in_features == l2.out_features == l3.in_features
                and l3.out_features <= 4 and all(p.dtype == torch.float32 and p.is_cuda and p.requires_grad
                                                  for m in (l1, l2, l3) for p in (m.weight, m.bias))):
            return False
        if x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
            return False
        if x.shape[0] * max(l1.out_features, x.stride(0)) >= 2 ** 31:
            return False
        hs.add(l1.out_features)
        slopes.add(slope)
    return len(hs) == 1 and hs.pop() in (128, 256) and len(slopes) == 1


class _FusedMLPsFn(torch.autograd.Function):
    """Up to two MLPs (the actor and the critic) on their input rows, forward and backward each as one set of
    whole-network fp32-MFMA launches for both networks (gr_mlp_forward / gr_mlp_backward, gr_mlp.hip).  Forward
    saves h1 and z2 per network; the backward returns every parameter gradient from one fixed-order reduction and
    leaves the saved tensors intact (a retained graph may run it again)."""

    @staticmethod
    def forward(ctx, nnets, slope, *args):
        xs, params = args[:nnets], args[nnets:]
        rows = xs[0].shape[0]
        dev = xs[0].device
        a = GrMlpArgs()
        a.rows, a.nets, a.slope = rows, nnets, float(slope)
        keep, outs = [], []
        for i in range(nnets):
            w1, b1, w2, b2, w3, b3 = params[6 * i:6 * i + 6]
            h = w1.shape[0]
            h1 = torch.empty(rows, h, device=dev, dtype=torch.float32)
            z2 = torch.empty(rows, h, device=dev, dtype=torch.float32)
            y = torch.empty(rows, w3.shape[0], device=dev, dtype=torch.float32)
            s = GrMlpNet()
            s.x, s.ldx, s.d, s.k = xs[i].data_ptr(), xs[i].stride(0), w1.shape[1], w3.shape[0]
            for name, t in (("w1", w1), ("b1", b1), ("w2", w2), ("b2", b2), ("w3", w3), ("b3", b3)):
                setattr(s, name, t.data_ptr())
            s.h1, s.z2, s.y = h1.data_ptr(), z2.data_ptr(), y.data_ptr()
            # the sign of h1 as bits (H = 256: the backward reads these instead of the h1 rows, mlp_bwd256h)
            mask = torch.empty(_mask_words(rows, h), device=dev, dtype=torch.int64)
            s.h1mask = mask.data_ptr() if mask.numel() else None
            a.net[i] = s
            a.hidden = h
            keep += [h1, z2, mask]
            outs.append(y)
        _lib_call("gr_mlp_forward", C.byref(a), _stream(xs[0]))
        ctx.nnets, ctx.slope = nnets, float(slope)
        ctx.save_for_backward(*xs, *keep, *params)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gys):
        from .. import _abi

        nnets = ctx.nnets
        saved = ctx.saved_tensors
        xs, keep, params = saved[:nnets], saved[nnets:4 * nnets], saved[4 * nnets:]
        rows = xs[0].shape[0]
        dev = xs[0].device
        a = GrMlpArgs()
        a.rows, a.nets, a.slope = rows, nnets, ctx.slope
        grads_out, gys_keep = [], []
        for i in range(nnets):
            w1, b1, w2, b2, w3, b3 = params[6 * i:6 * i + 6]
            h, d, k = w1.shape[0], w1.shape[1], w3.shape[0]
            h1, z2, mask = keep[3 * i], keep[3 * i + 1], keep[3 * i + 2]
            gy = gys[i]
            gy = torch.zeros(rows, k, device=dev, dtype=torch.float32) if gy is None else gy.float().contiguous()
            gys_keep.append(gy)
            grads = _sink_region(params[6 * i:6 * i + 6])
            if grads is None:
                grads = torch.empty(h * d + h + h * h + h + k * h + k, device=dev, dtype=torch.float32)
            s = GrMlpNet()
            s.x, s.ldx, s.d, s.k = xs[i].data_ptr(), xs[i].stride(0), d, k
            for name, t in (("w1", w1), ("b1", b1), ("w2", w2), ("b2", b2), ("w3", w3), ("b3", b3)):
                setattr(s, name, t.data_ptr())
            # (gz2 in its own buffer: a retained graph, e.g. PPO's first-mini-batch autograd.grad check, runs this
            # backward twice over the same saved z2)
            gz2 = torch.empty_like(z2)
            gys_keep.append(gz2)
            s.h1, s.z2, s.gy, s.gz2, s.grads = h1.data_ptr(), z2.data_ptr(), gy.data_ptr(), gz2.data_ptr(), grads.data_ptr()
            s.h1mask = mask.data_ptr() if mask.numel() else None
            a.net[i] = s
            a.hidden = h
            o = 0
            split = []
            for shape in ((h, d), (h,), (h, h), (h,), (k, h), (k,)):
                numel = 1
                for e in shape:
                    numel *= e
                split.append(grads[o:o + numel].view(shape))
                o += numel
            grads_out += split
        part = torch.empty(_abi.load().gr_mlp_partials(rows, a.hidden, nnets), device=dev, dtype=torch.float32)
        a.partial = part.data_ptr()
        _lib_call("gr_mlp_backward", C.byref(a), _stream(xs[0]))
        return (None, None) + (None,) * nnets + tuple(grads_out)


# True: the forward also writes the sign of h1 as bits and the backward (H = 256) reads those instead of the h1 rows
# (mlp_bwd256h, two workgroups per CU).  Measured no faster than mlp_bwd256 (C2 +2 %, 393 216 rows -3 %, the
# forward's mask +2 %; DESIGN §4f''), so off by default; tests run both.
_H1_MASKS = False


def _mask_words(rows: int, hidden: int) -> int:
    """gr_mlp_h1mask_words for H = 256 (mlp_bwd256h); 0 (no mask: the backward reads h1) for H = 128."""
    if hidden != 256 or not _H1_MASKS:
        return 0
    from .. import _abi

    return int(_abi.load().gr_mlp_h1mask_words(rows, hidden))


def _sink_region(params):
    """The span of the flat gradient buffer holding these six parameters' gradient views (_GRAD_SINK), when they
    are contiguous, back to back and in this order; else None."""
    if _GRAD_SINK is None:
        return None
    views = [_GRAD_SINK.get(id(p)) for p in params]
    if any(v is None for v in views):
        return None
    base, off = views[0], 0
    for p, v in zip(params, views):
        if v.dtype != torch.float32 or not v.is_contiguous() or v.numel() != p.numel() or \
                v.data_ptr() != base.data_ptr() + 4 * off:
            return None
        off += p.numel()
    return torch.as_strided(base, (off,), (1,), base.storage_offset())


def fused_mlps(nets, xs):
    """The outputs of `nets` (nn.Sequential MLPs) on `xs` through _FusedMLPsFn; call only when networks_fusable."""
    params, slope = [], None
    for net in nets:
        l1, l2, l3, slope = _mlp_layers(net)
        params += [l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias]
    return _FusedMLPsFn.apply(len(nets), slope, *xs, *params)
