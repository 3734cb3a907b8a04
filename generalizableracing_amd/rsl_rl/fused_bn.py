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
    return C.c_void_p(_abi.raw_stream(x.device))


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


def batch_norm_act(bn: nn.BatchNorm2d, act: nn.Module, x: torch.Tensor, uses: int = 1,
                   count_first: bool = False) -> torch.Tensor:
    """act(bn(x)) for rows x [M, C] in training mode, running statistics updated as nn.BatchNorm2d does
    (the caller has already counted the batch in num_batches_tracked, unless count_first);
    uses > 1: as `uses` forwards of the same rows would (_update_running)."""
    code, slope = _act_code(act)
    y, stats = _BatchNormAct.apply(x, bn.weight, bn.bias, bn.eps, code, slope)
    _update_running(bn, stats, uses, count_first)
    return y


class _Stem1(torch.autograd.Function):
    """Conv2d(1, C, 3, stride 3) -> BatchNorm2d (batch statistics) -> act from the depth images (gr_stem1_*).
    Returns the nimg x na table-a rows only (the next conv's input as it is): the nimg x nb table-b rows enter the
    statistics but nothing reads them, so no zero-filled [rows, C] gradient is built for them in the backward."""

    @staticmethod
    def forward(ctx, img, conv_w, bn_w, bn_b, pix, na, nb, eps, act, slope, rows=None):
        lib = _abi.load()
        nimg = img.shape[0] if rows is None else rows.numel()
        c = conv_w.shape[0]
        y = torch.empty(nimg * na, c, device=img.device, dtype=torch.float32)
        stats = torch.empty(4, c, device=img.device, dtype=torch.float32)
        part = torch.empty(int(lib.gr_stem1_scratch_doubles(nimg, na + nb, c)), device=img.device, dtype=torch.float64)
        w = conv_w.detach().reshape(c, 9).contiguous()
        bw, bb = bn_w.detach().contiguous(), bn_b.detach().contiguous()
        rc = lib.gr_stem1_forward(img.data_ptr(), img.stride(0), 0, _rows_ptr(rows), nimg, pix.data_ptr(), na, nb,
                                  w.data_ptr(), c, bw.data_ptr(), bb.data_ptr(), float(eps), act, float(slope),
                                  y.data_ptr(), nimg * na, stats.data_ptr(), part.data_ptr(), _stream(img))
        if rc != 0:
            raise RuntimeError(f"gr_stem1_forward failed (status {rc})")
        ctx.save_for_backward(img, w, bw, bb, stats)
        ctx.pix = pix  # a constant table (possibly made under inference mode): kept as an attribute
        ctx.rows = rows  # (the batch's row indices into img, or None)
        ctx.args = (na, nb, act, slope, conv_w.shape)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, gy, _gstats):
        if ctx.needs_input_grad[0]:
            raise RuntimeError("the fused stem computes no gradient for the image")
        lib = _abi.load()
        img, w, bw, bb, stats = ctx.saved_tensors
        pix = ctx.pix
        na, nb, act, slope, wshape = ctx.args
        rows = ctx.rows
        nimg, c = (img.shape[0] if rows is None else rows.numel()), w.shape[0]
        gy = gy.contiguous()
        gconv = torch.empty(c, 9, device=img.device, dtype=torch.float32)
        gbw = torch.empty(c, device=img.device, dtype=torch.float32)
        gbb = torch.empty(c, device=img.device, dtype=torch.float32)
        part = torch.empty(int(lib.gr_stem1_scratch_doubles(nimg, na + nb, c)), device=img.device, dtype=torch.float64)
        rc = lib.gr_stem1_backward(img.data_ptr(), img.stride(0), 0, _rows_ptr(rows), nimg, pix.data_ptr(), na, nb,
                                   w.data_ptr(), c, bw.data_ptr(), bb.data_ptr(), stats.data_ptr(), act, float(slope),
                                   gy.data_ptr(),
                                   gy.shape[0], gconv.data_ptr(), gbw.data_ptr(), gbb.data_ptr(), part.data_ptr(),
                                   _stream(img))
        if rc != 0:
            raise RuntimeError(f"gr_stem1_backward failed (status {rc})")
        return None, gconv.view(wshape), gbw, gbb, None, None, None, None, None, None, None


# conv2's weight gradient inside the first block's backward (gr_stem12_backward_w2: y1 recomputed there, so the forward
# stores no y1 and no separate gz2^T y1 pass runs); False: the round-5 form (y1 stored, gr_patch_wgrad) for A/B
STEM12_W2 = True
STEM12_W2_MAX_N2 = 80  # (gr_stem12_backward_w2 covers conv2 patch counts up to 80 per image: 72 x 96 images)
# the backward's sums of the pixels and of xhat x pixels (conv1's weight gradient) from the forward's pixel moments
# instead of 4 MFMA per tile and table b's tiles (gr_stem12_forward / gr_stem12_backward_w2 `moments`); False: A/B
STEM12_MOMENTS = True


def _w2_path(fused_forward: bool, na: int) -> bool:
    return STEM12_W2 and fused_forward and 1 <= na // 9 <= STEM12_W2_MAX_N2


class _Stem12(torch.autograd.Function):
    """The first block (as _Stem1, C = 16) followed by conv2: z2 = y1.view(-1, 144) @ w2^T, w2 [32, 144] in (position j,
    channel) column order.  The forward computes conv2 inside the first block's apply pass (gr_stem12_forward); the
    backward takes conv2's output gradient straight into the first block's passes: conv2's input gradient, a
    [rows, 144] matrix, is never written, and conv2's weight gradient gz2^T y1 is contracted there too from y1
    recomputed in registers (gr_stem12_backward_w2), so y1 itself is never written either.  (STEM12_W2 False: y1 is
    stored by the forward and conv2's weight gradient is the split-K product of gz2 and the saved y1.)"""

    @staticmethod
    def forward(ctx, img, conv_w, bn_w, bn_b, w2, pix, na, nb, eps, act, slope, fused_forward=True, rows=None,
                keep_y=True):
        lib = _abi.load()
        nimg = img.shape[0] if rows is None else rows.numel()
        # (keep_y False: no backward will run, so y1 — kept only for conv2's weight gradient — is not stored; nor when
        # that gradient is formed inside the first block's backward)
        w2_path = _w2_path(fused_forward, na)
        backward_follows = keep_y
        keep_y = (keep_y and not w2_path) or not fused_forward
        y = torch.empty(nimg * na if keep_y else 0, 16, device=img.device, dtype=torch.float32)
        stats = torch.empty(4, 16, device=img.device, dtype=torch.float32)
        part = torch.empty(int(lib.gr_stem1_scratch_doubles(nimg, na + nb, 16)), device=img.device, dtype=torch.float64)
        w = conv_w.detach().reshape(16, 9).contiguous()
        bw, bb = bn_w.detach().contiguous(), bn_b.detach().contiguous()
        w2d = w2.detach()
        # the statistics pass's pixel moments, when the backward will take conv1's A2 / A3 sums from them
        mom = torch.empty(64 if (w2_path and STEM12_MOMENTS and backward_follows) else 0, device=img.device,
                          dtype=torch.float64)
        if fused_forward:
            # conv2 inside the first block's apply pass: w2f[j][g][o][v] = W2[o][j * 16 + 4 g + v]
            w2f = w2d.reshape(32, 9, 4, 4).permute(1, 2, 0, 3).contiguous()
            z2 = torch.empty(nimg * (na // 9), 32, device=img.device, dtype=torch.float32)
            rc = lib.gr_stem12_forward(img.data_ptr(), img.stride(0), 0, _rows_ptr(rows), nimg, pix.data_ptr(), na, nb,
                                       w.data_ptr(), 16, bw.data_ptr(), bb.data_ptr(), float(eps), act, float(slope),
                                       w2f.data_ptr(),
                                       na // 9, y.data_ptr() if keep_y else None, z2.data_ptr(), stats.data_ptr(),
                                       mom.data_ptr() if mom.numel() else None, part.data_ptr(), _stream(img))
        else:  # the first block's kernels, then conv2 as a GEMM (the A/B reference of the fused forward)
            rc = lib.gr_stem1_forward(img.data_ptr(), img.stride(0), 0, _rows_ptr(rows), nimg, pix.data_ptr(), na, nb,
                                      w.data_ptr(), 16, bw.data_ptr(), bb.data_ptr(), float(eps), act, float(slope),
                                      y.data_ptr(), nimg * na, stats.data_ptr(), part.data_ptr(), _stream(img))
            z2 = y.view(-1, 144) @ w2d.t() if rc == 0 else None
        if rc != 0:
            raise RuntimeError(f"gr_stem12_forward failed (status {rc})")
        ctx.save_for_backward(img, w, bw, bb, stats, y, w2d, mom)
        ctx.pix = pix
        ctx.rows = rows
        ctx.args = (na, nb, act, slope, conv_w.shape)
        ctx.w2_path = w2_path
        ctx.mark_non_differentiable(stats)
        return z2, stats

    @staticmethod
    def backward(ctx, gz2, _gstats):
        if ctx.needs_input_grad[0]:
            raise RuntimeError("the fused stem computes no gradient for the image")
        lib = _abi.load()
        img, w, bw, bb, stats, y, w2d, mom = ctx.saved_tensors
        na, nb, act, slope, wshape = ctx.args
        rows = ctx.rows
        nimg = img.shape[0] if rows is None else rows.numel()
        gz2 = gz2.contiguous()
        if gz2.data_ptr() % 16:
            gz2 = gz2.clone()
        # w2t[j][g][ch][s] = W2[o = 8 g + s][j * 16 + ch]
        w2t = w2d.reshape(4, 8, 9, 16).permute(2, 0, 3, 1).contiguous()
        gconv = torch.empty(16, 9, device=img.device, dtype=torch.float32)
        gbw = torch.empty(16, device=img.device, dtype=torch.float32)
        gbb = torch.empty(16, device=img.device, dtype=torch.float32)
        if ctx.w2_path:  # the first block's backward with conv2's dgrad and wgrad (y1 recomputed)
            gw2 = torch.empty(32, 144, device=img.device, dtype=torch.float32)
            part = torch.empty(int(lib.gr_stem12_backward_w2_scratch_doubles(nimg)), device=img.device,
                               dtype=torch.float64)
            rc = lib.gr_stem12_backward_w2(img.data_ptr(), img.stride(0), 0, _rows_ptr(rows), nimg, ctx.pix.data_ptr(),
                                           na, nb, w.data_ptr(), 16, bw.data_ptr(), bb.data_ptr(), stats.data_ptr(),
                                           mom.data_ptr() if mom.numel() else None, act,
                                           float(slope), gz2.data_ptr(), na // 9, w2t.data_ptr(), gconv.data_ptr(),
                                           gbw.data_ptr(), gbb.data_ptr(), gw2.data_ptr(), part.data_ptr(), _stream(img))
            if rc != 0:
                raise RuntimeError(f"gr_stem12_backward_w2 failed (status {rc})")
            return (None, gconv.view(wshape), gbw, gbb, gw2 if ctx.needs_input_grad[4] else None, None, None, None,
                    None, None, None, None, None, None)
        gw2 = None
        if ctx.needs_input_grad[4]:  # conv2's weight: gz2^T y1 patches (gr_patch_wgrad: MFMA, fixed-order sums)
            from .linear import tall_wgrad

            gw2 = tall_wgrad(gz2, y.view(y.shape[0] // 9, 144))
        part = torch.empty(int(lib.gr_stem1_scratch_doubles(nimg, na + nb, 16)), device=img.device, dtype=torch.float64)
        rc = lib.gr_stem12_backward(img.data_ptr(), img.stride(0), 0, _rows_ptr(rows), nimg, ctx.pix.data_ptr(), na, nb,
                                    w.data_ptr(), 16, bw.data_ptr(), bb.data_ptr(), stats.data_ptr(), act, float(slope),
                                    gz2.data_ptr(),
                                    na // 9, w2t.data_ptr(), gconv.data_ptr(), gbw.data_ptr(), gbb.data_ptr(),
                                    part.data_ptr(), _stream(img))
        if rc != 0:
            raise RuntimeError(f"gr_stem12_backward failed (status {rc})")
        return None, gconv.view(wshape), gbw, gbb, gw2, None, None, None, None, None, None, None, None, None


class _BnActPatchGemm(torch.autograd.Function):
    """y = act(bn(z)).view(-1, k) @ w^T without writing act(bn(z)): the vision stem's block 2 (BatchNorm2d(32) ->
    LeakyReLU on conv2's output rows z [M, 32]) feeding conv3 (w [64, 128], its 2 x 2 patches of four consecutive
    rows).  Forward: the BatchNorm's statistics pass (gr_bn_stats), then conv3 with the BatchNorm and activation
    applied as the rows are loaded (gr_tsgemm_bnact).  Backward: conv3's input gradient (gr_tsgemm), its weight
    gradient recomputing act(bn(z)) on load (gr_patch_wgrad_bnact), and the BatchNorm + activation backward
    (gr_bn_act_backward) on z.  The same values as batch_norm_act then the patch GEMM (the applied rows are
    bit-identical to gr_bn_act_forward's)."""

    @staticmethod
    def forward(ctx, z, bn_w, bn_b, w, eps, act, slope):
        lib = _abi.load()
        m, c = z.shape
        n, k = w.shape
        stats = torch.empty(4, c, device=z.device, dtype=torch.float32)
        part = torch.empty(int(lib.gr_bn_scratch_doubles(m, c)), device=z.device, dtype=torch.float64)
        rc = lib.gr_bn_stats(z.data_ptr(), m, c, float(eps), stats.data_ptr(), part.data_ptr(), _stream(z))
        if rc != 0:
            raise RuntimeError(f"gr_bn_stats failed (status {rc})")
        bw, bb, wd = bn_w.detach().contiguous(), bn_b.detach().contiguous(), w.detach().contiguous()
        mp = m * c // k
        y = torch.empty(mp, n, device=z.device, dtype=torch.float32)
        rc = lib.gr_tsgemm_bnact(z.data_ptr(), k, wd.data_ptr(), y.data_ptr(), n, mp, k, n, c, stats.data_ptr(),
                                 bw.data_ptr(), bb.data_ptr(), act, float(slope), _stream(z))
        if rc != 0:
            raise RuntimeError(f"gr_tsgemm_bnact failed (status {rc})")
        ctx.save_for_backward(z, bw, bb, stats, wd)
        ctx.act, ctx.slope = act, slope
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, gy, _gstats):
        lib = _abi.load()
        z, bw, bb, stats, w = ctx.saved_tensors
        m, c = z.shape
        n, k = w.shape
        mp = m * c // k
        gy = gy.contiguous()
        dev = z.device
        gw = None
        if ctx.needs_input_grad[3]:  # conv3's weight: gy^T act(bn(z)), recomputed on load
            gw = torch.empty(n, k, device=dev, dtype=torch.float32)
            wpart = torch.empty(int(lib.gr_patch_wgrad_floats(mp, n, k)), device=dev, dtype=torch.float32)
            rc = lib.gr_patch_wgrad_bnact(z.data_ptr(), k, gy.data_ptr(), mp, n, k, wpart.data_ptr(), gw.data_ptr(), c,
                                          stats.data_ptr(), bw.data_ptr(), bb.data_ptr(), ctx.act, float(ctx.slope),
                                          _stream(z))
            if rc != 0:
                raise RuntimeError(f"gr_patch_wgrad_bnact failed (status {rc})")
        # the gradient of act(bn(z)) = gy w, then the BatchNorm + activation backward on z
        dblock = torch.empty(mp, k, device=dev, dtype=torch.float32)
        rc = lib.gr_tsgemm(gy.data_ptr(), n, w.data_ptr(), 0, dblock.data_ptr(), k, mp, n, k, _stream(z))
        if rc != 0:
            raise RuntimeError(f"gr_tsgemm failed (status {rc})")
        gx = torch.empty_like(z)
        gbw = torch.empty(c, device=dev, dtype=torch.float32)
        gbb = torch.empty(c, device=dev, dtype=torch.float32)
        part = torch.empty(int(lib.gr_bn_scratch_doubles(m, c)), device=dev, dtype=torch.float64)
        rc = lib.gr_bn_act_backward(z.data_ptr(), dblock.data_ptr(), m, c, bw.data_ptr(), bb.data_ptr(),
                                    stats.data_ptr(), ctx.act, float(ctx.slope), gx.data_ptr(), gbw.data_ptr(),
                                    gbb.data_ptr(), part.data_ptr(), _stream(z))
        if rc != 0:
            raise RuntimeError(f"gr_bn_act_backward failed (status {rc})")
        return gx, gbw, gbb, gw, None, None, None


def bn_act_conv_applicable(bn: nn.BatchNorm2d, act: nn.Module, z: torch.Tensor, w: torch.Tensor) -> bool:
    """_BnActPatchGemm covers block 2 -> conv3: fused_applicable(bn, act, z) with 32 channels, w [64, 128] fp32, the
    patches four consecutive rows."""
    return (fused_applicable(bn, act, z) and z.shape[1] == 32 and tuple(w.shape) == (64, 128)
            and w.dtype == torch.float32 and (z.shape[0] * 32) % 128 == 0)


def bn_act_conv(bn: nn.BatchNorm2d, act: nn.Module, z: torch.Tensor, w: torch.Tensor, uses: int = 1,
                count_first: bool = False) -> torch.Tensor:
    """act(bn(z)).view(-1, 128) @ w^T (block 2 into conv3) without materialising act(bn(z)); running statistics updated
    as batch_norm_act does."""
    code, slope = _act_code(act)
    y, stats = _BnActPatchGemm.apply(z, bn.weight, bn.bias, w, bn.eps, code, slope)
    _update_running(bn, stats, uses, count_first)
    return y


def stem12_applicable(bn: nn.BatchNorm2d, act: nn.Module, img: torch.Tensor, conv_w: torch.Tensor,
                      conv2_w: torch.Tensor, na: int) -> bool:
    """The fused first block + conv2 backward: stem1_applicable with 16 channels, conv2 = Conv2d(16, 32, 3, stride 3)
    without bias, and the table-a rows grouped as its patches (na = 9 n2)."""
    return (stem1_applicable(bn, act, img, conv_w) and conv_w.shape[0] == 16 and
            tuple(conv2_w.shape) == (32, 16, 3, 3) and conv2_w.dtype == torch.float32 and na % 9 == 0)


def stem12_bn_act_conv(bn: nn.BatchNorm2d, act: nn.Module, conv_w: torch.Tensor, w2: torch.Tensor, img: torch.Tensor,
                       pix: torch.Tensor, na: int, nb: int, uses: int = 1, fused_forward: bool = True,
                       count_first: bool = False, rows: torch.Tensor | None = None) -> torch.Tensor:
    """conv2's output rows [B * na / 9, 32] = patches(act(bn(conv(img)))) @ w2^T (w2 [32, 144], columns (j, c)),
    running statistics of the first BN updated as stem1_bn_act does.  rows: the batch is img[rows] (int64 device
    indices), read through them instead of a gathered copy."""
    code, slope = _act_code(act)
    keep_y = torch.is_grad_enabled() and any(t.requires_grad for t in (conv_w, bn.weight, bn.bias, w2))
    z2, stats = _Stem12.apply(img, conv_w, bn.weight, bn.bias, w2, pix, na, nb, bn.eps, code, slope, fused_forward,
                              _rows_arg(rows), keep_y)
    _update_running(bn, stats, uses, count_first)
    return z2


def stem1_applicable(bn: nn.BatchNorm2d, act: nn.Module, img: torch.Tensor, conv_w: torch.Tensor) -> bool:
    """The image-side HIP op: fp32 CUDA image rows (unit column stride), a 1-channel 3x3 conv without bias into
    C in {4, 8, 16, 32, 64} channels, training-mode BN, LeakyReLU / ELU(1)."""
    return (img.is_cuda and img.dtype == torch.float32 and img.dim() == 2 and img.stride(1) == 1
            and not img.requires_grad and tuple(conv_w.shape[1:]) == (1, 3, 3) and conv_w.shape[0] in _CHANNELS
            and conv_w.dtype == torch.float32 and bn.affine and bn.training and _act_code(act) is not None)


def stem1_bn_act(bn: nn.BatchNorm2d, act: nn.Module, conv_w: torch.Tensor, img: torch.Tensor, pix: torch.Tensor,
                 na: int, nb: int, uses: int = 1, count_first: bool = False,
                 rows: torch.Tensor | None = None) -> torch.Tensor:
    """act(bn(conv(img))) as the table-a patch rows of VisionActorCritic.stem_gemm (img [B, H*W] rows; pix int16
    [(na + nb) * 9] pixel offsets; the B * nb table-b rows count in the statistics and are not returned), running
    statistics updated as nn.BatchNorm2d does (the caller counts the batch in num_batches_tracked)."""
    code, slope = _act_code(act)
    y, stats = _Stem1.apply(img, conv_w, bn.weight, bn.bias, pix, na, nb, bn.eps, code, slope, _rows_arg(rows))
    _update_running(bn, stats, uses, count_first)
    return y


def _rows_arg(rows):
    """The batch's row indices as the kernels take them (contiguous int64 on the image's device), or None."""
    if rows is None:
        return None
    if rows.dtype != torch.int64 or rows.dim() != 1:
        raise ValueError("row indices: a 1-D int64 tensor")
    return rows.contiguous()


def _rows_ptr(rows):
    return rows.data_ptr() if rows is not None else None


def _update_running(bn: nn.BatchNorm2d, stats: torch.Tensor, uses: int = 1, count_first: bool = False):
    """The running-statistics update of one training-mode forward; uses > 1 replays it as `uses` forwards of the
    same rows would, in sequence (each forward after the first counted here in num_batches_tracked, the first too
    with count_first, else by the caller).  With a momentum on the GPU: one launch (gr_bn_running_update)."""
    if not bn.track_running_stats or bn.running_mean is None:
        return
    nbt = bn.num_batches_tracked
    count = uses if count_first else uses - 1
    rm, rv = bn.running_mean, bn.running_var
    if (bn.momentum is not None and stats.is_cuda and rm.is_cuda and rm.dtype == torch.float32
            and rv.dtype == torch.float32 and rm.is_contiguous() and rv.is_contiguous() and stats.is_contiguous()
            and (nbt is None or nbt.dtype == torch.int64)):
        m = float(bn.momentum)
        # (through raw pointers, as F.batch_norm updates them inside its kernel: no version bump, so a torch
        # batch_norm of the same forward that saved them for its backward stays valid)
        rc = _abi.load().gr_bn_running_update(rm.data_ptr(), rv.data_ptr(), nbt.data_ptr() if nbt is not None else None,
                                              stats.data_ptr(), rm.numel(), float(1.0 - m), m, int(uses),
                                              int(count) if nbt is not None else 0, _stream(stats))
        if rc != 0:
            raise RuntimeError(f"gr_bn_running_update failed (status {rc})")
        return
    for k in range(uses):
        if (k or count_first) and nbt is not None:
            nbt.add_(1)
        if bn.track_running_stats and bn.running_mean is not None:
            momentum = 0.0 if bn.momentum is None else bn.momentum
            if bn.momentum is None and bn.num_batches_tracked is not None:
                momentum = 1.0 / float(bn.num_batches_tracked)
            with torch.no_grad():
                # (through .data, as F.batch_norm updates them inside its kernel: no version bump, so a torch
                # batch_norm of the same forward that saved them for its backward stays valid)
                bn.running_mean.data.mul_(1.0 - momentum).add_(stats[0], alpha=momentum)
                bn.running_var.data.mul_(1.0 - momentum).add_(stats[3], alpha=momentum)


def reference_batch_norm_act(bn: nn.BatchNorm2d, act: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """torch's own ops for the same step (tests; eval mode)."""
    return act(F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                            0.0 if bn.momentum is None else bn.momentum, bn.eps))
