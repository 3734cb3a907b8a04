"""VisionActorCritic — the reference's depth-image policy
(standalone/rsl_rl/ext/modules/vision_actor_critic.py:43-144), used by the registered racing recipe
(quadcopter_diff/agents/rsl_rl_ppo_cfg.py:43-52,80-104: img_res (72, 96), dim_hidden_input 192,
128x128 heads, lrelu, PPOL2C2).

Observation rows are [state | H*W depth image] (racing_ctbr_env.py:141-160).  The image goes
through a strided conv stem (Conv 3x3/3 -> BN -> act, 3x3/3, 2x2/2, flatten, linear), the state
through one linear layer; their sum, activated, feeds the actor and critic MLPs.  Module names and
order match the reference so its checkpoints load as-is.  Convs / GEMMs run on MIOpen / hipBLASLt
through torch.

MI355X path: every stem convolution has stride == kernel and no padding, i.e. it convolves
non-overlapping patches.  `features()` therefore evaluates the stem as three patch GEMMs on
channels-last activations (hipBLASLt) instead of MIOpen direct convolutions, with the BatchNorm
statistics taken over the same (batch, height, width) set and the flatten order of the reference
(NCHW) kept by permuting the final Linear's columns.  The nn.Conv2d / nn.BatchNorm2d modules hold
the parameters and running statistics exactly as the reference's, so checkpoints are interchangeable;
`stem(img)` still runs the reference module as written (tests compare the two).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import linear as _lin
from .actor_critic import ActorCritic, resolve_nn_activation
from .fused_bn import (batch_norm_act, bn_act_conv, bn_act_conv_applicable, fused_applicable, stem1_applicable,
                       stem1_bn_act, stem12_applicable, stem12_bn_act_conv)


def _conv_out(n: int, k: int, s: int) -> int:
    return (n - k) // s + 1


class _PatchGemm(torch.autograd.Function):
    """y = x @ w^T for tall-skinny x [M, K] (M = batch * patches, millions) and a small w [N, K].

    The weight gradient w^T-shaped [N, K] = dy^T x reduces over all M rows; as one GEMM hipBLASLt
    tiles only its tiny N x K output (one or a few workgroups stream millions of rows).  Here it is
    split over M into chunks of SPLIT rows (a batched GEMM, one workgroup set per chunk) and the
    partial products are summed."""

    SPLIT = 8192

    @staticmethod
    def forward(ctx, x, w, b=None):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        if b is None:
            y = _tsgemm(x, w, True)
            return y if y is not None else x @ w.t()
        return torch.addmm(b, x, w.t())  # (the bias in the GEMM's epilogue)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = None
        if ctx.needs_input_grad[0]:
            gx = _tsgemm(gy, w, False)
            gx = gx if gx is not None else gy @ w
        # (the bias gradient by gr_column_sum: a fixed-order pass, and graph-safe where torch's multi-block sum is
        # not, linear.bias_grad)
        gb = _lin.bias_grad(gy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        gw = None
        if ctx.needs_input_grad[1]:
            m, c = x.shape[0], _PatchGemm.SPLIT
            s = m // c
            if gy.is_cuda and _abi_wgrad_ok(gy, x):  # gr_patch_wgrad: one MFMA pass, fixed-order sums
                gw = _lin.tall_wgrad(gy, x)
            elif s >= 2:
                gw = torch.bmm(gy[: s * c].view(s, c, -1).transpose(1, 2), x[: s * c].view(s, c, -1)).sum(0)
                if m > s * c:
                    gw = gw + gy[s * c:].t() @ x[s * c:]
            else:
                gw = gy.t() @ x
        return gx, gw, gb


def _tsgemm(a, w, b_nk: bool):
    """a @ w^T (b_nk) or a @ w on gr_tsgemm (the weight staged in LDS, the rows streamed once) when it covers the shape
    (conv3: [M, 128] x [64, 128]^T and [M, 64] x [64, 128]; the final Linear's input gradient [M, 192] x [192, 1280]),
    else None."""
    if not (a.is_cuda and a.dtype == torch.float32 and w.dtype == torch.float32 and a.dim() == 2 and a.stride(1) == 1):
        return None
    from .. import _abi

    k = a.shape[1]
    n = w.shape[0] if b_nk else w.shape[1]
    if not ((k == 128 and n == 64 and b_nk) or (k == 64 and n == 128 and not b_nk)
            or (k == 192 and not b_nk and n % 64 == 0 and n <= 4096)):
        return None
    w = w.contiguous()
    out = torch.empty(a.shape[0], n, device=a.device, dtype=torch.float32)
    rc = _abi.load().gr_tsgemm(a.data_ptr(), a.stride(0), w.data_ptr(), int(b_nk), out.data_ptr(), n, a.shape[0], k,
                               n, _abi.raw_stream(a.device))
    if rc != 0:
        raise RuntimeError(f"gr_tsgemm failed (status {rc})")
    return out


def _abi_wgrad_ok(gy, x) -> bool:
    """gr_patch_wgrad covers the shape (conv3: 64 x 128, the final Linear: 192 x 1280, conv2: 32 x 144)."""
    from .. import _abi

    return (gy.dtype == torch.float32 and x.dtype == torch.float32 and x.stride(-1) == 1
            and int(_abi.load().gr_patch_wgrad_floats(x.shape[0], gy.shape[1], x.shape[1])) > 0)


def _gemm(x, w, b=None):
    """x @ w^T (+ b): _PatchGemm with autograd on, else one GEMM (gr_tsgemm where it covers the shape; the bias in
    the GEMM's epilogue)."""
    if torch.is_grad_enabled():
        return _PatchGemm.apply(x, w, b)
    if b is None:
        y = _tsgemm(x, w, True)
        return y if y is not None else x @ w.t()
    return torch.addmm(b, x, w.t())


class VisionActorCritic(ActorCritic):
    is_recurrent = False
    # training-mode BatchNorm + activation of the stem as one HIP op on the GPU (rsl_rl/fused_bn.py); False:
    # torch's batch_norm and activation ops (tests compare the two)
    fused_bn = True
    # with fused_bn: conv2's input gradient formed inside the first block's backward passes (fused_bn._Stem12); False:
    # the first block alone, conv2 as a patch GEMM (tests and scripts/bench_vision.py --no-fused-conv2 compare the two)
    fused_conv2 = True
    # with fused_conv2: conv2's forward inside the first block's apply pass too (False: conv2's forward as a GEMM)
    fused_conv2_forward = True
    # with fused_conv2: block 2's BatchNorm + activation applied as conv3 loads its rows (never written)
    fused_conv3 = True

    def __init__(self, num_actor_obs: int, num_critic_obs: int, num_actions: int, img_res=(72, 96),
                 dim_hidden_input: int = 192, actor_hidden_dims=(256, 256, 256), critic_hidden_dims=(256, 256, 256),
                 activation="elu", init_noise_std=1.0, noise_std_type: str = "scalar", **kwargs):
        self.use_auxiliary_loss = bool(kwargs.pop("use_auxiliary_loss", False))
        super().__init__(dim_hidden_input, dim_hidden_input, num_actions, actor_hidden_dims=actor_hidden_dims,
                         critic_hidden_dims=critic_hidden_dims, activation=activation,
                         init_noise_std=init_noise_std, noise_std_type=noise_std_type, **kwargs)
        self.activation = resolve_nn_activation(activation)
        self.img_res = tuple(int(x) for x in img_res)
        h, w = self.img_res
        h1, w1 = _conv_out(h, 3, 3), _conv_out(w, 3, 3)
        h2, w2 = _conv_out(h1, 3, 3), _conv_out(w1, 3, 3)
        h3, w3 = _conv_out(h2, 2, 2), _conv_out(w2, 2, 2)
        if min(h3, w3) <= 0:
            raise ValueError(f"image {self.img_res} too small for the conv stem")
        self.stem = nn.Sequential(
            nn.Conv2d(1, 16, 3, 3, bias=False),
            nn.BatchNorm2d(16),
            self.activation,
            nn.Conv2d(16, 32, 3, 3, bias=False),
            nn.BatchNorm2d(32),
            self.activation,
            nn.Conv2d(32, 64, 2, 2, bias=False),
            nn.BatchNorm2d(64),
            self.activation,
            nn.Flatten(),
            nn.Linear(64 * h3 * w3, dim_hidden_input),  # 1280 at 72x96
        )
        self._dims = (h1, w1, h2, w2, h3, w3)
        self._pidx = None
        self.num_pixels = h * w
        if num_actor_obs <= self.num_pixels:
            raise ValueError(f"num_actor_obs {num_actor_obs} must exceed the image size {self.num_pixels}")
        self.state_enc = nn.Linear(num_actor_obs - self.num_pixels, dim_hidden_input)
        if self.use_auxiliary_loss:
            self.aux_decoder = nn.Linear(dim_hidden_input, 1)

    # how many forwards of the same rows one stem evaluation stands for (shared_features): each BatchNorm's running
    # statistics are updated that many times, as that many training-mode forwards would
    _bn_uses = 1

    def _bn(self, bn: nn.BatchNorm2d, x: torch.Tensor) -> torch.Tensor:
        """nn.BatchNorm2d.forward on channels-last rows [M, C] (M = batch*height*width)."""
        y = self._bn_once(bn, x)
        if self._bn_uses > 1 and bn.training and bn.track_running_stats and bn.running_mean is not None:
            from .fused_bn import _update_running

            with torch.no_grad():
                xd = x.detach().double()
                stats = torch.stack([xd.mean(0), xd.var(0, unbiased=False), xd.var(0, unbiased=False),
                                     xd.var(0, unbiased=True)]).float()
            for _ in range(self._bn_uses - 1):  # (F.batch_norm made the first update)
                if bn.num_batches_tracked is not None:
                    bn.num_batches_tracked.add_(1)
                _update_running(bn, stats)
        return y

    def _bn_once(self, bn: nn.BatchNorm2d, x: torch.Tensor) -> torch.Tensor:
        momentum = 0.0 if bn.momentum is None else bn.momentum
        if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            if bn.momentum is None:
                momentum = 1.0 / float(bn.num_batches_tracked)
        use_batch = bn.training or (bn.running_mean is None and bn.running_var is None)
        args = (bn.running_mean if not bn.training or bn.track_running_stats else None,
                bn.running_var if not bn.training or bn.track_running_stats else None,
                bn.weight, bn.bias, use_batch, momentum, bn.eps)
        if use_batch and x.device.type == "cpu":
            # torch's CPU batch_norm reduces an [M, C] (channels-last) input with ~1e-4 relative error at M ~ 2e5
            # rows when |mean| >> std (depth-image activations); on [1, C, M] it reduces as it does the
            # reference's NCHW tensors (~3e-7).  The GPU kernels are accurate in either layout.
            return F.batch_norm(x.t().contiguous().unsqueeze(0), *args)[0].t().contiguous()
        return F.batch_norm(x, *args)

    def _bn_act(self, bn: nn.BatchNorm2d, act: nn.Module, x: torch.Tensor) -> torch.Tensor:
        """act(bn(x)) on rows [M, C]: the fused HIP op in training mode on the GPU, else torch's ops."""
        if self.fused_bn and fused_applicable(bn, act, x):  # (the batch counted with the running statistics)
            return batch_norm_act(bn, act, x, self._bn_uses, count_first=True)
        return act(self._bn(bn, x))

    def _bn_statistics(self, bn: nn.BatchNorm2d, x: torch.Tensor) -> None:
        """A training-mode forward's effect on bn without its output: the running statistics and batch count."""
        if not (bn.training and bn.track_running_stats):
            return
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.is_contiguous() \
                and x.shape[1] in (4, 8, 16, 32, 64) and x.shape[0] >= 2 and self.fused_bn:
            from .. import _abi
            from .fused_bn import _stream, _update_running

            lib = _abi.load()
            m, c = x.shape
            stats = torch.empty(4, c, device=x.device, dtype=torch.float32)
            part = torch.empty(int(lib.gr_bn_scratch_doubles(m, c)), device=x.device, dtype=torch.float64)
            rc = lib.gr_bn_stats(x.data_ptr(), m, c, float(bn.eps), stats.data_ptr(), part.data_ptr(), _stream(x))
            if rc != 0:
                raise RuntimeError(f"gr_bn_stats failed (status {rc})")
            _update_running(bn, stats, self._bn_uses, count_first=True)
            return
        self._bn(bn, x.detach())

    def record_batch_statistics(self, observations: torch.Tensor, rows: torch.Tensor | None = None) -> None:
        """What a training-mode forward of these rows changes besides its output: every BatchNorm's running
        statistics and batch count (the stem up to block 3's statistics; no final Linear, state encoder or heads).
        PPOL2C2's update evaluates the policy on the successor observations only for that side effect
        (ppo_l2c2.py:188-189: `action_smoothness` is computed under inference mode and never used)."""
        if rows is None:
            img = observations[:, -self.num_pixels:].reshape(-1, 1, *self.img_res)
        else:
            img = observations[:, -self.num_pixels:]
        self.stem_gemm(img, rows=rows, statistics_only=True)

    def _patch_index(self, device):
        """Pixel indices of conv1's patches, rows ordered so that every later layer's input is a VIEW of
        the previous layer's output: conv1 rows feeding conv2 come grouped as conv2's 3x3 patches,
        those grouped as conv3's 2x2 patches; positions a later conv does not cover (conv1 columns
        30-31 at 72x96) follow at the end — they still enter the BatchNorm statistics."""
        if getattr(self, "_pidx", None) is not None and self._pidx[0].device == torch.device(device):
            return self._pidx
        h, w = self.img_res
        h1, w1, h2, w2, h3, w3 = self._dims
        g3 = [(2 * v3 + i, 2 * u3 + j) for v3 in range(h3) for u3 in range(w3) for i in range(2) for j in range(2)]
        s3 = set(g3)
        g2 = g3 + [(v, u) for v in range(h2) for u in range(w2) if (v, u) not in s3]
        l1 = [(3 * v2 + i, 3 * u2 + j) for v2, u2 in g2 for i in range(3) for j in range(3)]
        s1 = set(l1)
        l1_left = [(v, u) for v in range(h1) for u in range(w1) if (v, u) not in s1]

        def pix(cells):
            return torch.tensor([(3 * v + i) * w + 3 * u + j for v, u in cells for i in range(3) for j in range(3)],
                                dtype=torch.long, device=device)

        with torch.inference_mode(False):  # cached across rollouts (inference mode) and updates
            a, b = pix(l1), pix(l1_left)
            # the same cells as int16 offsets, table a then table b, for the fused first block (gr_stem1_*)
            pix16 = torch.cat([a, b]).to(torch.int16)
        self._pidx = (a, b, len(l1), len(l1_left), len(g3), len(g2), pix16)
        return self._pidx

    def stem_gemm(self, img: torch.Tensor, extra_bias: torch.Tensor | None = None,
                  rows: torch.Tensor | None = None, statistics_only: bool = False) -> torch.Tensor | None:
        """The conv stem as patch GEMMs (identical math to self.stem(img), other summation order); extra_bias is added
        to the final Linear's bias (features() passes the state encoder's).  rows: the batch is img[rows], read
        through the indices by the fused first block (the other paths gather it)."""
        conv1, bn1, act, conv2, bn2, _, conv3, bn3, _, _, lin = self.stem
        h1, w1, h2, w2, h3, w3 = self._dims
        flat = img.reshape(img.shape[0], -1)
        idx, idx_left, n1, n1_left, n3, n2, pix16 = self._patch_index(img.device)
        fused12 = (self.fused_bn and self.fused_conv2 and n1 == 9 * n2
                   and stem12_applicable(bn1, act, flat, conv1.weight, conv2.weight, n1))
        if rows is not None and not (fused12 or (self.fused_bn and stem1_applicable(bn1, act, flat, conv1.weight))):
            flat, rows = flat.index_select(0, rows), None
        B = flat.shape[0] if rows is None else rows.numel()
        w2m = conv2.weight.permute(0, 2, 3, 1).reshape(32, 144)  # conv2 on its 3x3 patches, columns (i, j, c)
        block2 = None
        w3m = conv3.weight.permute(0, 2, 3, 1).reshape(64, 128)  # conv3 on its 2x2 patches, columns (i, j, c)
        z3 = None
        if fused12:
            # conv1 + BN1 + act + conv2: the backward forms conv2's input gradient inside the first block's passes
            z2 = stem12_bn_act_conv(bn1, act, conv1.weight, w2m, flat, pix16, n1, n1_left, self._bn_uses,
                                    self.fused_conv2_forward, count_first=True, rows=rows)
            if self.fused_conv3 and n3 == n2 and bn_act_conv_applicable(bn2, act, z2, w3m):
                # block 2 straight into conv3: act(bn2(z2)) applied as conv3 loads its rows, never written
                z3 = bn_act_conv(bn2, act, z2, w3m, self._bn_uses, count_first=True)
            else:
                block2 = self._bn_act(bn2, act, z2)
        elif self.fused_bn and stem1_applicable(bn1, act, flat, conv1.weight):
            # conv1 + BN1 + act from the image itself: no patch matrix, no conv output (rsl_rl/fused_bn.py)
            y = stem1_bn_act(bn1, act, conv1.weight, flat, pix16, n1, n1_left, self._bn_uses, count_first=True,
                             rows=rows)
        else:
            x = flat.index_select(1, idx).view(B * n1, 9)
            if n1_left:
                x = torch.cat([x, flat.index_select(1, idx_left).view(B * n1_left, 9)])
            y = self._bn_act(bn1, act, _gemm(x, conv1.weight.reshape(16, 9)))
        if block2 is None and z3 is None:
            # conv2's 3x3 patches (i, j, c): a view (the fused block returns exactly these rows; a slice of the whole
            # tensor would still cost a zero-filled gradient plus a copy in the backward)
            x = (y if y.shape[0] == B * n1 else y[: B * n1]).view(B * n2, 144)
            block2 = self._bn_act(bn2, act, _gemm(x, w2m))
        if z3 is None:
            y = block2.view(B, n2, 32)
            x = (y if n3 == n2 else y[:, :n3]).reshape(B * h3 * w3, 128)  # conv3's 2x2 patches: a view at 72x96
            z3 = _gemm(x, w3m)
        if statistics_only:  # (record_batch_statistics: block 3's statistics are the last thing it needs)
            self._bn_statistics(bn3, z3)
            return None
        y = self._bn_act(bn3, act, z3).view(B, h3 * w3 * 64)
        # reference flatten is NCHW (c, h, w): permute the Linear's columns to (h, w, c) instead
        wl = lin.weight.view(-1, 64, h3, w3).permute(0, 2, 3, 1).reshape(lin.weight.shape[0], -1)
        return _gemm(y, wl, lin.bias if extra_bias is None else lin.bias + extra_bias)

    def features(self, observations: torch.Tensor) -> torch.Tensor:
        """act(stem(image) + state_enc(state)), vision_actor_critic.py:119-122."""
        img = observations[:, -self.num_pixels:].reshape(-1, 1, *self.img_res)
        state = observations[:, :-self.num_pixels]
        # the state encoder's GEMM takes the stem's output (with both biases) as its addend: no [B, 192] adds
        se = self.state_enc
        return self.activation(torch.addmm(self.stem_gemm(img, se.bias), state, se.weight.t()))

    def features_rows(self, observations: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
        """features(observations[rows]) without the gathered copy of the image rows: the state columns are gathered,
        the fused first block reads the images through `rows` (a PPO mini-batch straight from the rollout storage)."""
        state = observations[:, :-self.num_pixels].index_select(0, rows)
        img = observations[:, -self.num_pixels:]
        se = self.state_enc
        return self.activation(torch.addmm(self.stem_gemm(img, se.bias, rows=rows), state, se.weight.t()))

    def shared_features(self, observations: torch.Tensor, uses: int) -> torch.Tensor:
        """features(observations) evaluated once for `uses` consumers of the same rows (PPOL2C2's mixed batch feeds
        both the actor and the critic, ppo_l2c2.py:184-186, which the reference evaluates as two stem forwards):
        the same values, one backward through the stem for the summed feature gradient, and every BatchNorm's
        running statistics updated `uses` times, as `uses` training-mode forwards of these rows do."""
        self._bn_uses = int(uses)
        try:
            return self.features(observations)
        finally:
            self._bn_uses = 1

    def update_distribution(self, observations):
        mean = self.actor(self.features(observations))
        self.distribution = torch.distributions.Normal(mean, self._std(mean))

    # act: ActorCritic.act (the distribution's draw without torch.normal's per-call host read, the same bits)

    def act_inference(self, observations):
        """-> (mean, feature), as the reference (its exporters and PPOL2C2 take [0])."""
        feat = self.features(observations)
        return self.actor(feat), feat

    def evaluate(self, critic_observations, **kwargs):
        return self.critic(self.features(critic_observations))
