"""Policy exporters for deployment (reference: standalone/rsl_rl/ext/utils/exporter.py:19-140, and
Isaac Lab's export_policy_as_jit / export_policy_as_onnx used by standalone/rsl_rl/play.py:100-118).

* `export_policy_as_jit`: TorchScript of normalizer + actor MLP, input the 16-dim state obs.
* `export_vision_policy_as_jit`: TorchScript of the vision policy with the reference exporter's
  two-input signature forward(state [B,16], depth_image [B,1,72,96]) -> actions
  (+ sigmoid(aux) when the auxiliary head is exported).
* `export_vision_policy_as_onnx` / `export_policy_as_onnx`: the same modules through
  `torch.onnx.export` (opset 11, input/output names as the reference).  torch's exporter needs the
  `onnx` package; it is not installed in this image, so these raise a clear error here and work
  wherever `onnx` is importable.
"""
from __future__ import annotations

import copy
import os

import torch
import torch.nn as nn


class _PolicyExporter(nn.Module):
    def __init__(self, policy, normalizer=None):
        super().__init__()
        self.actor = copy.deepcopy(policy.actor).cpu()
        self.normalizer = copy.deepcopy(normalizer).cpu() if normalizer is not None else nn.Identity()

    def forward(self, x):
        return self.actor(self.normalizer(x))


class _VisionPolicyExporter(nn.Module):
    """exporter.py:34-98 (non-recurrent branch)."""

    def __init__(self, policy, normalizer=None, use_auxiliary_head: bool = False):
        super().__init__()
        self.stem = copy.deepcopy(policy.stem).cpu()
        self.state_enc = copy.deepcopy(policy.state_enc).cpu()
        self.activation = copy.deepcopy(policy.activation).cpu()
        self.actor = copy.deepcopy(policy.actor).cpu()
        self.use_aux = bool(use_auxiliary_head)
        self.auxiliary_head = copy.deepcopy(policy.aux_decoder).cpu() if use_auxiliary_head else nn.Identity()
        self.normalizer = copy.deepcopy(normalizer).cpu() if normalizer is not None else nn.Identity()

    def forward(self, state: torch.Tensor, depth_image: torch.Tensor):
        img_h, img_w = depth_image.shape[2], depth_image.shape[3]
        x_in = self.normalizer(torch.cat([state, depth_image.reshape(depth_image.shape[0], -1)], dim=1))
        img = x_in[:, x_in.shape[1] - img_h * img_w:].reshape(-1, 1, img_h, img_w)
        st = x_in[:, : x_in.shape[1] - img_h * img_w]
        feat = self.activation(self.stem(img) + self.state_enc(st))
        return self.actor(feat)

    def forward_with_aux(self, state: torch.Tensor, depth_image: torch.Tensor):
        img_h, img_w = depth_image.shape[2], depth_image.shape[3]
        x_in = self.normalizer(torch.cat([state, depth_image.reshape(depth_image.shape[0], -1)], dim=1))
        img = x_in[:, x_in.shape[1] - img_h * img_w:].reshape(-1, 1, img_h, img_w)
        st = x_in[:, : x_in.shape[1] - img_h * img_w]
        feat = self.activation(self.stem(img) + self.state_enc(st))
        return self.actor(feat), torch.sigmoid(self.auxiliary_head(feat))


class _VisionAuxWrapper(nn.Module):
    def __init__(self, inner: _VisionPolicyExporter):
        super().__init__()
        self.inner = inner

    def forward(self, state: torch.Tensor, depth_image: torch.Tensor):
        return self.inner.forward_with_aux(state, depth_image)


def _normalizer(n):
    return None if n is None or isinstance(n, nn.Identity) else n


def export_policy_as_jit(policy, normalizer, path: str, filename: str = "policy.pt") -> str:
    os.makedirs(path, exist_ok=True)
    m = _PolicyExporter(policy, _normalizer(normalizer)).eval()
    out = os.path.join(path, filename)
    torch.jit.script(m).save(out)
    return out


def export_vision_policy_as_jit(policy, path: str, normalizer=None, filename: str = "vision_policy.pt",
                                use_auxiliary_head: bool = False) -> str:
    os.makedirs(path, exist_ok=True)
    m = _VisionPolicyExporter(policy, _normalizer(normalizer), use_auxiliary_head).eval()
    mod = _VisionAuxWrapper(m).eval() if use_auxiliary_head else m
    out = os.path.join(path, filename)
    torch.jit.script(mod).save(out)
    return out


def _onnx_export(module, args, out, input_names, output_names, verbose):
    try:
        import onnx  # noqa: F401
    except ImportError as e:
        raise RuntimeError("ONNX export needs the `onnx` package, which is not installed in this environment; "
                           "use export_*_as_jit here, or run the export where onnx is available") from e
    torch.onnx.export(module, args, out, export_params=True, opset_version=11, verbose=verbose,
                      input_names=input_names, output_names=output_names, dynamic_axes={}, dynamo=False)
    return out


def export_policy_as_onnx(policy, path: str, normalizer=None, filename: str = "policy.onnx", verbose=False) -> str:
    os.makedirs(path, exist_ok=True)
    m = _PolicyExporter(policy, _normalizer(normalizer)).eval()
    x = torch.zeros(1, m.actor[0].in_features)
    return _onnx_export(m, (x,), os.path.join(path, filename), ["obs"], ["actions"], verbose)


def export_vision_policy_as_onnx(policy, path: str, normalizer=None, filename: str = "vision_policy.onnx",
                                 verbose=False, image_shape=(72, 96), state_shape=(24,),
                                 use_auxiliary_head: bool = False) -> str:
    """exporter.py:19-32 signature."""
    os.makedirs(path, exist_ok=True)
    m = _VisionPolicyExporter(policy, _normalizer(normalizer), use_auxiliary_head).eval()
    img = torch.zeros(1, 1, *image_shape)
    state = torch.zeros(1, *state_shape)
    if use_auxiliary_head:
        return _onnx_export(_VisionAuxWrapper(m).eval(), (state, img), os.path.join(path, filename),
                            ["state", "img"], ["actions", "auxiliary"], verbose)
    return _onnx_export(m, (state, img), os.path.join(path, filename), ["state", "img"], ["actions"], verbose)
