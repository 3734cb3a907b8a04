"""Policy exporters (standalone/rsl_rl/ext/utils/exporter.py:19-140; Isaac Lab export_policy_as_jit):
the TorchScript files reproduce the live policy's inference output."""
import pytest
import torch

from generalizableracing_amd.rsl_rl import ActorCritic, EmpiricalNormalization, VisionActorCritic
from generalizableracing_amd.rsl_rl import exporter


def test_state_policy_jit_round_trip(tmp_path):
    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [32, 32], [32, 32], "lrelu").eval()
    norm = EmpiricalNormalization([16])
    norm.train()
    norm(torch.randn(100, 16) * 3 + 1)
    norm.eval()
    path = exporter.export_policy_as_jit(pol, norm, str(tmp_path), "policy.pt")
    m = torch.jit.load(path)
    x = torch.randn(7, 16)
    torch.testing.assert_close(m(x), pol.act_inference(norm(x)))


def test_vision_policy_jit_two_inputs_and_aux(tmp_path):
    torch.manual_seed(1)
    pol = VisionActorCritic(16 + 72 * 96, 16 + 72 * 96, 4, img_res=(72, 96), dim_hidden_input=192,
                            actor_hidden_dims=[128, 128], critic_hidden_dims=[128, 128], activation="lrelu",
                            use_auxiliary_loss=True)
    pol.train()
    pol.act(torch.rand(32, 16 + 72 * 96))  # move the BatchNorm running statistics off their init
    pol.eval()
    state, img = torch.randn(3, 16), torch.rand(3, 1, 72, 96)
    obs = torch.cat([state, img.view(3, -1)], 1)
    mean, feat = pol.act_inference(obs)
    m = torch.jit.load(exporter.export_vision_policy_as_jit(pol, str(tmp_path), None, "v.pt"))
    torch.testing.assert_close(m(state, img), mean, rtol=1e-5, atol=1e-5)
    ma = torch.jit.load(exporter.export_vision_policy_as_jit(pol, str(tmp_path), None, "va.pt", use_auxiliary_head=True))
    act, aux = ma(state, img)
    torch.testing.assert_close(act, mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(aux, torch.sigmoid(pol.aux_decoder(feat)), rtol=1e-5, atol=1e-5)


def test_onnx_export_needs_the_onnx_package(tmp_path):
    try:
        import onnx  # noqa: F401
        pytest.skip("onnx is installed here")
    except ImportError:
        pass
    pol = ActorCritic(16, 16, 4, [8], [8], "lrelu")
    with pytest.raises(RuntimeError, match="onnx"):
        exporter.export_policy_as_onnx(pol, str(tmp_path))
