"""The build's VisionActorCritic on the GPU — the fused first block (gr_stem1_*), the fused BatchNorm +
activation ops (gr_bn_act_*), the patch GEMMs — against the reference module's outputs, BatchNorm running
statistics and gradients (tests/golden/make_golden_vision.py; vision_actor_critic.py:43-144)."""
import pytest

import vision_golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused_bn", [True, False])
def test_vision_actor_critic_matches_reference_module_gpu(fused_bn):
    got, f = vision_golden.build_and_run("cuda:0", fused_bn=fused_bn)
    worst = vision_golden.check(got, f)
    print(sorted(worst.items(), key=lambda kv: -kv[1])[:5])
