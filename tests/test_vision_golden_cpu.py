"""The build's VisionActorCritic (torch path, CPU) against the reference module's own outputs, BatchNorm
running statistics and gradients (tests/golden/make_golden_vision.py; vision_actor_critic.py:43-144)."""
import vision_golden


def test_vision_actor_critic_matches_reference_module_cpu():
    got, f = vision_golden.build_and_run("cpu")
    worst = vision_golden.check(got, f)
    print(sorted(worst.items(), key=lambda kv: -kv[1])[:5])
