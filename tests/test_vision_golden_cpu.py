"""The build's VisionActorCritic (torch path, CPU) against the reference module's own outputs, BatchNorm
running statistics and gradients (tests/golden/make_golden_vision.py; vision_actor_critic.py:43-144)."""
import vision_golden


def test_vision_actor_critic_matches_reference_module_cpu():
    got, f = vision_golden.build_and_run("cpu")
    worst = vision_golden.check(got, f)
    print(sorted(worst.items(), key=lambda kv: -kv[1])[:5])


def test_vision_fixture_inputs_reproduce_from_the_oracle():
    """The fixture's observation inputs are re-derived from the CPU oracle env (tests/oracle_vecenv.py, the same
    seeds as make_golden_vision.py) and must equal the stored rows bit for bit: a change of the oracle's draws
    (noise, resets, camera) then fails here instead of silently drifting the next regeneration's inputs."""
    import numpy as np

    f = vision_golden.load()
    pol, cri = vision_golden.observation_rows(f["obs_critic"].shape[0])
    assert np.array_equal(pol[:, :16].numpy(), f["obs_policy_state"].numpy())
    assert np.array_equal(cri.numpy(), f["obs_critic"].numpy())
