"""The build's PPO (TallLinear split-K weight gradients at 24 576-row mini-batches) against the reference's PPO
over plain nn.Linear layers at BASELINE C2 size, on the CPU (tests/ppo_c2_golden.py has the pins and their
tolerances; the GPU device path is tests/test_gpu_ppo_c2_golden.py)."""
import ppo_c2_golden as pc2


def test_ppo_c2_update_matches_reference_cpu():
    rep = pc2.replay(pc2.load(), "cpu")
    assert rep[0]["grad_err"] < 1e-5
