"""standalone/rsl_rl/train.py end to end on the HIP env (reference train.sh command line)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_train_cli_two_iterations(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "standalone", "rsl_rl"))
    import train

    runner = train.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-State-v0", "--num_envs", "1024", "--headless",
                         "--max_iterations", "2", "--log_root", str(tmp_path)])
    assert runner.last_log["fps"] > 0
    runs = list((tmp_path / "rsl_rl" / "racing_ppo").iterdir())
    assert len(runs) == 1 and (runs[0] / "params" / "env.yaml").exists()
    assert any(f.name.startswith("model_") for f in runs[0].iterdir())
    # resume from the latest checkpoint of the latest run
    r2 = train.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-State-v0", "--num_envs", "1024", "--max_iterations", "1",
                     "--log_root", str(tmp_path), "--resume", "1"])
    assert r2.current_learning_iteration >= 1


def test_train_cli_l2c2_recipe(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "standalone", "rsl_rl"))
    import train

    runner = train.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-State-v0", "--num_envs", "1024", "--headless",
                         "--max_iterations", "2", "--log_root", str(tmp_path),
                         "--agent", "rsl_rl_l2c2_cfg_entry_point"])
    assert type(runner.alg).__name__ == "PPOL2C2"
    assert runner.last_log["smooth_loss"] > 0.0
    assert (tmp_path / "rsl_rl" / "racing_ppo_l2c2").exists()


def test_play_exports_and_runs_the_checkpoint(tmp_path):
    """standalone/rsl_rl/play.py: latest checkpoint -> env + runner -> exported TorchScript -> play loop."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "standalone", "rsl_rl"))
    import play
    import train

    train.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-State-v0", "--num_envs", "512", "--max_iterations", "1",
                "--log_root", str(tmp_path)])
    out = play.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-State-v0", "--num_envs", "256", "--max_steps", "250",
                     "--log_root", str(tmp_path)])
    assert out["episodes"] > 0  # 250 steps > the 200-step episode limit
    m = torch.jit.load(out["exported"]["jit"])
    assert m(torch.zeros(3, 16)).shape == (3, 4)


def test_reference_command_line_trains_the_reference_recipe(tmp_path):
    """train.sh's own command line (`--task DiffLab-Quadcopter-CTBR-Racing-v0 --num_envs 1024 --headless`) gets the
    reference's pairing for that id (quadcopter_diff/__init__.py:50-63): depth camera + VisionActorCritic +
    PPOL2C2."""
    sys.path.insert(0, os.path.join(ROOT, "standalone", "rsl_rl"))
    import train

    runner = train.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-v0", "--num_envs", "1024", "--headless",
                         "--max_iterations", "1", "--log_root", str(tmp_path)])
    assert type(runner.alg).__name__ == "PPOL2C2" and type(runner.alg.policy).__name__ == "VisionActorCritic"
    assert runner.env.unwrapped.camera is not None
    assert runner.alg.storage.observations.shape[-1] == 16 + 72 * 96
    assert runner.last_log["fps"] > 0
    assert (tmp_path / "rsl_rl" / "racing_ppo_l2c2_vision").exists()


def test_vision_task_trains_and_plays(tmp_path):
    """The reference's registered recipe: depth camera + VisionActorCritic + PPOL2C2."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "standalone", "rsl_rl"))
    import play
    import train

    runner = train.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-Vision-v0", "--num_envs", "256",
                         "--max_iterations", "1", "--log_root", str(tmp_path)])
    assert type(runner.alg).__name__ == "PPOL2C2" and type(runner.alg.policy).__name__ == "VisionActorCritic"
    assert runner.alg.storage.observations.shape[-1] == 16 + 72 * 96
    out = play.main(["--task", "DiffLab-Quadcopter-CTBR-Racing-Vision-v0", "--num_envs", "64", "--max_steps", "30",
                     "--log_root", str(tmp_path), "--show_camera"])
    m = torch.jit.load(out["exported"]["jit"])
    assert m(torch.zeros(2, 16), torch.zeros(2, 1, 72, 96)).shape == (2, 4)
    cam_dir = os.path.join(os.path.dirname(out["checkpoint"]), "camera")
    assert len(os.listdir(cam_dir)) == 3
