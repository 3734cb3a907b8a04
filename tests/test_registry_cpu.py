"""Task ids resolve to the reference's pairings (extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/
__init__.py:50-63): `DiffLab-Quadcopter-CTBR-Racing-v0` is the depth-camera racing env with
QuadcopterVisionPPORunnerCfg (VisionActorCritic + PPOL2C2, rsl_rl_ppo_cfg.py:80-104), so train.sh trains the
reference's recipe; the state-only MLP task of the BASELINE configs has an id of its own."""
import importlib

registry = importlib.import_module("generalizableracing_amd.registry")


def test_reference_id_is_the_vision_recipe():
    env_cfg = registry.load_cfg_from_registry("DiffLab-Quadcopter-CTBR-Racing-v0", "env_cfg_entry_point")
    agent = registry.load_cfg_from_registry("DiffLab-Quadcopter-CTBR-Racing-v0", "rsl_rl_cfg_entry_point")
    assert env_cfg.camera is not None
    assert (env_cfg.camera.height, env_cfg.camera.width) == (72, 96)
    d = agent.to_dict()
    assert d["policy"]["class_name"] == "VisionActorCritic"
    assert d["algorithm"]["class_name"] == "PPOL2C2"
    assert d["algorithm"]["entropy_coef"] == 0.005


def test_state_id_is_the_mlp_recipe():
    env_cfg = registry.load_cfg_from_registry("DiffLab-Quadcopter-CTBR-Racing-State-v0", "env_cfg_entry_point")
    agent = registry.load_cfg_from_registry("DiffLab-Quadcopter-CTBR-Racing-State-v0", "rsl_rl_cfg_entry_point")
    assert env_cfg.camera is None
    d = agent.to_dict()
    assert d["policy"]["class_name"] == "ActorCritic" and d["algorithm"]["class_name"] == "PPO"
    assert list(d["policy"]["actor_hidden_dims"]) == [256, 256]
    l2c2 = registry.load_cfg_from_registry("DiffLab-Quadcopter-CTBR-Racing-State-v0", "rsl_rl_l2c2_cfg_entry_point")
    assert l2c2.to_dict()["algorithm"]["class_name"] == "PPOL2C2"


def test_vision_alias_matches_the_reference_id():
    a = registry.registry()["DiffLab-Quadcopter-CTBR-Racing-v0"]
    b = registry.registry()["DiffLab-Quadcopter-CTBR-Racing-Vision-v0"]
    assert a == b
