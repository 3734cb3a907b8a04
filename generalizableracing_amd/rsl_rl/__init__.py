"""rsl_rl surface (runner / PPO / storage / ActorCritic) in PyTorch-ROCm, mirroring
standalone/rsl_rl/ext of the reference, with RCCL data parallelism."""
from .actor_critic import ActorCritic, EmpiricalNormalization  # noqa: F401
from .config import QuadcopterL2C2PPORunnerCfg, QuadcopterPPORunnerCfg, QuadcopterVisionPPORunnerCfg, RslRlPpoActorCriticCfg, RslRlPpoAlgorithmCfg  # noqa: F401
from .on_policy_runner import OnPolicyRunner  # noqa: F401
from .ppo import PPO  # noqa: F401
from .rollout_storage import RolloutStorage  # noqa: F401
from .ppo_l2c2 import PPOL2C2  # noqa: F401
from .rollout_storage_l2c2 import RolloutStorageL2C2  # noqa: F401
from .vision_actor_critic import VisionActorCritic  # noqa: F401
