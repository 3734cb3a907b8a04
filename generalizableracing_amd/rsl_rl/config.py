"""Runner configuration (rsl_rl_ppo_cfg.py:15-41, QuadcopterPPORunnerCfg) as plain dataclasses.

`to_dict()` produces the dict layout Isaac Lab's RslRlOnPolicyRunnerCfg.to_dict()
hands to OnPolicyRunner (keys "policy", "algorithm", "num_steps_per_env", …).
Hidden dims are 256x256 (BASELINE.json); the reference's state-only cfg uses 128x128.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field


@dataclass
class RslRlPpoActorCriticCfg:
    class_name: str = "ActorCritic"
    init_noise_std: float = 1.0
    noise_std_type: str = "scalar"
    actor_hidden_dims: list = field(default_factory=lambda: [256, 256])
    critic_hidden_dims: list = field(default_factory=lambda: [256, 256])
    activation: str = "lrelu"


@dataclass
class RslRlPpoAlgorithmCfg:
    class_name: str = "PPO"
    value_loss_coef: float = 1.0
    use_clipped_value_loss: bool = True
    clip_param: float = 0.2
    entropy_coef: float = 0.0
    num_learning_epochs: int = 5
    num_mini_batches: int = 4
    learning_rate: float = 5.0e-4
    schedule: str = "adaptive"
    gamma: float = 0.99
    lam: float = 0.95
    desired_kl: float = 0.01
    max_grad_norm: float = 1.0
    # not in the reference: rollout inference (act / evaluate / log prob) as one bf16 MFMA launch
    # (rsl_rl/fused_inference.py); the update stays fp32.  MLP ActorCritic with 128 / 256 hidden units only.
    fused_rollout_inference: bool = False
    # precision of that launch: "bf16" (bf16 operands, BASELINE C5) or "fp32" (fp32 operands on fp32 MFMA, the
    # reference's arithmetic: the stored old mean / log prob then match the update's fp32 recompute)
    fused_rollout_precision: str = "bf16"
    # not in the reference: dtype of the rollout storage's observation buffers ("bfloat16" halves them;
    # mini-batches are cast back to fp32 for the update)
    storage_obs_dtype: str = "float32"
    # not in the reference: the update's mini-batch step captured once in a hipGraph and replayed (ppo.py
    # _GraphedStep; single rank; PPO only)
    graph_update: bool = False
    # not in the reference: the update's forward/backward under torch.autocast(bfloat16) (ppo.py)
    update_autocast_bf16: bool = False
    # not in the reference: the env writes each transition's observations straight into the rollout storage
    # slot (RacingEnv.set_obs_sink; PPO or PPOL2C2, state rows or fp32 camera rows, no empirical normalisation)
    # instead of add_transitions copying them — with storage_obs_dtype "bfloat16" (state rows) the kernel rounds
    # them to bf16 itself
    obs_sink: bool = True
    # not in the reference: the update's mini-batch losses (log prob, KL, clipped surrogate and value loss) as one
    # HIP op each way (rsl_rl/fused_loss.py); False keeps the torch ops
    fused_losses: bool = True
    # not in the reference: the grad-norm clip and Adam as four HIP launches over the parameter table
    # (rsl_rl/flat_adam.py); False keeps torch.optim.Adam + nn.utils.clip_grad_norm_
    fused_adam: bool = True
    # not in the reference: with fused_losses, the actor and critic MLPs of the update as whole-network fp32-MFMA
    # kernels, one launch per direction for both networks (gr_mlp_forward / gr_mlp_backward, csrc/gr_mlp.hip);
    # False keeps the per-layer path (fused first layer and head around hipBLASLt GEMMs, rsl_rl/linear.py MLP)
    fused_mlp: bool = True


@dataclass
class QuadcopterPPORunnerCfg:
    seed: int = 42
    device: str = "cuda:0"
    num_steps_per_env: int = 24
    max_iterations: int = 5000
    empirical_normalization: bool = False
    policy: RslRlPpoActorCriticCfg = field(default_factory=RslRlPpoActorCriticCfg)
    algorithm: RslRlPpoAlgorithmCfg = field(default_factory=RslRlPpoAlgorithmCfg)
    save_interval: int = 500
    experiment_name: str = "racing_ppo"
    run_name: str = ""
    logger: str = "tensorboard"
    resume: bool = False
    load_run: str = ".*"
    load_checkpoint: str = "model_.*.pt"

    def to_dict(self) -> dict:
        return asdict(self)


@dataclass
class QuadcopterL2C2PPORunnerCfg(QuadcopterPPORunnerCfg):
    """The reference's racing recipe algorithm (rsl_rl_ppo_cfg.py:80-104: class_name "PPOL2C2",
    entropy 0.005, 4000 iterations) on the state-only MLP policy.  The L2C2 knobs keep the
    PPOL2C2 constructor defaults (ppo_l2c2.py:26-28)."""

    max_iterations: int = 4000
    experiment_name: str = "racing_ppo_l2c2"
    algorithm: RslRlPpoAlgorithmCfg = field(
        default_factory=lambda: RslRlPpoAlgorithmCfg(class_name="PPOL2C2", entropy_coef=0.005))


@dataclass
class RslRlPpoVisionActorCriticCfg(RslRlPpoActorCriticCfg):
    """rsl_rl_ppo_cfg.py:43-52."""

    class_name: str = "VisionActorCritic"
    img_res: tuple = (72, 96)
    dim_hidden_input: int = 192
    actor_hidden_dims: list = field(default_factory=lambda: [128, 128])
    critic_hidden_dims: list = field(default_factory=lambda: [128, 128])
    use_auxiliary_loss: bool = True  # policy.__setattr__("use_auxiliary_loss", True), :104


@dataclass
class QuadcopterVisionPPORunnerCfg(QuadcopterPPORunnerCfg):
    """The reference's registered racing recipe (rsl_rl_ppo_cfg.py:80-104): VisionActorCritic + PPOL2C2."""

    max_iterations: int = 4000
    experiment_name: str = "racing_ppo_l2c2_vision"
    policy: RslRlPpoActorCriticCfg = field(default_factory=RslRlPpoVisionActorCriticCfg)
    algorithm: RslRlPpoAlgorithmCfg = field(
        default_factory=lambda: RslRlPpoAlgorithmCfg(class_name="PPOL2C2", entropy_coef=0.005))
