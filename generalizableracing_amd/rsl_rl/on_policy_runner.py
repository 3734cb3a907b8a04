"""OnPolicyRunner (standalone/rsl_rl/ext/runners/on_policy_runner.py:20-360).

Same constructor / learn / log / save / load / get_inference_policy surface
and the same `Perf/total_fps = num_steps_per_env * num_envs / (collection +
learn)` metric (:229).  Differences, all bookkeeping:
  * episode return / length statistics are accumulated on the device (the
    reference calls .cpu() every step, on_policy_runner.py:170-171); they
    are read once per iteration;
  * multi-GPU: rank 0 logs and saves; fps is whole-job (x world size);
  * TensorBoard is optional (not installed here): scalars go to a CSV
    writer when torch.utils.tensorboard is unavailable.
"""
from __future__ import annotations

import os
import time

import torch

from . import distributed as gdist
from .actor_critic import ActorCritic, EmpiricalNormalization
from .ppo import PPO
from .ppo_l2c2 import PPOL2C2
from .rollout_ops import EpisodeStats
from .vision_actor_critic import VisionActorCritic

ALGORITHMS = {"PPO": PPO, "PPOL2C2": PPOL2C2}
POLICIES = {"ActorCritic": ActorCritic, "VisionActorCritic": VisionActorCritic}


class _CsvWriter:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.f = open(os.path.join(log_dir, "scalars.csv"), "a", buffering=1)

    def add_scalar(self, key, value, step):
        self.f.write(f"{step},{key},{float(value)}\n")

    def close(self):
        self.f.close()


def _make_writer(log_dir, logger_type):
    if logger_type == "tensorboard":
        try:
            from torch.utils.tensorboard import SummaryWriter

            return SummaryWriter(log_dir=log_dir, flush_secs=10)
        except Exception:
            pass
    return _CsvWriter(log_dir)


# the reference's rewbuffer / lenbuffer deques and episode sums (on_policy_runner.py:128-173), on the device
_EpisodeStats = EpisodeStats


class OnPolicyRunner:
    """On-policy runner for training and evaluation."""

    def __init__(self, env, train_cfg: dict, log_dir=None, device="cpu"):
        self.cfg = train_cfg
        self.alg_cfg = dict(train_cfg["algorithm"])
        self.policy_cfg = dict(train_cfg["policy"])
        self.device = device
        self.env = env
        if self.alg_cfg["class_name"] not in ALGORITHMS:  # on_policy_runner.py:31-36
            raise ValueError(f"Training type not found for algorithm {self.alg_cfg['class_name']}.")
        self.training_type = "rl"
        obs, extras = self.env.get_observations()
        num_obs = obs.shape[1]
        self.privileged_obs_type = "critic" if "critic" in extras["observations"] else None
        num_privileged_obs = (extras["observations"][self.privileged_obs_type].shape[1]
                              if self.privileged_obs_type is not None else num_obs)
        policy_class = POLICIES[self.policy_cfg.pop("class_name")]
        policy = policy_class(num_obs, num_privileged_obs, self.env.num_actions, **self.policy_cfg).to(self.device)
        alg_class = ALGORITHMS[self.alg_cfg.pop("class_name")]
        want_sink = bool(self.alg_cfg.pop("obs_sink", True))
        self.alg = alg_class(policy, env=self.env, device=self.device, **self.alg_cfg)
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]
        self.empirical_normalization = self.cfg["empirical_normalization"]
        if self.empirical_normalization:
            self.obs_normalizer = EmpiricalNormalization(shape=[num_obs], until=1.0e8).to(self.device)
            self.privileged_obs_normalizer = EmpiricalNormalization(shape=[num_privileged_obs], until=1.0e8).to(self.device)
        else:
            self.obs_normalizer = torch.nn.Identity().to(self.device)
            self.privileged_obs_normalizer = torch.nn.Identity().to(self.device)
        self.alg.init_storage(self.training_type, self.env.num_envs, self.num_steps_per_env, [num_obs],
                              [num_privileged_obs], [self.env.num_actions])
        self.obs_sink = want_sink and self._sink_supported(obs, extras)
        if self.obs_sink:
            self.alg.storage.enable_obs_sink()
        self.log_dir = log_dir
        self.writer = None
        self.logger_type = self.cfg.get("logger", "tensorboard")
        self.tot_timesteps = 0
        self.tot_time = 0.0
        self.current_learning_iteration = 0
        self.is_main = gdist.rank() == 0
        self.last_log: dict = {}

    def _sink_supported(self, obs, extras) -> bool:
        """The observation sink (RacingEnv.set_obs_sink: the step kernel, or on the camera task the camera kernel,
        writes each transition's observations into the rollout storage slot) applies when the stored rows are
        exactly the env's rows: PPO or PPOL2C2 (whose successor pairs read the same slots), no empirical
        normalisation, separate critic rows, the env on the training device; the camera task's rows with fp32
        storage only."""
        if not isinstance(self.alg, PPO) or self.empirical_normalization or not hasattr(self.env, "set_obs_sink"):
            return False
        st = self.alg.storage
        if st.privileged_observations is None or self.privileged_obs_type is None:
            return False
        unwrapped = getattr(self.env, "unwrapped", self.env)
        if torch.device(self.env.device) != torch.device(self.device):
            return False
        if getattr(unwrapped, "camera", None) is not None and st.observations.dtype != torch.float32:
            return False
        width = getattr(unwrapped, "num_obs", 16)
        crit = extras["observations"][self.privileged_obs_type]
        return obs.dim() == 2 and obs.shape[1] == width and crit.dim() == 2 and crit.shape[1] == width

    def learn(self, num_learning_iterations: int, init_at_random_ep_len: bool = False):
        if self.log_dir is not None and self.writer is None and self.is_main:
            self.writer = _make_writer(self.log_dir, str(self.logger_type).lower())
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        obs, extras = self.env.get_observations()
        privileged_obs = extras["observations"].get(self.privileged_obs_type, obs)
        obs, privileged_obs = obs.to(self.device), privileged_obs.to(self.device)
        storage = self.alg.storage
        if self.obs_sink:
            storage.discard_sink()  # fresh observations: slot 0 is copied from them
        self.train_mode()
        ep_infos = []
        stats = EpisodeStats(self.env.num_envs, self.device, steps=self.num_steps_per_env)
        start_iter = self.current_learning_iteration
        tot_iter = start_iter + num_learning_iterations
        for it in range(start_iter, tot_iter):
            start = time.time()
            with torch.inference_mode():
                for _ in range(self.num_steps_per_env):
                    actions = self.alg.act(obs, privileged_obs)
                    if self.obs_sink:  # this step's observations land in the next transition's slot
                        self.env.set_obs_sink(*storage.sink_slot(storage.step + 1))
                    obs, rewards, dones, infos = self.env.step(actions.to(self.env.device))
                    obs, rewards, dones = obs.to(self.device), rewards.to(self.device), dones.to(self.device)
                    obs = self.obs_normalizer(obs)
                    if self.privileged_obs_type is not None:
                        privileged_obs = self.privileged_obs_normalizer(
                            infos["observations"][self.privileged_obs_type]).to(self.device)
                    else:
                        privileged_obs = obs
                    self.alg.process_env_step(rewards, dones, infos)
                    if self.log_dir is not None:
                        if "episode" in infos:
                            ep_infos.append(infos["episode"])
                        elif "log" in infos:
                            ep_infos.append(infos["log"])
                    stats.update(rewards, dones)
                if self.obs_sink:
                    self.env.set_obs_sink(None)
                if hasattr(self.env, "check_device_status"):
                    self.env.check_device_status()  # a kernel-flagged step fails the iteration loudly
                if torch.cuda.is_available() and str(self.device).startswith("cuda"):
                    torch.cuda.synchronize(self.device)
                stop = time.time()
                collection_time = stop - start
                start = stop
                self.alg.compute_returns(privileged_obs)
            loss_dict = self.alg.update()
            if torch.cuda.is_available() and str(self.device).startswith("cuda"):
                torch.cuda.synchronize(self.device)
            stop = time.time()
            learn_time = stop - start
            self.current_learning_iteration = it
            self.log(locals())
            if self.log_dir is not None and self.is_main and it % self.save_interval == 0:
                self.save(os.path.join(self.log_dir, f"model_{it}.pt"))
            ep_infos.clear()
        if self.log_dir is not None and self.is_main:
            self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))

    def log(self, locs: dict, width: int = 80, pad: int = 35):
        ws = gdist.world_size()
        steps = self.num_steps_per_env * self.env.num_envs * ws
        self.tot_timesteps += steps
        iteration_time = locs["collection_time"] + locs["learn_time"]
        self.tot_time += iteration_time
        fps = int(steps / iteration_time)
        means = locs["stats"].means()
        ep_vals = {}
        for key in (locs["ep_infos"][0] if locs["ep_infos"] else []):
            vals = []
            for ep_info in locs["ep_infos"]:
                if key not in ep_info:
                    continue
                v = ep_info[key]
                v = v if isinstance(v, torch.Tensor) else torch.tensor([float(v)])
                vals.append(v.reshape(-1).to(self.device))
            ep_vals[key] = float(torch.cat(vals).float().mean())
        with torch.no_grad():
            mean_std = float(self.alg.policy._std(torch.zeros(1, self.env.num_actions, device=self.device)).mean())
        self.last_log = {"fps": fps, "collection_time": locs["collection_time"], "learn_time": locs["learn_time"],
                         "mean_reward": means[0] if means else None, "mean_episode_length": means[1] if means else None,
                         "learning_rate": self.alg.learning_rate, **locs["loss_dict"], **ep_vals}
        if not self.is_main:
            return
        it = locs["it"]
        if self.writer is not None:
            for k, v in ep_vals.items():
                self.writer.add_scalar(k if "/" in k else "Episode/" + k, v, it)
            for k, v in locs["loss_dict"].items():
                self.writer.add_scalar(f"Loss/{k}", v, it)
            self.writer.add_scalar("Loss/learning_rate", self.alg.learning_rate, it)
            self.writer.add_scalar("Policy/mean_noise_std", mean_std, it)
            self.writer.add_scalar("Perf/total_fps", fps, it)
            self.writer.add_scalar("Perf/collection time", locs["collection_time"], it)
            self.writer.add_scalar("Perf/learning_time", locs["learn_time"], it)
            if means:
                self.writer.add_scalar("Train/mean_reward", means[0], it)
                self.writer.add_scalar("Train/mean_episode_length", means[1], it)
        if self.log_dir is None:
            return
        title = f" \033[1m Learning iteration {it}/{locs['tot_iter']} \033[0m "
        s = f"{'#' * width}\n{title.center(width, ' ')}\n\n"
        s += (f"{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, "
              f"learning {locs['learn_time']:.3f}s)\n")
        s += f"{'Mean action noise std:':>{pad}} {mean_std:.2f}\n"
        if means:
            s += f"{'Mean reward:':>{pad}} {means[0]:.2f}\n{'Mean episode length:':>{pad}} {means[1]:.2f}\n"
        for k, v in locs["loss_dict"].items():
            s += f"{f'Mean {k} loss:':>{pad}} {v:.4f}\n"
        for k, v in ep_vals.items():
            s += f"{(k + ':') if '/' in k else f'Mean episode {k}:':>{pad}} {v:.4f}\n"
        s += (f"{'-' * width}\n{'Total timesteps:':>{pad}} {self.tot_timesteps}\n"
              f"{'Iteration time:':>{pad}} {iteration_time:.2f}s\n{'Total time:':>{pad}} {self.tot_time:.2f}s\n")
        print(s, flush=True)

    def save(self, path, infos=None):
        saved = {"model_state_dict": self.alg.policy.state_dict(),
                 "optimizer_state_dict": self.alg.optimizer.state_dict(),
                 "iter": self.current_learning_iteration, "infos": infos}
        if self.empirical_normalization:
            saved["obs_norm_state_dict"] = self.obs_normalizer.state_dict()
            saved["privileged_obs_norm_state_dict"] = self.privileged_obs_normalizer.state_dict()
        torch.save(saved, path)

    def load(self, path, load_optimizer=True):
        loaded = torch.load(path, weights_only=True, map_location=self.device)
        resumed = self.alg.policy.load_state_dict(loaded["model_state_dict"])
        if self.empirical_normalization and resumed:
            self.obs_normalizer.load_state_dict(loaded["obs_norm_state_dict"])
            self.privileged_obs_normalizer.load_state_dict(loaded["privileged_obs_norm_state_dict"])
        if load_optimizer and resumed:
            self.alg.optimizer.load_state_dict(loaded["optimizer_state_dict"])
            for g in self.alg.optimizer.param_groups:  # a graph-captured update saves its rate as a tensor
                if torch.is_tensor(g["lr"]):
                    g["lr"] = float(g["lr"])
        if resumed:
            self.current_learning_iteration = loaded["iter"]
        return loaded["infos"]

    def get_inference_policy(self, device=None):
        self.eval_mode()
        if device is not None:
            self.alg.policy.to(device)
        policy = self.alg.policy.act_inference
        if self.cfg["empirical_normalization"]:
            if device is not None:
                self.obs_normalizer.to(device)
            return lambda x: self.alg.policy.act_inference(self.obs_normalizer(x))  # noqa: E731
        return policy

    def train_mode(self):
        self.alg.policy.train()
        if self.empirical_normalization:
            self.obs_normalizer.train()
            self.privileged_obs_normalizer.train()

    def eval_mode(self):
        self.alg.policy.eval()
        if self.empirical_normalization:
            self.obs_normalizer.eval()
            self.privileged_obs_normalizer.eval()

    def add_git_repo_to_log(self, repo_file_path):
        pass
