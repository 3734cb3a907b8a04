"""The racing env on the device: Python surface over libgr.so.

`RacingEnv` mirrors `ManagerBasedDiffRLEnv` (extensions/diff.lab/diff/lab/envs/
manager_based_diff_rl_env.py): `step(action) -> (obs_dict, reward, terminated,
time_outs, extras)`, `reset()`, `episode_length_buf`, `max_episode_length`, …
`RslRlVecEnvWrapper` mirrors Isaac Lab's rsl_rl wrapper, the VecEnv the
runner drives (standalone/rsl_rl/ext/runners/on_policy_runner.py:38,119-143).

Every step is ONE fused HIP launch (+ a one-workgroup log finalize) on the
current torch stream, with no host synchronisation.  Output tensors alternate
between two buffer sets (ping-pong) because rsl_rl keeps step t's `obs`
while step t+1 runs; a tensor returned by step t stays valid until step t+2.
`extras["log"]` entries come from a ring of 64 steps (the runner reads them at
the end of its 24-step rollout).
"""
from __future__ import annotations

import ctypes as C
import time
from collections.abc import Mapping
from concurrent.futures import ThreadPoolExecutor

import torch

from .. import _abi
from .racing_cfg import RacingEnvCfg
from .tracks import build_tracks

LOG_RING = 64
# diagnostics (scripts/prof_regen.py): a list to append (label, time.perf_counter()) stamps to inside
# regenerate_terrain; None = off
REGEN_STAMPS = None


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)  # (torch's own raw-stream accessor)


def _stamp(label):
    if REGEN_STAMPS is not None:
        REGEN_STAMPS.append((label, time.perf_counter()))


_EMPTY_MEAN_SLOTS = [_abi.LOG_EPSUM0 + j for j in range(7)] + [_abi.LOG_ACC, _abi.LOG_M_ACTRATE, _abi.LOG_M_LINSPD,
                                                               _abi.LOG_M_ANGSPD]
_EMPTY_COUNT_SLOTS = [_abi.LOG_T_TIMEOUT, _abi.LOG_T_CONTACT, _abi.LOG_T_BADPOSE]


class _EpisodeLog(Mapping):
    """extras["log"] of one call: the kernel leaves per-wave partial sums in a
    ring slot; the means Isaac Lab's managers log are formed on first access
    (gr_log_finalize, one small launch, no host sync).  Valid for LOG_RING calls."""

    __slots__ = ("_env", "_k", "_vals", "_keys", "_empty_reset")

    def __init__(self, env: "RacingEnv", k: int, keys: dict):
        self._env = env
        self._k = k
        self._vals = None
        self._keys = keys
        self._empty_reset = False  # reset(env_ids=[]): _reset_idx over an empty set

    def values(self) -> torch.Tensor:  # type: ignore[override]
        if self._vals is None:
            env = self._env
            if env._calls - self._k > LOG_RING:
                raise RuntimeError("extras['log'] read more than LOG_RING calls after its step")
            chain = [self]
            prev = env._log_at(self._k - 1)
            while prev is not None and prev._vals is None and len(chain) < LOG_RING:
                chain.append(prev)
                prev = env._log_at(prev._k - 1)
            for lg in reversed(chain):
                out = torch.empty(_abi.LOG_SLOTS, dtype=torch.float32, device=env.device)
                pv = prev._vals.data_ptr() if prev is not None and prev._vals is not None else None
                env._call("gr_log_finalize", env._log_slab[lg._k % LOG_RING].data_ptr(), pv, out.data_ptr(),
                          env._stream())
                if lg._empty_reset:
                    # the reference's _reset_idx over no envs (manager_based_diff_rl_env.py:362-407): the means
                    # over the reset envs are torch.mean of an empty set (NaN), the termination counts 0
                    out[_EMPTY_MEAN_SLOTS] = float("nan")
                    out[_EMPTY_COUNT_SLOTS] = 0.0
                lg._vals = out
                prev = lg
        return self._vals

    def __getitem__(self, k):
        return self.values()[self._keys[k]]

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)


class RacingEnv:
    """Vectorised drone-racing env (one shard of envs on one GPU)."""

    metadata = {"render_modes": [None]}

    def __init__(self, cfg: RacingEnvCfg, render_mode=None, **kwargs):
        self.cfg = cfg
        self.render_mode = render_mode
        self.device = torch.device(cfg.sim.device)
        if self.device.type != "cuda":
            raise RuntimeError(
                "RacingEnv runs on an MI355X (torch 'cuda' device on ROCm); got device "
                f"{self.device}.  The env step is HIP-only, there is no CPU path."
            )
        if not torch.cuda.is_available():
            raise RuntimeError("RacingEnv needs a GPU: torch.cuda.is_available() is False")
        self._lib = _abi.load()
        self._gcfg = cfg.to_gr_config()
        self.num_envs = int(cfg.scene.num_envs)
        self.num_actions = 4
        self.step_dt = cfg.step_dt
        self.physics_dt = cfg.sim.dt
        self.common_step_counter = 0
        dev = self.device

        ctx = C.c_void_p()
        _abi.check(self._lib, None, self._lib.gr_create(C.byref(self._gcfg), C.byref(ctx)), "gr_create")
        self._ctx = ctx

        # ---- track table + obstacles (host-generated, then device-resident) ----
        self.terrain_generation = 0
        interval = cfg.terrain.regen_interval_s
        self._regen_steps = None if interval is None else max(1, int(round(interval / self.step_dt)))
        # periodic regeneration: the context owns the terrain arrays (gr_terrain_reserve); the next generation is
        # built on a background host thread from half-way through the interval and uploaded into the context's
        # staging arrays on a side stream (gr_terrain_stage), so the interval step only commits it on the stream
        # (gr_terrain_commit: fixed arguments, graph-capturable)
        self._resident = False
        self._captured_epoch = None  # terrain epoch of the last call captured into a graph (_call)
        self._builder = ThreadPoolExecutor(max_workers=1, thread_name_prefix="gr-terrain") \
            if self._regen_steps is not None else None
        self._next_terrain = None
        # the builder's pinned upload sources: two persistent sets with the reservation's capacities, generation g
        # staged from set g % 2 (the interval step never allocates or frees pinned memory: a pinned free took
        # ~0.5 ms of its host time)
        self._pin_pool = [None, None]
        # host objects of replaced generations, released on the builder thread when it starts the next build
        self._retired = []
        self._scratch_set = None  # the interval step's reset outputs (allocated with the output sets below)
        self._load_terrain(self._terrain_seed(0))

        # ---- state (SoA float4 planes) and outputs ----
        n = self.num_envs
        self.state = torch.zeros(_abi.NUM_PLANES, n, 4, dtype=torch.float32, device=dev)
        self.istate = torch.zeros(n, 4, dtype=torch.int32, device=dev)
        self._sets = [self._alloc_outputs(n, dev) for _ in range(2)]
        if self._regen_steps is not None:
            self._scratch_set = self._alloc_outputs(n, dev)
        self._nrows = self._lib.gr_num_log_rows(ctx)
        self._log_slab = torch.zeros(LOG_RING, self._nrows, _abi.LOG_SLOTS, dtype=torch.float32, device=dev)
        self._logs: list = [None] * LOG_RING
        self._counters = torch.zeros(2, dtype=torch.int32, device=dev)
        self._calls = 0
        self._cur = 0  # index of the output set written by the last call
        self._bufs = [self._make_buffers(k) for k in range(LOG_RING)]
        self._log_keys = self._build_log_keys()
        # ---- optional front depth camera (the reference's vision task)
        self.camera = cfg.camera
        self.num_obs = _abi.OBS_DIM
        if self.camera is not None:
            self._cam_cfg = self.camera.to_gr()
            self._call("gr_enable_camera", C.byref(self._cam_cfg))
            npix = self.camera.num_pixels
            self.num_obs = _abi.OBS_DIM + npix
            # the sensor's data buffer (distance_to_image_plane) and its age; -1 = outdated
            self.depth = torch.zeros(n, npix, dtype=torch.float32, device=dev)
            self.camera_age = torch.full((n,), -1, dtype=torch.int32, device=dev)
            self._img_sets = [{"policy": torch.zeros(n, self.num_obs, dtype=torch.float32, device=dev),
                               "critic": torch.zeros(n, self.num_obs, dtype=torch.float32, device=dev)}
                              for _ in range(2)]
            self._cam_bufs = []
            for k in range(2):
                cb = _abi.GrCameraBuffers()
                cb.depth = self.depth.data_ptr()
                cb.age = self.camera_age.data_ptr()
                cb.obs_policy = self._img_sets[k]["policy"].data_ptr()
                cb.obs_critic = self._img_sets[k]["critic"].data_ptr()
                self._cam_bufs.append(cb)
        self.extras: dict = {}
        self._sink = None  # (policy, critic) tensors of the bound observation sink
        # fp32 sink = the calls' observation OUTPUT (set_obs_sink): the rows are written once, into the storage slot
        self._sink_out = None
        self._last_rows = None  # (policy, critic) rows the last call wrote, if not the output set's
        # camera task: the fp32 sink is the camera kernel's [16 state terms | image] output instead
        self._cam_sink_out = None
        self._last_img = None
        # startup (gr_init): nominal state, startup DR events, initial terrain levels
        self._bind(0)
        self._call("gr_init", self._stream())
        self._calls, self._cur = 1, 1  # gr_init wrote output set 1 (binding 0); counters zeroed

    # ------------------------------------------------------------------ terrain
    def _terrain_seed(self, generation: int) -> int:
        """The track seed of terrain generation g of this shard (generation 0 at start-up)."""
        return self.cfg.terrain.seed + self.cfg.track_seed_offset + 1000003 * generation

    def _build_terrain(self, seed: int):
        t = self.cfg.terrain
        return build_tracks(num_types=t.num_cols, num_levels=t.num_rows, num_gates=t.num_gates, seed=seed,
                            obstacles=t.obstacles, cell=t.obstacle_cell)

    @staticmethod
    def _pin_generation(gates, recs, obst) -> dict:
        """Pinned host copies of a generation's arrays (the asynchronous upload's source)."""
        pin = {"gates": torch.from_numpy(gates).pin_memory(), "records": torch.from_numpy(recs).pin_memory()}
        if obst is not None:
            for k in ("records", "counts", "grid_f", "grid_i", "cells", "items"):
                pin["o_" + k] = torch.from_numpy(getattr(obst, k)).pin_memory()
        return pin

    @staticmethod
    def _host_obstacles(pin, obst):
        """gr_obstacles over the pinned host arrays (gr_terrain_stage)."""
        if obst is None:
            return None
        o = _abi.GrObstacles()
        for k in ("records", "counts", "grid_f", "grid_i", "cells", "items"):
            setattr(o, k, pin["o_" + k].data_ptr())
        o.max_obstacles = obst.max_obstacles
        o.num_cells = int(obst.cells.shape[0])
        o.num_items = int(obst.items.shape[0])
        return o

    def _pinned_set(self, k, gates, recs, obst):
        """Pinned set k of the pool holding this generation's arrays (views with its shapes into buffers with the
        reservation's capacities; allocated on first use, reused every other generation).  None when the generation
        does not fit (a new reservation follows in _stage_now)."""
        caps = self._capacity
        if obst is not None and (obst.max_obstacles > caps[0] or obst.cells.shape[0] > caps[1]
                                 or obst.items.shape[0] > caps[2]):
            return None
        ps = self._pin_pool[k]
        if ps is None or ps["gates"].shape != gates.shape or ps["caps"] != caps:
            ps = {"caps": caps, "gates": torch.empty(gates.shape, dtype=torch.float32, pin_memory=True),
                  "records": torch.empty(recs.shape, dtype=torch.float32, pin_memory=True)}
            if obst is not None:
                ntr = obst.counts.shape[0]
                ps["o_records"] = torch.empty(ntr * caps[0] * obst.records.shape[2], dtype=torch.float32,
                                              pin_memory=True)
                ps["o_counts"] = torch.empty(ntr, dtype=torch.int32, pin_memory=True)
                ps["o_grid_f"] = torch.empty(ntr, 4, dtype=torch.float32, pin_memory=True)
                ps["o_grid_i"] = torch.empty(ntr, 4, dtype=torch.int32, pin_memory=True)
                ps["o_cells"] = torch.empty(caps[1] * 2, dtype=torch.int32, pin_memory=True)
                ps["o_items"] = torch.empty(caps[2] * obst.items.shape[1], dtype=torch.float32, pin_memory=True)
            self._pin_pool[k] = ps
        pin = {"gates": ps["gates"], "records": ps["records"]}
        pin["gates"].copy_(torch.from_numpy(gates))
        pin["records"].copy_(torch.from_numpy(recs))
        if obst is not None:
            for key in ("records", "counts", "grid_f", "grid_i", "cells", "items"):
                a = getattr(obst, key)
                v = ps["o_" + key].view(-1)[:a.size].view(a.shape)
                v.copy_(torch.from_numpy(a))
                pin["o_" + key] = v
        return pin

    @property
    def terrain_epoch(self) -> int:
        """gr_terrain_epoch: how often the context (re)allocated its terrain arrays.  A hipGraph captured over this
        env's calls bakes in the arrays of the epoch it was captured in."""
        return int(self._lib.gr_terrain_epoch(self._ctx))

    def forget_captures(self):
        """The caller destroyed every graph it captured over this env's calls: the terrain arrays may move again."""
        self._captured_epoch = None

    def _reserve_terrain(self, obst):
        """gr_terrain_reserve with room for generations somewhat larger than `obst` (the generator's sizes vary by
        ~1 % between seeds; a larger one reallocates, outside any graph).  Refused while a graph captured over this
        env's calls may still be replayed (it would read the freed arrays): forget_captures() first."""
        if self._resident and getattr(self, "_captured_epoch", None) is not None:
            raise RuntimeError(
                "the terrain generation outgrew its reservation, and reallocating would leave the hipGraphs captured "
                f"over this env (terrain epoch {self._captured_epoch}) pointing at freed arrays: destroy them and call "
                "env.forget_captures(), then regenerate again")
        if obst is None:
            caps = (0, 0, 0)
        else:
            caps = (obst.max_obstacles + max(8, obst.max_obstacles // 4), int(obst.cells.shape[0] * 1.25) + 64,
                    int(obst.items.shape[0] * 1.25) + 256)
        self._call("gr_terrain_reserve", *caps)
        self._resident = True
        self._capacity = caps

    def _stage(self, pin, obst, stream) -> int:
        """gr_terrain_stage (status returned: GR_ERR_CAPACITY is handled by the caller)."""
        o = self._host_obstacles(pin, obst)
        return self._lib.gr_terrain_stage(self._ctx, pin["gates"].data_ptr(), pin["records"].data_ptr(),
                                          C.byref(o) if o is not None else None, stream)

    def _stage_now(self, gates, recs, obst) -> dict:
        """Stage a generation on the env's stream (start-up, or a regeneration the builder did not prepare); grows
        the reservation if the generation does not fit."""
        if not self._resident:
            self._reserve_terrain(obst)
        pin = self._pin_generation(gates, recs, obst)
        rc = self._stage(pin, obst, self._stream())
        if rc == _abi.GR_ERR_CAPACITY:
            self._reserve_terrain(obst)
            rc = self._stage(pin, obst, self._stream())
        if rc != 0:
            raise RuntimeError(f"gr_terrain_stage failed (status {rc}): {self._lib.gr_last_error(self._ctx).decode()}")
        # the upload is a raw hipMemcpyAsync that torch's pinned-memory cache does not track: the set is released only
        # after this event (_release_retired), never back into the cache while the copy may still read it
        pin["_uploaded"] = torch.cuda.Event()
        pin["_uploaded"].record(torch.cuda.current_stream(self.device))
        return pin

    @staticmethod
    def _release_retired(retired: list):
        """Drop replaced generations' host objects, after the uploads from their pinned sets (if any) completed."""
        for entry in retired:
            pin = entry[-1]
            if isinstance(pin, dict) and pin.get("_uploaded") is not None:
                pin["_uploaded"].synchronize()
        retired.clear()

    def _commit(self, pin, gates, recs, obst):
        """gr_terrain_commit on the env's stream; the generation's host arrays become the env's track_gates /
        track_records / obstacle_table."""
        self._call("gr_terrain_commit", self._stream())
        _stamp("commit_call")
        # the replaced generation's host objects (and a fresh pin set, _stage_now) are released by the builder when
        # it starts the next build, not here: no host free in the interval step (nor in its graph capture)
        self._retired.append((getattr(self, "track_gates", None), getattr(self, "track_records", None),
                              getattr(self, "obstacle_table", None), pin))
        if len(self._retired) > 2:  # (no builder ran in between: one-step intervals, direct regenerate_terrain calls)
            old, self._retired = self._retired[:-2], self._retired[-2:]
            self._release_retired(old)
        self.track_gates = gates if torch.is_tensor(gates) else torch.from_numpy(gates)
        self.track_records = recs if torch.is_tensor(recs) else torch.from_numpy(recs)
        self.obstacle_table = obst
        self.obstacles = None

    def _start_next_terrain(self):
        """Build generation terrain_generation + 1 on the background thread (host numpy, the reference's generator
        restated: tracks.py) and upload it into the context's staging arrays on a side stream, after the previous
        commit (gr_terrain_stage)."""
        if self._builder is None:
            return
        g = self.terrain_generation + 1
        dev = self.device
        side = self._upload_stream = getattr(self, "_upload_stream", None) or torch.cuda.Stream(dev)
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("the terrain builder starts half-way through the interval: capture whole intervals "
                               "outside this step, or only the interval step")
        # the staging arrays are free once everything enqueued so far (the last commit, eager or a graph replay) ran
        after = torch.cuda.Event()
        after.record(torch.cuda.current_stream(dev))
        retired, self._retired = self._retired, []

        def work():
            self._release_retired(retired)  # (the previous generations' host objects, released here)
            gates, recs, obst = self._build_terrain(self._terrain_seed(g))
            pin = self._pinned_set(g % 2, gates, recs, obst)
            if pin is None:  # larger than the reservation: staged again by the interval step (_stage_now)
                return g, gates, recs, obst, None, None, _abi.GR_ERR_CAPACITY
            gates, recs = torch.from_numpy(gates), torch.from_numpy(recs)  # (the env's track_gates / records, here)
            with torch.cuda.stream(side):
                side.wait_event(after)
                rc = self._stage(pin, obst, side.cuda_stream)
                done = torch.cuda.Event()
                done.record(side)
            done.synchronize()  # (on this thread: the interval step then finds the upload complete, no stream wait)
            return g, gates, recs, obst, pin, done, rc

        self._next_terrain = self._builder.submit(work)

    def _load_terrain(self, seed: int):
        """Generate the track table (gates + obstacles) for `seed` and bind it: resident (gr_terrain_reserve / stage /
        commit) when the env regenerates its terrain, else gr_bind_tracks + gr_bind_obstacles over env-owned device
        tensors (track_gates / track_records / obstacles)."""
        gates, recs, obst = self._build_terrain(seed)
        dev = self.device
        if self._regen_steps is not None:
            pin = self._stage_now(gates, recs, obst)
            self._commit(pin, gates, recs, obst)
            torch.cuda.synchronize(dev)
            return
        self.track_gates = torch.from_numpy(gates).to(dev).contiguous()
        self.track_records = torch.from_numpy(recs).to(dev).contiguous()
        self._call("gr_bind_tracks", self.track_gates.data_ptr(), self.track_records.data_ptr())
        self.obstacle_table = obst
        if obst is None:
            self.obstacles = None
            if hasattr(self._lib, "gr_bind_obstacles"):  # (older timing builds predate obstacles)
                self._call("gr_bind_obstacles", None)
            return
        self.obstacles = {k: torch.from_numpy(getattr(obst, k)).to(dev).contiguous()
                          for k in ("records", "counts", "grid_f", "grid_i", "cells", "items")}
        o = _abi.GrObstacles()
        for k, v in self.obstacles.items():
            setattr(o, k, v.data_ptr())
        o.max_obstacles = obst.max_obstacles
        o.num_cells = int(obst.cells.shape[0])
        o.num_items = int(obst.items.shape[0])
        self._obst_struct = o
        self._call("gr_bind_obstacles", C.byref(o))

    def regenerate_terrain(self, out_set: dict | None = None):
        """EventCfg.reset_terrain -> reset_terrain_period (mdp/events.py:180-204): a new terrain
        (next seed of this shard's stream), then env.reset() of every env.

        The builder staged the generation ahead (validated on the host, uploaded on the side stream, its completion
        awaited on the builder thread); here the env's stream commits it (gr_terrain_commit: one kernel with fixed
        arguments), so the interval step is gr_terrain_commit + gr_reset + gr_observe, graph-capturable.  The host
        only waits for the builder if the interval was shorter than a build and its upload.  Under a graph capture the staged generation must
        be complete already (a replay commits whatever was staged last)."""
        g = self.terrain_generation + 1
        staged = None
        _stamp("enter")
        if self._next_terrain is not None and self._resident:
            g_built, gates, recs, obst, pin, done, rc = self._next_terrain.result()
            _stamp("result")
            assert g_built == g
            if rc == 0:
                # the builder waited for its upload before returning: the staged arrays are complete, so the stream
                # needs no dependency on it (and under a graph capture no event may be touched)
                _stamp("wait_event")
                staged = (gates, recs, obst, pin)
            elif rc != _abi.GR_ERR_CAPACITY:
                raise RuntimeError(f"gr_terrain_stage failed (status {rc}): "
                                   f"{self._lib.gr_last_error(self._ctx).decode()}")
        self._next_terrain = None
        if staged is None:  # (not started, an interval of one step, a direct call, or a larger generation) here
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("regenerate_terrain under a graph capture needs the next generation staged "
                                   "(the builder's upload complete)")
            gates, recs, obst = self._build_terrain(self._terrain_seed(g))
            pin = self._stage_now(gates, recs, obst)
            staged = (gates, recs, obst, pin)
        gates, recs, obst, pin = staged
        self._commit(pin, gates, recs, obst)
        _stamp("commit")
        self.terrain_generation = g
        out = self.reset(out_set=out_set)
        _stamp("reset")
        return out

    # ------------------------------------------------------------------ plumbing
    @staticmethod
    def _alloc_outputs(n, dev):
        return {
            "policy": torch.zeros(n, _abi.OBS_DIM, dtype=torch.float32, device=dev),
            "critic": torch.zeros(n, _abi.OBS_DIM, dtype=torch.float32, device=dev),
            "auxiliary": torch.zeros(n, 1, dtype=torch.float32, device=dev),
            "reward": torch.zeros(n, dtype=torch.float32, device=dev),
            "terminated": torch.zeros(n, dtype=torch.bool, device=dev),
            "time_out": torch.zeros(n, dtype=torch.bool, device=dev),
            "dones": torch.zeros(n, dtype=torch.int64, device=dev),
        }

    def _make_buffers(self, k: int) -> _abi.GrBuffers:
        """Buffers for call number k: outputs -> set (k+1)%2, previous -> set k%2, log slab k % LOG_RING,
        observation-noise counter parity k % 2."""
        out, prev = self._sets[(k + 1) % 2], self._sets[k % 2]
        b = _abi.GrBuffers()
        b.state = self.state.data_ptr()
        b.istate = self.istate.data_ptr()
        b.obs_policy = out["policy"].data_ptr()
        b.obs_critic = out["critic"].data_ptr()
        b.obs_aux = out["auxiliary"].data_ptr()
        b.reward = out["reward"].data_ptr()
        b.terminated = out["terminated"].data_ptr()
        b.time_out = out["time_out"].data_ptr()
        b.dones = out["dones"].data_ptr()
        b.prev_obs_critic = prev["critic"].data_ptr()
        b.prev_obs_aux = prev["auxiliary"].data_ptr()
        b.prev_time_out = prev["time_out"].data_ptr()
        b.log_partial = self._log_slab[k % LOG_RING].data_ptr()
        b.counters = self._counters.data_ptr()
        b.counter_index = k % 2
        return b

    def _bind(self, k: int, out_set: dict | None = None, prev_set: dict | None = None):
        """Bind call k's buffers; out_set / prev_set (output-set dicts) replace the call's output / previous rows
        (the terrain interval step's reset writes a scratch set: _regenerate_in_step)."""
        b = self._bufs[k % LOG_RING]
        if self._sink_out is not None or self._last_rows is not None or out_set is not None or prev_set is not None:
            b = _abi.GrBuffers.from_buffer_copy(b)
            if self._last_rows is not None:  # gr_reset / gr_observe carry the last action from the rows last written
                b.prev_obs_critic = self._last_rows[1].data_ptr()
            if prev_set is not None:
                b.prev_obs_critic = prev_set["critic"].data_ptr()
                b.prev_obs_aux = prev_set["auxiliary"].data_ptr()
                b.prev_time_out = prev_set["time_out"].data_ptr()
            if out_set is not None:
                for f, key in (("obs_policy", "policy"), ("obs_critic", "critic"), ("obs_aux", "auxiliary"),
                               ("reward", "reward"), ("terminated", "terminated"), ("time_out", "time_out"),
                               ("dones", "dones")):
                    setattr(b, f, out_set[key].data_ptr())
            elif self._sink_out is not None:
                b.obs_policy, b.obs_critic = self._sink_out[0].data_ptr(), self._sink_out[1].data_ptr()
        self._call("gr_bind_buffers", C.byref(b))
        if getattr(self, "camera", None) is not None:
            cb = self._cam_bufs[(k + 1) % 2]
            if self._cam_sink_out is not None:
                cb = _abi.GrCameraBuffers.from_buffer_copy(cb)
                cb.obs_policy, cb.obs_critic = self._cam_sink_out[0].data_ptr(), self._cam_sink_out[1].data_ptr()
            self._call("gr_bind_camera_buffers", C.byref(cb))

    def _render(self, mode: int, mask_ptr=None):
        if self.camera is not None:
            self._call("gr_camera_render", mode, mask_ptr, self._stream())

    def _stream(self):
        # the raw handle of the device's current stream: torch.cuda.current_stream(device) builds a Stream object
        # under a device guard on every env call (a few µs of each step's host time)
        if _RAW_STREAM is not None and self.device.index is not None:
            return _RAW_STREAM(self.device.index)
        return torch.cuda.current_stream(self.device).cuda_stream

    def _call(self, name, *args):
        if torch.cuda.is_current_stream_capturing():  # a graph now holds this epoch's terrain arrays (_reserve_terrain)
            self._captured_epoch = self.terrain_epoch
        rc = getattr(self._lib, name)(self._ctx, *args)
        if rc != 0:
            raise RuntimeError(f"{name} failed (status {rc}): {self._lib.gr_last_error(self._ctx).decode()}")

    def _advance(self, out_set: dict | None = None, prev_set: dict | None = None):
        """Bind the next output set + log slab; returns (output set, extras["log"] of this call)."""
        k = self._calls
        self._bind(k, out_set, prev_set)
        self._calls += 1
        self._cur = (k + 1) % 2
        self._last_rows = self._sink_out if out_set is None else None
        self._last_img = self._cam_sink_out
        lg = _EpisodeLog(self, k, self._log_keys)
        self._logs[k % LOG_RING] = lg
        return self._sets[self._cur], lg

    def _log_at(self, k: int):
        if k < 0:
            return None
        lg = self._logs[k % LOG_RING]
        return lg if lg is not None and lg._k == k else None

    def _build_log_keys(self) -> dict:
        c = self.cfg
        keys = {}
        for j, name in enumerate(c.reward_term_names()):
            keys[f"Episode_Reward/{name}"] = _abi.LOG_EPSUM0 + j
        cur = c.curriculum_term_names()
        keys[f"Curriculum/{cur[0]}"] = _abi.LOG_LEVEL
        if len(cur) > 1:
            keys[f"Curriculum/{cur[1]}"] = _abi.LOG_NOISE
        for name, slot in (("accumulate_gates", _abi.LOG_ACC), ("action_rate", _abi.LOG_M_ACTRATE),
                           ("avg_lin_spd", _abi.LOG_M_LINSPD), ("avg_ang_spd", _abi.LOG_M_ANGSPD)):
            keys[f"Metrics/next_gate_pose/{name}"] = slot
        tnames = c.termination_term_names()
        slots = [_abi.LOG_T_TIMEOUT, _abi.LOG_T_CONTACT, _abi.LOG_T_BADPOSE]
        for name, slot in zip(tnames, slots):
            keys[f"Episode_Termination/{name}"] = slot
        return keys

    def _obs_dict(self, s):
        if self.camera is not None:
            img = self._img_sets[self._cur]
            if self._last_img is not None:  # the camera kernel wrote its rows into the bound fp32 sink
                return {"policy": self._last_img[0], "critic": self._last_img[1], "auxiliary": s["auxiliary"]}
            return {"policy": img["policy"], "critic": img["critic"], "auxiliary": s["auxiliary"]}
        if self._last_rows is not None:  # the last call wrote its rows into the bound fp32 sink
            return {"policy": self._last_rows[0], "critic": self._last_rows[1], "auxiliary": s["auxiliary"]}
        return {"policy": s["policy"], "critic": s["critic"], "auxiliary": s["auxiliary"]}

    def state_obs(self) -> dict:
        """The 16 state terms of the last call (without the image)."""
        if self._last_rows is not None:
            return {"policy": self._last_rows[0], "critic": self._last_rows[1]}
        s = self._sets[self._cur]
        return {"policy": s["policy"], "critic": s["critic"]}

    # ------------------------------------------------------------------ properties
    @property
    def unwrapped(self):
        return self

    @property
    def max_episode_length_s(self) -> float:
        return self.cfg.episode_length_s

    @property
    def max_episode_length(self) -> int:
        return self.cfg.max_episode_length

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self.istate[:, _abi.I_EPLEN]

    @episode_length_buf.setter
    def episode_length_buf(self, value: torch.Tensor):
        self.istate[:, _abi.I_EPLEN].copy_(value.to(self.device))

    @property
    def obs_buf(self) -> dict:
        return self._obs_dict(self._sets[self._cur])

    @property
    def gr_config(self) -> _abi.GrConfig:
        return self._gcfg

    def bytes_per_env_step(self) -> tuple[int, int]:
        r, w = C.c_int64(), C.c_int64()
        self._call("gr_bytes_per_env_step", C.byref(r), C.byref(w))
        return r.value, w.value

    def step_kernel_name(self) -> str:
        """The step_kernel instantiation gr_step launches with the current bindings (gr_step_kernel_variant)."""
        v = self._lib.gr_step_kernel_variant(self._ctx)
        if v < 0:
            raise RuntimeError(f"gr_step_kernel_variant failed (status {v})")
        return _abi.STEP_KERNEL_NAMES[v]

    def device_status(self, clear: bool = True) -> int:
        """gr_device_status: the GR_STATUS_* bits the step kernels raised since the last clear (synchronises the
        env's stream)."""
        st = C.c_uint32()
        self._call("gr_device_status", C.byref(st), int(bool(clear)), self._stream())
        return st.value

    def check_device_status(self):
        """Raise if a kernel flagged an untrustworthy step since the last check (the runner calls this once per
        rollout, where it synchronises anyway)."""
        from ..rsl_rl import distributed as gdist

        st = self.device_status(clear=True)
        # data parallel: the bits are OR-ed over the ranks first (max of the words, which suffices for one bit;
        # the local word is reported), so every rank raises together instead of one rank raising while the
        # others block in the update's all-reduces until the collective timeout
        any_st = gdist.allreduce_max_int(st, self.device) if gdist.is_dist() else st
        if any_st:
            why = "; ".join(t for b, t in _abi.STATUS_TEXT.items() if (st or any_st) & b) or "unknown"
            where = "" if st else f" (raised on another rank; rank {gdist.rank()} is clean)"
            raise RuntimeError(f"gr step kernel status 0x{any_st:x}{where}: {why}")

    def state_field(self, name: str) -> torch.Tensor:
        """Gather a named per-env state field ([N, k] copy) from the SoA planes."""
        parts = [self.state[p, :, c0:c0 + k] for p, c0, k in _abi.STATE_FIELDS[name]]
        return torch.cat(parts, dim=1)

    def set_state_field(self, name: str, value: torch.Tensor):
        j = 0
        for p, c0, k in _abi.STATE_FIELDS[name]:
            self.state[p, :, c0:c0 + k].copy_(value[:, j:j + k])
            j += k

    @property
    def gate_id(self) -> torch.Tensor:
        return self.istate[:, _abi.I_PACKED] & 0xFF

    @property
    def terrain_levels(self) -> torch.Tensor:
        return (self.istate[:, _abi.I_PACKED] >> 8) & 0xFF

    @property
    def terrain_types(self) -> torch.Tensor:
        return (self.istate[:, _abi.I_PACKED] >> 24) & 0xFF

    # ------------------------------------------------------------------ MDP
    def step(self, action: torch.Tensor):
        """ManagerBasedDiffRLEnv.step (manager_based_diff_rl_env.py:160-267)."""
        if action.dim() != 2 or action.shape[1] != self.num_actions:
            raise ValueError(f"Invalid action shape, expected: {self.num_actions}, received: {action.shape[-1]}.")
        if action.shape[0] != self.num_envs:
            raise ValueError(f"Invalid action batch {action.shape[0]}, expected {self.num_envs}")
        a = action
        if a.device != self.device or a.dtype != torch.float32 or not a.is_contiguous() or a.data_ptr() % 16:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        out, log = self._advance()
        self._call("gr_step", a.data_ptr(), self._stream())
        self._render(_abi.GR_CAM_STEP)
        self.common_step_counter += 1
        self.extras = {"log": log}
        if self._regen_steps is not None:
            phase = self.common_step_counter % self._regen_steps
            if phase == 0:
                self._regenerate_in_step()
            elif phase == self._regen_steps // 2 and self._next_terrain is None:
                self._start_next_terrain()
        return self._obs_dict(out), out["reward"], out["terminated"], out["time_out"], self.extras

    def _regenerate_in_step(self):
        """The terrain interval event inside step (manager_based_diff_rl_env.py:259-264): after the step's
        resets and command update, reset_terrain_period (mdp/events.py:180-204) rebuilds the terrain and
        calls env.reset(); the observations are computed after it.  So the step returns its own reward /
        terminated / time-outs / dones with the post-reset observations and the reset's extras["log"].

        Call k (this step) wrote output set B.  The reset (call k+1) writes set A, which still holds the
        previous step's observations that the runner keeps in its transition until process_env_step; the
        observation pass (call k+2) writes the post-reset observations back into set B, over the step's
        observation rows only; set A's rows are then restored.  The next step (call k+3) writes set A and
        reads the post-reset rows of set B as its previous observation."""
        if self.camera is None:
            # the reset's own observation (discarded by the reference: the step computes them again) goes to a scratch
            # output set, so the runner's held set is never written and nothing is saved / restored: the interval step
            # is gr_swap_terrain + gr_reset(all) + gr_observe on the stream
            scratch = self._scratch_set
            if scratch is None:  # (a direct call on an env built without an interval)
                scratch = self._scratch_set = self._alloc_outputs(self.num_envs, self.device)
            _, extras = self.regenerate_terrain(out_set=scratch)
            self._observe_after(scratch)
            self.extras = {"log": extras["log"], "terrain_regenerated": True}
            return
        held = self._sets[(self._cur + 1) % 2]
        # (with the fp32 sink as the output the reset and observation passes write the step's slot, which is what
        # the step returns; the runner's previous slot is not touched)
        keys = ("auxiliary",) if self._sink_out is not None else ("policy", "critic", "auxiliary")
        saved = [held[k].clone() for k in keys]
        sink_img = self.camera is not None and self._cam_sink_out is not None
        if self.camera is not None and not sink_img:  # (with the camera sink bound the held set is not written)
            held_img = self._img_sets[(self._cur + 1) % 2]
            saved_img = [held_img[k].clone() for k in ("policy", "critic")]
        _, extras = self.regenerate_terrain()
        self.observe()
        for k, v in zip(keys, saved):
            held[k].copy_(v)
        if self.camera is not None and not sink_img:
            for k, v in zip(("policy", "critic"), saved_img):
                held_img[k].copy_(v)
        self.extras = {"log": extras["log"], "terrain_regenerated": True}

    def reset(self, seed: int | None = None, env_ids=None, options=None, out_set: dict | None = None):
        """ManagerBasedEnv.reset -> _reset_idx(env_ids) (+ curriculum), then observations.  out_set: write the
        call's outputs into this output-set dict instead of the next ping-pong set (_regenerate_in_step)."""
        mask_t = None
        empty = False
        if env_ids is not None:
            ids = torch.as_tensor(env_ids, device=self.device, dtype=torch.long)
            empty = ids.numel() == 0
            mask_t = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
            mask_t[ids] = 1
        out, log = self._advance(out_set)
        if out_set is not None:
            out = out_set
        log._empty_reset = empty
        mp = mask_t.data_ptr() if mask_t is not None else None
        self._call("gr_reset", mp, self._stream())
        self._render(_abi.GR_CAM_RESET, mp)
        self.extras = {"log": log}
        return self._obs_dict(out), self.extras

    def set_obs_sink(self, policy: torch.Tensor | None, critic: torch.Tensor | None = None):
        """The following step / reset / observe calls put their policy and critic rows into these [num_envs, 16]
        tensors — the rollout storage's slot for the next transition — instead of the storage copying them
        (rollout_storage.py:74-88).  float32: the tensors become the calls' observation output (written once, and
        returned by the calls); bfloat16 (config C5's bf16 rollout buffers): gr_bind_obs_sink, the kernel writes
        the fp32 output rows and their round-to-nearest-even bf16 copy.  None unbinds.  Camera task: [num_envs,
        16 + pixels] float32 tensors become the camera kernel's output ([16 state terms | image] rows,
        observation.py:65-94 into rollout_storage.py:74-88's slot, written once)."""
        if policy is None:
            self._sink = None
            self._sink_out = None
            self._cam_sink_out = None
            self._bind_obs_sink(None, None, _abi.GR_DTYPE_F32)
            return
        width = self.num_obs
        dtypes = (torch.float32,) if self.camera is not None else (torch.float32, torch.bfloat16)
        for t in (policy, critic):
            if (t is None or t.device != self.device or tuple(t.shape) != (self.num_envs, width)
                    or not t.is_contiguous() or t.dtype not in dtypes or t.data_ptr() % 16):
                raise ValueError(f"set_obs_sink: need contiguous 16-byte aligned [{self.num_envs}, {width}] "
                                 f"{' / '.join(str(d) for d in dtypes)} tensors on {self.device}")
        if critic.dtype != policy.dtype:
            raise ValueError("set_obs_sink: policy and critic sinks must share a dtype")
        self._sink = (policy, critic)  # kept alive while bound
        if self.camera is not None:
            self._cam_sink_out = (policy, critic)
            return
        if policy.dtype == torch.float32:
            # fp32: the tensors ARE the calls' observation output (the rows are written once; the calls return
            # these tensors), rollout_storage.py:74-88's copy with no second write
            self._sink_out = (policy, critic)
            self._bind_obs_sink(None, None, _abi.GR_DTYPE_F32)
            return
        # bf16: the fp32 rows stay the output (the rollout inference reads them) and the kernel also writes the
        # rounded rows into the slot
        self._sink_out = None
        self._bind_obs_sink(policy.data_ptr(), critic.data_ptr(), _abi.GR_DTYPE_BF16)

    def _bind_obs_sink(self, p, c, dtype):
        """gr_bind_obs_sink unless the context already holds exactly this binding (an fp32 sink rebinds nothing
        per step: its tensors are the calls' outputs, set in _bind)."""
        state = (p, c, dtype)
        if getattr(self, "_obs_sink_state", None) != state:
            self._call("gr_bind_obs_sink", p, c, dtype)
            self._obs_sink_state = state

    def observe(self) -> dict:
        """ObservationManager.compute(): fresh observation noise, no state change."""
        out, _ = self._advance()
        self._call("gr_observe", self._stream())
        self._render(_abi.GR_CAM_OBSERVE)
        return self._obs_dict(out)

    def _observe_after(self, prev_set: dict):
        """observe() whose previous rows (the last action the rows carry) are prev_set's."""
        self._advance(prev_set=prev_set)
        self._call("gr_observe", self._stream())

    def seed(self, seed: int = -1) -> int:
        return seed

    def close(self):
        if getattr(self, "_builder", None) is not None:
            # (a running build stages into the context's arrays: wait for it before the context goes)
            self._builder.shutdown(wait=True, cancel_futures=True)
            self._builder = None
        if getattr(self, "_ctx", None):
            self._lib.gr_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RslRlVecEnvWrapper:
    """Isaac Lab's omni.isaac.lab_tasks.utils.wrappers.rsl_rl.RslRlVecEnvWrapper surface
    (call sites: standalone/rsl_rl/train.py:120, on_policy_runner.py:38,119-122,143)."""

    def __init__(self, env: RacingEnv):
        self.env = env
        self.num_envs = env.num_envs
        self.device = env.device
        self.max_episode_length = env.max_episode_length
        self.num_actions = env.num_actions
        self.num_obs = env.num_obs
        self.num_privileged_obs = env.num_obs
        self.env.reset()

    @property
    def cfg(self):
        return self.env.cfg

    @property
    def unwrapped(self) -> RacingEnv:
        return self.env

    @property
    def render_mode(self):
        return self.env.render_mode

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self.env.episode_length_buf

    @episode_length_buf.setter
    def episode_length_buf(self, value: torch.Tensor):
        self.env.episode_length_buf = value

    def seed(self, seed: int = -1) -> int:
        return self.env.seed(seed)

    def check_device_status(self):
        """RacingEnv.check_device_status."""
        self.env.check_device_status()

    def set_obs_sink(self, policy, critic=None):
        """RacingEnv.set_obs_sink (rollout storage slots written by the kernel; None unbinds)."""
        self.env.set_obs_sink(policy, critic)

    def get_observations(self):
        obs_dict = self.env.observe()
        return obs_dict["policy"], {"observations": obs_dict}

    def reset(self):
        obs_dict, _ = self.env.reset()
        return obs_dict["policy"], {"observations": obs_dict}

    def step(self, actions: torch.Tensor):
        obs_dict, rew, terminated, truncated, extras = self.env.step(actions)
        extras["observations"] = obs_dict
        if not self.env.cfg.is_finite_horizon:
            extras["time_outs"] = truncated
        # dones = (terminated | truncated).long(), written by the kernel directly
        dones = self.env._sets[self.env._cur]["dones"]
        return obs_dict["policy"], rew, dones, extras

    def close(self):
        return self.env.close()
