"""ctypes front-end of the CPU oracle (oracle/gr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the generalizableracing_amd package.
Also converts between the oracle's array-of-structs env records and the HIP
kernel's struct-of-float4-planes state so both can be driven from one state.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_F = np.float32
_I = np.int32
ENV_DTYPE = np.dtype([
    ("p", _F, 3), ("q", _F, 4), ("v", _F, 3), ("w", _F, 3), ("alpha", _F, 3), ("T", _F), ("tau", _F, 3),
    ("lag", _F, 4), ("thr_err", _F), ("noise_level", _F), ("k2", _F, 3), ("k1", _F, 3), ("ep_sum", _F, 7),
    ("m_actrate", _F), ("Kp", _F, 3), ("cT", _F), ("Kd", _F, 3), ("m_plant", _F), ("ctau", _F, 3),
    ("m_ctrl", _F), ("J", _F, 3), ("motor_w", _F, 4), ("rotor", _F, 4),
    ("ep_len", _I), ("acc", _I), ("epoch", _I), ("gate_id", _I), ("level", _I), ("type", _I), ("azero", _I),
])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        vp = C.c_void_p
        lib.gro_env_size.restype = C.c_size_t
        for name, args in {
            "gro_type_starts": [vp, vp],
            "gro_init": [vp, vp, C.c_int, vp],
            "gro_reset": [vp, vp, C.c_int, vp, vp, vp, vp],
            "gro_step": [vp, vp, C.c_int, vp, vp, vp, vp],
            "gro_observe": [vp, vp, C.c_int, vp, vp, vp],
            "gro_test_dynamics": [vp, C.c_int, C.c_int] + [vp] * 9,
            "gro_test_math": [C.c_int, C.c_int, vp, vp, vp],
            "gro_test_philox": [C.c_int] + [C.c_uint32] * 6 + [vp],
            "gro_test_fields6": [C.c_int, vp, vp],
            "gro_test_normal24": [C.c_int, vp, vp],
            "gro_test_cam_noise": [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, vp],
            "gro_num_threads": [],
            "gro_camera": [vp, vp, vp, C.c_int, vp, C.c_int, vp, vp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp],
            "gro_camera_frame": [vp, vp, vp, vp, vp],
            "gro_camera_cull_check": [vp, vp, vp, C.c_int, vp, vp, vp],
            "gro_draws": [vp, C.c_int, C.c_int, C.c_uint32, C.c_uint32, vp],
        }.items():
            f = getattr(lib, name)
            f.restype = None
            f.argtypes = args
        lib.gro_camera_ray.restype = C.c_float
        lib.gro_camera_ray.argtypes = [vp, vp, vp, C.c_int, vp, vp, C.c_int, C.c_int]
        lib.gro_collision_count.restype = C.c_int
        lib.gro_collision_count.argtypes = [vp, vp, C.c_int, vp, vp]
        if lib.gro_env_size() != ENV_DTYPE.itemsize:
            raise RuntimeError(f"gro_env size {lib.gro_env_size()} != numpy {ENV_DTYPE.itemsize}")
        _lib = lib
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class GroOut(C.Structure):
    _fields_ = [("obs_policy", C.c_void_p), ("obs_critic", C.c_void_p), ("obs_aux", C.c_void_p),
                ("reward", C.c_void_p), ("terminated", C.c_void_p), ("time_out", C.c_void_p),
                ("dones", C.c_void_p), ("log_out", C.c_void_p)]


class GroTracks(C.Structure):
    _fields_ = [("gates", C.c_void_p), ("tracks", C.c_void_p), ("obst", C.c_void_p), ("obst_count", C.c_void_p),
                ("max_obst", C.c_int32)]


def from_env(env):
    """An Oracle over the same config and tables as a device RacingEnv (gates, records, obstacles)."""
    ot = getattr(env, "obstacle_table", None)
    return Oracle(env.gr_config, env.track_gates.cpu().numpy(), env.track_records.cpu().numpy(),
                  None if ot is None else ot.records, None if ot is None else ot.counts)


class Oracle:
    """Stateful CPU env mirroring the device env (same config struct, same track table).
    obst_records [T*L][M][20] / obst_counts [T*L]: the obstacle table (None: no obstacles)."""

    def __init__(self, cfg, gates: np.ndarray, recs: np.ndarray, obst_records: np.ndarray | None = None,
                 obst_counts: np.ndarray | None = None):
        self.lib = load()
        self.cfg = cfg  # generalizableracing_amd._abi.GrConfig (plain ctypes struct)
        n = cfg.num_envs
        self.n = n
        self.gates = np.ascontiguousarray(gates, dtype=np.float32)
        self.recs = np.ascontiguousarray(recs, dtype=np.float32)
        if obst_records is not None:
            self.obst = np.ascontiguousarray(obst_records, dtype=np.float32)
            self.obst_counts = np.ascontiguousarray(obst_counts, dtype=np.int32)
            self.tracks = GroTracks(_p(self.gates), _p(self.recs), _p(self.obst), _p(self.obst_counts),
                                    self.obst.shape[1])
        else:
            self.tracks = GroTracks(_p(self.gates), _p(self.recs), None, None, 0)
        self.envs = np.zeros(n, dtype=ENV_DTYPE)
        self.obs_policy = np.zeros((n, 16), np.float32)
        self.obs_critic = np.zeros((n, 16), np.float32)
        self.obs_aux = np.zeros(n, np.float32)
        self.reward = np.zeros(n, np.float32)
        self.terminated = np.zeros(n, np.uint8)
        self.time_out = np.zeros(n, np.uint8)
        self.dones = np.zeros(n, np.int64)
        self.log = np.zeros(20, np.float32)
        self.counter = np.zeros(1, np.uint32)
        self.out = GroOut(_p(self.obs_policy), _p(self.obs_critic), _p(self.obs_aux), _p(self.reward),
                          _p(self.terminated), _p(self.time_out), _p(self.dones), _p(self.log))

    def init(self):
        self.lib.gro_init(C.byref(self.cfg), _p(self.envs), self.n, C.byref(self.out))
        self.counter[0] = 0

    def reset(self, mask: np.ndarray | None = None):
        mp = None if mask is None else _p(np.ascontiguousarray(mask, dtype=np.uint8))
        self.lib.gro_reset(C.byref(self.cfg), _p(self.envs), self.n, mp, C.byref(self.tracks), _p(self.counter),
                           C.byref(self.out))

    def step(self, actions: np.ndarray):
        a = np.ascontiguousarray(actions, dtype=np.float32)
        self.lib.gro_step(C.byref(self.cfg), _p(self.envs), self.n, _p(a), C.byref(self.tracks), _p(self.counter),
                          C.byref(self.out))

    def observe(self):
        self.lib.gro_observe(C.byref(self.cfg), _p(self.envs), self.n, C.byref(self.tracks), _p(self.counter),
                             C.byref(self.out))

    # ---- depth camera (gro_camera): state lives next to the env records
    def enable_camera(self, cam_cfg):
        """cam_cfg: generalizableracing_amd._abi.GrCameraConfig."""
        self.cam_cfg = cam_cfg
        npix = cam_cfg.width * cam_cfg.height
        self.depth = np.zeros((self.n, npix), np.float32)
        self.cam_age = np.full(self.n, -1, np.int32)
        self.img_policy = np.zeros((self.n, 16 + npix), np.float32)
        self.img_critic = np.zeros((self.n, 16 + npix), np.float32)

    def camera(self, mode: int, mask: np.ndarray | None = None):
        """Image observation of the call just made (cnt = the counter that call used)."""
        mp = None if mask is None else _p(np.ascontiguousarray(mask, dtype=np.uint8))
        cnt = (int(self.counter[0]) - 1) & 0xFFFFFFFF
        self.lib.gro_camera(C.byref(self.cfg), C.byref(self.cam_cfg), _p(self.envs), self.n, C.byref(self.tracks),
                            mode, mp, _p(self.terminated), _p(self.time_out), cnt, _p(self.depth), _p(self.cam_age),
                            _p(self.obs_policy), _p(self.obs_critic), _p(self.img_policy), _p(self.img_critic))

    def camera_ray(self, track: int, p, q, u: int, v: int) -> float:
        p = np.ascontiguousarray(p, dtype=np.float32)
        q = np.ascontiguousarray(q, dtype=np.float32)
        return float(self.lib.gro_camera_ray(C.byref(self.cfg), C.byref(self.cam_cfg), C.byref(self.tracks), track,
                                             _p(p), _p(q), u, v))

    def camera_frame(self, p, q):
        """-> (o[3], c0, c1, c2, ray_a[W], ray_b[H]) as the oracle computes them (fp32)."""
        W, H = self.cam_cfg.width, self.cam_cfg.height
        out = np.zeros(12 + W + H, np.float32)
        self.lib.gro_camera_frame(C.byref(self.cfg), C.byref(self.cam_cfg),
                                  _p(np.ascontiguousarray(p, np.float32)), _p(np.ascontiguousarray(q, np.float32)),
                                  _p(out))
        return out[0:3], out[3:6], out[6:9], out[9:12], out[12:12 + W], out[12 + W:]

    def camera_cull_check(self, track: int, p, q) -> np.ndarray:
        """gro_camera_cull_check: [[pairs, culled pairs, culled pairs with a hit (must be 0), culled window pixels]
        of the gates, the same of the obstacles]."""
        out = np.zeros(8, np.int64)
        self.lib.gro_camera_cull_check(C.byref(self.cfg), C.byref(self.cam_cfg), C.byref(self.tracks), track,
                                       _p(np.ascontiguousarray(p, np.float32)), _p(np.ascontiguousarray(q, np.float32)),
                                       _p(out))
        return out.reshape(2, 4)

    def collision_count(self, track: int, p, q) -> int:
        p = np.ascontiguousarray(p, dtype=np.float32)
        q = np.ascontiguousarray(q, dtype=np.float32)
        return self.lib.gro_collision_count(C.byref(self.cfg), C.byref(self.tracks), track, _p(p), _p(q))


def test_dynamics(cfg, mode, state_in, ab, cmd, ctrl_in, par, drag):
    lib = load()
    n = state_in.shape[0]
    arrs = [np.ascontiguousarray(x, dtype=np.float32) for x in (state_in, ab, cmd, ctrl_in, par, drag)]
    so = np.zeros((n, 13), np.float32)
    co = np.zeros((n, 4), np.float32)
    xo = np.zeros((n, 13), np.float32)
    lib.gro_test_dynamics(C.byref(cfg), n, mode, *[_p(a) for a in arrs], _p(so), _p(co), _p(xo))
    return so, co, xo


def test_math(fn, x, y=None):
    lib = load()
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.ascontiguousarray(np.ones_like(x) if y is None else y, dtype=np.float32)
    out = np.zeros_like(x)
    lib.gro_test_math(fn, x.size, _p(x), _p(y), _p(out))
    return out


def test_philox(n, c0, c1, c2, c3, k0, k1):
    lib = load()
    out = np.zeros((n, 4), np.uint32)
    lib.gro_test_philox(n, c0, c1, c2, c3, k0, k1, _p(out))
    return out


DRAW_OBS, DRAW_GATE, DRAW_RESET, DRAW_STATIC = 0, 1, 2, 3
DRAW_LEN = {DRAW_OBS: 6, DRAW_GATE: 6, DRAW_RESET: 25, DRAW_STATIC: 16}


def draws(cfg, i: int, kind: int, c1: int = 0, c3: int = 0) -> np.ndarray:
    """gro_draws: the random values env i (of cfg's shard) consumes for `kind` (DRAW_*), as fp32."""
    out = np.zeros(25, np.float32)
    load().gro_draws(C.byref(cfg), int(i), int(kind), C.c_uint32(c1 & 0xFFFFFFFF), C.c_uint32(c3 & 0xFFFFFFFF),
                     _p(out))
    return out[:DRAW_LEN[kind]]


def num_threads() -> int:
    lib = load()
    lib.gro_num_threads.restype = C.c_int
    return int(lib.gro_num_threads())


def test_fields6(words: np.ndarray) -> np.ndarray:
    lib = load()
    w = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1, 4)
    out = np.zeros((w.shape[0], 6), np.uint32)
    lib.gro_test_fields6(w.shape[0], _p(w), _p(out))
    return out


def type_starts(cfg):
    lib = load()
    out = np.zeros(cfg.num_types + 1, np.int32)
    lib.gro_type_starts(C.byref(cfg), _p(out))
    return out


# ---------------------------------------------------------------- layout bridge
# kernel planes (include/gr.h GR_P_*) <-> oracle records
_PLANE_MAP = [  # (plane, comp) for each float of the kernel state, in ENV_DTYPE field order
    ("p", [(0, 0), (0, 1), (0, 2)]), ("q", [(0, 3), (1, 0), (1, 1), (1, 2)]), ("v", [(1, 3), (2, 0), (2, 1)]),
    ("w", [(2, 2), (2, 3), (3, 0)]), ("alpha", [(3, 1), (3, 2), (3, 3)]), ("T", [(4, 0)]),
    ("tau", [(4, 1), (4, 2), (4, 3)]), ("lag", [(5, 0), (5, 1), (5, 2), (5, 3)]), ("thr_err", [(6, 0)]),
    ("noise_level", [(6, 1)]), ("k2", [(6, 2), (6, 3), (7, 0)]), ("k1", [(7, 1), (7, 2), (7, 3)]),
    ("ep_sum", [(8, 0), (8, 1), (8, 2), (8, 3), (9, 0), (9, 1), (9, 2)]), ("m_actrate", [(9, 3)]),
    ("Kp", [(10, 0), (10, 1), (10, 2)]), ("cT", [(10, 3)]), ("Kd", [(11, 0), (11, 1), (11, 2)]),
    ("m_plant", [(11, 3)]), ("ctau", [(12, 0), (12, 1), (12, 2)]), ("m_ctrl", [(12, 3)]),
    ("J", [(13, 0), (13, 1), (13, 2)]), ("motor_w", [(14, 0), (14, 1), (14, 2), (14, 3)]),
    ("rotor", [(16, 0), (16, 1), (16, 2), (16, 3)]),
]


def planes_to_envs(state: np.ndarray, istate: np.ndarray) -> np.ndarray:
    n = state.shape[1]
    envs = np.zeros(n, dtype=ENV_DTYPE)
    for name, comps in _PLANE_MAP:
        vals = np.stack([state[p, :, c] for p, c in comps], axis=1)
        envs[name] = vals if len(comps) > 1 else vals[:, 0]
    envs["ep_len"] = istate[:, 0]
    envs["acc"] = istate[:, 1]
    envs["epoch"] = istate[:, 2]
    packed = istate[:, 3]
    envs["gate_id"] = packed & 0xFF
    envs["level"] = (packed >> 8) & 0xFF
    envs["azero"] = (packed >> 16) & 1
    envs["type"] = (packed >> 24) & 0xFF
    return envs


def envs_to_planes(envs: np.ndarray, num_planes: int = 17):
    n = envs.shape[0]
    state = np.zeros((num_planes, n, 4), np.float32)
    for name, comps in _PLANE_MAP:
        vals = envs[name].reshape(n, -1)
        for j, (p, c) in enumerate(comps):
            state[p, :, c] = vals[:, j]
    istate = np.zeros((n, 4), np.int32)
    istate[:, 0] = envs["ep_len"]
    istate[:, 1] = envs["acc"]
    istate[:, 2] = envs["epoch"]
    istate[:, 3] = (envs["gate_id"] & 0xFF) | ((envs["level"] & 0xFF) << 8) | ((envs["azero"] & 1) << 16) | \
        ((envs["type"] & 0xFF) << 24)
    return state, istate


def test_normal24(words: np.ndarray) -> np.ndarray:
    """gr_normal24 (the camera noise's inverse-CDF normal) of each uint32 word."""
    w = np.ascontiguousarray(words, dtype=np.uint32).ravel()
    out = np.zeros(w.size, np.float32)
    load().gro_test_normal24(w.size, _p(w), _p(out))
    return out


def test_cam_noise(gid: int, cnt: int, q0: int, nq: int, k0: int, k1: int) -> np.ndarray:
    """The camera's image noise (gr_cam_noise4) of env id gid, call counter cnt, quads q0 .. q0 + nq - 1: [4 nq]."""
    out = np.zeros(4 * nq, np.float32)
    load().gro_test_cam_noise(gid & 0xFFFFFFFF, cnt & 0xFFFFFFFF, q0 & 0xFFFFFFFF, nq, k0 & 0xFFFFFFFF,
                              k1 & 0xFFFFFFFF, _p(out))
    return out
