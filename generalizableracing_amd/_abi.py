"""ctypes mirror of include/gr.h and the loader for libgr.so.

The product path talks to the HIP step only through this C ABI (plain
pointers, sizes and a hipStream_t; no torch types cross it).  `load()` fails
loudly when the in-tree libgr.so is missing — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must be imported first: libgr.so binds to torch's libamdhip64)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgr.so")

# ---- constants (include/gr.h) ----
GR_ABI_VERSION = 6
GR_INTEGRATOR_DD_EXPLICIT = 0
GR_INTEGRATOR_SEMI_IMPLICIT = 1

P_POSQ, P_QV, P_VW, P_WA, P_CTRL, P_LAG, P_RST0, P_RST1, P_EP0, P_EP1, P_PAR0, P_PAR1, P_PAR2, P_PAR3, P_MOTOR = range(15)
P_OHINT, P_ROTOR = 15, 16
NUM_PLANES = 17
I_EPLEN, I_ACC, I_EPOCH, I_PACKED = range(4)
OBS_DIM = 16
GATE_FLOATS = 20
TRACK_FLOATS = 4
OBST_FLOATS = 20

LOG_NRESET = 0
LOG_EPSUM0 = 1
LOG_ACC = 8
LOG_M_ACTRATE = 9
LOG_M_LINSPD = 10
LOG_M_ANGSPD = 11
LOG_T_TIMEOUT = 12
LOG_T_CONTACT = 13
LOG_T_BADPOSE = 14
LOG_LEVEL = 15
LOG_NOISE = 16
LOG_SLOTS = 20

# named fields of the float planes: name -> (plane, first component, count)
STATE_FIELDS = {
    "pos": [(P_POSQ, 0, 3)],
    "quat": [(P_POSQ, 3, 1), (P_QV, 0, 3)],
    "lin_vel_w": [(P_QV, 3, 1), (P_VW, 0, 2)],
    "ang_vel_b": [(P_VW, 2, 2), (P_WA, 0, 1)],
    "ang_acc_b": [(P_WA, 1, 3)],
    "ctrl": [(P_CTRL, 0, 4)],
    "lag": [(P_LAG, 0, 4)],  # tanh(previous raw action): the lag buffer, squashed once
    "thr_est_error": [(P_RST0, 0, 1)],
    "noise_level": [(P_RST0, 1, 1)],
    "drag2": [(P_RST0, 2, 2), (P_RST1, 0, 1)],
    "drag1": [(P_RST1, 1, 3)],
    "episode_sums": [(P_EP0, 0, 4), (P_EP1, 0, 3)],
    "metric_action_rate": [(P_EP1, 3, 1)],
    "rate_gain_p": [(P_PAR0, 0, 3)],
    "thrust_filter": [(P_PAR0, 3, 1)],
    "rate_gain_d": [(P_PAR1, 0, 3)],
    "mass_plant": [(P_PAR1, 3, 1)],
    "torque_filter": [(P_PAR2, 0, 3)],
    "mass_ctrl": [(P_PAR2, 3, 1)],
    "inertia_plant": [(P_PAR3, 0, 3)],
    "motor_omega": [(P_MOTOR, 0, 4)],
    "rotor_constants": [(P_ROTOR, 0, 4)],
}


class GrConfig(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32),
        ("env_id_offset", C.c_int32),
        ("seed_lo", C.c_uint32),
        ("seed_hi", C.c_uint32),
        ("num_types", C.c_int32),
        ("num_levels", C.c_int32),
        ("max_gates", C.c_int32),
        ("max_init_level", C.c_int32),
        ("stage", C.c_int32),
        ("integrator", C.c_int32),
        ("decimation", C.c_int32),
        ("max_episode_length", C.c_int32),
        ("sim_dt", C.c_float),
        ("step_dt", C.c_float),
        ("episode_length_s", C.c_float),
        ("gravity", C.c_float),
        ("mass", C.c_float),
        ("inertia", C.c_float * 3),
        ("arm_length", C.c_float),
        ("kappa", C.c_float),
        ("motor_tau", C.c_float),
        ("motor_omega", C.c_float * 2),
        ("thrustmap", C.c_float * 3),
        ("max_thrust_weight_ratio", C.c_float),
        ("body_rate_bound", C.c_float),
        ("rate_gain_p", C.c_float * 3),
        ("rate_gain_d", C.c_float * 3),
        ("thrust_ctrl_delay", C.c_float),
        ("torque_ctrl_delay", C.c_float * 3),
        ("use_motor_model", C.c_int32),
        ("action_lag", C.c_int32),
        ("drag1", C.c_float * 3),
        ("drag1_rand", C.c_float),
        ("drag2", C.c_float * 3),
        ("drag2_rand", C.c_float),
        ("z_drag", C.c_float),
        ("z_drag_rand", C.c_float),
        ("random_drag", C.c_int32),
        ("mass_add_range", C.c_float * 2),
        ("inertia_scale_range", C.c_float * 2),
        ("pid_scale_range", C.c_float * 2),
        ("delay_scale_range", C.c_float * 2),
        ("dr_startup", C.c_int32),
        ("dr_plant", C.c_int32),
        ("spawn_pos", C.c_float * 3),
        ("reset_pos_half", C.c_float * 3),
        ("reset_att_half", C.c_float * 3),
        ("reset_vel_half", C.c_float * 6),
        ("gate_threshold", C.c_float),
        ("gate_noise_pos", C.c_float * 3),
        ("add_gate_noise", C.c_int32),
        ("level_up_threshold", C.c_int32),
        ("level_down_threshold", C.c_int32),
        ("noise_curriculum", C.c_int32),
        ("noise_enhance_threshold", C.c_int32),
        ("noise_decay_threshold", C.c_int32),
        ("noise_enhance", C.c_float),
        ("noise_decay", C.c_float),
        ("obs_noise", C.c_int32),
        ("obs_lin_vel_noise", C.c_float),
        ("obs_att_noise", C.c_float),
        ("w_progress", C.c_float),
        ("w_body_rate", C.c_float),
        ("w_action_rate", C.c_float),
        ("w_collision", C.c_float),
        ("w_perception", C.c_float),
        ("w_success", C.c_float),
        ("w_bad_pose", C.c_float),
        ("collider_half", C.c_float * 3),
        ("collision_count_threshold", C.c_int32),
        ("out_of_bound", C.c_float * 2),
        ("term_contact", C.c_int32),
        ("term_bad_pose", C.c_int32),
        ("dr_rotor", C.c_int32),
        ("rotor_scale_range", C.c_float * 2),
        ("reserved", C.c_int32 * 5),
    ]

    def to_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = list(v) if hasattr(v, "__len__") else v
        return out


class GrBuffers(C.Structure):
    _fields_ = [
        ("state", C.c_void_p),
        ("istate", C.c_void_p),
        ("obs_policy", C.c_void_p),
        ("obs_critic", C.c_void_p),
        ("obs_aux", C.c_void_p),
        ("reward", C.c_void_p),
        ("terminated", C.c_void_p),
        ("time_out", C.c_void_p),
        ("dones", C.c_void_p),
        ("prev_obs_critic", C.c_void_p),
        ("prev_obs_aux", C.c_void_p),
        ("prev_time_out", C.c_void_p),
        ("log_partial", C.c_void_p),
        ("counters", C.c_void_p),
        ("counter_index", C.c_int32),
        ("reserved", C.c_int32),
    ]


class GrCameraConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
        ("offset_pos", C.c_float * 3), ("offset_rot", C.c_float * 4),
        ("max_distance", C.c_float), ("update_period", C.c_float), ("noise_std", C.c_float),
        ("add_noise", C.c_int32), ("obs_scale", C.c_float), ("reserved", C.c_int32 * 6),
    ]


class GrCameraBuffers(C.Structure):
    _fields_ = [("depth", C.c_void_p), ("age", C.c_void_p), ("obs_policy", C.c_void_p), ("obs_critic", C.c_void_p)]


class GrObstacles(C.Structure):
    _fields_ = [("records", C.c_void_p), ("counts", C.c_void_p), ("grid_f", C.c_void_p), ("grid_i", C.c_void_p),
                ("cells", C.c_void_p), ("items", C.c_void_p), ("max_obstacles", C.c_int32), ("num_cells", C.c_int32),
                ("num_items", C.c_int32), ("reserved", C.c_int32)]


class GrPolicyNet(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p),
                ("b2", C.c_void_p), ("w3", C.c_void_p), ("b3", C.c_void_p), ("out", C.c_void_p),
                ("num_obs", C.c_int32), ("num_out", C.c_int32), ("reserved", C.c_int32 * 2)]


class GrPolicyArgs(C.Structure):
    _fields_ = [("net", GrPolicyNet * 2), ("std", C.c_void_p), ("actions", C.c_void_p), ("log_prob", C.c_void_p),
                ("counters", C.c_void_p), ("counter_index", C.c_int32), ("num_envs", C.c_int32),
                ("hidden", C.c_int32), ("activation", C.c_int32), ("env_id_offset", C.c_int32),
                ("seed_lo", C.c_uint32), ("seed_hi", C.c_uint32), ("precision", C.c_int32), ("reserved", C.c_int32)]


GR_POLICY_ACT_LRELU, GR_POLICY_ACT_ELU = 0, 1
GR_POLICY_BF16, GR_POLICY_FP32 = 0, 1
GR_POLICY_LRELU_PRESCALE = 0.505
GR_CAM_STEP, GR_CAM_RESET, GR_CAM_OBSERVE = 0, 1, 2
GR_DTYPE_F32, GR_DTYPE_BF16 = 0, 1
GR_STEP_L2, GR_STEP_LDS, GR_STEP_LDS8, GR_STEP_LDS8_LEAN, GR_STEP_OBST, GR_STEP_OBST_LEAN = range(6)
STEP_KERNEL_NAMES = ["step_kernel<false, false>", "step_kernel<true, false>", "step_kernel<true, false, 8>",
                     "step_kernel<true, false, 8, 1>", "step_kernel<false, true>", "step_kernel<false, true, 0, 1>"]
GR_STATUS_OBST_WAIT_TIMEOUT = 1
GR_ERR_CAPACITY = -4
GR_FAULT_NONE, GR_FAULT_OBST_NO_SIGNAL = 0, 1
STATUS_TEXT = {GR_STATUS_OBST_WAIT_TIMEOUT: "a physics wave gave up waiting for its obstacle mask (stale mask used)"}

EXPORTS = [
    "gr_abi_version", "gr_source_sha256", "gr_config_default", "gr_config_size", "gr_create", "gr_destroy", "gr_last_error",
    "gr_num_blocks", "gr_num_log_rows", "gr_log_finalize", "gr_bytes_per_env_step", "gr_bind_tracks", "gr_bind_obstacles", "gr_swap_terrain", "gr_bind_buffers", "gr_bind_obs_sink", "gr_init", "gr_reset",
    "gr_step", "gr_observe", "gr_device_status", "gr_test_inject_fault", "gr_test_camera_slots", "gr_set_timing", "gr_read_timing", "gr_test_dynamics", "gr_test_math",
    "gr_test_philox",
    "gr_debug_read_stamps", "gr_debug_read_policy_stamps",
    "gr_camera_config_default", "gr_camera_config_size", "gr_enable_camera", "gr_bind_camera_buffers",
    "gr_camera_render", "gr_camera_bytes_per_env", "gr_policy_forward", "gr_policy_args_size", "gr_column_sum_partials", "gr_column_sum",
    "gr_head_partials", "gr_head_forward", "gr_head_backward", "gr_mlp_in_partials", "gr_mlp_in_forward",
    "gr_mlp_in_backward", "gr_ppo_loss_partials", "gr_ppo_loss_forward", "gr_ppo_loss_backward",
    "gr_adam_prepare", "gr_adam_clip", "gr_adam_step", "gr_adam_clip_step", "gr_ppo_loss_forward_backward",
    "gr_store_transition", "gr_episode_accumulate", "gr_gae", "gr_l2c2_mix",
    "gr_ppo_loss_forward_loss", "gr_ppo_loss_backward_loss", "gr_adaptive_lr",
    "gr_bn_scratch_doubles", "gr_bn_act_forward", "gr_bn_act_backward", "gr_stem1_scratch_doubles",
    "gr_stem1_forward", "gr_stem1_backward", "gr_mlp_partials", "gr_mlp_forward", "gr_mlp_backward",
    "gr_mlp_args_size", "gr_step_kernel_variant", "gr_terrain_reserve", "gr_terrain_stage", "gr_terrain_commit",
    "gr_terrain_epoch", "gr_mlp_h1mask_words", "gr_stem12_backward", "gr_stem12_forward",
    "gr_patch_wgrad_floats", "gr_patch_wgrad", "gr_bn_running_update", "gr_tsgemm", "gr_l2c2_mix_rows", "gr_tsgemm_bnact",
    "gr_patch_wgrad_bnact", "gr_bn_stats", "gr_stem12_backward_w2_scratch_doubles", "gr_stem12_backward_w2",
]

_lib = None


def _declare(lib):
    vp = C.c_void_p
    sig = {
        "gr_abi_version": (C.c_int, []),
        "gr_config_default": (C.c_int, [C.POINTER(GrConfig)]),
        "gr_config_size": (C.c_size_t, []),
        "gr_create": (C.c_int, [C.POINTER(GrConfig), C.POINTER(vp)]),
        "gr_destroy": (C.c_int, [vp]),
        "gr_last_error": (C.c_char_p, [vp]),
        "gr_num_blocks": (C.c_int, [vp]),
        "gr_num_log_rows": (C.c_int, [vp]),
        "gr_log_finalize": (C.c_int, [vp, vp, vp, vp, vp]),
        "gr_bytes_per_env_step": (C.c_int, [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "gr_bind_tracks": (C.c_int, [vp, vp, vp]),
        "gr_bind_obstacles": (C.c_int, [vp, C.POINTER(GrObstacles)]),
        "gr_swap_terrain": (C.c_int, [vp, vp, vp, vp, C.POINTER(GrObstacles), C.POINTER(GrObstacles), vp]),
        "gr_terrain_reserve": (C.c_int, [vp, C.c_int32, C.c_int32, C.c_int32]),
        "gr_terrain_stage": (C.c_int, [vp, vp, vp, C.POINTER(GrObstacles), vp]),
        "gr_terrain_commit": (C.c_int, [vp, vp]),
        "gr_terrain_epoch": (C.c_int64, [vp]),
        "gr_mlp_h1mask_words": (C.c_int64, [C.c_int64, C.c_int32]),
        "gr_bind_buffers": (C.c_int, [vp, C.POINTER(GrBuffers)]),
        "gr_bind_obs_sink": (C.c_int, [vp, vp, vp, C.c_int]),
        "gr_init": (C.c_int, [vp, vp]),
        "gr_reset": (C.c_int, [vp, vp, vp]),
        "gr_step": (C.c_int, [vp, vp, vp]),
        "gr_observe": (C.c_int, [vp, vp]),
        "gr_step_kernel_variant": (C.c_int, [vp]),
        "gr_device_status": (C.c_int, [vp, C.POINTER(C.c_uint32), C.c_int, vp]),
        "gr_source_sha256": (C.c_char_p, []),
        "gr_test_inject_fault": (C.c_int, [vp, C.c_int]),
        "gr_test_camera_slots": (C.c_int, [vp, C.c_int32]),
        "gr_set_timing": (C.c_int, [vp, C.c_int]),
        "gr_read_timing": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
        "gr_test_dynamics": (C.c_int, [vp, C.c_int, C.c_int] + [vp] * 9 + [vp]),
        "gr_test_math": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, vp, vp]),
        "gr_test_philox": (C.c_int, [vp, C.c_int] + [C.c_uint32] * 4 + [vp, vp]),
        "gr_debug_read_stamps": (C.c_int, [vp, C.c_int]),
        "gr_debug_read_policy_stamps": (C.c_int, [vp, C.c_int]),
        "gr_camera_config_default": (C.c_int, [C.POINTER(GrCameraConfig)]),
        "gr_camera_config_size": (C.c_size_t, []),
        "gr_enable_camera": (C.c_int, [vp, C.POINTER(GrCameraConfig)]),
        "gr_bind_camera_buffers": (C.c_int, [vp, C.POINTER(GrCameraBuffers)]),
        "gr_camera_render": (C.c_int, [vp, C.c_int, vp, vp]),
        "gr_camera_bytes_per_env": (C.c_int, [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "gr_policy_forward": (C.c_int, [C.POINTER(GrPolicyArgs), vp]),
        "gr_policy_args_size": (C.c_size_t, []),
        "gr_column_sum_partials": (C.c_int, [C.c_int64]),
        "gr_column_sum": (C.c_int, [vp, C.c_int, C.c_int64, C.c_int32, vp, vp, vp]),
        "gr_head_partials": (C.c_int64, [C.c_int64, C.c_int32, C.c_int32]),
        "gr_head_forward": (C.c_int, [vp, C.c_int64, C.c_int32, vp, vp, C.c_int32, C.c_float, vp, vp]),
        "gr_head_backward": (C.c_int, [vp, vp, C.c_int64, C.c_int32, vp, C.c_int32, C.c_float, vp, vp, vp, vp]),
        "gr_mlp_in_partials": (C.c_int64, [C.c_int64, C.c_int32, C.c_int32]),
        "gr_ppo_loss_partials": (C.c_int64, [C.c_int64]),
        "gr_adam_prepare": (C.c_int, [vp, C.c_int32, vp]),
        "gr_store_transition": (C.c_int, [vp, vp]),
        "gr_ppo_loss_forward_loss": (C.c_int, [vp, vp, vp, C.c_float, vp, vp, vp, vp, vp]),
        "gr_ppo_loss_backward_loss": (C.c_int, [vp, vp, C.c_float, vp, vp, vp, vp, vp]),
        "gr_adaptive_lr": (C.c_int, [vp, vp, C.c_double, C.c_double, C.c_double, vp]),
        "gr_episode_accumulate": (C.c_int, [C.c_int64, vp, vp, C.c_int32, vp, vp, vp, vp, vp, vp]),
        "gr_gae": (C.c_int, [C.c_int64, C.c_int32, C.c_float, C.c_float, vp, vp, vp, vp, C.c_int64, vp, vp, vp]),
        "gr_l2c2_mix": (C.c_int, [vp, vp, vp, C.c_int64, C.c_int32, vp, vp]),
        "gr_l2c2_mix_rows": (C.c_int, [vp, vp, C.c_int64, vp, vp, vp, C.c_int64, C.c_int32, vp, vp]),
        "gr_tsgemm_bnact": (C.c_int, [vp, C.c_int64, vp, vp, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp,
                                      vp, vp, C.c_int32, C.c_float, vp]),
        "gr_patch_wgrad_bnact": (C.c_int, [vp, C.c_int64, vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, C.c_int32, vp,
                                           vp, vp, C.c_int32, C.c_float, vp]),
        "gr_bn_stats": (C.c_int, [vp, C.c_int64, C.c_int32, C.c_float, vp, vp, vp]),
        "gr_adam_clip": (C.c_int, [vp, C.c_float, vp, vp]),
        "gr_adam_step": (C.c_int, [vp, vp]),
        "gr_adam_clip_step": (C.c_int, [vp, C.c_float, vp, vp, vp, C.c_double, C.c_double, C.c_double, vp]),
        "gr_ppo_loss_forward_backward": (C.c_int, [vp, vp, C.c_float, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "gr_ppo_loss_forward": (C.c_int, [vp, vp, vp, vp]),
        "gr_ppo_loss_backward": (C.c_int, [vp, vp, vp, vp, vp, vp, vp]),
        "gr_mlp_in_forward": (C.c_int, [vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, C.c_int32, C.c_float, vp, vp]),
        "gr_mlp_in_backward": (C.c_int, [vp, vp, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_float, vp, vp,
                                         vp]),
        "gr_mlp_partials": (C.c_int64, [C.c_int64, C.c_int32, C.c_int32]),
        "gr_mlp_forward": (C.c_int, [vp, vp]),
        "gr_mlp_backward": (C.c_int, [vp, vp]),
        "gr_mlp_args_size": (C.c_size_t, []),
        "gr_bn_scratch_doubles": (C.c_int64, [C.c_int64, C.c_int32]),
        "gr_bn_act_forward": (C.c_int, [vp, C.c_int64, C.c_int32, vp, vp, C.c_float, C.c_int32, C.c_float, vp, vp, vp,
                                        vp]),
        "gr_bn_act_backward": (C.c_int, [vp, vp, C.c_int64, C.c_int32, vp, vp, vp, C.c_int32, C.c_float, vp, vp, vp,
                                         vp, vp]),
        "gr_stem1_scratch_doubles": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
        "gr_stem1_forward": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int32, vp, C.c_int32, C.c_int32, vp, C.c_int32,
                                       vp, vp, C.c_float, C.c_int32, C.c_float, vp, C.c_int64, vp, vp, vp]),
        "gr_stem1_backward": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int32, vp, C.c_int32, C.c_int32, vp, C.c_int32,
                                        vp, vp, vp, C.c_int32, C.c_float, vp, C.c_int64, vp, vp, vp, vp, vp]),
        "gr_patch_wgrad_floats": (C.c_int64, [C.c_int64, C.c_int32, C.c_int32]),
        "gr_patch_wgrad": (C.c_int, [vp, C.c_int64, vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp]),
        "gr_bn_running_update": (C.c_int, [vp, vp, vp, vp, C.c_int32, C.c_float, C.c_float, C.c_int32, C.c_int32, vp]),
        "gr_tsgemm": (C.c_int, [vp, C.c_int64, vp, C.c_int32, vp, C.c_int64, C.c_int64, C.c_int32, C.c_int32, vp]),
        "gr_stem12_forward": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int32, vp, C.c_int32, C.c_int32, vp, C.c_int32,
                                        vp, vp, C.c_float, C.c_int32, C.c_float, vp, C.c_int32, vp, vp, vp, vp, vp, vp]),
        "gr_stem12_backward": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int32, vp, C.c_int32, C.c_int32, vp, C.c_int32,
                                         vp, vp, vp, C.c_int32, C.c_float, vp, C.c_int32, vp, vp, vp, vp, vp, vp]),
        "gr_stem12_backward_w2_scratch_doubles": (C.c_int64, [C.c_int32]),
        "gr_stem12_backward_w2": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int32, vp, C.c_int32, C.c_int32, vp,
                                            C.c_int32, vp, vp, vp, vp, C.c_int32, C.c_float, vp, C.c_int32, vp, vp, vp,
                                            vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name) and os.environ.get("GR_LIB_PATH"):
            continue  # an older timing build (GR_LIB_PATH) may predate an entry point
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def tree_source_sha256() -> str | None:
    """The SHA-256 gr_source_sha256() reports for a library built from this tree's sources: csrc/Makefile's SRCS then
    HDRS, in its order, concatenated (None when the sources are not here)."""
    import hashlib

    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    mk = os.path.join(csrc, "Makefile")
    if not os.path.exists(mk):
        return None
    lists = {}
    for line in open(mk):
        for var in ("SRCS", "HDRS"):
            if line.startswith(var + " :="):
                lists[var] = line.split(":=", 1)[1].split()
    h = hashlib.sha256()
    for f in lists.get("SRCS", []) + lists.get("HDRS", []):
        path = os.path.normpath(os.path.join(csrc, f.replace("$(HERE)", "")))
        if not os.path.exists(path):
            return None
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def load(path: str | None = None):
    """Load libgr.so (the HIP step).  Raises if it is missing: no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("GR_LIB_PATH") or LIB_PATH  # override: timing-only ablation builds
    if not os.path.exists(p):
        raise RuntimeError(
            f"libgr.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C generalizableracing_amd/csrc`.  The racing env has no CPU fallback."
        )
    lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
    _declare(lib)
    if lib.gr_abi_version() != GR_ABI_VERSION:
        raise RuntimeError(f"libgr.so ABI {lib.gr_abi_version()} != expected {GR_ABI_VERSION}")
    if lib.gr_config_size() != C.sizeof(GrConfig):
        raise RuntimeError(f"gr_config size mismatch: C {lib.gr_config_size()} vs ctypes {C.sizeof(GrConfig)}")
    if lib.gr_camera_config_size() != C.sizeof(GrCameraConfig):
        raise RuntimeError("gr_camera_config size mismatch between libgr.so and the ctypes mirror")
    if lib.gr_policy_args_size() != C.sizeof(GrPolicyArgs):
        raise RuntimeError(f"gr_policy_args size mismatch: C {lib.gr_policy_args_size()} vs ctypes "
                           f"{C.sizeof(GrPolicyArgs)}")
    if hasattr(lib, "gr_mlp_args_size"):
        from .rsl_rl.linear import GrMlpArgs

        if lib.gr_mlp_args_size() != C.sizeof(GrMlpArgs):
            raise RuntimeError("gr_mlp_args size mismatch between libgr.so and the ctypes mirror")
    if path is None:
        _lib = lib
    return lib


def default_config() -> GrConfig:
    cfg = GrConfig()
    rc = load().gr_config_default(C.byref(cfg))
    if rc != 0:
        raise RuntimeError("gr_config_default failed")
    return cfg


def default_camera_config() -> GrCameraConfig:
    cfg = GrCameraConfig()
    rc = load().gr_camera_config_default(C.byref(cfg))
    if rc != 0:
        raise RuntimeError("gr_camera_config_default failed")
    return cfg


def check(lib, ctx, rc: int, what: str):
    if rc != 0:
        msg = lib.gr_last_error(ctx) if ctx else b""
        raise RuntimeError(f"{what} failed (status {rc}): {msg.decode() if msg else ''}")


_RAW_STREAM = None


def raw_stream(device) -> int:
    """The raw handle of `device`'s current HIP stream for the C ABI's `stream` argument: torch's accessor when the
    device has an index (torch.cuda.current_stream(device) builds a Stream object under a device guard per call)."""
    global _RAW_STREAM
    import torch

    if _RAW_STREAM is None:
        _RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", False)
    index = device.index if isinstance(device, torch.device) else None
    if _RAW_STREAM and index is not None:
        return _RAW_STREAM(index)
    return torch.cuda.current_stream(device).cuda_stream
