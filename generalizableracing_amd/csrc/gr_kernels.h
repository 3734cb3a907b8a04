// gr_kernels.h — kernel argument block and launchers (internal to libgr.so).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gr.h"

#define GR_BLOCK 256
#define GR_MAX_TYPES 64

namespace gr {

enum { KMODE_STEP = 0, KMODE_RESET = 1, KMODE_OBSERVE = 2 };

// Passed by value (kernarg segment -> scalar registers).  Everything derived
// from the config that would otherwise be recomputed per lane lives here.
struct KArgs {
  gr_config cfg;
  gr_buffers buf;
  const float* table;  // packed track table [T*L][track_stride]
  int track_stride;    // floats per track: max_gates*GR_GATE_FLOATS + GR_TRACK_FLOATS
  int lds_bytes;       // dynamic LDS per workgroup (0: read the table from global memory)
  int type_start[GR_MAX_TYPES + 1];
  float thrust_lo, thrust_hi;  // 4 * f(omega_min/max), controller_diff.py:96-99
  float lat_reach;             // > max |lattice offset|: ground-test cull radius
  float w[7];                  // reward weights in RewardsCfg order
  // motor model (controller_diff.py:140-144, thrust_controller_diff.py)
  float B[4][4], Bi[4][4];
  float motor_fmax, motor_c;
  float tm_k2, tm_k1, tm_k0, tm_k1sq, tm_4k2, tm_inv2k2, tm_negk1;
};

hipError_t launch_env(int mode, const KArgs& a, const float* actions, const uint8_t* mask, hipStream_t s,
                      hipEvent_t t0, hipEvent_t t1);
hipError_t launch_init(const KArgs& a, hipStream_t s);
hipError_t launch_log_finalize(const float* rows, int nrows, const float* prev, float* out, float ep_len_s,
                               float num_envs, hipStream_t s);
hipError_t launch_test_dynamics(const KArgs& a, int n, int mode, const float* si, const float* ab, const float* cmd,
                                const float* ci, const float* par, const float* drag, float* so, float* co, float* xo,
                                hipStream_t s);
hipError_t launch_test_math(int fn, int n, const float* x, const float* y, float* out, hipStream_t s);
hipError_t launch_test_philox(int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                              uint32_t* out, hipStream_t s);

}  // namespace gr
