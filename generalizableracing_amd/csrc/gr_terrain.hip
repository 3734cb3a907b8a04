// gr_terrain.hip — gr_terrain_commit's kernel (include/gr.h "Resident terrain").
//
// The periodic terrain regeneration (EventCfg.reset_terrain -> reset_terrain_period, .../quadcopter_diff/mdp/
// events.py:180-204) makes a new generation of tracks live between two steps.  The generation was validated and
// uploaded ahead into the context's staging block (gr_terrain_stage, on a side stream, while the env stepped); here,
// in one launch on the env's stream, with arguments that never change (so the interval step is graph-capturable):
//   1. the packed gate table: [track][max_gates * GR_GATE_FLOATS | GR_TRACK_FLOATS] from the staged gates and
//      track records (what pack_tracks' two 2-D copies do for gr_bind_tracks / gr_swap_terrain);
//   2. the obstacle block [records | counts | grid_f | grid_i | cells | items] staging -> live, through the last
//      staged item (the extent is the staged header's first word: the generation's item count varies);
//   3. the per-env obstacle hints (state plane GR_P_OHINT) cleared: they index the previous generation's cells.
// HBM-bound copy: ~2 MB records + ~0.2 MB cells + ~4 MB items + 1 MB hints at 65 536 envs (the 8-gate obstacle
// tracks); float4 loads / stores, grid-stride.
#include <hip/hip_runtime.h>

#include "gr_kernels.h"

namespace gr {

__global__ __launch_bounds__(256) void terrain_commit_kernel(TerrainCommitArgs a) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nt = (long long)gridDim.x * blockDim.x;
  const long long ntab = (long long)a.ntr * a.stride4;
  for (long long q = tid; q < ntab; q += nt) {
    const int t = (int)(q / a.stride4), o = (int)(q % a.stride4);
    a.table[q] = o < a.g4 ? a.s_gates[(long long)t * a.g4 + o] : a.s_tracks[t];
  }
  if (a.l_obst) {
    long long nob = a.hdr[0];
    nob = nob < a.max_obst4 ? nob : a.max_obst4;
    for (long long q = tid; q < nob; q += nt) a.l_obst[q] = a.s_obst[q];
  }
  if (a.hints) {
    for (long long q = tid; q < a.n_hints; q += nt) a.hints[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

hipError_t launch_terrain_commit(const TerrainCommitArgs& a, hipStream_t s) {
  // the grid from the capacities only (a graph replay launches the same grid for any staged generation)
  long long work = (long long)a.ntr * a.stride4;
  if (a.max_obst4 > work) work = a.max_obst4;
  if (a.n_hints > work) work = a.n_hints;
  long long blocks = (work + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  hipLaunchKernelGGL(terrain_commit_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace gr
