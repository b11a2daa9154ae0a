// sgd_sf16.h — argument blocks and launchers of the split-fp16 SGD-step kernels (sgd_sf16.hip).
#pragma once

#include "mlp_common.h"

namespace rlks {
constexpr int SF_F1_W = 8;    // waves per F1a / F1b workgroup (two workgroups per CU); 16 rows each
constexpr int SF_F1F_W = 16;  // waves per fused-F1 (k_sf_f1) workgroup: one workgroup per CU (sgd_sf16.hip)
constexpr int SF_FWD_W = 8;   // waves per rollout-forward (k_sf_fwd16) workgroup (two per CU)
constexpr int SF_PMAX = 1024;       // weight-max entries per (parity, kind)
constexpr int SF_W2_PSTRIDE = 256 * 256;  // floats between F2's dW2 partials (padding them apart: no gain)
}  // namespace rlks

#include <hip/hip_ext.h>

namespace rlks {

// In-pipeline kernel timing (rlks_ppo_grad_profile): while a profile runs, the SGD step's kernels are
// launched through hipExtLaunchKernelGGL with a start / stop event pair each (the events bracket the
// kernel itself, as rocprofv3's kernel trace does, not the launch gaps); null otherwise.
enum { KEV_SPLIT, KEV_F1A, KEV_F1B, KEV_F2, KEV_REDUCE, KEV_N };
extern hipEvent_t* g_kernel_events;  // [2 KEV_N]: start, stop per kernel
template <typename K, typename... Args>
inline void launch_timed(int idx, K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
  if (g_kernel_events)
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, g_kernel_events[2 * idx], g_kernel_events[2 * idx + 1], 0u,
                          args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}

struct SfNetW {
  const float *w1, *b1, *w2;
  _Float16 *w1h, *w1l, *w2ph, *w2pl, *w2th, *w2tl;
  _Float16 *w2rh, *w2rl;  // rollout: w2p in wave-fragment order [q 4][kt 8][s 2][i 2][64 lanes][8]
  float* sc;          // [8]: s_w1, 1/s_w1, s_w2, 1/s_w2, e_w1, e_w2
  float* pmax;        // [2 parity][2 kind: W2, W1a][SF_PMAX] per-block max |w| (k_sf_wmax: entries
                      // 0..15 of each kind; the fused reduce: one entry per reduce block)
  unsigned* tag;      // [2 parity]: the Adam step whose fused reduce filled pmax[parity] (0: none)
};
// parity: which half of pmax holds this prep's maxima; the split zeroes the other half, which the
// fused reduce + Adam of the coming SGD step fills (one entry per reduce block, no atomics) for the
// next prep.  skip_wmax: the maxima are already there (the previous SGD step was fused).
struct SfPrepArgs {
  SfNetW n[2];
  int D, KD;
  int parity, skip_wmax, write_roll;
  unsigned expect_tag;  // skip_wmax: pmax[parity] is valid only if tag[parity] == expect_tag; else
                        // every split block scans the weights for their maxima itself
};

struct SfNet {
  const float *b2, *w3, *b3;
  const _Float16 *w1h, *w1l, *w2ph, *w2pl, *w2th, *w2tl;
  const float* sc;
  _Float16* dz2s;  // [M/16 tiles][8 n-steps][hi, lo][64 lanes][8]: dZ2 of each 16-row tile split at
                  // 2^tile_edz, in F1a's lane order (sgd_sf16.hip F1)
  int* tile_edz;  // [M/16]: each 16-row tile's dZ2 split exponent (F1a -> F1b, F2)
  int* tile_ex;   // [M/16]: each 16-row tile's X split exponent (F1a -> F2)
  float *part_w1, *part_b1;                 // [F1 blocks of 128 rows][...] (F1b)
  float *part_w3, *part_b3, *part_stat;     // [sf_f1a_parts][...] (F1a)
  float *part_w2, *part_b2;                                   // [splits][...]
};
struct SfArgs {
  SfNet n[2];
  const float* x;
  int x_stride, M, D, A_pi;
  int tiles_per_split;
  int net0;  // F1: first net of the grid (blockIdx.y + net0)
  int products;  // MFMA products per split product: 1 = RLKS_PRECISION_F16 (hi hi), else 3 (fp32-accurate)
  _Float16* xsp;  // [2 hi, lo][M][KD]: Xa = [X | 1 | 0] of every row split by F1a at its 16-row tile's
                  // exponent and sign (tile_ex, tile_sign), written by the policy net's F1a, read by F2
  rlks_ppo_coeffs co;
  const float* dyn;
};

// rollout step on split-fp16 (rollout_sf16.hip): both nets' forward + sample + env step
struct SfRollNet {
  const _Float16 *w1h, *w1l, *w2rh, *w2rl;
  const float *b2, *w3, *b3;
  const float* sc;
};
struct SfRollArgs {
  SfRollNet n[2];
  float* x;        // FWD_ONLY: [M][D] observations; FWD_ROLLOUT: obs [T+1][M][D] (obs[0] read)
  int M, D, A, T;  // T: rollout steps (FWD_ROLLOUT); buffers below are time-major [T(+1)][M]
  float* logits;   // [(T)][M][A] or null
  float* values;   // [(T+1)][M] or null
  // FWD_ROLLOUT: sample, step the env lane m = row m
  EnvView env;
  const double* tab_cost;
  const double* tab_lat;
  int explore;
  float* obs_next;
  float* logp;
  int32_t* actions;
  float* rewards;
  uint8_t* dones;
};
int launch_sf_roll(const SfRollArgs& a, int mode, hipStream_t s);

// forward of both nets on 16-row tiles (sgd_sf16.hip k_sf_fwd16): out[0] = logits [M][A] (or null:
// the value net alone), out[1] = values [M] (or null)
struct SfFwdArgs {
  SfNet n[2];  // weights: w1h/w1l, w2ph/w2pl, sc, b2, w3, b3
  const float* x;  // [M][D] observations
  int M, D, net0;
  float* out[2];
};
int launch_sf_fwd16(const SfFwdArgs& a, int A, hipStream_t s);

int sf_kd(int D);
int launch_sf_prep(const SfPrepArgs& a, hipStream_t s);
// halves: 1 = F1a (k_sf_fwd), 2 = F1b (k_sf_bwd), 3 = both, SF_F1_FUSED = the fused kernel (k_sf_f1)
constexpr int SF_F1_FUSED = 7;
int launch_sf_f1(const SfArgs& a, int net0, int nets, int A, hipStream_t s, int halves = 3);  // needs M % 256 == 0
int launch_sf_dw2(const SfArgs& a, int splits, hipStream_t s);
// whether F2 is k_sf_dw2r (H1 in registers; its dW2 partials in [k / 4][n][4] order, the default)
// rather than round 3-5's k_sf_dw2 ([n][k] partials; RLKS_F2_IMAGE=1, kept for same-box A/B runs)
bool sf_f2_regs();
// F1's partials per net (one per F1 workgroup): dW1 / db1, and dW3 / db3 / stats; the workspace holds
// the split kernels' count (the larger), the fused kernel writes half as many
int sf_f1_parts(int M, bool fused);
// whether a whole gradient (part 0: one rank, or the multi-rank step's one-bucket form) runs the fused
// F1 kernel at A actions: by default up to 4 actions; RLKS_F1_FUSED=1 / RLKS_F1_SPLIT=1 force it
// 
bool sf_f1_fused(int A);

}  // namespace rlks
