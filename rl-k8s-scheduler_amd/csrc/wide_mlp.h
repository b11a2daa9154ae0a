// wide_mlp.h — the generic-width PPO MLP path (wide_mlp.hip) over the split-fp16 GEMM.
#pragma once

#include "mlp_common.h"

namespace rlks {

struct WideNet {
  _Float16 *h1h, *h1l;          // H1 as fp16 planes [M][H] at 2^14 (the pre-split GEMMs' operand)
  float *h2, *out, *dout;       // [M][H], [M][A_net], [M][A_net]
  _Float16 *w2h, *w2l;          // W2 planes [H][H] (this SGD step's / forward's weights)
  _Float16 *w1h, *w1l;          // W1 planes [H][D] (obs_dim D a multiple of 32: Z1 on the pre-split GEMM)
  unsigned* slots;              // operand max |x| slots
  float* part_stat;             // [blocks][4]
};
struct WideWs {
  WideNet n[2];
  float* dzb;  // [M][H] dZ1 (dZ2 goes straight to the dzh / dzl planes)
  _Float16 *dzh, *dzl;  // dZ2 planes [M][H]
  _Float16 *xh, *xl;    // X planes [M][D] (obs_dim D a multiple of 32)
  double* rew64;     // [M] env-step scratch (rollout)
  float* part;       // split-K / split column-sum partials of the weight gradients
  unsigned* stat_slots;
  int64_t bytes;
  int M, blocks;
};

bool wide_needed(const rlks_mlp_desc* d);
WideWs wide_ws_layout(int D, int H, int A, int M, char* base);
int wide_forward(const rlks_mlp_desc* d, const float* params, const float* x, int ldx, int M, const WideWs& w,
                 float* logits, float* values, hipStream_t s);
int wide_grad(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
              const float* mb, int M, float* grad, double* stats, const WideWs& w, hipStream_t s);
// TorchCategorical over [N][A] logits (Philox sample, or argmax when explore == 0) -> actions, logp
int launch_sample(const EnvView& v, const float* logits, int A, int explore, int32_t* actions, float* logp,
                  hipStream_t s);
int wide_rollout(rlks_env* env, const rlks_mlp_desc* d, const float* params, const rlks_rollout_bufs* b, int explore,
                 const WideWs& w, hipStream_t s);

}  // namespace rlks
