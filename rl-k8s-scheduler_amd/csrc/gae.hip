// gae.hip — K3: advantages / value targets (RLlib compute_advantages, use_gae=True, restated).
//
// The reference calls RLlib PPO (train_ppo.py:9-23, gamma=0.99 :19; train_final.py:16 0.995;
// lambda default 1.0).  RLlib computes, per trajectory fragment,
//   delta_t = r_t + gamma*V_{t+1} - V_t ; A = discount_cumsum(delta, gamma*lambda) ; vt = A + V
// with V_{T} = 0 after a terminal step and V(s_T) when the fragment is cut.  Over a time-major
// [T][N] rollout with auto-reset lanes this is the reverse recurrence below (one lane per env,
// coalesced across lanes at every t).  HBM-bound: 17 B per env-step (r, V, done in; A, vt out).
#include <hip/hip_runtime.h>

#include "rlks_internal.h"

namespace rlks {

constexpr int GAE_BLOCK = 256;

__global__ __launch_bounds__(GAE_BLOCK) void k_gae(const float* __restrict__ r, const float* __restrict__ v,
                                                   const uint8_t* __restrict__ d, float gamma, float gl,
                                                   int T, int N, float* __restrict__ adv,
                                                   float* __restrict__ vt, double* __restrict__ partials) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (n < N) {
    float a = 0.f;
    float vnext = v[(size_t)T * N + n];
#pragma unroll 4
    for (int t = T - 1; t >= 0; --t) {
      const size_t i = (size_t)t * N + n;
      const float vt_ = v[i];
      const float nd = d[i] ? 0.f : 1.f;
      const float delta = r[i] + gamma * vnext * nd - vt_;
      a = delta + gl * nd * a;
      adv[i] = a;
      vt[i] = a + vt_;
      vnext = vt_;
      s1 += (double)a;
      s2 += (double)a * (double)a;
    }
  }
  if (!partials) return;
  __shared__ double sh[2][GAE_BLOCK / 64];
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[0][w] = s1; sh[1][w] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a1 = 0.0, a2 = 0.0;
    for (int i = 0; i < GAE_BLOCK / 64; ++i) { a1 += sh[0][i]; a2 += sh[1][i]; }
    partials[2 * blockIdx.x] = a1;
    partials[2 * blockIdx.x + 1] = a2;
  }
}

__global__ void k_adv_stats(const double* __restrict__ p, int n, double count, double* __restrict__ out) {
  __shared__ double s1[256], s2[256];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) { a += p[2 * i]; b += p[2 * i + 1]; }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) { s1[threadIdx.x] += s1[threadIdx.x + o]; s2[threadIdx.x] += s2[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = s1[0]; out[1] = s2[0]; out[2] = count; }
}

// RLlib standardize_fields: (x - mean) / max(1e-4, std), numpy std (ddof = 0)
__global__ void k_adv_finalize(const double* __restrict__ s, float* __restrict__ dyn) {
  if (threadIdx.x != 0) return;
  const double n = s[2] > 0 ? s[2] : 1.0;
  const double mean = s[0] / n;
  double var = s[1] / n - mean * mean;
  if (var < 0) var = 0;
  double sd = sqrt(var);
  if (sd < 1e-4) sd = 1e-4;
  dyn[RLKS_DYN_ADV_MEAN] = (float)mean;
  dyn[RLKS_DYN_ADV_INVSTD] = (float)(1.0 / sd);
}

}  // namespace rlks

using namespace rlks;

extern "C" {

int rlks_gae_partials_count(int N) { return (int)cdiv(N, GAE_BLOCK); }

int rlks_gae(const float* rewards, const float* values, const uint8_t* dones, float gamma, float lam, int T,
             int N, float* adv, float* vtarg, double* partials, void* stream) {
  RLKS_REQUIRE(rewards && values && dones && adv && vtarg, RLKS_ERR_ARG, "rlks_gae: null argument");
  RLKS_REQUIRE(T > 0 && N > 0, RLKS_ERR_ARG, "rlks_gae: T and N must be positive");
  hipLaunchKernelGGL(k_gae, dim3(cdiv(N, GAE_BLOCK)), dim3(GAE_BLOCK), 0, (hipStream_t)stream, rewards, values,
                     dones, gamma, gamma * lam, T, N, adv, vtarg, partials);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_adv_stats(const double* partials, int n, double count, double* sums, void* stream) {
  RLKS_REQUIRE(partials && sums && n > 0, RLKS_ERR_ARG, "rlks_adv_stats: bad argument");
  hipLaunchKernelGGL(k_adv_stats, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, n, count, sums);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_adv_finalize(const double* sums, float* dyn, void* stream) {
  RLKS_REQUIRE(sums && dyn, RLKS_ERR_ARG, "rlks_adv_finalize: null argument");
  hipLaunchKernelGGL(k_adv_finalize, dim3(1), dim3(64), 0, (hipStream_t)stream, sums, dyn);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

}  // extern "C"
