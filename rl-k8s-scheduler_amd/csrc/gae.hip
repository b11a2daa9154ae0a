// gae.hip — K3: advantages / value targets (RLlib compute_advantages, use_gae=True, restated).
//
// The reference calls RLlib PPO (train_ppo.py:9-23, gamma=0.99 :19; train_final.py:16 0.995;
// lambda default 1.0).  RLlib computes, per trajectory fragment,
//   delta_t = r_t + gamma*V_{t+1} - V_t ; A = discount_cumsum(delta, gamma*lambda) ; vt = A + V
// with V_{T} = 0 after a terminal step and V(s_T) when the fragment is cut.  Over a time-major
// [T][N] rollout with auto-reset lanes this is the first-order linear recurrence
//   a_t = delta_t + c_t a_{t+1},  c_t = gamma lambda (1 - done_t),  a_T = 0,
// computed as a reverse scan over time (k_gae_scan); rollouts longer than 256 steps (c1: one lane,
// 4,000 steps) use the serial per-lane recurrence (k_gae).  HBM-bound: 17 B per env-step (r, V,
// done in; A, vt out).
#include <hip/hip_runtime.h>

#include "rlks_internal.h"

namespace rlks {

constexpr int GAE_BLOCK = 256;
// 64 lanes (256-byte rows) per scan workgroup: 128 x 131,072 (c4) in 56 us vs 68 us at 32 lanes,
// 128 x 4,096 (c2) in 6.1 vs 5.5 us
constexpr int GAE_LANES = 64;       // lanes per advantage-sum partial (and per scan workgroup)
constexpr int GAE_SERIAL_T = 256;   // longer rollouts (c1's single 4,000-step lane) run the serial recurrence
constexpr int GAE_MAX_SEG = 16;  // time segments per scan workgroup

// per-partial (GAE_LANES-lane group) sums of a and a^2: scan workgroups are one group (thread =
// (lane, segment)); the serial kernel's blocks hold GAE_BLOCK / GAE_LANES groups
__device__ __forceinline__ void gae_partials(double s1, double s2, double* __restrict__ partials, int group,
                                             int n_groups) {
  __shared__ double sh[2][1024 / GAE_LANES];
#pragma unroll
  for (int o = GAE_LANES / 2; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  const int q = threadIdx.x / GAE_LANES;
  if ((threadIdx.x & (GAE_LANES - 1)) == 0) { sh[0][q] = s1; sh[1][q] = s2; }
  __syncthreads();
  if (group >= 0) {  // scan: all of the workgroup's segments belong to the same lanes
    if (threadIdx.x == 0) {
      double a1 = 0.0, a2 = 0.0;
      for (int i = 0; i < (int)(blockDim.x / GAE_LANES); ++i) { a1 += sh[0][i]; a2 += sh[1][i]; }
      partials[2 * group] = a1;
      partials[2 * group + 1] = a2;
    }
  } else if ((threadIdx.x & (GAE_LANES - 1)) == 0) {  // serial: one group per GAE_LANES threads
    const int g = blockIdx.x * (GAE_BLOCK / GAE_LANES) + q;
    if (g < n_groups) { partials[2 * g] = sh[0][q]; partials[2 * g + 1] = sh[1][q]; }
  }
}

// Reverse scan.  A workgroup owns 32 lanes x W time segments of S consecutive steps (thread =
// (lane, segment); every row it reads or writes is 128 contiguous bytes across the lanes).
// Pass 1: each thread forms its segment's deltas and the affine map a_in -> (A + C a_in) of its S
// steps in registers; the W maps of a lane meet in LDS and one thread per lane composes them from
// the last segment back (W fused multiply-adds); pass 2: each thread replays its segment's
// recurrence from its incoming value and writes A and the value targets.
template <int S>
__global__ __launch_bounds__(1024) void k_gae_scan(
    const float* __restrict__ r, const float* __restrict__ v, const uint8_t* __restrict__ d, float gamma, float gl,
    int T, int N, float* __restrict__ adv, float* __restrict__ vt, double* __restrict__ partials) {
  __shared__ float sA[GAE_MAX_SEG][GAE_LANES], sC[GAE_MAX_SEG][GAE_LANES], sIn[GAE_MAX_SEG][GAE_LANES];
  const int ll = threadIdx.x & (GAE_LANES - 1), seg = threadIdx.x / GAE_LANES, W = blockDim.x / GAE_LANES;
  const int n = blockIdx.x * GAE_LANES + ll, t0 = seg * S;
  const bool live = n < N;
  float dl[S], cc[S], vv[S];
  float A = 0.f, Cm = 1.f;
  if (live) {
    float vnext = v[(size_t)min(t0 + S, T) * N + n];
#pragma unroll
    for (int j = S - 1; j >= 0; --j) {
      const int t = t0 + j;
      dl[j] = 0.f; cc[j] = 1.f; vv[j] = 0.f;
      if (t < T) {
        const size_t i = (size_t)t * N + n;
        const float vt_ = v[i];
        const float nd = d[i] ? 0.f : 1.f;
        dl[j] = r[i] + gamma * vnext * nd - vt_;
        cc[j] = gl * nd;
        vv[j] = vt_;
        A = dl[j] + cc[j] * A;
        Cm = cc[j] * Cm;
        vnext = vt_;
      }
    }
  }
  sA[seg][ll] = A;
  sC[seg][ll] = Cm;
  __syncthreads();
  if (seg == 0) {
    float a_in = 0.f;
    for (int w = W - 1; w >= 0; --w) {
      sIn[w][ll] = a_in;
      a_in = sA[w][ll] + sC[w][ll] * a_in;
    }
  }
  __syncthreads();
  double s1 = 0.0, s2 = 0.0;
  if (live) {
    float a = sIn[seg][ll];
#pragma unroll
    for (int j = S - 1; j >= 0; --j) {
      const int t = t0 + j;
      if (t < T) {
        a = dl[j] + cc[j] * a;
        const size_t i = (size_t)t * N + n;
        adv[i] = a;
        vt[i] = a + vv[j];
        s1 += (double)a;
        s2 += (double)a * (double)a;
      }
    }
  }
  if (partials) gae_partials(s1, s2, partials, blockIdx.x, 0);
}

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
  if (partials) gae_partials(s1, s2, partials, -1, (N + GAE_LANES - 1) / GAE_LANES);
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

int rlks_gae_partials_count(int N) { return (int)cdiv(N, GAE_LANES); }

int rlks_gae(const float* rewards, const float* values, const uint8_t* dones, float gamma, float lam, int T,
             int N, float* adv, float* vtarg, double* partials, void* stream) {
  RLKS_REQUIRE(rewards && values && dones && adv && vtarg, RLKS_ERR_ARG, "rlks_gae: null argument");
  RLKS_REQUIRE(T > 0 && N > 0, RLKS_ERR_ARG, "rlks_gae: T and N must be positive");
  hipStream_t s = (hipStream_t)stream;
  const float gl = gamma * lam;
  if (T > GAE_SERIAL_T) {
    hipLaunchKernelGGL(k_gae, dim3(cdiv(N, GAE_BLOCK)), dim3(GAE_BLOCK), 0, s, rewards, values, dones, gamma, gl, T,
                       N, adv, vtarg, partials);
  } else if (T <= 8 * GAE_MAX_SEG) {
    const unsigned W = cdiv(T, 8);
    hipLaunchKernelGGL(k_gae_scan<8>, dim3(cdiv(N, GAE_LANES)), dim3(GAE_LANES * W), 0, s, rewards, values, dones,
                       gamma, gl, T, N, adv, vtarg, partials);
  } else if (T <= 16 * GAE_MAX_SEG) {
    const unsigned W = cdiv(T, 16);
    hipLaunchKernelGGL(k_gae_scan<16>, dim3(cdiv(N, GAE_LANES)), dim3(GAE_LANES * W), 0, s, rewards, values, dones,
                       gamma, gl, T, N, adv, vtarg, partials);
  } else {
    hipLaunchKernelGGL(k_gae, dim3(cdiv(N, GAE_BLOCK)), dim3(GAE_BLOCK), 0, s, rewards, values, dones, gamma, gl, T,
                       N, adv, vtarg, partials);
  }
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
