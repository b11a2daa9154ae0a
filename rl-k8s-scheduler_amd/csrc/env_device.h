// env_device.h — device side of the K8sMultiCloudEnv lane model (K1), shared by env.hip (the
// step / reset / sample kernels) and rollout.hip (policy forward fused with sample + step).
//
// Reference: /root/reference/rl_scheduler/env/k8s_multi_cloud_env.py
//   _get_live_cpu (:84-88), _get_obs (:90-103), reset (:106-112), step (:115-144).
// Layout: lane state is structure-of-arrays in HBM (int32 step[N], int32 episode[N], f64
// ep_ret[N], ...; MT19937 words as [625][N] so that lane i's word k is coalesced across a wave).
// The [T][C] cost/latency tables are staged in LDS by every workgroup.  Reward arithmetic is f64
// with explicit round-to-nearest multiplies/adds so that 100*(0.6*cost + 0.4*latency) is
// bit-identical to CPython (no FMA contraction).
#pragma once

#include <hip/hip_runtime.h>

#include "rlks_internal.h"

struct rlks_env {
  rlks_env_cfg cfg;
  double span;        // cpu_hi - cpu_lo, computed in f64 exactly as CPython does
  double* d_cost;     // [T][C]
  double* d_lat;      // [T][C]
  int32_t* d_step;    // [N]
  int32_t* d_episode; // [N]
  double* d_ep_ret;   // [N] running return of the current episode
  double* d_ret_sum;  // [N] sum of completed-episode returns since last clear
  int32_t* d_ep_cnt;  // [N] completed episodes since last clear
  uint32_t* d_mt;     // [625][N] (MT19937 mode only)
  int32_t* d_status;  // [4] scratch
};

namespace rlks {

constexpr int ENV_BLOCK = 256;
constexpr int MAX_TABLE_BYTES = 96 * 1024;  // LDS budget for the staged tables

struct EnvView {
  int N, T, C, max_steps, noise_mode, autoreset, env_offset;
  uint32_t k0, k1;
  double cpu_lo, span, w_cost, w_lat, scale;
  int32_t* step;
  int32_t* episode;
  double* ep_ret;
  double* ret_sum;
  int32_t* ep_cnt;
  uint32_t* mt;
};

inline EnvView view(const rlks_env* e) {
  EnvView v;
  v.N = e->cfg.n_envs; v.T = e->cfg.n_rows; v.C = e->cfg.n_clouds; v.max_steps = e->cfg.max_steps;
  v.noise_mode = e->cfg.noise_mode; v.autoreset = e->cfg.autoreset; v.env_offset = e->cfg.env_offset;
  v.k0 = (uint32_t)e->cfg.seed; v.k1 = (uint32_t)(e->cfg.seed >> 32);
  v.cpu_lo = e->cfg.cpu_lo; v.span = e->span; v.w_cost = e->cfg.w_cost; v.w_lat = e->cfg.w_lat;
  v.scale = e->cfg.scale;
  v.step = e->d_step; v.episode = e->d_episode; v.ep_ret = e->d_ep_ret; v.ret_sum = e->d_ret_sum;
  v.ep_cnt = e->d_ep_cnt; v.mt = e->d_mt;
  return v;
}

// stage [T][C] cost then latency tables into LDS (f64)
__device__ __forceinline__ void stage_tables(double* s_tab, const double* __restrict__ cost,
                                             const double* __restrict__ lat, int TC) {
  for (int i = threadIdx.x; i < TC; i += blockDim.x) {
    s_tab[i] = cost[i];
    s_tab[TC + i] = lat[i];
  }
  __syncthreads();
}

// utilisation noise for cloud c at row t: random.uniform(0.1, 0.8) (:87)
__device__ __forceinline__ double noise(const EnvView& v, int lane, int t, int c, int episode) {
  double u;
  if (v.noise_mode == RLKS_NOISE_MT19937) {
    u = mt_random(v.mt, v.N, lane);
  } else {
    u32x4 x = philox4x32_10(u32x4{(uint32_t)(v.env_offset + lane), (uint32_t)episode, (uint32_t)t,
                                  ((uint32_t)RLKS_PURPOSE_OBS << 16) | (uint32_t)(c >> 1)},
                            v.k0, v.k1);
    u = (c & 1) ? u53(x.z, x.w) : u53(x.x, x.y);
  }
  return __dadd_rn(v.cpu_lo, __dmul_rn(v.span, u));
}

// _get_obs (:90-103): f32[cost[0..C), lat[0..C), cpu[0..C)] of row t
__device__ __forceinline__ void emit_obs(const EnvView& v, const double* s_tab, int lane, int t,
                                         int episode, float* __restrict__ o) {
  const int C = v.C, TC = v.T * v.C;
  for (int c = 0; c < C; ++c) o[c] = (float)s_tab[t * C + c];
  for (int c = 0; c < C; ++c) o[C + c] = (float)s_tab[TC + t * C + c];
  for (int c = 0; c < C; ++c) o[2 * C + c] = (float)noise(v, lane, t, c, episode);
}

struct StepOut {
  double reward;
  int step;
  bool done;
  bool overrun;
};

// step (:115-144) for one lane with a valid action; writes next obs (auto-reset aware)
__device__ __forceinline__ StepOut step_lane(const EnvView& v, const double* s_tab, int lane, int a,
                                             float* __restrict__ o, float* __restrict__ final_o) {
  StepOut r{0.0, 0, false, false};
  int t = v.step[lane];
  const int C = v.C, TC = v.T * v.C;
  if (t >= v.T) {  // iloc[t] out of bounds before any change
    r.step = t;
    r.overrun = true;
    return r;
  }
  const double cost = s_tab[t * C + a];
  const double lat = s_tab[TC + t * C + a];
  r.reward = __dmul_rn(v.scale, __dadd_rn(__dmul_rn(v.w_cost, cost), __dmul_rn(v.w_lat, lat)));
  t += 1;
  v.step[lane] = t;
  r.step = t;
  r.done = t >= v.max_steps;
  if (t >= v.T) {  // iloc[t] of the next obs raises after current_step was incremented
    r.overrun = true;
    return r;
  }
  int ep = v.episode[lane];
  emit_obs(v, s_tab, lane, t, ep, o);
  // episode return bookkeeping (PPO result episode_reward_mean)
  double ret = v.ep_ret[lane] + r.reward;
  if (r.done) {
    v.ret_sum[lane] += ret;
    v.ep_cnt[lane] += 1;
    ret = 0.0;
  }
  v.ep_ret[lane] = ret;
  if (r.done && v.autoreset) {
    const int D = 3 * C;
    if (final_o)
      for (int j = 0; j < D; ++j) final_o[j] = o[j];
    v.step[lane] = 0;
    v.episode[lane] = ep + 1;
    emit_obs(v, s_tab, lane, 0, ep + 1, o);
  }
  return r;
}

inline size_t table_lds(const rlks_env* e) {
  return (size_t)2 * e->cfg.n_rows * e->cfg.n_clouds * sizeof(double);
}

}  // namespace rlks
