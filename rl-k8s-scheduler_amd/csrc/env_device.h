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
  // node-level extension, allocated when cfg.nodes_per_cluster > 0
  int32_t* d_cap;       // [3][C]: node cpu (m), node mem (MiB), max initial pods per node
  double* d_lam;        // [2][n_trace]: arrival rate, exp(-rate)
  int n_trace;
  int maxp;             // most pods a node can hold (over all clusters)
  uint32_t* d_skip;     // [n_skip] departure-skip survival table round((1 - depart_prob)^j 2^32)
  int n_skip;
  int2* d_free;         // [n_envs][C][N] {free millicores, free MiB}
  uint16_t* d_chunk;    // [n_envs][C][N/8] pods per 8-node chunk (the step's index into d_free)
  int32_t* d_used_cpu;  // [C][n_envs]
  unsigned long long* d_counters;  // [5] node checks, pods placed, pods rejected, pods departed,
                                   // nodes written (opt-in)
  int counters_on;
  // completed-episode log since the last rlks_env_episode_log(clear): the first RLKS_EPLOG_CAP
  // returns with key (episode << 32 | global lane); the count keeps running past the capacity
  double* d_eplog;
  long long* d_eplog_key;
  unsigned* d_eplog_n;
  double* d_epstat;  // [ceil(n_envs / EPS_LANES)][2] partial (sum, count) of rlks_env_episode_stats
  // node rollouts in two lane halves (ppo.hip node_rollout): the second half's stream and the fork /
  // join events, created on first use
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

namespace rlks {

constexpr int ENV_BLOCK = 256;
constexpr int MAX_TABLE_BYTES = 128 * 1024;  // LDS budget for the staged tables (gfx950: 160 KB per workgroup)

struct EnvView {
  int N, T, C, max_steps, noise_mode, autoreset, env_offset, track_returns;
  int lane0, lane_end;  // the lanes a node step / sample launch covers: [lane0, lane_end) (view(): all N);
                        // N stays the stride of the per-lane arrays
  uint32_t k0, k1;
  double cpu_lo, span, w_cost, w_lat, scale;
  int32_t* step;
  int32_t* episode;
  double* ep_ret;
  double* ret_sum;
  int32_t* ep_cnt;
  uint32_t* mt;
  // node-level extension; nodes == 0 is the reference env
  int nodes, pod_cpu, pod_mem, arrival_mode, n_trace, n_skip;
  uint32_t pod_mag;     // pods on a node = mul_u24(cap - free, pod_mag) >> pod_shift (exact: see view())
  int pod_shift;
  double penalty;
  const int32_t* cap;   // [3][C]
  const double* lam;    // [2][n_trace]
  const uint32_t* skip; // [n_skip] departure-skip survival table
  double depart_prob;
  int2* free;           // [n_envs][C][N] {free millicores, free MiB}: a lane's nodes are contiguous
  uint16_t* chunk;      // [n_envs][C][N/8] pods held by each 8-node chunk (64-byte line of free)
  int32_t* used_cpu;    // [C][n_envs]
  unsigned long long* counters;  // null unless enabled
  double* eplog;        // [RLKS_EPLOG_CAP] completed-episode returns (see rlks_env)
  long long* eplog_key;
  unsigned* eplog_n;
};

bool node_step_range(rlks_env* e, int lane0, int lane_end, const int32_t* actions, float* obs, float* rew32,
                     uint8_t* term, hipStream_t s);  // (env.hip)

inline EnvView view(const rlks_env* e) {
  EnvView v;
  v.N = e->cfg.n_envs; v.lane0 = 0; v.lane_end = e->cfg.n_envs; v.T = e->cfg.n_rows; v.C = e->cfg.n_clouds; v.max_steps = e->cfg.max_steps;
  v.noise_mode = e->cfg.noise_mode; v.autoreset = e->cfg.autoreset; v.env_offset = e->cfg.env_offset;
  v.track_returns = e->cfg.skip_returns ? 0 : 1;
  v.k0 = (uint32_t)e->cfg.seed; v.k1 = (uint32_t)(e->cfg.seed >> 32);
  v.cpu_lo = e->cfg.cpu_lo; v.span = e->span; v.w_cost = e->cfg.w_cost; v.w_lat = e->cfg.w_lat;
  v.scale = e->cfg.scale;
  v.step = e->d_step; v.episode = e->d_episode; v.ep_ret = e->d_ep_ret; v.ret_sum = e->d_ret_sum;
  v.ep_cnt = e->d_ep_cnt; v.mt = e->d_mt;
  v.nodes = e->cfg.nodes_per_cluster; v.pod_cpu = e->cfg.pod_cpu_m; v.pod_mem = e->cfg.pod_mem_mi;
  v.arrival_mode = e->cfg.arrival_mode; v.n_trace = e->n_trace; v.n_skip = e->n_skip;
  v.depart_prob = e->cfg.depart_prob;
  // (cap - free) = pods * pod_cpu with pods <= 64 and cap < 2^22: with m = ceil(2^24 / pod_cpu),
  // pods * pod_cpu * m / 2^24 = pods + pods * pod_cpu * delta / 2^24, delta < 1, and the error term
  // stays below 1 for pod_cpu < 2^18; the 24-bit product stays below 2^32.  pod_cpu = 1: identity.
  v.pod_shift = v.pod_cpu > 1 ? 24 : 0;
  v.pod_mag = v.pod_cpu > 1 ? (uint32_t)((16777216u + (uint32_t)v.pod_cpu - 1u) / (uint32_t)v.pod_cpu) : 1u;
  v.penalty = e->cfg.reject_penalty;
  v.cap = e->d_cap; v.lam = e->d_lam; v.skip = e->d_skip; v.free = e->d_free; v.chunk = e->d_chunk;
  v.used_cpu = e->d_used_cpu; v.counters = e->counters_on ? e->d_counters : nullptr;
  v.eplog = e->d_eplog; v.eplog_key = e->d_eplog_key; v.eplog_n = e->d_eplog_n;
  return v;
}

// Append the returns of the lanes whose episode just ended.  Called by exactly those lanes (a
// divergent branch): one atomic per wave, slots by rank among the active lanes.  The log order is
// restored on the host by the key (episode, global lane), i.e. completion order (all lanes step in
// lockstep), so the atomic's order does not matter.
__device__ __forceinline__ void eplog_append(const EnvView& v, int lane, int episode, double ret) {
  const unsigned long long m = __ballot(1);
  const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
  unsigned base = 0;
  if (rank == 0) base = atomicAdd(v.eplog_n, (unsigned)__popcll(m));
  base = __builtin_amdgcn_readfirstlane(base);
  const unsigned i = base + rank;
  if (i < (unsigned)RLKS_EPLOG_CAP) {
    v.eplog[i] = ret;
    v.eplog_key[i] = ((long long)episode << 32) | (long long)(unsigned)(v.env_offset + lane);
  }
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

// ---------------------------------------------------------------- node-level extension
// DESIGN.md §4 (builder-defined; same algorithm and the same Philox counters as
// oracle/rlks_oracle.c).  Node state is int2 {free cpu, free mem}, [env][C][N]: each lane walks
// its own contiguous nodes (a step touches only the clusters where a pod leaves and the chosen
// cluster's first-fit prefix, different clusters in different lanes).
__device__ __forceinline__ int2* node_col(const EnvView& v, int lane) {  // node 0 of `lane`
  return v.free + (size_t)lane * v.C * v.nodes;
}
__device__ __forceinline__ size_t node_off(size_t g) { return g; }
// chunk totals of cluster c of `lane`: N/8 entries padded to a multiple of 8 (16-byte groups)
__device__ __forceinline__ int chunk_stride(int nodes) { return ((nodes >> 3) + 7) & ~7; }
__device__ __forceinline__ uint16_t* chunk_tot(const EnvView& v, int lane, int c) {
  return v.chunk + ((size_t)lane * v.C + c) * chunk_stride(v.nodes);
}

// initial occupancy of cluster c for one lane (episode `episode`); col = node_col(lane) + c*N,
// tot = the cluster's chunk totals.  Returns the cluster's used millicores.
__device__ __forceinline__ int32_t nodes_reset_cluster(const EnvView& v, int2* col, uint16_t* tot, int c,
                                                       uint32_t gid, int episode) {
  const int C = v.C, N = v.nodes;
  const int32_t cc = v.cap[c], cm = v.cap[C + c], m1 = v.cap[2 * C + c] + 1;
  int32_t used = 0;
  for (int n8 = 0; n8 < N; n8 += 8) {
    int32_t ct = 0;
#pragma unroll
    for (int h = 0; h < 8; h += 4) {
      const int n4 = n8 + h;
      const u32x4 x = philox4x32_10(u32x4{gid, (uint32_t)episode, (uint32_t)((c * N + n4) >> 2),
                                          (uint32_t)RLKS_PURPOSE_OCCUPANCY << 16}, v.k0, v.k1);
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t pods = (int32_t)(((uint64_t)w[j] * (uint64_t)m1) >> 32);
        col[node_off(n4 + j)] = make_int2(cc - pods * v.pod_cpu, cm - pods * v.pod_mem);
        ct += pods;
      }
    }
    tot[n8 >> 3] = (uint16_t)ct;
    used += ct * v.pod_cpu;
  }
  return used;
}

__device__ __forceinline__ void nodes_reset_lane(const EnvView& v, int lane, int episode) {
  const uint32_t gid = (uint32_t)(v.env_offset + lane);
  int2* col = node_col(v, lane);
  for (int c = 0; c < v.C; ++c)
    v.used_cpu[(size_t)c * v.N + lane] =
        nodes_reset_cluster(v, col + (size_t)c * v.nodes, chunk_tot(v, lane, c), c, gid, episode);
}

// pods arriving at row t: Poisson(lam) by inverse transform (f64, no contraction)
__device__ __forceinline__ int arrivals(const EnvView& v, uint32_t gid, int episode, int t) {
  const u32x4 x = philox4x32_10(u32x4{gid, (uint32_t)episode, (uint32_t)t, (uint32_t)RLKS_PURPOSE_ARRIVAL << 16},
                                v.k0, v.k1);
  const double u = u53(x.x, x.y);
  const int j = v.arrival_mode ? t % v.n_trace : 0;
  const double lam = v.lam[j];
  double p = v.lam[v.n_trace + j], F = p;
  int k = 0;
  while (u > F && k < 64) {
    k += 1;
    p = __ddiv_rn(__dmul_rn(p, lam), (double)k);
    F = __dadd_rn(F, p);
  }
  return k;
}

// _get_obs (:90-103): f32[cost[0..C), lat[0..C), cpu[0..C)] of row t
__device__ __forceinline__ void emit_obs(const EnvView& v, const double* s_tab, int lane, int t,
                                         int episode, float* __restrict__ o) {
  const int C = v.C, TC = v.T * v.C;
  for (int c = 0; c < C; ++c) o[c] = (float)s_tab[t * C + c];
  for (int c = 0; c < C; ++c) o[C + c] = (float)s_tab[TC + t * C + c];
  if (v.nodes > 0) {  // utilisation of each cluster from its nodes (extension): exact ints, IEEE f32 divide
    for (int c = 0; c < C; ++c)
      o[2 * C + c] = __fdiv_rn((float)v.used_cpu[(size_t)c * v.N + lane], (float)(v.nodes * v.cap[c]));
  } else {
    for (int c = 0; c < C; ++c) o[2 * C + c] = (float)noise(v, lane, t, c, episode);
  }
}

// episode return bookkeeping (PPO result episode_reward_mean)
// (ep_ret: the lane's running return, v.ep_ret[lane], loaded by the caller)
__device__ __forceinline__ void track_return_from(const EnvView& v, int lane, int ep, double reward, bool done,
                                                  double ep_ret) {
  double ret = ep_ret + reward;
  if (done) {
    v.ret_sum[lane] += ret;
    v.ep_cnt[lane] += 1;
    eplog_append(v, lane, ep, ret);
    ret = 0.0;
  }
  v.ep_ret[lane] = ret;
}
__device__ __forceinline__ void track_return(const EnvView& v, int lane, int ep, double reward, bool done) {
  track_return_from(v, lane, ep, reward, done, v.ep_ret[lane]);
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
  int ep = v.episode[lane];
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
  emit_obs(v, s_tab, lane, t, ep, o);
  if (v.track_returns) track_return(v, lane, ep, r.reward, r.done);
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
