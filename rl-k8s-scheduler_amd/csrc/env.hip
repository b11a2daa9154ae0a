// env.hip — K1: the batched K8sMultiCloudEnv step kernel (one lane per environment).
//
// Reference: /root/reference/rl_scheduler/env/k8s_multi_cloud_env.py
//   _get_live_cpu (:84-88), _get_obs (:90-103), reset (:106-112), step (:115-144).
// Layout: lane state is structure-of-arrays in HBM (int32 step[N], int32 episode[N], f64
// ep_ret[N]...; MT19937 words as [625][N] so that lane i's word k is coalesced across a wave).
// The [T][C] cost/latency tables (3.2 KB for the reference 2-cloud table) are staged in LDS by
// every workgroup.  Reward arithmetic is f64 with explicit round-to-nearest multiplies/adds so
// that 100*(0.6*cost + 0.4*latency) is bit-identical to CPython (no FMA contraction).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include <mutex>
#include <new>

#include "env_device.h"

namespace rlks {

// ----------------------------------------------------------------------------- kernels
__global__ void k_mt_seed(EnvView v, const uint8_t* __restrict__ mask, const uint32_t* __restrict__ keys,
                          const int32_t* __restrict__ keylen, int key_stride, uint64_t default_seed) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= v.N) return;
  if (mask && !mask[lane]) return;
  uint32_t kdef[2];
  const uint32_t* key;
  int klen;
  if (keys) {
    key = keys + (size_t)lane * key_stride;
    klen = keylen[lane];
  } else {
    const uint64_t s = default_seed + (uint64_t)(v.env_offset + (int64_t)lane);
    kdef[0] = (uint32_t)s;
    kdef[1] = (uint32_t)(s >> 32);
    key = kdef;
    klen = kdef[1] ? 2 : 1;
  }
  uint32_t* mt = v.mt;
  const int S = v.N;
  // init_genrand(19650218)
  uint32_t prev = 19650218u;
  mt[lane] = prev;
  for (int i = 1; i < MT_N; ++i) {
    prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
    mt[i * S + lane] = prev;
  }
  // init_by_array
  int i = 1, j = 0;
  for (int k = (MT_N > klen ? MT_N : klen); k; --k) {
    const uint32_t pm = mt[(i - 1) * S + lane];
    mt[i * S + lane] = (mt[i * S + lane] ^ ((pm ^ (pm >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i; ++j;
    if (i >= MT_N) { mt[lane] = mt[(MT_N - 1) * S + lane]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = MT_N - 1; k; --k) {
    const uint32_t pm = mt[(i - 1) * S + lane];
    mt[i * S + lane] = (mt[i * S + lane] ^ ((pm ^ (pm >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= MT_N) { mt[lane] = mt[(MT_N - 1) * S + lane]; i = 1; }
  }
  mt[lane] = 0x80000000u;
  mt[MT_N * S + lane] = MT_N;
}

__global__ void k_env_reset(EnvView v, const double* __restrict__ cost, const double* __restrict__ lat,
                            const uint8_t* __restrict__ mask, float* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) double s_tab[];
  stage_tables(s_tab, cost, lat, v.T * v.C);
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= v.N) return;
  if (mask && !mask[lane]) return;
  const int ep = v.episode[lane] + 1;
  v.episode[lane] = ep;
  v.step[lane] = 0;
  v.ep_ret[lane] = 0.0;
  if (v.nodes > 0) nodes_reset_lane(v, lane, ep);
  emit_obs(v, s_tab, lane, 0, ep, obs + (size_t)lane * 3 * v.C);
}

// node occupancy at creation (episode 0), so that stepping before the first reset is defined
__global__ void k_nodes_init(EnvView v) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane < v.N) nodes_reset_lane(v, lane, v.episode[lane]);
}

__global__ void k_validate(int N, int C, const int32_t* __restrict__ actions, int32_t* __restrict__ status) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (lane < N) {
    const int a = actions[lane];
    bad = a < 0 || a >= C;
  }
  const unsigned long long m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&status[0], (int)__popcll(m));
}

__global__ void k_env_step(EnvView v, const double* __restrict__ cost, const double* __restrict__ lat,
                           const int32_t* __restrict__ actions, float* __restrict__ obs,
                           double* __restrict__ rew64, float* __restrict__ rew32, uint8_t* __restrict__ term,
                           uint8_t* __restrict__ trunc, int32_t* __restrict__ step_out,
                           float* __restrict__ final_obs, int32_t* __restrict__ status) {
  if (status[0] != 0) return;  // some action was invalid: nothing steps (reference assert, :116)
  extern __shared__ __attribute__((aligned(16))) double s_tab[];
  stage_tables(s_tab, cost, lat, v.T * v.C);
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  bool over = false;
  if (lane < v.N) {
    const int D = 3 * v.C;
    StepOut r = step_lane(v, s_tab, lane, actions[lane], obs + (size_t)lane * D,
                          final_obs ? final_obs + (size_t)lane * D : nullptr);
    over = r.overrun;
    rew64[lane] = r.reward;
    if (rew32) rew32[lane] = (float)r.reward;
    term[lane] = (uint8_t)r.done;
    if (trunc) trunc[lane] = 0;
    if (step_out) step_out[lane] = r.step;
  }
  const unsigned long long m = __ballot(over);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&status[1], (int)__popcll(m));
}

// TorchCategorical sample / argmax over A logits, then step
__global__ void k_sample_step(EnvView v, const double* __restrict__ cost, const double* __restrict__ lat,
                              const float* __restrict__ logits, int explore, int32_t* __restrict__ actions,
                              float* __restrict__ logp, float* __restrict__ obs, float* __restrict__ rew,
                              uint8_t* __restrict__ done) {
  extern __shared__ __attribute__((aligned(16))) double s_tab[];
  stage_tables(s_tab, cost, lat, v.T * v.C);
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= v.N) return;
  const int A = v.C;
  const float* l = logits + (size_t)lane * A;
  float mx = l[0];
  int amax = 0;
  for (int a = 1; a < A; ++a)
    if (l[a] > mx) { mx = l[a]; amax = a; }
  float s = 0.f;
  for (int a = 0; a < A; ++a) s += expf(l[a] - mx);
  int act = amax;
  if (explore) {
    const int t = v.step[lane];
    const int ep = v.episode[lane];
    u32x4 x = philox4x32_10(u32x4{(uint32_t)(v.env_offset + lane), (uint32_t)ep, (uint32_t)t,
                                  (uint32_t)RLKS_PURPOSE_ACTION << 16},
                            v.k0, v.k1);
    const float u = (float)u53(x.x, x.y) * s;
    float c = 0.f;
    act = A - 1;
    for (int a = 0; a < A; ++a) {
      c += expf(l[a] - mx);
      if (u < c) { act = a; break; }
    }
  }
  actions[lane] = act;
  logp[lane] = l[act] - mx - logf(s);
  StepOut r = step_lane(v, s_tab, lane, act, obs + (size_t)lane * 3 * v.C, nullptr);
  rew[lane] = (float)r.reward;
  done[lane] = (uint8_t)r.done;
}

// deterministic single-workgroup reduction of the per-lane episode accumulators
__global__ void k_episode_stats(EnvView v, double* __restrict__ out, int clear) {
  __shared__ double s_sum[ENV_BLOCK];
  __shared__ double s_cnt[ENV_BLOCK];
  double sum = 0.0, cnt = 0.0;
  for (int i = threadIdx.x; i < v.N; i += blockDim.x) {
    sum += v.ret_sum[i];
    cnt += (double)v.ep_cnt[i];
    if (clear) { v.ret_sum[i] = 0.0; v.ep_cnt[i] = 0; }
  }
  s_sum[threadIdx.x] = sum;
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + o];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = s_sum[0]; out[1] = s_cnt[0]; }
}

__global__ void k_lane_state(int N, const int32_t* __restrict__ step, const int32_t* __restrict__ ep,
                             int32_t* __restrict__ step_out, int32_t* __restrict__ ep_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (step_out) step_out[i] = step[i];
  if (ep_out) ep_out[i] = ep[i];
}

// [C*N][n_envs] -> [n_envs][C][N] (test / inspection surface)
__global__ void k_node_transpose(EnvView v, int32_t* __restrict__ fc, int32_t* __restrict__ fm) {
  const size_t cn = (size_t)v.C * v.nodes;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // destination index
  if (i >= cn * v.N) return;
  const size_t lane = i / cn, g = i % cn;
  if (fc) fc[i] = v.free_cpu[g * v.N + lane];
  if (fm) fm[i] = v.free_mem[g * v.N + lane];
}

__global__ void k_used_transpose(EnvView v, int32_t* __restrict__ used) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)v.C * v.N) return;
  const size_t lane = i / v.C, c = i % v.C;
  used[i] = v.used_cpu[c * v.N + lane];
}

__global__ void k_philox(const uint32_t* __restrict__ ctr, const uint32_t* __restrict__ key,
                         uint32_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u32x4 c{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
  u32x4 r = philox4x32_10(c, key[0], key[1]);
  out[4 * i] = r.x; out[4 * i + 1] = r.y; out[4 * i + 2] = r.z; out[4 * i + 3] = r.w;
}

__global__ void k_mt_draws(uint32_t* __restrict__ mt, double* __restrict__ out, int n) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int i = 0; i < n; ++i) out[i] = mt_random(mt, 1, 0);
}

}  // namespace rlks

using namespace rlks;

extern "C" {

int rlks_env_create(const rlks_env_cfg* cfg, const double* cost, const double* lat, rlks_env** out) {
  RLKS_REQUIRE(cfg, RLKS_ERR_ARG, "rlks_env_create: null cfg");
  RLKS_REQUIRE(cfg->nodes_per_cluster == 0, RLKS_ERR_ARG,
               "rlks_env_create: node-level clusters need per-cluster capacities (rlks_env_create_ext)");
  return rlks_env_create_ext(cfg, cost, lat, nullptr, nullptr, nullptr, 0, out);
}

int rlks_env_create_ext(const rlks_env_cfg* cfg, const double* cost, const double* lat, const int32_t* node_cpu_m,
                        const int32_t* node_mem_mi, const double* arrival_trace, int n_trace, rlks_env** out) {
  RLKS_REQUIRE(cfg && cost && lat && out, RLKS_ERR_ARG, "rlks_env_create: null argument");
  RLKS_REQUIRE(cfg->n_envs > 0 && cfg->n_rows > 0 && cfg->n_clouds > 0, RLKS_ERR_ARG,
               "rlks_env_create: n_envs, n_rows and n_clouds must be positive");
  RLKS_REQUIRE(cfg->max_steps > 0, RLKS_ERR_ARG, "rlks_env_create: max_steps must be positive");
  RLKS_REQUIRE(cfg->noise_mode == RLKS_NOISE_PHILOX || cfg->noise_mode == RLKS_NOISE_MT19937,
               RLKS_ERR_ARG, "rlks_env_create: unknown noise_mode");
  RLKS_REQUIRE((size_t)2 * cfg->n_rows * cfg->n_clouds * sizeof(double) <= (size_t)MAX_TABLE_BYTES,
               RLKS_ERR_UNSUPPORTED, "rlks_env_create: tables exceed the LDS budget");
  const int C = cfg->n_clouds, NN = cfg->nodes_per_cluster;
  if (NN > 0) {
    RLKS_REQUIRE(node_cpu_m && node_mem_mi, RLKS_ERR_ARG, "rlks_env_create_ext: per-cluster capacities required");
    RLKS_REQUIRE(NN % 4 == 0, RLKS_ERR_ARG, "rlks_env_create_ext: nodes_per_cluster must be a multiple of 4");
    RLKS_REQUIRE(cfg->pod_cpu_m > 0 && cfg->pod_mem_mi > 0, RLKS_ERR_ARG, "rlks_env_create_ext: bad pod request");
    RLKS_REQUIRE(cfg->arrival_mode == 0 || (arrival_trace && n_trace > 0), RLKS_ERR_ARG,
                 "rlks_env_create_ext: bursty arrivals need a trace");
    RLKS_REQUIRE(cfg->arrival_rate >= 0 && cfg->depart_prob >= 0 && cfg->init_occupancy >= 0, RLKS_ERR_ARG,
                 "rlks_env_create_ext: rates must be non-negative");
    for (int c = 0; c < C; ++c)
      RLKS_REQUIRE(node_cpu_m[c] > 0 && node_mem_mi[c] > 0, RLKS_ERR_ARG, "rlks_env_create_ext: bad capacity");
  }
  *out = nullptr;
  rlks_env* e = new (std::nothrow) rlks_env();
  RLKS_REQUIRE(e, RLKS_ERR_STATE, "rlks_env_create: out of host memory");
  e->cfg = *cfg;
  e->span = cfg->cpu_hi - cfg->cpu_lo;
  const size_t N = cfg->n_envs, TC = (size_t)cfg->n_rows * C;
  hipError_t err = hipSuccess;
  auto alloc = [&](void** p, size_t bytes) {
    if (err == hipSuccess) err = hipMalloc(p, bytes);
    if (err == hipSuccess) err = hipMemset(*p, 0, bytes);
  };
  alloc((void**)&e->d_cost, TC * sizeof(double));
  alloc((void**)&e->d_lat, TC * sizeof(double));
  alloc((void**)&e->d_step, N * sizeof(int32_t));
  alloc((void**)&e->d_episode, N * sizeof(int32_t));
  alloc((void**)&e->d_ep_ret, N * sizeof(double));
  alloc((void**)&e->d_ret_sum, N * sizeof(double));
  alloc((void**)&e->d_ep_cnt, N * sizeof(int32_t));
  alloc((void**)&e->d_status, 4 * sizeof(int32_t));
  alloc((void**)&e->d_counters, 4 * sizeof(unsigned long long));
  if (cfg->noise_mode == RLKS_NOISE_MT19937) alloc((void**)&e->d_mt, (size_t)(MT_N + 1) * N * sizeof(uint32_t));
  if (err == hipSuccess) err = hipMemcpy(e->d_cost, cost, TC * sizeof(double), hipMemcpyHostToDevice);
  if (err == hipSuccess) err = hipMemcpy(e->d_lat, lat, TC * sizeof(double), hipMemcpyHostToDevice);
  if (NN > 0) {
    // host-side constants, computed exactly as oracle/rlks_oracle.c:ro_env_enable_nodes does
    std::vector<int32_t> cap(3 * C);
    for (int c = 0; c < C; ++c) {
      cap[c] = node_cpu_m[c];
      cap[C + c] = node_mem_mi[c];
      const int mp = std::min(node_cpu_m[c] / cfg->pod_cpu_m, node_mem_mi[c] / cfg->pod_mem_mi);
      cap[2 * C + c] = (int32_t)std::floor(cfg->init_occupancy * (double)mp);
    }
    e->n_trace = cfg->arrival_mode ? n_trace : 1;
    std::vector<double> lam(2 * e->n_trace);
    for (int i = 0; i < e->n_trace; ++i) {
      lam[i] = cfg->arrival_mode ? arrival_trace[i] : cfg->arrival_rate;
      lam[e->n_trace + i] = std::exp(-lam[i]);
    }
    const double pd = cfg->depart_prob * 4294967296.0;
    e->p_dep = pd >= 4294967295.0 ? 0xffffffffu : (pd <= 0 ? 0u : (uint32_t)pd);
    const size_t cells = (size_t)C * NN * N;
    alloc((void**)&e->d_cap, cap.size() * sizeof(int32_t));
    alloc((void**)&e->d_lam, lam.size() * sizeof(double));
    alloc((void**)&e->d_free_cpu, cells * sizeof(int32_t));
    alloc((void**)&e->d_free_mem, cells * sizeof(int32_t));
    alloc((void**)&e->d_used_cpu, (size_t)C * N * sizeof(int32_t));
    if (err == hipSuccess) err = hipMemcpy(e->d_cap, cap.data(), cap.size() * sizeof(int32_t), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(e->d_lam, lam.data(), lam.size() * sizeof(double), hipMemcpyHostToDevice);
    if (err == hipSuccess) {
      hipLaunchKernelGGL(k_nodes_init, dim3(cdiv(N, ENV_BLOCK)), dim3(ENV_BLOCK), 0, 0, view(e));
      err = hipGetLastError();
    }
  }
  if (err == hipSuccess && e->d_mt) {
    hipLaunchKernelGGL(k_mt_seed, dim3(cdiv(N, ENV_BLOCK)), dim3(ENV_BLOCK), 0, 0, view(e), nullptr,
                       nullptr, nullptr, 0, cfg->seed);
    err = hipGetLastError();
  }
  if (err == hipSuccess) err = hipDeviceSynchronize();
  if (err != hipSuccess) {
    rlks_env_destroy(e);
    return fail(RLKS_ERR_HIP, std::string("rlks_env_create: ") + hipGetErrorString(err));
  }
  *out = e;
  return RLKS_OK;
}

int rlks_env_destroy(rlks_env* e) {
  if (!e) return RLKS_OK;
  hipDeviceSynchronize();
  hipFree(e->d_cost); hipFree(e->d_lat); hipFree(e->d_step); hipFree(e->d_episode);
  hipFree(e->d_ep_ret); hipFree(e->d_ret_sum); hipFree(e->d_ep_cnt); hipFree(e->d_status);
  hipFree(e->d_counters);
  if (e->d_mt) hipFree(e->d_mt);
  if (e->d_cap) hipFree(e->d_cap);
  if (e->d_lam) hipFree(e->d_lam);
  if (e->d_free_cpu) hipFree(e->d_free_cpu);
  if (e->d_free_mem) hipFree(e->d_free_mem);
  if (e->d_used_cpu) hipFree(e->d_used_cpu);
  delete e;
  return RLKS_OK;
}

int rlks_env_config(const rlks_env* e, rlks_env_cfg* out) {
  RLKS_REQUIRE(e && out, RLKS_ERR_ARG, "rlks_env_config: null argument");
  *out = e->cfg;
  return RLKS_OK;
}

int rlks_env_seed(rlks_env* e, const uint8_t* mask, const uint32_t* keys, const int32_t* keylen,
                  int key_stride, void* stream) {
  RLKS_REQUIRE(e, RLKS_ERR_ARG, "rlks_env_seed: null env");
  RLKS_REQUIRE(e->cfg.noise_mode == RLKS_NOISE_MT19937, RLKS_ERR_STATE,
               "rlks_env_seed: only the MT19937 noise mode has per-lane generator state");
  RLKS_REQUIRE(!keys || (keylen && key_stride > 0), RLKS_ERR_ARG, "rlks_env_seed: bad key arrays");
  hipLaunchKernelGGL(k_mt_seed, dim3(cdiv(e->cfg.n_envs, ENV_BLOCK)), dim3(ENV_BLOCK), 0,
                     (hipStream_t)stream, view(e), mask, keys, keylen, key_stride, e->cfg.seed);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_reset(rlks_env* e, const uint8_t* mask, float* obs, void* stream) {
  RLKS_REQUIRE(e && obs, RLKS_ERR_ARG, "rlks_env_reset: null argument");
  hipLaunchKernelGGL(k_env_reset, dim3(cdiv(e->cfg.n_envs, ENV_BLOCK)), dim3(ENV_BLOCK), table_lds(e),
                     (hipStream_t)stream, view(e), e->d_cost, e->d_lat, mask, obs);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_step(rlks_env* e, const int32_t* actions, float* obs, double* rew64, float* rew32,
                  uint8_t* term, uint8_t* trunc, int32_t* step_out, float* final_obs, int32_t* status,
                  void* stream) {
  RLKS_REQUIRE(e && actions && obs && rew64 && term && status, RLKS_ERR_ARG,
               "rlks_env_step: null argument");
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = cdiv(e->cfg.n_envs, ENV_BLOCK);
  RLKS_HIP(hipMemsetAsync(status, 0, 2 * sizeof(int32_t), s));
  hipLaunchKernelGGL(k_validate, dim3(grid), dim3(ENV_BLOCK), 0, s, e->cfg.n_envs, e->cfg.n_clouds,
                     actions, status);
  RLKS_LAUNCHED();
  hipLaunchKernelGGL(k_env_step, dim3(grid), dim3(ENV_BLOCK), table_lds(e), s, view(e), e->d_cost,
                     e->d_lat, actions, obs, rew64, rew32, term, trunc, step_out, final_obs, status);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_sample_step(rlks_env* e, const float* logits, int explore, int32_t* actions, float* logp,
                         float* obs_next, float* reward, uint8_t* done, void* stream) {
  RLKS_REQUIRE(e && logits && actions && logp && obs_next && reward && done, RLKS_ERR_ARG,
               "rlks_env_sample_step: null argument");
  RLKS_REQUIRE(e->cfg.autoreset, RLKS_ERR_STATE, "rlks_env_sample_step: needs autoreset lanes");
  hipLaunchKernelGGL(k_sample_step, dim3(cdiv(e->cfg.n_envs, ENV_BLOCK)), dim3(ENV_BLOCK), table_lds(e),
                     (hipStream_t)stream, view(e), e->d_cost, e->d_lat, logits, explore, actions, logp,
                     obs_next, reward, done);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_episode_stats(rlks_env* e, double* out, int clear, void* stream) {
  RLKS_REQUIRE(e && out, RLKS_ERR_ARG, "rlks_env_episode_stats: null argument");
  hipLaunchKernelGGL(k_episode_stats, dim3(1), dim3(ENV_BLOCK), 0, (hipStream_t)stream, view(e), out, clear);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_lane_state(rlks_env* e, int32_t* steps, int32_t* episodes, void* stream) {
  RLKS_REQUIRE(e, RLKS_ERR_ARG, "rlks_env_lane_state: null env");
  hipLaunchKernelGGL(k_lane_state, dim3(cdiv(e->cfg.n_envs, ENV_BLOCK)), dim3(ENV_BLOCK), 0,
                     (hipStream_t)stream, e->cfg.n_envs, e->d_step, e->d_episode, steps, episodes);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_node_state(rlks_env* e, int32_t* free_cpu, int32_t* free_mem, int32_t* used_cpu, void* stream) {
  RLKS_REQUIRE(e, RLKS_ERR_ARG, "rlks_env_node_state: null env");
  RLKS_REQUIRE(e->cfg.nodes_per_cluster > 0, RLKS_ERR_STATE, "rlks_env_node_state: env has no nodes");
  const EnvView v = view(e);
  const size_t cells = (size_t)v.C * v.nodes * v.N;
  hipStream_t s = (hipStream_t)stream;
  if (free_cpu || free_mem) {
    hipLaunchKernelGGL(k_node_transpose, dim3(cdiv((long)cells, 256)), dim3(256), 0, s, v, free_cpu, free_mem);
    RLKS_LAUNCHED();
  }
  if (used_cpu) {
    hipLaunchKernelGGL(k_used_transpose, dim3(cdiv((long)v.C * v.N, 256)), dim3(256), 0, s, v, used_cpu);
    RLKS_LAUNCHED();
  }
  return RLKS_OK;
}

int rlks_env_counters(rlks_env* e, int enable, unsigned long long* out_dev, void* stream) {
  RLKS_REQUIRE(e, RLKS_ERR_ARG, "rlks_env_counters: null env");
  hipStream_t s = (hipStream_t)stream;
  if (out_dev) RLKS_HIP(hipMemcpyAsync(out_dev, e->d_counters, 3 * sizeof(unsigned long long),
                                       hipMemcpyDeviceToDevice, s));
  if (enable >= 0) {
    if (enable && !e->counters_on) RLKS_HIP(hipMemsetAsync(e->d_counters, 0, 3 * sizeof(unsigned long long), s));
    e->counters_on = enable;
  }
  return RLKS_OK;
}

int rlks_philox4x32_10(const uint32_t* ctr, const uint32_t* key, uint32_t* out, int n, void* stream) {
  RLKS_REQUIRE(ctr && key && out && n >= 0, RLKS_ERR_ARG, "rlks_philox4x32_10: bad argument");
  if (n == 0) return RLKS_OK;
  hipLaunchKernelGGL(k_philox, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, ctr, key, out, n);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_mt_random(const uint32_t* key, int keylen, double* out, int n, void* stream) {
  RLKS_REQUIRE(key && out && keylen > 0 && n >= 0, RLKS_ERR_ARG, "rlks_mt_random: bad argument");
  hipStream_t s = (hipStream_t)stream;
  // one-lane generator in a temporary state buffer (test surface only; allocation is fine here)
  uint32_t* mt = nullptr;
  RLKS_HIP(hipMalloc(&mt, (MT_N + 1) * sizeof(uint32_t)));
  int32_t* kl = nullptr;
  RLKS_HIP(hipMalloc(&kl, sizeof(int32_t)));
  RLKS_HIP(hipMemcpyAsync(kl, &keylen, sizeof(int32_t), hipMemcpyHostToDevice, s));
  EnvView v{};
  v.N = 1;
  v.mt = mt;
  hipLaunchKernelGGL(k_mt_seed, dim3(1), dim3(64), 0, s, v, nullptr, key, kl, keylen, 0ull);
  RLKS_LAUNCHED();
  if (n) hipLaunchKernelGGL(k_mt_draws, dim3(1), dim3(64), 0, s, mt, out, n);
  RLKS_LAUNCHED();
  RLKS_HIP(hipStreamSynchronize(s));
  hipFree(mt);
  hipFree(kl);
  return RLKS_OK;
}

}  // extern "C"
