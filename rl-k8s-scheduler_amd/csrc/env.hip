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

#include <cstring>
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
  emit_obs(v, s_tab, lane, 0, ep, obs + (size_t)lane * 3 * v.C);
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
  RLKS_REQUIRE(cfg && cost && lat && out, RLKS_ERR_ARG, "rlks_env_create: null argument");
  RLKS_REQUIRE(cfg->n_envs > 0 && cfg->n_rows > 0 && cfg->n_clouds > 0, RLKS_ERR_ARG,
               "rlks_env_create: n_envs, n_rows and n_clouds must be positive");
  RLKS_REQUIRE(cfg->max_steps > 0, RLKS_ERR_ARG, "rlks_env_create: max_steps must be positive");
  RLKS_REQUIRE(cfg->noise_mode == RLKS_NOISE_PHILOX || cfg->noise_mode == RLKS_NOISE_MT19937,
               RLKS_ERR_ARG, "rlks_env_create: unknown noise_mode");
  RLKS_REQUIRE(cfg->nodes_per_cluster == 0, RLKS_ERR_UNSUPPORTED,
               "rlks_env_create: node-level clusters are built by rlks_cluster_create");
  RLKS_REQUIRE((size_t)2 * cfg->n_rows * cfg->n_clouds * sizeof(double) <= (size_t)MAX_TABLE_BYTES,
               RLKS_ERR_UNSUPPORTED, "rlks_env_create: tables exceed the LDS budget");
  *out = nullptr;
  rlks_env* e = new (std::nothrow) rlks_env();
  RLKS_REQUIRE(e, RLKS_ERR_STATE, "rlks_env_create: out of host memory");
  e->cfg = *cfg;
  e->span = cfg->cpu_hi - cfg->cpu_lo;
  const size_t N = cfg->n_envs, TC = (size_t)cfg->n_rows * cfg->n_clouds;
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
  if (cfg->noise_mode == RLKS_NOISE_MT19937) alloc((void**)&e->d_mt, (size_t)(MT_N + 1) * N * sizeof(uint32_t));
  if (err == hipSuccess) err = hipMemcpy(e->d_cost, cost, TC * sizeof(double), hipMemcpyHostToDevice);
  if (err == hipSuccess) err = hipMemcpy(e->d_lat, lat, TC * sizeof(double), hipMemcpyHostToDevice);
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
  if (e->d_mt) hipFree(e->d_mt);
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
