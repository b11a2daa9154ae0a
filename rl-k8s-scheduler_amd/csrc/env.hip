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
// Skip n_draws[lane] calls of random() (2 words each) on every masked lane: positions lane e of a
// batched evaluation at the point of the process-global stream that episode e of the reference's
// sequential loop starts from (final_evaluation.py:42-49: 200 draws per 99-step episode).
__global__ void k_mt_discard(EnvView v, const uint8_t* __restrict__ mask, const int64_t* __restrict__ n_draws) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= v.N) return;
  if (mask && !mask[lane]) return;
  for (int64_t i = 2 * n_draws[lane]; i > 0; --i) (void)mt_next(v.mt, v.N, lane);
}

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
  if (status && status[0] != 0) return;  // some action was invalid: nothing steps (reference assert, :116)
  extern __shared__ __attribute__((aligned(16))) double s_tab[];
  stage_tables(s_tab, cost, lat, v.T * v.C);
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  bool over = false;
  if (lane < v.N) {
    const int D = 3 * v.C;
    StepOut r = step_lane(v, s_tab, lane, actions[lane], obs + (size_t)lane * D,
                          final_obs ? final_obs + (size_t)lane * D : nullptr);
    over = r.overrun;
    if (rew64) rew64[lane] = r.reward;
    if (rew32) rew32[lane] = (float)r.reward;
    term[lane] = (uint8_t)r.done;
    if (trunc) trunc[lane] = 0;
    if (step_out) step_out[lane] = r.step;
  }
  const unsigned long long m = __ballot(over);
  if (status && (threadIdx.x & 63) == 0 && m) atomicAdd(&status[1], (int)__popcll(m));
}

// The reference env's step at HBM rate: two clouds, Philox utilisation noise, no node extension.
// Same arithmetic, counters and write order as step_lane + emit_obs (bit-identical outputs), laid
// out for streaming: the four table entries a step reads come from L1/L2 (the 3.2 KB table is
// read by every lane of a wave at the same few rows, so no LDS staging and no barrier), one Philox
// call gives both clouds' noise, the 24-byte obs row is three 8-byte stores, and every lane-state
// word is read once and written once.  Per env-step it moves action 4 + step 4 + 4 + episode 4 +
// obs 24 + reward 8 (f64) + terminated 1 = 49 B, plus ep_ret 8 + 8 when returns are tracked
// (cfg.skip_returns = 0) and 1 + 4 for the optional truncated / step outputs.
// Outputs are written with non-temporal (streaming) stores: nothing reads them back before they
// leave the cache, and at 16M lanes that took the step from 0.195 to 0.130 ms (4.2 -> 6.3 TB/s).
template <typename V>
__device__ __forceinline__ void st_stream(V* p, V x) {
  __builtin_nontemporal_store(x, p);
}

__device__ __forceinline__ void obs_row2(const EnvView& v, const double* __restrict__ cost,
                                         const double* __restrict__ lat, int lane, int row, int ep,
                                         float* __restrict__ o) {
  const double2 cr = *reinterpret_cast<const double2*>(cost + 2 * row);
  const double2 lr = *reinterpret_cast<const double2*>(lat + 2 * row);
  const u32x4 x = philox4x32_10_mad(u32x4{(uint32_t)(v.env_offset + lane), (uint32_t)ep, (uint32_t)row,
                                          (uint32_t)RLKS_PURPOSE_OBS << 16},
                                    v.k0, v.k1);
  const double n0 = __dadd_rn(v.cpu_lo, __dmul_rn(v.span, u53(x.x, x.y)));
  const double n1 = __dadd_rn(v.cpu_lo, __dmul_rn(v.span, u53(x.z, x.w)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2* o2 = reinterpret_cast<f32x2*>(o);
  st_stream(o2, f32x2{(float)cr.x, (float)cr.y});
  st_stream(o2 + 1, f32x2{(float)lr.x, (float)lr.y});
  st_stream(o2 + 2, f32x2{(float)n0, (float)n1});
}

__global__ __launch_bounds__(256) void k_env_step2(EnvView v, const double* __restrict__ cost,
                                                   const double* __restrict__ lat, const int32_t* __restrict__ actions,
                                                   float* __restrict__ obs, double* __restrict__ rew64,
                                                   float* __restrict__ rew32, uint8_t* __restrict__ term,
                                                   uint8_t* __restrict__ trunc, int32_t* __restrict__ step_out,
                                                   float* __restrict__ final_obs, int32_t* __restrict__ status) {
  if (status && status[0] != 0) return;  // some action was invalid: nothing steps (reference assert, :116)
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  bool over = false;
  if (lane < v.N) {
    int t = v.step[lane];
    const int a = actions[lane];
    double reward = 0.0;
    bool done = false;
    if (t >= v.T) {  // iloc[t] out of bounds before any change
      over = true;
    } else {
      const int ep = v.episode[lane];
      reward = __dmul_rn(v.scale, __dadd_rn(__dmul_rn(v.w_cost, cost[2 * t + a]), __dmul_rn(v.w_lat, lat[2 * t + a])));
      t += 1;
      done = t >= v.max_steps;
      if (t >= v.T) {  // iloc[t] of the next obs raises after current_step was incremented
        v.step[lane] = t;
        over = true;
      } else {
        if (v.track_returns) track_return(v, lane, ep, reward, done);
        if (done && v.autoreset) {
          if (final_obs) obs_row2(v, cost, lat, lane, t, ep, final_obs + (size_t)lane * 6);
          v.step[lane] = 0;
          v.episode[lane] = ep + 1;
          obs_row2(v, cost, lat, lane, 0, ep + 1, obs + (size_t)lane * 6);
        } else {
          v.step[lane] = t;
          obs_row2(v, cost, lat, lane, t, ep, obs + (size_t)lane * 6);
        }
      }
    }
    if (rew64) st_stream(rew64 + lane, reward);
    if (rew32) st_stream(rew32 + lane, (float)reward);
    st_stream(term + lane, (uint8_t)done);
    if (trunc) trunc[lane] = 0;
    if (step_out) step_out[lane] = t;
  }
  const unsigned long long m = __ballot(over);
  if (status && (threadIdx.x & 63) == 0 && m) atomicAdd(&status[1], (int)__popcll(m));
}

// ---------------------------------------------------------------- node-level step (c3 / c5)
// One lane per env; the same algorithm, Philox counters and counters as
// oracle/rlks_oracle.c:nodes_step_lane.  Departures: per cluster with pods, geometric skips over its
// pods (one 32-bit draw per departure plus one to stop; the survival table is in LDS when it fits),
// each departing pod located by a forward scan of the cluster's nodes, a node written back once
// when the scan leaves it; arrivals: first fit from node 0 of the chosen cluster.  A lane reads
// only the clusters where a pod leaves and the first-fit prefix: per env-step about one cluster of
// nodes at c3's stationary churn instead of all C x N.
constexpr int SKIP_LDS_MAX = 4096;  // survival-table entries staged in LDS (16 KB)
// k_node_step_wl's shape (profiles/r04x, r04y: 1 or 4 pairs a thread and 2-4 waves a workgroup were slower)
constexpr int NODE_WL_NP = 2;  // (env, cluster) pairs per thread
constexpr int NODE_WL_W = 1;   // waves per workgroup
constexpr int NODE_WL_MAX_C = 64;  // clusters per env up to which the work-list kernel runs (2^cs lanes an env)

__device__ __forceinline__ int node_pods(const EnvView& v, int32_t cc, int32_t free_cpu) {
  return (int)(__umul24((uint32_t)(cc - free_cpu), v.pod_mag) >> v.pod_shift);
}
// the 8 nodes of a chunk: one 64-byte line, four 16-byte loads
__device__ __forceinline__ void load_chunk(const int2* p, int2 (&f)[8]) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4* q = reinterpret_cast<const i32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const i32x4 x = q[i];
    f[2 * i] = make_int2(x[0], x[1]);
    f[2 * i + 1] = make_int2(x[2], x[3]);
  }
}
// 8 chunk totals (16 bytes) unpacked; returns their sum
__device__ __forceinline__ int unpack_tot8(const uint4 x, int (&t)[8]) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  int s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    t[2 * i] = (int)(w[i] & 0xffffu);
    t[2 * i + 1] = (int)(w[i] >> 16);
    s += t[2 * i] + t[2 * i + 1];
  }
  return s;
}
__device__ __forceinline__ int load_tot8(const uint16_t* p, int (&t)[8]) {
  return unpack_tot8(*reinterpret_cast<const uint4*>(p), t);
}
// a cluster's chunk totals read on demand, a 16-byte group at a time
struct TotLoad {
  const uint16_t* tot;
  __device__ __forceinline__ int operator()(int g, int (&t)[8]) const { return load_tot8(tot + 8 * g, t); }
  __device__ __forceinline__ void left(int, int) {}
};
// ... or with the first 4 groups (256 nodes) loaded up front, together: one memory round trip
// where the on-demand walk has one per group it passes
struct TotPf {
  uint4 g0, g1, g2, g3;  // (named, not an array: an array here is put in scratch memory)
  __device__ __forceinline__ TotPf(const uint16_t* p, int nodes) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const int last = (nodes - 1) >> 6;  // the cluster's last group (fewer than 4: reread, never past it)
    g0 = q[0];
    g1 = q[min(1, last)];
    g2 = q[min(2, last)];
    g3 = q[min(3, last)];
  }
  // (clusters of at most 256 nodes only: a load here for the groups past the fourth would be merged
  // with the selects below into one load through a pointer into scratch memory)
  // d pods left chunk ch (written back to memory): the same in the registers, so a first fit after
  // the departures reads the totals it would load
  __device__ __forceinline__ void left(int ch, int d) {
    const uint32_t sub = (uint32_t)d << (16 * (ch & 1));
    const int w = (ch >> 1) & 3, g = ch >> 3;
    g0.x -= g == 0 && w == 0 ? sub : 0u; g0.y -= g == 0 && w == 1 ? sub : 0u;
    g0.z -= g == 0 && w == 2 ? sub : 0u; g0.w -= g == 0 && w == 3 ? sub : 0u;
    g1.x -= g == 1 && w == 0 ? sub : 0u; g1.y -= g == 1 && w == 1 ? sub : 0u;
    g1.z -= g == 1 && w == 2 ? sub : 0u; g1.w -= g == 1 && w == 3 ? sub : 0u;
    g2.x -= g == 2 && w == 0 ? sub : 0u; g2.y -= g == 2 && w == 1 ? sub : 0u;
    g2.z -= g == 2 && w == 2 ? sub : 0u; g2.w -= g == 2 && w == 3 ? sub : 0u;
    g3.x -= g == 3 && w == 0 ? sub : 0u; g3.y -= g == 3 && w == 1 ? sub : 0u;
    g3.z -= g == 3 && w == 2 ? sub : 0u; g3.w -= g == 3 && w == 3 ? sub : 0u;
  }
  __device__ __forceinline__ static void opaque(uint4& a) {
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w));
  }
  __device__ __forceinline__ int operator()(int grp, int (&t)[8]) const {
    // (the selects act on register values: selects of the members' loads would become one load at
    // a computed offset, which keeps the object in scratch memory)
    uint4 a = g0, b = g1, c = g2, d = g3;
    opaque(a);
    opaque(b);
    opaque(c);
    opaque(d);
    uint4 x;
    x.x = grp == 0 ? a.x : grp == 1 ? b.x : grp == 2 ? c.x : d.x;
    x.y = grp == 0 ? a.y : grp == 1 ? b.y : grp == 2 ? c.y : d.y;
    x.z = grp == 0 ? a.z : grp == 1 ? b.z : grp == 2 ? c.z : d.z;
    x.w = grp == 0 ? a.w : grp == 1 ? b.w : grp == 2 ? c.w : d.w;
    return unpack_tot8(x, t);
  }
};
// write back the chunk's nodes that lost pods and its new total
__device__ __forceinline__ int flush_chunk(int2* col, uint16_t* tot, int ch, int ctot, const int2 (&f)[8],
                                           const int (&dep)[8], unsigned long long& n_wr) {
  int d = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (dep[q]) {
      col[8 * ch + q] = f[q];
      ++n_wr;
      d += dep[q];
    }
  tot[ch] = (uint16_t)(ctot - d);
  return d;
}

// obs row `row` from the lane's used millicores (exact ints, IEEE f32 divide)
__device__ __forceinline__ void node_obs_row(const EnvView& v, const double* __restrict__ cost,
                                             const double* __restrict__ lat, int lane, int row,
                                             float* __restrict__ o) {
  const int C = v.C;
  for (int c = 0; c < C; ++c) o[c] = (float)cost[row * C + c];
  for (int c = 0; c < C; ++c) o[C + c] = (float)lat[row * C + c];
  for (int c = 0; c < C; ++c)
    o[2 * C + c] = __fdiv_rn((float)v.used_cpu[(size_t)c * v.N + lane], (float)(v.nodes * v.cap[c]));
}

// step counters of one lane (summed per wave into v.counters when enabled)
struct NodeCounters {
  unsigned long long checks = 0, placed = 0, rej = 0, dep = 0, wr = 0, rd = 0;
};

// u < S[x], the survival table's entry x (0 past the table), decided without reading the table
// wherever the fp32 estimate (1 - p)^x 2^32 = exp2(x lg1p) 2^32 is more than 2^16 from u: the
// estimate is within ~400 of S[x] for every x and p (tests/test_nodes_host.py checks the bound), so
// only u within 2^16 of S[x] (~2^-15 of the draws) needs the table, and the answer is the table's.
__device__ __forceinline__ bool u_below_S(const EnvView& v, const uint32_t* S, int x, uint32_t u, float lg1p) {
  const float e = exp2f((float)x * lg1p) * 0x1p32f;
  const float fu = (float)u;
  if (fu < e - 0x1p16f) return true;
  if (fu > e + 0x1p16f) return false;
  return u < (x < v.n_skip ? S[x] : 0u);
}

// 1. departures of cluster c (nodes `col`, chunk totals `tot`, `used` millicores in/out): the pods
// are numbered in node order at the start of the step; a geometric skip over the survival table S
// picks the next departing pod, the chunk holding it is located from the chunk totals (8 totals a
// 16-byte load) and loaded once, and written back when the walk moves past it.  Philox counter
// {gid, episode, t | draw << 16, DEPART << 16 | c}.
// `get` reads the chunk totals (TotLoad or TotPf) and is told what left each chunk written back.
template <class Tot>
__device__ __forceinline__ void depart_cluster(const EnvView& v, const uint32_t* S, uint32_t gid, int ep, int t, int c,
                                               int2* col, uint16_t* tot, int32_t& used, NodeCounters& k,
                                               Tot& get) {
  const int N = v.nodes;
  const int32_t pc = v.pod_cpu, pm = v.pod_mem, cc = v.cap[c];
  const int P = used / pc;
  if (P == 0) return;
  int pos = 0, n = 0;
  int grp = 0, gcum = 0, gsum = -1;  // group of 8 chunk totals holding the next pod
  int gt[8];
  int ch = -1, ccum = 0, ctot = 0;    // loaded chunk, pods before it, its pods at the start
  int2 f[8];
  int dep[8];
  u32x4 x{0u, 0u, 0u, 0u};
  const float lg1p = log1pf(-(float)v.depart_prob) * 1.4426950408889634f;  // log2(1 - p) < 0
  const float inv_lg1p = 0.6931471805599453f / log1pf(-(float)v.depart_prob);  // 1 / log2(1 - p) = ln 2 / ln(1 - p) < 0
  while (pos < P) {
    if ((n & 3) == 0)
      x = philox4x32_10_mad(u32x4{gid, (uint32_t)ep, (uint32_t)t | ((uint32_t)(n >> 2) << 16),
                                  ((uint32_t)RLKS_PURPOSE_DEPART << 16) | (uint32_t)c},
                            v.k0, v.k1);
    const uint32_t u = (n & 3) == 0 ? x.x : (n & 3) == 1 ? x.y : (n & 3) == 2 ? x.z : x.w;
    ++n;
    const int R = P - pos;
    // none of the remaining R pods leaves iff u < S[R]
    if (u_below_S(v, S, R, u, lg1p)) break;
    // surviving pods before the departure: the largest s in [0, min(R, L)) with S[s] > u (0 if
    // none), as the oracle's binary search finds it.  S[s] ~ (1 - p)^s 2^32, so s ~ log2(u 2^-32) /
    // log2(1 - p): start there and step to the exact answer (u_below_S: the table is read only
    // where the estimate cannot tell)
    const int hi = min(R, v.n_skip) - 1;
    int s = (int)fminf(fmaxf(__log2f((float)u * 0x1p-32f) * inv_lg1p, 0.f), (float)hi);
    while (s > 0 && !u_below_S(v, S, s, u, lg1p)) --s;
    while (s < hi && u_below_S(v, S, s + 1, u, lg1p)) ++s;
    const int idx = pos + s;
    pos = idx + 1;
    // pod idx: its group, chunk, node
    for (;;) {
      if (!dcheck(8 * grp < (N >> 3), DC_NODE_GROUP, grp)) grp = ((N >> 3) - 1) >> 3;
      if (gsum < 0) gsum = get(grp, gt);
      if (idx < gcum + gsum) break;
      gcum += gsum;
      ++grp;
      gsum = -1;
    }
    int j = 0, cj = gcum, tj = gt[0];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (j == q && idx >= cj + gt[q]) { cj += gt[q]; j = q + 1; }
#pragma unroll
    for (int q = 0; q < 8; ++q) tj = (q == j) ? gt[q] : tj;
    if (!dcheck(8 * grp + j < (N >> 3), DC_NODE_CHUNK, 8 * grp + j)) j = (N >> 3) - 1 - 8 * grp;
    if (8 * grp + j != ch) {
      if (ch >= 0) get.left(ch, flush_chunk(col, tot, ch, ctot, f, dep, k.wr));
      ch = 8 * grp + j;
      ccum = cj;
      ctot = tj;
      load_chunk(col + 8 * ch, f);
#pragma unroll
      for (int q = 0; q < 8; ++q) dep[q] = 0;
      ++k.rd;
    }
    int qn = 0, cq = ccum;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int pq = node_pods(v, cc, f[q].x) + dep[q];
      if (qn == q && idx >= cq + pq) { cq += pq; qn = q + 1; }
    }
    if (!dcheck(qn < 8, DC_NODE_POD, idx)) qn = 7;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q == qn) {
        ++dep[q];
        f[q].x += pc;
        f[q].y += pm;
      }
    used -= pc;
    ++k.dep;
  }
  if (ch >= 0) get.left(ch, flush_chunk(col, tot, ch, ctot, f, dep, k.wr));  // some pod left this cluster
}

// 2. `rem` arriving pods onto cluster a, first fit: chunks whose 8 nodes are all full are skipped
// by their totals, the others are loaded and filled node by node in order.  rem: pods left over.
template <class Tot>
__device__ __forceinline__ void first_fit_cluster(const EnvView& v, int a, int2* col, uint16_t* tot, int& rem,
                                                  int32_t& used, NodeCounters& k, Tot get) {
  const int N = v.nodes, C = v.C;
  const int32_t pc = v.pod_cpu, pm = v.pod_mem;
  const int32_t cc = v.cap[a], cm = v.cap[C + a];
  const int full = 8 * min(cc / pc, cm / pm);
  const int NC = N >> 3;
  int placed = 0, last = -1;
  for (int g = 0; 8 * g < NC && rem > 0; ++g) {
    int gt[8];
    (void)get(g, gt);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int chn = 8 * g + j;
      if (rem > 0 && chn < NC && gt[j] < full) {
        int2 f[8];
        load_chunk(col + 8 * chn, f);
        ++k.rd;
        int here = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          int put = 0;
          while (rem > 0 && f[q].x >= pc && f[q].y >= pm) {
            f[q].x -= pc;
            f[q].y -= pm;
            --rem;
            ++put;
          }
          if (put) {
            col[8 * chn + q] = f[q];
            ++k.wr;
            here += put;
            last = 8 * chn + q;
          }
        }
        if (here) tot[chn] = (uint16_t)(gt[j] + here);
        placed += here;
      }
    }
  }
  used += placed * pc;
  const int nfin = rem > 0 ? N : (placed ? last : 0);
  k.checks += (unsigned long long)(placed + nfin);
  k.placed += (unsigned long long)placed;
  k.rej += (unsigned long long)rem;
}

__device__ __forceinline__ void depart_cluster(const EnvView& v, const uint32_t* S, uint32_t gid, int ep, int t, int c,
                                               int2* col, uint16_t* tot, int32_t& used, NodeCounters& k) {
  TotLoad get{tot};
  depart_cluster(v, S, gid, ep, t, c, col, tot, used, k, get);
}
__device__ __forceinline__ void first_fit_cluster(const EnvView& v, int a, int2* col, uint16_t* tot, int& rem,
                                                  int32_t& used, NodeCounters& k) {
  first_fit_cluster(v, a, col, tot, rem, used, k, TotLoad{tot});
}

__device__ __forceinline__ void node_counters_flush(const EnvView& v, NodeCounters k) {
  if (!v.counters) return;
  k.checks = wave_sum_u64(k.checks);
  k.placed = wave_sum_u64(k.placed);
  k.rej = wave_sum_u64(k.rej);
  k.dep = wave_sum_u64(k.dep);
  k.wr = wave_sum_u64(k.wr);
  k.rd = wave_sum_u64(k.rd);
  if ((threadIdx.x & 63) == 0) {
    if (k.checks) atomicAdd(&v.counters[0], k.checks);
    if (k.placed) atomicAdd(&v.counters[1], k.placed);
    if (k.rej) atomicAdd(&v.counters[2], k.rej);
    if (k.dep) atomicAdd(&v.counters[3], k.dep);
    if (k.wr) atomicAdd(&v.counters[4], k.wr);
    if (k.rd) atomicAdd(&v.counters[5], k.rd);
  }
}

// reward of row t's cost and latency of the chosen cluster, `rem` pods rejected
__device__ __forceinline__ double node_reward_of(const EnvView& v, double cost_ta, double lat_ta, int rem) {
  double r = __dmul_rn(v.scale, __dadd_rn(__dmul_rn(v.w_cost, cost_ta), __dmul_rn(v.w_lat, lat_ta)));
  if (v.penalty != 0.0) r = __dsub_rn(r, __dmul_rn(v.penalty, (double)rem));
  return r;
}
__device__ __forceinline__ double node_reward(const EnvView& v, const double* __restrict__ cost,
                                              const double* __restrict__ lat, int t, int a, int rem) {
  return node_reward_of(v, cost[t * v.C + a], lat[t * v.C + a], rem);
}

// whether cluster c loses a pod this step: the first departure draw of depart_cluster, decided as it
// decides it (false: its first draw stops the walk, or the cluster has no pods)
__device__ __forceinline__ bool depart_any(const EnvView& v, const uint32_t* S, uint32_t gid, int ep, int t, int c,
                                           int32_t used) {
  const int P = used / v.pod_cpu;
  if (P == 0) return false;
  const u32x4 x = philox4x32_10_mad(u32x4{gid, (uint32_t)ep, (uint32_t)t, ((uint32_t)RLKS_PURPOSE_DEPART << 16) | (uint32_t)c},
                                    v.k0, v.k1);
  const float lg1p = log1pf(-(float)v.depart_prob) * 1.4426950408889634f;
  return !u_below_S(v, S, P, x.x, lg1p);
}

// barrier for LDS traffic only: waits for the workgroup's LDS accesses, not its global stores (a
// __syncthreads() also waits for every store the wave has in flight)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Work-list form of the lane-per-(env, cluster) step (the same results, counters included), a
// workgroup of W waves over NP * 64 W (env, cluster) pairs.  The step is a chain of dependent
// memory round trips, so the kernel is laid out to keep that chain short: the divergent paths a wave
// of round 3's k_node_step_ec ran for the few lanes that need them (a departing pod's chunk walk in ~1 pair in
// 8, the chosen cluster's Poisson draw and first fit in 1 in 8) run over one compact list per
// workgroup, so a workgroup covers NP times the pairs for the same chain:
//   A (every pair): the step's loads, all issued together (step, episode, action, used millicores,
//     the obs and reward rows); the first departure draw's decision; a pair whose cluster loses a
//     pod, and each env's chosen cluster, go on the list;
//   B (the list, items spread over the W waves): depart_cluster, then for the chosen cluster the
//     arrivals and first fit, in one thread; the chunk totals the walks need come in one load (TotPf);
//   D (every pair): obs, auto-reset, reward and bookkeeping, from the used millicores B left in LDS.
// Between B and D only LDS is exchanged (lds_barrier), unless an env of the workgroup auto-resets:
// its clusters' nodes are then rewritten in D by other threads than B's, after a full barrier.
// A cluster's nodes are touched by one item of B only, so the order of the list does not matter.
template <int NP, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4))) k_node_step_wl(EnvView v, const double* __restrict__ cost,
                                                      const double* __restrict__ lat,
                                                      const int32_t* __restrict__ actions, float* __restrict__ obs,
                                                      double* __restrict__ rew64, float* __restrict__ rew32,
                                                      uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                                      int32_t* __restrict__ step_out, float* __restrict__ final_obs,
                                                      int32_t* __restrict__ status, int cs) {
  if (status && status[0] != 0) return;  // some action was invalid: nothing steps (reference assert, :116)
  constexpr int NT = 64 * W, PB = NP * NT;  // threads, pairs per workgroup
  constexpr uint16_t ARR = 0x8000, DEP = 0x4000;  // list item flags over the pair index
  static_assert(PB <= 0x4000, "pair index must fit below the flags");
  __shared__ int32_t s_used[PB];               // per pair: used millicores after B
  __shared__ int s_t[PB], s_ep[PB], s_rem[PB];  // per env of the workgroup: step, episode, pods rejected
  __shared__ uint16_t s_list[PB];              // work list: pair index | ARR | DEP
  __shared__ double s_oc[PB], s_ol[PB];        // per pair: obs row t + 1 (0 on reset) cost, latency
  __shared__ double s_rc[PB], s_rl[PB], s_er[PB];  // per env: reward row t cost, latency; running return
  __shared__ int s_n, s_reset;
  const int tid = threadIdx.x;
  const int cm = (1 << cs) - 1;
  const int env0 = v.lane0 + blockIdx.x * (PB >> cs);  // (a lane range: node_rollout's halves)
  const int C = v.C, N = v.nodes, D = 3 * C;
  // ---- A: loads
  int t[NP], ep[NP], a[NP];
  int32_t used0[NP];
  double ocost[NP], olat[NP], rcost[NP], rlat[NP];  // obs row t + 1 (or 0 on reset), reward row t
  double eret[NP];                                  // the chosen cluster's pair: the running return
  // (these five wait for D in LDS, not in registers, through B's walks)
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int p = tid + j * NT, c = p & cm, lane = env0 + (p >> cs);
    t[j] = ep[j] = a[j] = used0[j] = 0;
    ocost[j] = olat[j] = rcost[j] = rlat[j] = eret[j] = 0.0;
    if (lane < v.lane_end && c < C) {
      t[j] = v.step[lane];
      ep[j] = v.episode[lane];
      a[j] = actions[lane];
      used0[j] = v.used_cpu[(size_t)c * v.N + lane];
      if (t[j] < v.T) {
        const int t1 = t[j] + 1;
        const int row = t1 < v.T && !(t1 >= v.max_steps && v.autoreset) ? t1 : 0;
        ocost[j] = cost[row * C + c];
        olat[j] = lat[row * C + c];
        rcost[j] = cost[t[j] * C + c];
        rlat[j] = lat[t[j] * C + c];
        if (v.track_returns && c == a[j]) eret[j] = v.ep_ret[lane];
      }
    }
  }
  if (tid == 0) s_n = s_reset = 0;
  __syncthreads();
  // (the survival table stays in global memory, L2-resident: u_below_S reads it for ~2^-15 of the draws)
  const uint32_t* S = v.skip;
  // ---- A: the list
  bool any_reset = false;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int p = tid + j * NT, c = p & cm, el = p >> cs, lane = env0 + el;
    if (lane < v.lane_end && c < C) {
      if (!dcheck(a[j] >= 0 && a[j] < C, DC_NODE_ACTION, a[j])) a[j] = 0;
      if (t[j] < v.T) {
        if (c == 0) {
          s_t[el] = t[j];
          s_ep[el] = ep[j];
        }
        s_oc[p] = ocost[j];
        s_ol[p] = olat[j];
        if (c == a[j]) {
          s_rc[el] = rcost[j];
          s_rl[el] = rlat[j];
          s_er[el] = eret[j];
        }
        const int t1 = t[j] + 1;
        any_reset |= t1 < v.T && t1 >= v.max_steps && v.autoreset;
        const bool dep =
            v.depart_prob > 0.0 && depart_any(v, S, (uint32_t)(v.env_offset + lane), ep[j], t[j], c, used0[j]);
        if (dep || c == a[j]) s_list[atomicAdd(&s_n, 1)] = (uint16_t)(p | (dep ? DEP : 0) | (c == a[j] ? ARR : 0));
      }
    }
    s_used[p] = used0[j];
  }
  if (any_reset) s_reset = 1;
  lds_barrier();
  // ---- B: item i of the list goes to wave i % W, so the items spread over the workgroup's waves
  NodeCounters k;
  const int n = s_n;
  for (int i = (tid & 63) * W + (tid >> 6); i < n; i += NT) {
    const int it = s_list[i], p = it & (DEP - 1), ci = p & cm, ei = p >> cs, li = env0 + ei;
    const uint32_t gid = (uint32_t)(v.env_offset + li);
    int2* col = node_col(v, li) + (size_t)ci * N;
    uint16_t* tot = chunk_tot(v, li, ci);
    int32_t used = s_used[p];
    if (N <= 256) {
      TotPf pf(tot, N);  // (kept equal to memory through the departures)
      if (it & DEP) depart_cluster(v, S, gid, s_ep[ei], s_t[ei], ci, col, tot, used, k, pf);
      if (it & ARR) {
        int rem = arrivals(v, gid, s_ep[ei], s_t[ei]);
        first_fit_cluster(v, ci, col, tot, rem, used, k, pf);
        s_rem[ei] = rem;
      }
    } else {
      TotLoad tl{tot};
      if (it & DEP) depart_cluster(v, S, gid, s_ep[ei], s_t[ei], ci, col, tot, used, k, tl);
      if (it & ARR) {
        int rem = arrivals(v, gid, s_ep[ei], s_t[ei]);
        first_fit_cluster(v, ci, col, tot, rem, used, k, tl);
        s_rem[ei] = rem;
      }
    }
    s_used[p] = used;
  }
  if (s_reset) __syncthreads();  // (uniform: written before the last barrier)
  else lds_barrier();
  // ---- D: step (:115-144): row t1 = t + 1, done, auto-reset, obs
  int n_over = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int p = tid + j * NT, c = p & cm, el = p >> cs, lane = env0 + el;
    if (!(lane < v.lane_end && c < C)) continue;
    if (t[j] >= v.T) {  // iloc[t] out of bounds before any change
      if (c == 0) {
        ++n_over;
        if (rew64) rew64[lane] = 0.0;
        if (rew32) rew32[lane] = 0.f;
        term[lane] = 0;
        if (step_out) step_out[lane] = t[j];
        if (trunc) trunc[lane] = 0;
      }
      continue;
    }
    const uint32_t gid = (uint32_t)(v.env_offset + lane);
    int32_t used = s_used[p];
    const int t1 = t[j] + 1;
    const bool done = t1 >= v.max_steps;
    const bool reset = t1 < v.T && done && v.autoreset;
    if (reset) {
      if (final_obs) {
        float* o = final_obs + (size_t)lane * D;
        o[c] = (float)cost[t1 * C + c];
        o[C + c] = (float)lat[t1 * C + c];
        o[2 * C + c] = __fdiv_rn((float)used, (float)(N * v.cap[c]));
      }
      used = nodes_reset_cluster(v, node_col(v, lane) + (size_t)c * N, chunk_tot(v, lane, c), c, gid, ep[j] + 1);
    }
    if (used != used0[j] || reset) v.used_cpu[(size_t)c * v.N + lane] = used;
    if (t1 < v.T) {
      float* o = obs + (size_t)lane * D;
      o[c] = (float)s_oc[p];
      o[C + c] = (float)s_ol[p];
      o[2 * C + c] = __fdiv_rn((float)used, (float)(N * v.cap[c]));
    }
    if (c == a[j]) {
      const int rem = s_rem[el];
      const double r = node_reward_of(v, s_rc[el], s_rl[el], rem);
      v.step[lane] = reset ? 0 : t1;
      if (t1 >= v.T) ++n_over;
      else if (v.track_returns) track_return_from(v, lane, ep[j], r, done, s_er[el]);
      if (reset) v.episode[lane] = ep[j] + 1;
      if (rew64) rew64[lane] = r;
      if (rew32) rew32[lane] = (float)r;
      term[lane] = (uint8_t)done;
      if (step_out) step_out[lane] = t1;
      if (trunc) trunc[lane] = 0;
    }
  }
  node_counters_flush(v, k);
  if (status) {
    const int m = (int)wave_sum_u64((unsigned long long)n_over);
    if ((tid & 63) == 0 && m) atomicAdd(&status[1], m);
  }
}

// One lane per env, clusters in turn (C > 64: more clusters than a wave has lanes)
template <bool LDS_SKIP>
__global__ void __launch_bounds__(256) k_node_step(EnvView v, const double* __restrict__ cost,
                                                   const double* __restrict__ lat,
                                                   const int32_t* __restrict__ actions, float* __restrict__ obs,
                                                   double* __restrict__ rew64, float* __restrict__ rew32,
                                                   uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                                   int32_t* __restrict__ step_out, float* __restrict__ final_obs,
                                                   int32_t* __restrict__ status) {
  if (status && status[0] != 0) return;  // some action was invalid: nothing steps (reference assert, :116)
  __shared__ uint32_t s_skip[LDS_SKIP ? SKIP_LDS_MAX : 1];
  if (LDS_SKIP) {
    for (int i = threadIdx.x; i < v.n_skip; i += blockDim.x) s_skip[i] = v.skip[i];
    __syncthreads();
  }
  const uint32_t* S = LDS_SKIP ? s_skip : v.skip;
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  const int C = v.C, N = v.nodes, D = 3 * C;
  bool over = false;
  NodeCounters k;
  if (lane < v.N) {
    const int t = v.step[lane], ep = v.episode[lane];
    int a = actions[lane];
    if (t >= v.T) {  // iloc[t] out of bounds before any change
      over = true;
      if (rew64) rew64[lane] = 0.0;
      if (rew32) rew32[lane] = 0.f;
      term[lane] = 0;
      if (step_out) step_out[lane] = t;
    } else {
      const uint32_t gid = (uint32_t)(v.env_offset + lane);
      int2* nodes = node_col(v, lane);
      for (int c = 0; c < C && v.depart_prob > 0.0; ++c) {
        int32_t used = v.used_cpu[(size_t)c * v.N + lane];
        const int32_t used0 = used;
        depart_cluster(v, S, gid, ep, t, c, nodes + (size_t)c * N, chunk_tot(v, lane, c), used, k);
        if (used != used0) v.used_cpu[(size_t)c * v.N + lane] = used;
      }
      int rem = arrivals(v, gid, ep, t);
      if (!dcheck(a >= 0 && a < C, DC_NODE_ACTION, a)) a = 0;
      {
        int32_t used = v.used_cpu[(size_t)a * v.N + lane];
        const int32_t used0 = used;
        first_fit_cluster(v, a, nodes + (size_t)a * N, chunk_tot(v, lane, a), rem, used, k);
        if (used != used0) v.used_cpu[(size_t)a * v.N + lane] = used;
      }
      const double r = node_reward(v, cost, lat, t, a, rem);
      const int t1 = t + 1;
      v.step[lane] = t1;
      const bool done = t1 >= v.max_steps;
      if (t1 >= v.T) {
        over = true;
      } else {
        if (v.track_returns) track_return(v, lane, ep, r, done);
        if (done && v.autoreset) {
          if (final_obs) node_obs_row(v, cost, lat, lane, t1, final_obs + (size_t)lane * D);
          v.step[lane] = 0;
          v.episode[lane] = ep + 1;
          nodes_reset_lane(v, lane, ep + 1);
          node_obs_row(v, cost, lat, lane, 0, obs + (size_t)lane * D);
        } else {
          node_obs_row(v, cost, lat, lane, t1, obs + (size_t)lane * D);
        }
      }
      if (rew64) rew64[lane] = r;
      if (rew32) rew32[lane] = (float)r;
      term[lane] = (uint8_t)done;
      if (step_out) step_out[lane] = t1;
    }
    if (trunc) trunc[lane] = 0;
  }
  node_counters_flush(v, k);
  const unsigned long long m = __ballot(over);
  if (status && (threadIdx.x & 63) == 0 && m) atomicAdd(&status[1], (int)__popcll(m));
}

// TorchCategorical over the A logits l[0..A): explore -> u = f32(u53(Philox(ctr, key) words 0, 1)) *
// sum exp(l - max), the first a with u < cumsum; else argmax.  logp of the choice.  Shared by the
// rollout's fused sample + step and the standalone sampler (oracle.sample_actions restates it).
__device__ __forceinline__ int categorical(const float* __restrict__ l, int A, bool explore, u32x4 ctr, uint32_t k0,
                                          uint32_t k1, float& logp) {
  float mx = l[0];
  int amax = 0;
  for (int a = 1; a < A; ++a)
    if (l[a] > mx) { mx = l[a]; amax = a; }
  float s = 0.f;
  for (int a = 0; a < A; ++a) s += expf(l[a] - mx);
  int act = amax;
  if (explore) {
    const u32x4 x = philox4x32_10(ctr, k0, k1);
    const float u = (float)u53(x.x, x.y) * s;
    float c = 0.f;
    act = A - 1;
    for (int a = 0; a < A; ++a) {
      c += expf(l[a] - mx);
      if (u < c) { act = a; break; }
    }
  }
  logp = l[act] - mx - logf(s);
  return act;
}

// rows i < n: ctr = {ids[3i], ids[3i + 1], ids[3i + 2], ACTION << 16}
__global__ void k_sample_categorical(const float* __restrict__ logits, int n, int A, const uint32_t* __restrict__ ids,
                                     uint32_t k0, uint32_t k1, int explore, int32_t* __restrict__ actions,
                                     float* __restrict__ logp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float lp;
  u32x4 ctr{0u, 0u, 0u, (uint32_t)RLKS_PURPOSE_ACTION << 16};
  if (explore) {  // ids may be NULL for argmax
    ctr.x = ids[3 * i];
    ctr.y = ids[3 * i + 1];
    ctr.z = ids[3 * i + 2];
  }
  actions[i] = categorical(logits + (size_t)i * A, A, explore != 0, ctr, k0, k1, lp);
  if (logp) logp[i] = lp;
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
  const u32x4 ctr{(uint32_t)(v.env_offset + lane), (uint32_t)v.episode[lane], (uint32_t)v.step[lane],
                  (uint32_t)RLKS_PURPOSE_ACTION << 16};
  float lp;
  const int act = categorical(logits + (size_t)lane * v.C, v.C, explore != 0, ctr, v.k0, v.k1, lp);
  actions[lane] = act;
  logp[lane] = lp;
  StepOut r = step_lane(v, s_tab, lane, act, obs + (size_t)lane * 3 * v.C, nullptr);
  rew[lane] = (float)r.reward;
  done[lane] = (uint8_t)r.done;
}

// deterministic single-workgroup reduction of the per-lane episode accumulators
// fixed-order sum of n (sum, count) pairs from the block's threads: each thread adds items
// tid, tid + 256, ... of its range, then a pairwise LDS tree (the same bits on every run)
__device__ __forceinline__ void block_sum2(double sum, double cnt, double* __restrict__ out) {
  __shared__ double s_sum[ENV_BLOCK];
  __shared__ double s_cnt[ENV_BLOCK];
  s_sum[threadIdx.x] = sum;
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = ENV_BLOCK / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + o];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = s_sum[0]; out[1] = s_cnt[0]; }
}
// completed-episode sums over the lanes in two fixed-order stages: block b reduces lanes
// [b EPS_LANES, (b + 1) EPS_LANES) into part[b], then one block sums the parts
constexpr int EPS_LANES = 8 * ENV_BLOCK;
__global__ __launch_bounds__(ENV_BLOCK) void k_episode_stats_part(EnvView v, double* __restrict__ part, int clear) {
  double sum = 0.0, cnt = 0.0;
  const int i1 = min(v.N, (int)(blockIdx.x + 1) * EPS_LANES);
  for (int i = blockIdx.x * EPS_LANES + threadIdx.x; i < i1; i += ENV_BLOCK) {
    sum += v.ret_sum[i];
    cnt += (double)v.ep_cnt[i];
    if (clear) { v.ret_sum[i] = 0.0; v.ep_cnt[i] = 0; }
  }
  block_sum2(sum, cnt, part + 2 * blockIdx.x);
}
__global__ __launch_bounds__(ENV_BLOCK) void k_episode_stats_final(const double* __restrict__ part, int nb,
                                                                   double* __restrict__ out) {
  double sum = 0.0, cnt = 0.0;
  for (int b = threadIdx.x; b < nb; b += ENV_BLOCK) {
    sum += part[2 * b];
    cnt += part[2 * b + 1];
  }
  block_sum2(sum, cnt, out);
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
  const int2 f = node_col(v, (int)lane)[node_off(g)];
  if (fc) fc[i] = f.x;
  if (fm) fm[i] = f.y;
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

// the trusted node step (rlks_env_step with status / truncated / step / final obs null) over the lanes
// [lane0, lane_end) only, for node_rollout's two halves; false: this env has no lane-range step (C >
// NODE_WL_MAX_C or no nodes), use rlks_env_step
bool node_step_range(rlks_env* e, int lane0, int lane_end, const int32_t* actions, float* obs, float* rew32,
                     uint8_t* term, hipStream_t s) {
  const int C = e->cfg.n_clouds;
  if (e->cfg.nodes_per_cluster <= 0 || C > NODE_WL_MAX_C) return false;
  int cs = 0;
  while ((1 << cs) < C) ++cs;
  EnvView v = view(e);
  v.lane0 = lane0;
  v.lane_end = lane_end;
  const dim3 gridw(cdiv(lane_end - lane0, (NODE_WL_NP * 64 * NODE_WL_W) >> cs)), blkw(64 * NODE_WL_W);
  hipLaunchKernelGGL((k_node_step_wl<NODE_WL_NP, NODE_WL_W>), gridw, blkw, 0, s, v, e->d_cost, e->d_lat, actions, obs,
                     nullptr, rew32, term, nullptr, nullptr, nullptr, nullptr, cs);
  return hipGetLastError() == hipSuccess;
}
}  // namespace rlks

using namespace rlks;

namespace {
// Departure-skip survival table S[j] = round((1 - p)^j 2^32) capped at 2^32 - 1, j <
// min(pmax, first j with S[j] == 0) + 1: computed in f64 exactly as oracle/rlks_oracle.c:ro_skip32.
std::vector<uint32_t> skip32(int pmax, double p) {
  std::vector<uint32_t> out;
  const double q = 1.0 - p;
  double acc = 1.0;
  for (int j = 0; j <= pmax; ++j) {
    double x = acc * 4294967296.0;
    x = x + 0.5;
    const uint32_t v = x >= 4294967295.0 ? 0xffffffffu : (uint32_t)x;
    if (v == 0u) break;
    out.push_back(v);
    acc = acc * q;
  }
  return out;
}
}  // namespace

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
    RLKS_REQUIRE(NN % 8 == 0, RLKS_ERR_ARG, "rlks_env_create_ext: nodes_per_cluster must be a multiple of 8");
    RLKS_REQUIRE((long)C * NN <= 262144, RLKS_ERR_UNSUPPORTED,
                 "rlks_env_create_ext: at most 262,144 nodes per env (16-bit Philox block index)");
    RLKS_REQUIRE(C <= 1024, RLKS_ERR_UNSUPPORTED, "rlks_env_create_ext: at most 1,024 clusters");
    RLKS_REQUIRE(cfg->n_rows <= 65535, RLKS_ERR_UNSUPPORTED,
                 "rlks_env_create_ext: at most 65,535 table rows (16-bit step field of the departure counter)");
    RLKS_REQUIRE(cfg->depart_prob <= 1.0, RLKS_ERR_ARG, "rlks_env_create_ext: depart_prob must be <= 1");
    RLKS_REQUIRE(cfg->pod_cpu_m > 0 && cfg->pod_mem_mi > 0, RLKS_ERR_ARG, "rlks_env_create_ext: bad pod request");
    RLKS_REQUIRE(cfg->arrival_mode == 0 || (arrival_trace && n_trace > 0), RLKS_ERR_ARG,
                 "rlks_env_create_ext: bursty arrivals need a trace");
    RLKS_REQUIRE(cfg->arrival_rate >= 0 && cfg->depart_prob >= 0 && cfg->init_occupancy >= 0, RLKS_ERR_ARG,
                 "rlks_env_create_ext: rates must be non-negative");
    for (int c = 0; c < C; ++c) {
      RLKS_REQUIRE(node_cpu_m[c] > 0 && node_mem_mi[c] > 0 && node_cpu_m[c] < (1 << 22), RLKS_ERR_ARG,
                   "rlks_env_create_ext: bad capacity");
      RLKS_REQUIRE(std::min(node_cpu_m[c] / cfg->pod_cpu_m, node_mem_mi[c] / cfg->pod_mem_mi) <= 64,
                   RLKS_ERR_UNSUPPORTED, "rlks_env_create_ext: at most 64 pods per node");
    }
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
  alloc((void**)&e->d_counters, 8 * sizeof(unsigned long long));
  alloc((void**)&e->d_eplog, RLKS_EPLOG_CAP * sizeof(double));
  alloc((void**)&e->d_eplog_key, RLKS_EPLOG_CAP * sizeof(long long));
  alloc((void**)&e->d_eplog_n, sizeof(unsigned));
  alloc((void**)&e->d_epstat, 2 * cdiv(N, EPS_LANES) * sizeof(double));
  if (cfg->noise_mode == RLKS_NOISE_MT19937) alloc((void**)&e->d_mt, (size_t)(MT_N + 1) * N * sizeof(uint32_t));
  if (err == hipSuccess) err = hipMemcpy(e->d_cost, cost, TC * sizeof(double), hipMemcpyHostToDevice);
  if (err == hipSuccess) err = hipMemcpy(e->d_lat, lat, TC * sizeof(double), hipMemcpyHostToDevice);
  if (NN > 0) {
    // host-side constants, computed exactly as oracle/rlks_oracle.c:ro_env_enable_nodes does
    std::vector<int32_t> cap(3 * C);
    e->maxp = 0;
    for (int c = 0; c < C; ++c) {
      cap[c] = node_cpu_m[c];
      cap[C + c] = node_mem_mi[c];
      const int mp = std::min(node_cpu_m[c] / cfg->pod_cpu_m, node_mem_mi[c] / cfg->pod_mem_mi);
      cap[2 * C + c] = std::min(mp, (int32_t)std::floor(cfg->init_occupancy * (double)mp));
      e->maxp = std::max(e->maxp, mp);
    }
    std::vector<uint32_t> skip = skip32(NN * e->maxp, cfg->depart_prob);
    e->n_skip = (int)skip.size();
    if (skip.empty()) skip.push_back(0u);
    e->n_trace = cfg->arrival_mode ? n_trace : 1;
    std::vector<double> lam(2 * e->n_trace);
    for (int i = 0; i < e->n_trace; ++i) {
      lam[i] = cfg->arrival_mode ? arrival_trace[i] : cfg->arrival_rate;
      lam[e->n_trace + i] = std::exp(-lam[i]);
    }
    const size_t cells = (size_t)C * NN * N;  // [env][C][N]
    alloc((void**)&e->d_cap, cap.size() * sizeof(int32_t));
    alloc((void**)&e->d_lam, lam.size() * sizeof(double));
    alloc((void**)&e->d_skip, skip.size() * sizeof(uint32_t));
    alloc((void**)&e->d_free, cells * sizeof(int2));
    alloc((void**)&e->d_chunk, (size_t)C * (((NN >> 3) + 7) & ~7) * N * sizeof(uint16_t));
    alloc((void**)&e->d_used_cpu, (size_t)C * N * sizeof(int32_t));
    if (err == hipSuccess) err = hipMemcpy(e->d_cap, cap.data(), cap.size() * sizeof(int32_t), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(e->d_lam, lam.data(), lam.size() * sizeof(double), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(e->d_skip, skip.data(), skip.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
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
  (void)hipDeviceSynchronize();  // teardown: errors are not actionable here
  (void)hipFree(e->d_cost); (void)hipFree(e->d_lat); (void)hipFree(e->d_step); (void)hipFree(e->d_episode);
  (void)hipFree(e->d_ep_ret); (void)hipFree(e->d_ret_sum); (void)hipFree(e->d_ep_cnt); (void)hipFree(e->d_status);
  (void)hipFree(e->d_counters);
  (void)hipFree(e->d_eplog); (void)hipFree(e->d_eplog_key); (void)hipFree(e->d_eplog_n);
  (void)hipFree(e->d_epstat);
  if (e->d_mt) (void)hipFree(e->d_mt);
  if (e->d_cap) (void)hipFree(e->d_cap);
  if (e->d_lam) (void)hipFree(e->d_lam);
  if (e->d_skip) (void)hipFree(e->d_skip);
  if (e->d_free) (void)hipFree(e->d_free);
  if (e->d_chunk) (void)hipFree(e->d_chunk);
  if (e->d_used_cpu) (void)hipFree(e->d_used_cpu);
  if (e->side) (void)hipStreamDestroy(e->side);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
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

int rlks_env_mt_discard(rlks_env* e, const uint8_t* mask, const int64_t* n_draws, void* stream) {
  RLKS_REQUIRE(e && n_draws, RLKS_ERR_ARG, "rlks_env_mt_discard: null argument");
  RLKS_REQUIRE(e->cfg.noise_mode == RLKS_NOISE_MT19937, RLKS_ERR_STATE,
               "rlks_env_mt_discard: only the MT19937 noise mode has per-lane generator state");
  hipLaunchKernelGGL(k_mt_discard, dim3(cdiv(e->cfg.n_envs, ENV_BLOCK)), dim3(ENV_BLOCK), 0,
                     (hipStream_t)stream, view(e), mask, n_draws);
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
  RLKS_REQUIRE(e && actions && obs && (rew64 || rew32) && term, RLKS_ERR_ARG, "rlks_env_step: null argument");
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = cdiv(e->cfg.n_envs, ENV_BLOCK);
  if (status) {  // NULL: trusted actions (e.g. from the sampler), no validation / overrun report
    RLKS_HIP(hipMemsetAsync(status, 0, 2 * sizeof(int32_t), s));
    hipLaunchKernelGGL(k_validate, dim3(grid), dim3(ENV_BLOCK), 0, s, e->cfg.n_envs, e->cfg.n_clouds,
                       actions, status);
    RLKS_LAUNCHED();
  }
  if (e->cfg.nodes_per_cluster > 0) {
    const int C = e->cfg.n_clouds;
    if (C <= NODE_WL_MAX_C) {  // (env, cluster) pairs: 2^cs >= C lanes per env
      int cs = 0;
      while ((1 << cs) < C) ++cs;
      const dim3 gridw(cdiv(e->cfg.n_envs, (NODE_WL_NP * 64 * NODE_WL_W) >> cs)), blkw(64 * NODE_WL_W);
      hipLaunchKernelGGL((k_node_step_wl<NODE_WL_NP, NODE_WL_W>), gridw, blkw, 0, s, view(e), e->d_cost, e->d_lat, actions,
                         obs, rew64, rew32, term, trunc, step_out, final_obs, status, cs);
      RLKS_LAUNCHED();
      return RLKS_OK;
    }
    const dim3 grid(cdiv(e->cfg.n_envs, 256)), blk(256);
    if (e->n_skip <= SKIP_LDS_MAX)
      hipLaunchKernelGGL(k_node_step<true>, grid, blk, 0, s, view(e), e->d_cost, e->d_lat, actions, obs, rew64, rew32,
                         term, trunc, step_out, final_obs, status);
    else
      hipLaunchKernelGGL(k_node_step<false>, grid, blk, 0, s, view(e), e->d_cost, e->d_lat, actions, obs, rew64,
                         rew32, term, trunc, step_out, final_obs, status);
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
  if (e->cfg.n_clouds == 2 && e->cfg.noise_mode == RLKS_NOISE_PHILOX) {
    hipLaunchKernelGGL(k_env_step2, dim3(grid), dim3(ENV_BLOCK), 0, s, view(e), e->d_cost, e->d_lat, actions, obs,
                       rew64, rew32, term, trunc, step_out, final_obs, status);
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
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
  RLKS_REQUIRE(e->cfg.nodes_per_cluster == 0, RLKS_ERR_UNSUPPORTED,
               "rlks_env_sample_step: node-level envs step through rlks_env_step");
  hipLaunchKernelGGL(k_sample_step, dim3(cdiv(e->cfg.n_envs, ENV_BLOCK)), dim3(ENV_BLOCK), table_lds(e),
                     (hipStream_t)stream, view(e), e->d_cost, e->d_lat, logits, explore, actions, logp,
                     obs_next, reward, done);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_episode_stats(rlks_env* e, double* out, int clear, void* stream) {
  RLKS_REQUIRE(e && out, RLKS_ERR_ARG, "rlks_env_episode_stats: null argument");
  const int nb = (int)cdiv(e->cfg.n_envs, EPS_LANES);
  hipLaunchKernelGGL(k_episode_stats_part, dim3(nb), dim3(ENV_BLOCK), 0, (hipStream_t)stream, view(e), e->d_epstat,
                     clear);
  RLKS_LAUNCHED();
  hipLaunchKernelGGL(k_episode_stats_final, dim3(1), dim3(ENV_BLOCK), 0, (hipStream_t)stream, e->d_epstat, nb, out);
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

int rlks_sample_categorical(const float* logits, int n, int A, const uint32_t* ids, unsigned long long seed, int explore,
                            int32_t* actions, float* logp, void* stream) {
  RLKS_REQUIRE(logits && actions && n >= 0 && A >= 1 && (ids || !explore), RLKS_ERR_ARG,
               "rlks_sample_categorical: bad argument");
  if (n == 0) return RLKS_OK;
  hipLaunchKernelGGL(k_sample_categorical, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, logits, n, A, ids,
                     (uint32_t)seed, (uint32_t)(seed >> 32), explore, actions, logp);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_env_mt_words(rlks_env* e, int lane, uint32_t* words, int to_env, void* stream) {
  RLKS_REQUIRE(e && words, RLKS_ERR_ARG, "rlks_env_mt_words: null argument");
  RLKS_REQUIRE(e->d_mt, RLKS_ERR_ARG, "rlks_env_mt_words: the env is not in MT19937 noise mode");
  RLKS_REQUIRE(lane >= 0 && lane < e->cfg.n_envs, RLKS_ERR_ARG, "rlks_env_mt_words: lane out of range");
  // lane's word k at d_mt[k * n_envs + lane]: a 625-row column, 4 bytes wide
  const size_t pitch = (size_t)e->cfg.n_envs * sizeof(uint32_t);
  uint32_t* col = e->d_mt + lane;
  if (to_env)
    RLKS_HIP(hipMemcpy2DAsync(col, pitch, words, sizeof(uint32_t), sizeof(uint32_t), MT_N + 1, hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
  else
    RLKS_HIP(hipMemcpy2DAsync(words, sizeof(uint32_t), col, pitch, sizeof(uint32_t), MT_N + 1, hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
  return RLKS_OK;
}

int rlks_env_episode_log(rlks_env* e, double* returns, long long* keys, unsigned* count, int clear, void* stream) {
  RLKS_REQUIRE(e, RLKS_ERR_ARG, "rlks_env_episode_log: null env");
  hipStream_t s = (hipStream_t)stream;
  if (returns) RLKS_HIP(hipMemcpyAsync(returns, e->d_eplog, RLKS_EPLOG_CAP * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (keys) RLKS_HIP(hipMemcpyAsync(keys, e->d_eplog_key, RLKS_EPLOG_CAP * sizeof(long long), hipMemcpyDeviceToDevice, s));
  if (count) RLKS_HIP(hipMemcpyAsync(count, e->d_eplog_n, sizeof(unsigned), hipMemcpyDeviceToDevice, s));
  if (clear) RLKS_HIP(hipMemsetAsync(e->d_eplog_n, 0, sizeof(unsigned), s));
  return RLKS_OK;
}

// The per-lane state a resumed run needs, in a fixed order: step, episode, running and completed
// returns, completed counts, MT19937 words (MT mode), node free cpu / mem and per-cluster used cpu
// (node envs).  Philox draws need no state (counter = lane, episode, step, purpose).
namespace {
struct Seg { void* p; size_t bytes; };
int env_segments(const rlks_env* e, Seg* out) {
  const size_t N = e->cfg.n_envs;
  int n = 0;
  out[n++] = {e->d_step, N * sizeof(int32_t)};
  out[n++] = {e->d_episode, N * sizeof(int32_t)};
  out[n++] = {e->d_ep_ret, N * sizeof(double)};
  out[n++] = {e->d_ret_sum, N * sizeof(double)};
  out[n++] = {e->d_ep_cnt, N * sizeof(int32_t)};
  if (e->d_mt) out[n++] = {e->d_mt, (size_t)(MT_N + 1) * N * sizeof(uint32_t)};
  if (e->cfg.nodes_per_cluster > 0) {
    out[n++] = {e->d_free, (size_t)e->cfg.n_clouds * e->cfg.nodes_per_cluster * (size_t)N * sizeof(int2)};
    out[n++] = {e->d_chunk, (size_t)e->cfg.n_clouds * (((e->cfg.nodes_per_cluster >> 3) + 7) & ~7) * N * sizeof(uint16_t)};
    out[n++] = {e->d_used_cpu, (size_t)e->cfg.n_clouds * N * sizeof(int32_t)};
  }
  return n;
}
size_t aligned(size_t b) { return (b + 255) / 256 * 256; }
}  // namespace

int rlks_env_state_bytes(const rlks_env* e, int64_t* bytes) {
  RLKS_REQUIRE(e && bytes, RLKS_ERR_ARG, "rlks_env_state_bytes: null argument");
  Seg seg[12];
  const int n = env_segments(e, seg);
  size_t b = 0;
  for (int i = 0; i < n; ++i) b += aligned(seg[i].bytes);
  *bytes = (int64_t)b;
  return RLKS_OK;
}

int rlks_env_save_state(const rlks_env* e, void* dst, void* stream) {
  RLKS_REQUIRE(e && dst, RLKS_ERR_ARG, "rlks_env_save_state: null argument");
  Seg seg[12];
  const int n = env_segments(e, seg);
  char* o = (char*)dst;
  for (int i = 0; i < n; ++i) {
    RLKS_HIP(hipMemcpyAsync(o, seg[i].p, seg[i].bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    o += aligned(seg[i].bytes);
  }
  return RLKS_OK;
}

int rlks_env_load_state(rlks_env* e, const void* src, void* stream) {
  RLKS_REQUIRE(e && src, RLKS_ERR_ARG, "rlks_env_load_state: null argument");
  Seg seg[12];
  const int n = env_segments(e, seg);
  const char* o = (const char*)src;
  for (int i = 0; i < n; ++i) {
    RLKS_HIP(hipMemcpyAsync(seg[i].p, o, seg[i].bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    o += aligned(seg[i].bytes);
  }
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
  if (out_dev) RLKS_HIP(hipMemcpyAsync(out_dev, e->d_counters, 6 * sizeof(unsigned long long),
                                       hipMemcpyDeviceToDevice, s));
  if (enable >= 0) {
    if (enable && !e->counters_on) RLKS_HIP(hipMemsetAsync(e->d_counters, 0, 6 * sizeof(unsigned long long), s));
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
  RLKS_HIP(hipFree(mt));
  RLKS_HIP(hipFree(kl));
  return RLKS_OK;
}

}  // extern "C"
