// ppo.hip — host API of the policy/value MLP and the PPO update (include/rlks.h, section K4):
// layout, forward, minibatch gather, gradient orchestration (F1 -> F2 -> F3 -> reduce), Adam,
// KL-coefficient update and the rollout loop.
//
// Reference: RLlib PPO behind train_ppo.py:9-31 (train_batch_size 4000, sgd_minibatch_size 256,
// num_sgd_iter 10, lr 3e-4, gamma 0.99) and train_final.py:6-20.  RLlib is third-party and absent
// from /root/reference: the restated semantics are pinned against oracle/oracle.py.
#include <cmath>

#include "sgd_sf16.h"
#include "wide_mlp.h"

namespace rlks {


// ----------------------------------------------------------------------------- reduce
// out[i] = sum_p part[p * pstride + i] (i < len, p < P) in a fixed order with f64 accumulation.
// A block = 256 threads = OPB output vectors x G partial-groups; a vector is 4 consecutive outputs
// (one 16-byte load per partial) when the task's length and stride allow it, else 1.  G is chosen
// per task so that every thread sums about 16 partials.
struct RedTask {
  const float* part;
  float* out;        // float output ...
  double* out64;     // ... or double output (stats)
  int64_t pstride;
  int P, len, G, V;
  int blk0;
  int mslot;         // fused Adam: -1, or the max |w| slot (net * 2 + 0: W2, + 1: W1a) of the output
  int mbase;         // first entry of this task's blocks in the slot
  int kq;            // 0: output vector iv at element 4 iv; 1 (k_sf_dw2r's [k / 4][n][4] partials of a
                     // [256][256] weight): at n * 256 + 4 (iv >> 8), n = iv & 255
};
constexpr int MAX_TASKS = 20;
// torch.optim.Adam (single-tensor path) on element i: exp_avg.lerp_(g, 1-b1); exp_avg_sq =
// b2*v + (1-b2)*g*g; p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).  Shared by
// k_adam and the fused reduce so that both paths compute the same bits; every rounding is spelled out
// (__fmul_rn / __fadd_rn / fmaf) so that no inlining context contracts them differently (an -fno-slp-vectorize
// build fused m + w1 (g - m) into an fma in one kernel and not in the other, profiles/r06_noslp).
struct AdamCo {
  float w1, b2, omb2, step_size, bc2_sqrt, eps;
};
__device__ __forceinline__ float adam_elem(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                           int64_t i, float gi, const AdamCo& c) {
  const float mi = __fadd_rn(m[i], __fmul_rn(c.w1, __fsub_rn(gi, m[i])));
  const float vi = fmaf(gi, __fmul_rn(c.omb2, gi), __fmul_rn(c.b2, v[i]));
  m[i] = mi;
  v[i] = vi;
  const float denom = __fadd_rn(__fdiv_rn(sqrtf(vi), c.bc2_sqrt), c.eps);
  const float pn = fmaf(-c.step_size, __fdiv_rn(mi, denom), p[i]);
  p[i] = pn;
  return pn;
}

struct RedArgs {
  RedTask t[MAX_TASKS];
  int ntasks;
  double* stats;     // optional: stats[4] = rows, stats[5..7] = 0 (the sums come from tasks)
  double rows;
  // fused Adam (p != null): every parameter-gradient output element is also applied to its
  // parameter (index = out - grad), and the new |w| maxima of W2 / W1a go to the split's slots
  float *p, *m, *v;
  const float* grad;
  AdamCo co;
  float* slot[4];     // [net * 2 + 0] W2, [net * 2 + 1] W1a: per-block max entries (task mbase + block)
  unsigned* tag[2];   // set to tag_val: the slots hold the maxima of Adam step tag_val
  unsigned tag_val;
};

__device__ __forceinline__ void reduce_block(const RedArgs& g, const int bx) {
  __shared__ double sh[4][256];
  int ti = 0;
  while (ti + 1 < g.ntasks && bx >= g.t[ti + 1].blk0) ++ti;
  const RedTask T = g.t[ti];
  const int opb = 256 / T.G;
  const int o = threadIdx.x % opb, grp = threadIdx.x / opb;
  const int iv = (bx - T.blk0) * opb + o;  // output vector
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  // the partials of a thread RB loads at a time, summed in the same (increasing p) order: one
  // dependent load round trip per RB partials instead of per partial (c4 reduce + next gather
  // 17.5 -> 14.2-14.5 us at RB = 4 or 8, ~5.6 TB/s; profiles/r04c/reduce_batched_loads*.txt)
  constexpr int RB = 8;
  if (T.V == 4) {
    if (4 * iv < T.len) {
      const float* base = T.part + 4 * iv;
      int p = grp;
      for (; p + (RB - 1) * T.G < T.P; p += RB * T.G) {
        float4 v[RB];
#pragma unroll
        for (int q = 0; q < RB; ++q) v[q] = *reinterpret_cast<const float4*>(base + (int64_t)(p + q * T.G) * T.pstride);
#pragma unroll
        for (int q = 0; q < RB; ++q) {
          s[0] += (double)v[q].x; s[1] += (double)v[q].y; s[2] += (double)v[q].z; s[3] += (double)v[q].w;
        }
      }
      for (; p < T.P; p += T.G) {
        const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)p * T.pstride);
        s[0] += (double)v.x; s[1] += (double)v.y; s[2] += (double)v.z; s[3] += (double)v.w;
      }
    }
  } else if (iv < T.len) {
    int p = grp;
    for (; p + (RB - 1) * T.G < T.P; p += RB * T.G) {
      float v[RB];
#pragma unroll
      for (int q = 0; q < RB; ++q) v[q] = T.part[(int64_t)(p + q * T.G) * T.pstride + iv];
#pragma unroll
      for (int q = 0; q < RB; ++q) s[0] += (double)v[q];
    }
    for (; p < T.P; p += T.G) s[0] += (double)T.part[(int64_t)p * T.pstride + iv];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) sh[j][threadIdx.x] = s[j];
  // groups summed pairwise in a fixed tree order: log2 G LDS steps (the G group values summed
  // serially by each output's thread: 35 us instead of 19 us per c4 reduce, a few threads per
  // block doing G dependent LDS reads each)
  for (int h = T.G / 2; h >= 1; h /= 2) {
    __syncthreads();
    if (grp < h)
#pragma unroll
      for (int j = 0; j < 4; ++j) sh[j][threadIdx.x] += sh[j][threadIdx.x + h * opb];
  }
  __syncthreads();
  float wmax = 0.f;
  if (grp == 0) {
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < T.V; ++j) t[j] = sh[j][o];
    const int i0 = T.kq ? (iv & 255) * 256 + 4 * (iv >> 8) : T.V * iv;
    if (T.out64) {
      for (int j = 0; j < T.V && i0 + j < T.len; ++j) T.out64[i0 + j] = t[j];
    } else if (T.V == 4 && i0 + 3 < T.len) {
      const float4 gv = make_float4((float)t[0], (float)t[1], (float)t[2], (float)t[3]);
      *reinterpret_cast<float4*>(T.out + i0) = gv;
      if (g.p) {  // Adam on the four parameters (16-byte aligned: tensors start on 64-float boundaries)
        const int64_t pi = (T.out - g.grad) + i0;
        float4 pv = *reinterpret_cast<const float4*>(g.p + pi), mv = *reinterpret_cast<const float4*>(g.m + pi),
               vv = *reinterpret_cast<const float4*>(g.v + pi);
        float* pp = &pv.x; float* mm = &mv.x; float* vq = &vv.x;
        const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wmax = fmaxf(wmax, fabsf(adam_elem(pp, mm, vq, j, gg[j], g.co)));
        }
        *reinterpret_cast<float4*>(g.p + pi) = pv;
        *reinterpret_cast<float4*>(g.m + pi) = mv;
        *reinterpret_cast<float4*>(g.v + pi) = vv;
      }
    } else {
      for (int j = 0; j < T.V && i0 + j < T.len; ++j) {
        T.out[i0 + j] = (float)t[j];
        if (g.p) wmax = fmaxf(wmax, fabsf(adam_elem(g.p, g.m, g.v, (T.out - g.grad) + i0 + j, (float)t[j], g.co)));
      }
    }
  }
  if (g.p && T.mslot >= 0) {  // block-uniform: this block's max |w_new| -> the slot
    __shared__ float smax[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wmax = fmaxf(wmax, __shfl_xor(wmax, off, 64));
    if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = wmax;
    __syncthreads();
    if (threadIdx.x == 0)
      g.slot[T.mslot][T.mbase + bx - T.blk0] = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
  }
  if (g.stats && bx == 0 && threadIdx.x == 0) {
    g.stats[RLKS_STAT_ROWS] = g.rows;
    g.stats[5] = g.stats[6] = g.stats[7] = 0.0;
  }
  if (g.p && bx == 0 && threadIdx.x == 0) {
    *g.tag[0] = g.tag_val;
    *g.tag[1] = g.tag_val;
  }
}

__global__ __launch_bounds__(256) void k_reduce(RedArgs g) { reduce_block(g, (int)blockIdx.x); }

struct Reducer {
  RedArgs a{};
  int blocks = 0;
  int mnext[4] = {0, 0, 0, 0};  // next free entry per max slot
  void add(const float* part, float* out, double* out64, int64_t pstride, int P, int len, int mslot = -1) {
    RedTask& t = a.t[a.ntasks++];
    t.mslot = mslot;
    t.mbase = 0;
    t.kq = 0;
    int G = 1;
    constexpr int PPT = 32;  // partials per thread (c4 reduce: 16 -> 19.0 us, 32 -> 19.0 us, 8 -> 23.9 us)
    while (G < 256 && G * PPT < P) G *= 2;
    const bool vec = len % 4 == 0 && pstride % 4 == 0 && ((uintptr_t)part & 15) == 0;
    t.part = part; t.out = out; t.out64 = out64; t.pstride = pstride; t.P = P; t.len = len; t.G = G;
    t.V = vec ? 4 : 1;
    t.blk0 = blocks;
    const int nb = (int)cdiv(cdiv(len, t.V), 256 / G);
    blocks += nb;
    if (mslot >= 0) {
      t.mbase = mnext[mslot];
      mnext[mslot] += nb;
    }
  }
};

// fp32 path: per-net stat sums -> RLKS_STAT_* layout
__global__ void k_stats_finish(double* __restrict__ st, const double* __restrict__ s_pi,
                               const double* __restrict__ s_vf, int rows) {
  if (threadIdx.x) return;
  st[RLKS_STAT_POLICY_LOSS] = s_pi[0];
  st[RLKS_STAT_VF_LOSS] = s_vf[1];
  st[RLKS_STAT_KL] = s_pi[2];
  st[RLKS_STAT_ENTROPY] = s_pi[3];
  st[RLKS_STAT_ROWS] = (double)rows;
  st[5] = st[6] = st[7] = 0.0;
}

// ----------------------------------------------------------------------------- Adam
// torch.optim.Adam (single-tensor path): exp_avg.lerp_(g, 1-b1); exp_avg_sq = b2*v + (1-b2)*g*g;
// p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, int64_t n, AdamCo co) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  (void)adam_elem(p, m, v, i, g[i], co);
}

// RLlib PPO update_kl
__global__ void k_kl_update(float* __restrict__ dyn, const double* __restrict__ kc, float target) {
  if (threadIdx.x) return;
  const double kl = kc[1] > 0 ? kc[0] / kc[1] : 0.0;
  float c = dyn[RLKS_DYN_KL_COEFF];
  if (kl > 2.0 * target) c *= 1.5f;
  else if (kl < 0.5 * target) c *= 0.5f;
  dyn[RLKS_DYN_KL_COEFF] = c;
}

// ----------------------------------------------------------------------------- gather
// Balanced Feistel bijection on [0, 2^(2*half)) with per-epoch round keys, cycle-walked into
// [0, S): a fresh uniform-looking permutation of the train batch every epoch with no sort.
struct Perm {
  uint32_t key[4];
  uint32_t half, mask;
  uint64_t S;
};

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint64_t perm_apply(const Perm& P, uint64_t x) {
  do {
    uint32_t L = (uint32_t)(x >> P.half), R = (uint32_t)x & P.mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t nl = R;
      R = (L ^ mix32(R ^ P.key[r])) & P.mask;
      L = nl;
    }
    x = ((uint64_t)L << P.half) | R;
  } while (x >= P.S);
  return x;
}

constexpr int MAX_GROUPS = 64;
struct GatherArgs {
  rlks_rollout_bufs b;
  Perm perm[MAX_GROUPS];  // one bijection of [0, T * Ng) per lane group
  int64_t row0g;          // first row of this minibatch within each group's permutation
  int rows, rows_g, Ng, D, A, stride;
  float* mb;
  const float* packed;    // rlks_ppo_pack records [T N][pstride] (gather_packed), else null
  int pstride;
};

// source index t * N + n of minibatch row i: rows [k rows_g, (k+1) rows_g) come from lane group
// k, whose permutation p -> (t = p / Ng, lane k Ng + p mod Ng).  groups: the entries of `perm`
// (debug checks: the group index against it, and the permutation's input against its domain --
// its output is in [0, S) by construction)
__device__ __forceinline__ int64_t gather_src(const Perm* perm, int64_t row0g, int rows_g, int Ng, int N, uint32_t i,
                                              int groups) {
  uint32_t k = i / (uint32_t)rows_g;
  uint64_t ii = i - k * (uint32_t)rows_g;
  if (!dcheck(k < (uint32_t)groups, DC_GATHER_GROUP, k)) k = 0;
  if (!dcheck((uint64_t)row0g + ii < perm[k].S, DC_GATHER_SRC, (long long)(row0g + ii))) ii = 0;
  const uint64_t p = perm_apply(perm[k], (uint64_t)(row0g + ii));
  uint64_t t, nl;
  if (p >> 32) {
    t = p / (uint64_t)Ng;
    nl = p - t * (uint64_t)Ng;
  } else {  // 32-bit division (every train batch below 2^32 rows per group)
    const uint32_t t32 = (uint32_t)p / (uint32_t)Ng;
    t = t32;
    nl = (uint32_t)p - t32 * (uint32_t)Ng;
  }
  return (int64_t)(t * (uint64_t)N + (uint64_t)k * Ng + nl);
}
__device__ __forceinline__ int64_t gather_src(const GatherArgs& g, uint32_t i) {
  return gather_src(g.perm, g.row0g, g.rows_g, g.Ng, g.b.N, i, (g.rows + g.rows_g - 1) / g.rows_g);
}

// narrow records (stride 12 / 20 / 36: 2, 4 or 8 clouds): one thread per row computes the row's permuted source
// once, loads its fields (obs and logits contiguous, four scalars) and writes the record as
// 16-byte stores; consecutive threads write consecutive records
template <int S>
__global__ __launch_bounds__(256) void k_gather_rows(GatherArgs g) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint32_t)g.rows) return;
  const int64_t tn = gather_src(g, i);
  const int D = g.D, A = g.A;
  float rec[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    float v = 0.f;
    if (j < D) v = g.b.obs[tn * D + j];
    else if (j < D + A) v = g.b.logits[tn * A + (j - D)];
    else if (j == D + A) v = g.b.adv[tn];
    else if (j == D + A + 1) v = g.b.vtarg[tn];
    else if (j == D + A + 2) v = g.b.logp[tn];
    else if (j == D + A + 3) v = (float)g.b.actions[tn];
    rec[j] = v;
  }
  float4* dst = reinterpret_cast<float4*>(g.mb + (size_t)i * S);
#pragma unroll
  for (int q = 0; q < S / 4; ++q) {
    dst[q] = make_float4(rec[4 * q], rec[4 * q + 1], rec[4 * q + 2], rec[4 * q + 3]);
  }
}

// wide records: one thread per record element (row i = e / stride, field j), so the record
// stores are fully coalesced and each row's fields are read contiguously; the row's permuted
// source index is recomputed per element
__global__ void k_gather(GatherArgs g) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (uint32_t)g.rows * (uint32_t)g.stride) return;
  const uint32_t i = e / (uint32_t)g.stride, j = e - i * (uint32_t)g.stride;
  const int64_t tn = gather_src(g, i);
  const int D = g.D, A = g.A;
  float v = 0.f;
  if ((int)j < D) v = g.b.obs[tn * D + j];
  else if ((int)j < D + A) v = g.b.logits[tn * A + (j - D)];
  else if ((int)j == D + A) v = g.b.adv[tn];
  else if ((int)j == D + A + 1) v = g.b.vtarg[tn];
  else if ((int)j == D + A + 2) v = g.b.logp[tn];
  else if ((int)j == D + A + 3) v = (float)g.b.actions[tn];
  g.mb[(size_t)e] = v;
}

// Sample records in rollout order, one 64-byte-aligned record per sample (c2 / c4: exactly one
// 64-byte line), so that a minibatch gather reads one line per row instead of one line from each
// of the six rollout arrays (obs, logits, adv, vtarg, logp, action): one thread per sample, 16-byte
// streaming stores.
template <int PS>
__global__ __launch_bounds__(256) void k_pack(rlks_rollout_bufs b, int D, int A, float* __restrict__ packed) {
  constexpr int TPR = PS / 4;  // threads per record, thread q writes floats [4q, 4q + 4)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tn = e / TPR;
  const int q = (int)(e % TPR);
  if (tn >= (int64_t)b.T * b.N) return;
  float rec[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int j = 4 * q + c;
    float v = 0.f;
    if (j < D) v = b.obs[tn * D + j];
    else if (j < D + A) v = b.logits[tn * A + (j - D)];
    else if (j == D + A) v = b.adv[tn];
    else if (j == D + A + 1) v = b.vtarg[tn];
    else if (j == D + A + 2) v = b.logp[tn];
    else if (j == D + A + 3) v = (float)b.actions[tn];
    rec[c] = v;
  }
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f32x4{rec[0], rec[1], rec[2], rec[3]}, reinterpret_cast<f32x4*>(packed + tn * PS) + q);
}

// minibatch rows from packed records: PS / 4 consecutive threads per row, thread q moving the
// record's 16-byte piece q, so that every load instruction reads whole 64-byte lines (one line
// per row for PS = 16) and the stores are contiguous
template <int S, int PS>
__device__ __forceinline__ void gather_packed_elem(const Perm* perm, int64_t row0g, int rows_g, int Ng, int N, int rows,
                                                   const float* packed, float* mb, uint32_t e) {
  constexpr int TPR = PS / 4;
  const uint32_t i = e / TPR, q = e % TPR;
  if (i >= (uint32_t)rows) return;
  const int64_t tn = gather_src(perm, row0g, rows_g, Ng, N, i, (rows + rows_g - 1) / rows_g);
  const float4 v = reinterpret_cast<const float4*>(packed + tn * PS)[q];
  if (4 * q < (uint32_t)S) reinterpret_cast<float4*>(mb + (size_t)i * S)[q] = v;
}
template <int S, int PS>
__global__ __launch_bounds__(256) void k_gather_packed(GatherArgs g) {
  gather_packed_elem<S, PS>(g.perm, g.row0g, g.rows_g, g.Ng, g.b.N, g.rows, g.packed, g.mb,
                            blockIdx.x * blockDim.x + threadIdx.x);
}

// The next SGD step's packed gather, run by extra blocks of this step's reduce (single rank): the
// reduce reads only gradient partials, and every kernel reading the minibatch buffer has finished
// when it starts, so the gather may rewrite that buffer; one launch instead of two, and the gather's
// latency-bound reads hide under the reduce's streaming.
constexpr int NEXT_GROUPS = 8;
struct NextGather {
  Perm perm[NEXT_GROUPS];
  int64_t row0g;
  int rows, rows_g, Ng, N;
  float* mb;
  const float* packed;
  int blk0;  // blocks [0, blk0) reduce, the rest gather
};
template <int S, int PS>
__global__ __launch_bounds__(256) void k_reduce_gather(RedArgs g, NextGather n) {
  if ((int)blockIdx.x < n.blk0) {
    reduce_block(g, (int)blockIdx.x);
    return;
  }
  gather_packed_elem<S, PS>(n.perm, n.row0g, n.rows_g, n.Ng, n.N, n.rows, n.packed, n.mb,
                            ((uint32_t)blockIdx.x - (uint32_t)n.blk0) * 256u + threadIdx.x);
}

static Perm make_perm(uint64_t seed, int epoch, uint64_t S) {
  Perm P{};
  uint32_t bits = 2;
  while ((1ull << bits) < S) ++bits;
  if (bits & 1) ++bits;
  P.half = bits / 2;
  P.mask = (P.half >= 32) ? 0xffffffffu : ((1u << P.half) - 1u);
  P.S = S;
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(epoch + 1));
  for (int r = 0; r < 4; ++r) {  // splitmix64 round keys
    z += 0x9E3779B97F4A7C15ull;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    P.key[r] = (uint32_t)(x ^ (x >> 31));
  }
  return P;
}

// ----------------------------------------------------------------------------- workspace
struct NetWs {
  float *dz2, *part_b2, *part_w3, *part_b3, *part_stat, *part_w2, *part_w1, *part_b1;
};
struct Ws {
  NetWs n[2];
  double* stat64;  // [2][4]
  int64_t bytes;
  int tiles, splits;
};

static int pick_splits(int M) {
  // F2 grid = 4 tiles x 2 nets x S: about four workgroups per CU, >= 4 chunks of rows per split
  int s = 1;
  while (s * 2 * 8 <= 1024 && (M / (s * 2)) % BK == 0 && M / (s * 2) >= 4 * BK) s *= 2;
  return s;
}

static Ws ws_layout(int D, int A, int M, char* base) {
  Ws w{};
  w.tiles = M / GB;
  w.splits = pick_splits(M);
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + o : nullptr;
    o += (bytes + 255) / 256 * 256;
    return p;
  };
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    NetWs& n = w.n[net];
    n.dz2 = (float*)take(4LL * M * HID);
    n.part_b2 = (float*)take(4LL * w.tiles * HID);
    n.part_w3 = (float*)take(4LL * w.tiles * An * HID);
    n.part_b3 = (float*)take(4LL * w.tiles * (net == 0 ? A : 2));  // value net: [tile][hi, lo] (vf_row)
    n.part_stat = (float*)take(4LL * w.tiles * 4);
    n.part_w2 = (float*)take(4LL * w.splits * HID * HID);
    n.part_w1 = (float*)take(4LL * w.tiles * HID * D);
    n.part_b1 = (float*)take(4LL * w.tiles * HID);
  }
  w.stat64 = (double*)take(8 * 8);
  w.bytes = o;
  return w;
}

// split-fp16 path: pre-split weights, dZ2^T, per-F1-block and per-F2-split partials
struct SfWs {
  SfNetW w[2];
  SfNet n[2];
  double* stat64;
  float* pmax_roll[2];  // the rollout's weight-max slots (the SGD steps' pmax keeps its parity state)
  _Float16* xsp;        // F1a's Xa split for F2 (SfArgs::xsp)
  int64_t bytes, weight_bytes;
  int blocks, splits, tiles_per_split;
  int fa_parts;  // F1's dW3 / db3 / stats partials per net (the split kernels' count: the allocation)
};

static SfWs sf_ws_layout(int D, int A, int M, char* base) {
  SfWs w{};
  const int KD = sf_kd(D), tiles = M / 32;  // F2's 32-row tiles
  w.blocks = M / (16 * SF_F1_W);  // F1 workgroups of SF_F1_W x 16 rows
  w.fa_parts = sf_f1_parts(M, false);
  w.splits = 1;
  constexpr int F2_MAX_SPLITS = 128;  // F2 row splits per net (one 512-thread workgroup each)
  while (w.splits * 2 <= F2_MAX_SPLITS && tiles % (w.splits * 2) == 0) w.splits *= 2;
  w.tiles_per_split = tiles > 0 ? tiles / w.splits : 0;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + o : nullptr;
    o += (bytes + 255) / 256 * 256;
    return p;
  };
  // split weights of both nets first: their offsets do not depend on M (the rollout shares them)
  for (int net = 0; net < 2; ++net) {
    SfNetW& W = w.w[net];
    SfNet& n = w.n[net];
    W.w1h = (_Float16*)take(2LL * HID * KD);
    W.w1l = (_Float16*)take(2LL * HID * KD);
    W.w2ph = (_Float16*)take(2LL * HID * HID);
    W.w2pl = (_Float16*)take(2LL * HID * HID);
    W.w2th = (_Float16*)take(2LL * HID * HID);
    W.w2tl = (_Float16*)take(2LL * HID * HID);
    W.w2rh = (_Float16*)take(2LL * HID * HID);
    W.w2rl = (_Float16*)take(2LL * HID * HID);
    W.sc = (float*)take(4 * 8);
    W.pmax = (float*)take(4LL * 4 * SF_PMAX);
    W.tag = (unsigned*)take(4 * 2);
    w.pmax_roll[net] = (float*)take(4LL * 4 * SF_PMAX);
    n.w1h = W.w1h; n.w1l = W.w1l; n.w2ph = W.w2ph; n.w2pl = W.w2pl; n.w2th = W.w2th; n.w2tl = W.w2tl;
    n.sc = W.sc;
  }
  w.weight_bytes = o;
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    SfNet& n = w.n[net];
    n.dz2s = (_Float16*)take(4LL * M * HID);
    n.tile_edz = (int*)take(4LL * (M / 16));
    n.tile_ex = (int*)take(4LL * (M / 16));
    n.part_w1 = (float*)take(4LL * w.blocks * HID * D);
    n.part_b1 = (float*)take(4LL * w.blocks * HID);
    n.part_w3 = (float*)take(4LL * w.fa_parts * An * HID);
    n.part_b3 = (float*)take(4LL * w.fa_parts * (net == 0 ? A : 2));  // value net: [part][hi, lo] (vf_row)
    n.part_stat = (float*)take(4LL * w.fa_parts * 4);
    n.part_w2 = (float*)take(4LL * w.splits * SF_W2_PSTRIDE);
    n.part_b2 = (float*)take(4LL * w.splits * HID);
  }
  w.stat64 = (double*)take(8 * 8);
  w.xsp = (_Float16*)take(2LL * 2 * M * KD);
  w.bytes = o;
  return w;
}

// Weight splits for the split-fp16 kernels.  rollout: also the rollout's fragment-order copy of W2,
// with the max |w| slots of its own.  SGD step: `parity` selects the max slots (see SfPrepArgs);
// skip_wmax when the previous fused SGD step left this step's maxima there.
static int sf_prep(const rlks_mlp_desc* d, const SfWs& w, const float* params, hipStream_t s, bool rollout,
                   int parity = 0, bool skip_wmax = false, unsigned expect_tag = 0) {
  const int D = d->obs_dim;
  const Layout L = make_layout(D, HID, d->n_actions);
  SfPrepArgs pa{};
  pa.D = D;
  pa.KD = sf_kd(D);
  pa.parity = rollout ? 0 : parity;
  pa.skip_wmax = rollout ? 0 : (skip_wmax ? 1 : 0);
  pa.write_roll = rollout ? 1 : 0;
  pa.expect_tag = expect_tag;
  for (int net = 0; net < 2; ++net) {
    pa.n[net] = w.w[net];
    if (rollout) pa.n[net].pmax = w.pmax_roll[net];
    const NetPtrs P = net_ptrs_host(params, L, net);
    pa.n[net].w1 = P.w1; pa.n[net].b1 = P.b1; pa.n[net].w2 = P.w2;
  }
  return launch_sf_prep(pa, s);
}

// 2-cloud split-fp16 rollouts: up to this many lanes one persistent k_sf_roll launch runs the whole
// rollout (each workgroup loops over the T steps of its 32 lanes: a latency design, c2's 4,096 lanes
// are 128 workgroups); above it each step is k_sf_fwd16 + k_sample_step over all lanes (c4: 131,072
// lanes, 24.5 -> 14.5 ms per rollout, profiles/r04c)
constexpr int SF_ROLL_FUSED_MAX_LANES = 16384;

static bool is_wide(const rlks_mlp_desc* d) { return d->precision == RLKS_PRECISION_WIDE || wide_needed(d); }
// the split-fp16 fused kernels (fp32-accurate, or the one-product throughput mode)
static bool is_sf(const rlks_mlp_desc* d) {
  return d->precision == RLKS_PRECISION_SF16 || d->precision == RLKS_PRECISION_F16;
}

// the fused kernels (mlp_fwd / mlp_bwd / sgd_sf16 / rollout_sf16) cover hidden 256, obs < 32 and
// 2 / 4 / 8 actions; everything else runs on the generic-width path (wide_mlp.hip)
static int check_desc(const rlks_mlp_desc* d) {
  RLKS_REQUIRE(d, RLKS_ERR_ARG, "null mlp desc");
  RLKS_REQUIRE(d->precision == RLKS_PRECISION_FP32 || d->precision == RLKS_PRECISION_SF16 ||
                   d->precision == RLKS_PRECISION_WIDE || d->precision == RLKS_PRECISION_F16, RLKS_ERR_ARG,
               "unknown precision");
  RLKS_REQUIRE(d->obs_dim > 0 && d->hidden > 0 && d->hidden % 32 == 0 && d->hidden <= 8192 && d->n_actions > 0 &&
                   d->n_actions <= 64, RLKS_ERR_UNSUPPORTED,
               "MLP: hidden must be a multiple of 32 (<= 8192), 1 <= n_actions <= 64");
  if (!is_wide(d))
    RLKS_REQUIRE(d->obs_dim <= DMAX && (d->n_actions == 2 || d->n_actions == 4 || d->n_actions == 8),
                 RLKS_ERR_UNSUPPORTED, "fused MLP kernels: obs_dim in [1, 32], 2, 4 or 8 actions");
  return RLKS_OK;
}

// Node-level envs (nodes_per_cluster > 0): the node sweep has its own workgroup shape (k_node_step:
// 64 envs x W waves), so a rollout step is three launches on the stream: forward of both nets on
// obs[t] (logits[t], values[t]) -> Categorical sample (actions[t], logp[t]) -> trusted env step
// (obs[t + 1], f32 rewards[t], dones[t]); then the bootstrap V(obs[T]).  `w` = the split-fp16
// weights (SF16) or nullptr (fp32 kernels).
static int node_rollout(rlks_env* env, const rlks_mlp_desc* d, const float* params, const rlks_rollout_bufs* b,
                        int explore, const SfWs* w, hipStream_t s) {
  const int N = b->N, D = d->obs_dim, A = d->n_actions;
  const Layout L = make_layout(D, HID, A);
  SfFwdArgs r{};
  if (w) {
    if (int rc = sf_prep(d, *w, params, s, true)) return rc;
    for (int net = 0; net < 2; ++net) {
      const NetPtrs P = net_ptrs_host(params, L, net);
      r.n[net] = w->n[net];
      r.n[net].b2 = P.b2; r.n[net].w3 = P.w3; r.n[net].b3 = P.b3;
    }
    r.M = N; r.D = D;
  }
  auto forward = [&](const float* x, float* logits, float* values, int M = -1, hipStream_t fs = nullptr) -> int {
    if (w) {  // 16-row tiles of both nets (sgd_sf16.hip k_sf_fwd16)
      SfFwdArgs a = r;
      a.x = x;
      a.M = M < 0 ? N : M;
      a.out[0] = logits;
      a.out[1] = values;
      return launch_sf_fwd16(a, A, fs ? fs : s);
    }
    for (int net = 0; net < 2; ++net) {
      float* out = net == 0 ? logits : values;
      if (!out) continue;
      FwdArgs f{};
      f.P = net_ptrs_host(params, L, net);
      f.x = x; f.x_stride = D; f.M = N; f.D = D; f.A_pi = A; f.out = out;
      if (int rc = launch_fwd_head(f, net, A, FWD_ONLY, s)) return rc;
    }
    return RLKS_OK;
  };
  const EnvView v = view(env);
  // Two lane halves on two streams (opt-in: RLKS_NODE_TWO_STREAMS=1): each half runs
  // forward -> sample -> node step on its own stream, so that one half's latency-bound node step could
  // run beside the other half's forward.  Same launches per lane, Philox counters per lane: the same
  // rollout bit for bit.  Measured at c3 (profiles/r06_node): 12.9-13.0 ms a rollout against 12.7 ms in
  // one stream -- the half-size forward keeps every CU's wave slots (4 waves per SIMD at 128
  // registers), so the node step finds none free beside it and the split only adds its overheads.
  const int half = (N / 2) / 128 * 128;
  if (w && N >= 8192 && env->cfg.nodes_per_cluster > 0 && env->cfg.n_clouds <= 64 && getenv("RLKS_NODE_TWO_STREAMS")) {
    if (!env->side) {
      RLKS_HIP(hipStreamCreateWithFlags(&env->side, hipStreamNonBlocking));
      RLKS_HIP(hipEventCreateWithFlags(&env->ev_fork, hipEventDisableTiming));
      RLKS_HIP(hipEventCreateWithFlags(&env->ev_join, hipEventDisableTiming));
    }
    RLKS_HIP(hipEventRecord(env->ev_fork, s));
    RLKS_HIP(hipStreamWaitEvent(env->side, env->ev_fork, 0));
    const int lo[2] = {0, half}, hi[2] = {half, N};
    const hipStream_t hs[2] = {s, env->side};
    for (int t = 0; t < b->T; ++t) {
      const size_t tN = (size_t)t * N;
      for (int h = 0; h < 2; ++h) {
        const size_t o = tN + lo[h];
        if (int rc = forward(b->obs + o * D, b->logits + o * A, b->values + o, hi[h] - lo[h], hs[h])) return rc;
        EnvView vh = v;
        vh.lane0 = lo[h];
        vh.lane_end = hi[h];
        if (int rc = launch_sample(vh, b->logits + tN * A, A, explore, b->actions + tN, b->logp + tN, hs[h])) return rc;
        if (!node_step_range(env, lo[h], hi[h], b->actions + tN, b->obs + (tN + N) * D, b->rewards + tN,
                             b->dones + tN, hs[h]))
          return fail(RLKS_ERR_HIP, "node_rollout: lane-range node step");
      }
    }
    for (int h = 0; h < 2; ++h) {
      const size_t o = (size_t)b->T * N + lo[h];
      if (int rc = forward(b->obs + o * D, nullptr, b->values + o, hi[h] - lo[h], hs[h])) return rc;
    }
    RLKS_HIP(hipEventRecord(env->ev_join, env->side));
    RLKS_HIP(hipStreamWaitEvent(s, env->ev_join, 0));
    return RLKS_OK;
  }
  for (int t = 0; t < b->T; ++t) {
    const size_t tN = (size_t)t * N;
    if (int rc = forward(b->obs + tN * D, b->logits + tN * A, b->values + tN)) return rc;
    if (int rc = launch_sample(v, b->logits + tN * A, A, explore, b->actions + tN, b->logp + tN, s)) return rc;
    if (int rc = rlks_env_step(env, b->actions + tN, b->obs + (tN + N) * D, nullptr, b->rewards + tN, b->dones + tN,
                               nullptr, nullptr, nullptr, nullptr, s))
      return rc;
  }
  return forward(b->obs + (size_t)b->T * N * D, nullptr, b->values + (size_t)b->T * N);
}

__global__ void k_empty() {}  // (rlks_ppo_grad_profile: the event bracket's own time)

}  // namespace rlks

using namespace rlks;

extern "C" {

int rlks_mlp_layout(const rlks_mlp_desc* d, int64_t* offsets, int64_t* padded, int64_t* real) {
  RLKS_REQUIRE(d && d->obs_dim > 0 && d->hidden > 0 && d->n_actions > 0, RLKS_ERR_ARG, "rlks_mlp_layout: bad desc");
  const Layout L = make_layout(d->obs_dim, d->hidden, d->n_actions);
  if (offsets)
    for (int i = 0; i < RLKS_N_TENSORS; ++i) offsets[i] = L.off[i];
  if (padded) *padded = L.padded;
  if (real) *real = L.real;
  return RLKS_OK;
}

int rlks_policy_forward(const rlks_mlp_desc* d, const float* params, const float* obs, int n, float* logits,
                        float* values, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(!is_wide(d), RLKS_ERR_UNSUPPORTED, "rlks_policy_forward: this MLP needs rlks_policy_forward_ws");
  RLKS_REQUIRE(params && obs && n >= 0, RLKS_ERR_ARG, "rlks_policy_forward: bad argument");
  if (n == 0) return RLKS_OK;
  const Layout L = make_layout(d->obs_dim, d->hidden, d->n_actions);
  hipStream_t s = (hipStream_t)stream;
  for (int net = 0; net < 2; ++net) {
    float* out = net == 0 ? logits : values;
    if (!out) continue;
    FwdArgs a{};
    a.P = net_ptrs_host(params, L, net);
    a.x = obs; a.x_stride = d->obs_dim; a.M = n; a.D = d->obs_dim; a.A_pi = d->n_actions; a.out = out;
    if (int rc = launch_fwd_head(a, net, d->n_actions, FWD_ONLY, s)) return rc;
  }
  return RLKS_OK;
}

int rlks_minibatch_stride(const rlks_mlp_desc* d) { return d ? mb_stride(d->obs_dim, d->n_actions) : 0; }

int rlks_ppo_gather(const rlks_mlp_desc* d, const rlks_rollout_bufs* b, uint64_t perm_seed, int epoch,
                    int64_t row0, int rows, const float* dyn, float* mb, void* stream) {
  return rlks_ppo_gather_grouped(d, b, perm_seed, epoch, 1, 0, row0, rows, dyn, mb, stream);
}

static int gather_args(const rlks_mlp_desc* d, int T, int N, uint64_t perm_seed, int epoch, int groups, int group0,
                       int64_t row0, int rows, float* mb, GatherArgs& g) {
  RLKS_REQUIRE(groups >= 1 && groups <= MAX_GROUPS && group0 >= 0 && N % groups == 0 && rows % groups == 0 &&
                   row0 % groups == 0, RLKS_ERR_ARG,
               "rlks_ppo_gather: groups must divide the lanes, the rows and row0 (at most 64 groups)");
  const int Ng = N / groups;
  const uint64_t Sg = (uint64_t)T * (uint64_t)Ng;
  RLKS_REQUIRE(row0 >= 0 && (uint64_t)(row0 + rows) / groups <= Sg, RLKS_ERR_ARG, "rlks_ppo_gather: rows out of range");
  g = GatherArgs{};
  // group k's key: perm_seed for global group 0 (the single-group gather), else perm_seed offset by
  // an odd 64-bit multiple of the global group id
  for (int k = 0; k < groups; ++k)
    g.perm[k] = make_perm(perm_seed + 0x632BE59BD9B4E019ull * (uint64_t)(group0 + k), epoch, Sg);
  g.row0g = row0 / groups;
  g.rows_g = rows / groups;
  g.Ng = Ng;
  g.rows = rows;
  g.D = d->obs_dim;
  g.A = d->n_actions;
  g.stride = mb_stride(d->obs_dim, d->n_actions);
  g.mb = mb;
  RLKS_REQUIRE((int64_t)rows * g.stride < (int64_t)1 << 31, RLKS_ERR_UNSUPPORTED,
               "rlks_ppo_gather: at most 2^31 record elements per call");
  return RLKS_OK;
}

int rlks_ppo_gather_grouped(const rlks_mlp_desc* d, const rlks_rollout_bufs* b, uint64_t perm_seed, int epoch,
                            int groups, int group0, int64_t row0, int rows, const float* dyn, float* mb,
                            void* stream) {
  RLKS_REQUIRE(d && b && mb && rows >= 0, RLKS_ERR_ARG, "rlks_ppo_gather: bad argument");
  (void)dyn;  // advantages are standardised inside the loss kernel from dyn
  GatherArgs g;
  if (int rc = gather_args(d, b->T, b->N, perm_seed, epoch, groups, group0, row0, rows, mb, g)) return rc;
  if (rows == 0) return RLKS_OK;
  g.b = *b;
  const dim3 rg(cdiv(rows, 256));
  if (g.stride == 12) hipLaunchKernelGGL(k_gather_rows<12>, rg, dim3(256), 0, (hipStream_t)stream, g);
  else if (g.stride == 20) hipLaunchKernelGGL(k_gather_rows<20>, rg, dim3(256), 0, (hipStream_t)stream, g);
  else if (g.stride == 36) hipLaunchKernelGGL(k_gather_rows<36>, rg, dim3(256), 0, (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL(k_gather, dim3(cdiv(rows * g.stride, 256)), dim3(256), 0, (hipStream_t)stream, g);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_packed_stride(const rlks_mlp_desc* d) {
  if (!d) return 0;
  const int s = mb_stride(d->obs_dim, d->n_actions);
  return s == 12 ? 16 : s == 20 ? 32 : s == 36 ? 48 : 0;
}

int rlks_ppo_pack(const rlks_mlp_desc* d, const rlks_rollout_bufs* b, float* packed, void* stream) {
  RLKS_REQUIRE(d && b && packed && b->T > 0 && b->N > 0, RLKS_ERR_ARG, "rlks_ppo_pack: bad argument");
  const int ps = rlks_packed_stride(d);
  RLKS_REQUIRE(ps > 0, RLKS_ERR_UNSUPPORTED, "rlks_ppo_pack: records of 2, 4 or 8 clouds (obs 6 / 12 / 24) only");
  const int64_t n = (int64_t)b->T * b->N;
  const dim3 grid(cdiv(n * (ps / 4), 256));
  hipStream_t s = (hipStream_t)stream;
  const int D = d->obs_dim, A = d->n_actions;
  if (ps == 16) hipLaunchKernelGGL(k_pack<16>, grid, dim3(256), 0, s, *b, D, A, packed);
  else if (ps == 32) hipLaunchKernelGGL(k_pack<32>, grid, dim3(256), 0, s, *b, D, A, packed);
  else hipLaunchKernelGGL(k_pack<48>, grid, dim3(256), 0, s, *b, D, A, packed);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_ppo_gather_packed(const rlks_mlp_desc* d, const float* packed, int T, int N, uint64_t perm_seed, int epoch,
                           int groups, int group0, int64_t row0, int rows, float* mb, void* stream) {
  RLKS_REQUIRE(d && packed && mb && rows >= 0 && T > 0 && N > 0, RLKS_ERR_ARG, "rlks_ppo_gather_packed: bad argument");
  const int ps = rlks_packed_stride(d);
  RLKS_REQUIRE(ps > 0, RLKS_ERR_UNSUPPORTED, "rlks_ppo_gather_packed: records of 2, 4 or 8 clouds only");
  GatherArgs g;
  if (int rc = gather_args(d, T, N, perm_seed, epoch, groups, group0, row0, rows, mb, g)) return rc;
  if (rows == 0) return RLKS_OK;
  g.b.T = T;
  g.b.N = N;
  g.packed = packed;
  g.pstride = ps;
  hipStream_t s = (hipStream_t)stream;
  const dim3 rg(cdiv((int64_t)rows * ps / 4, 256));
  if (g.stride == 12) hipLaunchKernelGGL((k_gather_packed<12, 16>), rg, dim3(256), 0, s, g);
  else if (g.stride == 20) hipLaunchKernelGGL((k_gather_packed<20, 32>), rg, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_gather_packed<36, 48>), rg, dim3(256), 0, s, g);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_policy_forward_ws(const rlks_mlp_desc* d, const float* params, const float* obs, int n, float* logits,
                           float* values, void* workspace, int64_t ws_bytes, void* stream) {
  if (int rc = check_desc(d)) return rc;
  if (!is_wide(d)) return rlks_policy_forward(d, params, obs, n, logits, values, stream);
  RLKS_REQUIRE(params && obs && n >= 0 && workspace, RLKS_ERR_ARG, "rlks_policy_forward_ws: bad argument");
  if (n == 0) return RLKS_OK;
  const WideWs w = wide_ws_layout(d->obs_dim, d->hidden, d->n_actions, n, (char*)workspace);
  RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_policy_forward_ws: workspace too small");
  return wide_forward(d, params, obs, d->obs_dim, n, w, logits, values, (hipStream_t)stream);
}

int rlks_ppo_workspace_bytes(const rlks_mlp_desc* d, int rows, int64_t* bytes) {
  if (int rc = check_desc(d)) return rc;
  if (is_wide(d)) {
    RLKS_REQUIRE(bytes && rows > 0, RLKS_ERR_ARG, "rlks_ppo_workspace_bytes: bad argument");
    *bytes = wide_ws_layout(d->obs_dim, d->hidden, d->n_actions, rows, nullptr).bytes;
    return RLKS_OK;
  }
  if (is_sf(d)) {
    RLKS_REQUIRE(bytes && rows > 0 && rows % 256 == 0, RLKS_ERR_ARG,
                 "rlks_ppo_workspace_bytes: split-fp16 rows must be a positive multiple of 256");
    *bytes = sf_ws_layout(d->obs_dim, d->n_actions, rows, nullptr).bytes;
    return RLKS_OK;
  }
  RLKS_REQUIRE(bytes && rows > 0 && rows % GB == 0, RLKS_ERR_ARG,
               "rlks_ppo_workspace_bytes: rows must be a positive multiple of 128");
  *bytes = ws_layout(d->obs_dim, d->n_actions, rows, nullptr).bytes;
  return RLKS_OK;
}

int rlks_debug_sf_handoff(const rlks_mlp_desc* d, int rows, void* ws, void** out) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(out && ws && rows > 0 && rows % 256 == 0 && is_sf(d) && !is_wide(d),
               RLKS_ERR_ARG, "rlks_debug_sf_handoff: split-fp16 descriptor, rows % 256 == 0");
  const SfWs w = sf_ws_layout(d->obs_dim, d->n_actions, rows, (char*)ws);
  for (int net = 0; net < 2; ++net) {
    out[net] = w.n[net].dz2s;
    out[2 + net] = w.n[net].tile_edz;
  }
  return RLKS_OK;
}

int rlks_debug_wide_bufs(const rlks_mlp_desc* d, int rows, void* ws, void** out) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(out && ws && rows > 0 && is_wide(d), RLKS_ERR_ARG, "rlks_debug_wide_bufs: wide descriptor");
  const WideWs w = wide_ws_layout(d->obs_dim, d->hidden, d->n_actions, rows, (char*)ws);
  for (int net = 0; net < 2; ++net) {
    out[3 * net] = w.n[net].h2;
    out[3 * net + 1] = w.n[net].out;
    out[3 * net + 2] = w.n[net].dout;
  }
  return RLKS_OK;
}

// SGD step with Adam fused into the gradient reduction (single rank: no gradient all-reduce between
// them).  step: the Adam step performed (1-based); prev_fused: the previous SGD step on these
// parameters was fused, so its reduce left this step's weight maxima in the split's slots.
struct FusedAdam {
  float *p, *m, *v;
  AdamCo co;
  int step, prev_fused;
  bool apply = true;  // false: the prep uses the previous step's maxima, the reduce only sums (an
                      // all-reduce follows; rlks_ppo_adam_apply then applies Adam)
};

// part: 0 = the whole gradient; 1 = the weight split, F1a, F2 and the reduce of W2 / b2 / W3 / b3 and
// the stats; 2 = F1b and the reduce of W1 / b1 (rlks_ppo_grad_step_part: the caller all-reduces part
// 1's buckets while part 2 runs)
static int sf_grad(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                   const float* mb, int M, float* grad, double* stats, void* workspace, int64_t ws_bytes, int phases,
                   hipStream_t s, const FusedAdam* fa = nullptr, const NextGather* nx = nullptr, int part = 0) {
  RLKS_REQUIRE(M > 0 && M % 256 == 0, RLKS_ERR_ARG, "rlks_ppo_grad: split-fp16 rows must be a positive multiple of 256");
  const int D = d->obs_dim, A = d->n_actions, H = HID;
  const SfWs w = sf_ws_layout(D, A, M, (char*)workspace);
  RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_ppo_grad: workspace too small");
  const Layout L = make_layout(D, H, A);
  const bool f_pi = phases & (RLKS_PHASE_FWD | RLKS_PHASE_FWD_PI), f_vf = phases & (RLKS_PHASE_FWD | RLKS_PHASE_FWD_VF);
  if (part == 2) phases &= ~(RLKS_PHASE_PREP | RLKS_PHASE_DW2);
  if ((phases & (RLKS_PHASE_FWD | RLKS_PHASE_PREP)) && part != 2) {
    const int parity = fa ? ((fa->step - 1) & 1) : 0;
    if (int rc = sf_prep(d, w, params, s, false, parity, fa && fa->prev_fused, fa ? (unsigned)fa->step : 0u))
      return rc;
  }
  SfArgs a{};
  a.x = mb; a.x_stride = mb_stride(D, A); a.M = M; a.D = D; a.A_pi = A;
  a.tiles_per_split = w.tiles_per_split; a.co = *co; a.dyn = dyn; a.xsp = w.xsp;
  a.products = d->precision == RLKS_PRECISION_F16 ? 1 : 3;
  for (int net = 0; net < 2; ++net) {
    a.n[net] = w.n[net];
    const NetPtrs P = net_ptrs_host(params, L, net);
    a.n[net].b2 = P.b2; a.n[net].w3 = P.w3; a.n[net].b3 = P.b3;
  }
  // F1 (forward, loss, dZ2, dH1 -> dW1 / db1, dW3 / db3) per net; F2 (dW2, db2) for both.  F1 is the
  // fused kernel for a whole gradient (part 0: rlks_ppo_grad, the fused-Adam SGD step, the multi-rank
  // step's one-bucket form) where sf_f1_fused says so, else the two kernels F1a, F1b; the overlapped
  // multi-rank form (part 1 / 2: F1b under the all-reduce) always runs the two
  const bool fused_f1 = part == 0 && sf_f1_fused(A);
  if (f_pi || f_vf) {
    const int net0 = f_pi ? 0 : 1, nets = (f_pi && f_vf) ? 2 : 1;
    if (fused_f1 || part != 0) {
      if (int rc = launch_sf_f1(a, net0, nets, A, s, fused_f1 ? SF_F1_FUSED : part)) return rc;
    } else {
      if (int rc = launch_sf_f1(a, net0, nets, A, s, 3)) return rc;
    }
  }
  // split F1 halves alone, both nets (profiling: each reads what a full F1 left in the workspace)
  if (!(f_pi || f_vf) && (phases & (RLKS_PHASE_F1A | RLKS_PHASE_F1B)))
    if (int rc = launch_sf_f1(a, 0, 2, A, s, (phases & RLKS_PHASE_F1A ? 1 : 0) | (phases & RLKS_PHASE_F1B ? 2 : 0)))
      return rc;
  if (phases & RLKS_PHASE_DW2)
    if (int rc = launch_sf_dw2(a, w.splits, s)) return rc;
  if (!(phases & RLKS_PHASE_REDUCE)) return RLKS_OK;
  // F1's partial count: the fused kernel has half the split kernels' workgroups
  const int f1p = sf_f1_parts(M, fused_f1);
  Reducer R;
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    const int64_t* o = L.off + 6 * net;
    const SfNet& n = w.n[net];
    if (part != 1) {
      R.add(n.part_w1, grad + o[0], nullptr, (int64_t)H * D, f1p, H * D, 2 * net + 1);
      R.add(n.part_b1, grad + o[1], nullptr, H, f1p, H, 2 * net + 1);
    }
    if (part != 2) {
      R.add(n.part_w2, grad + o[2], nullptr, SF_W2_PSTRIDE, w.splits, H * H, 2 * net);
      R.a.t[R.a.ntasks - 1].kq = sf_f2_regs() ? 1 : 0;
      R.add(n.part_b2, grad + o[3], nullptr, H, w.splits, H);
      R.add(n.part_w3, grad + o[4], nullptr, (int64_t)An * H, f1p, An * H);
      if (net == 0) R.add(n.part_b3, grad + o[5], nullptr, An, f1p, An);
      else R.add(n.part_b3, grad + o[5], nullptr, 1, 2 * f1p, 1);  // every hi and lo, in f64
    }
  }
  if (stats && part != 2) {  // per-block columns [policy loss, vf loss, kl, entropy] -> RLKS_STAT_* directly
    const int tiles = f1p;
    R.add(w.n[0].part_stat + 0, nullptr, stats + RLKS_STAT_POLICY_LOSS, 4, tiles, 1);
    R.add(w.n[1].part_stat + 1, nullptr, stats + RLKS_STAT_VF_LOSS, 4, tiles, 1);
    R.add(w.n[0].part_stat + 2, nullptr, stats + RLKS_STAT_KL, 4, tiles, 1);
    R.add(w.n[0].part_stat + 3, nullptr, stats + RLKS_STAT_ENTROPY, 4, tiles, 1);
    R.a.stats = stats;
    R.a.rows = (double)M;
  }
  if (fa && fa->apply) {  // Adam on every parameter as its gradient is summed; W2 / W1a maxima -> the next prep
    RLKS_REQUIRE(part == 0, RLKS_ERR_ARG, "sf_grad: fused Adam needs the whole gradient");
    for (int k = 0; k < 4; ++k)
      RLKS_REQUIRE(R.mnext[k] <= SF_PMAX, RLKS_ERR_UNSUPPORTED, "rlks_ppo_sgd_step: too many reduce blocks per weight");
    R.a.p = fa->p; R.a.m = fa->m; R.a.v = fa->v; R.a.grad = grad; R.a.co = fa->co;
    const int par = fa->step & 1;
    for (int net = 0; net < 2; ++net) {
      R.a.slot[2 * net] = w.w[net].pmax + (par * 2 + 0) * SF_PMAX;
      R.a.slot[2 * net + 1] = w.w[net].pmax + (par * 2 + 1) * SF_PMAX;
    }
    // the slots are complete when the reduce is (the next prep is a later launch): mark them as
    // this step's
    R.a.tag[0] = w.w[0].tag + par;
    R.a.tag[1] = w.w[1].tag + par;
    R.a.tag_val = (unsigned)fa->step + 1u;  // tag of step s = s + 1 (0: none), expected by step s + 1's prep
  }
  if (nx && nx->rows > 0) {  // + the next step's gather (blocks after the reduce's)
    NextGather n = *nx;
    n.blk0 = R.blocks;
    const int ps = rlks_packed_stride(d), stride = mb_stride(D, A);
    const dim3 grid(R.blocks + (int)cdiv((int64_t)n.rows * ps / 4, 256));
    if (stride == 12) hipLaunchKernelGGL((k_reduce_gather<12, 16>), grid, dim3(256), 0, s, R.a, n);
    else if (stride == 20) hipLaunchKernelGGL((k_reduce_gather<20, 32>), grid, dim3(256), 0, s, R.a, n);
    else hipLaunchKernelGGL((k_reduce_gather<36, 48>), grid, dim3(256), 0, s, R.a, n);
  } else {
    launch_timed(KEV_REDUCE, k_reduce, dim3(R.blocks), dim3(256), 0, s, R.a);
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_ppo_grad_phases(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                         const float* mb, int M, float* grad, double* stats, void* workspace, int64_t ws_bytes,
                         int phases, void* stream) {
  if (int rc = check_desc(d)) return rc;
  if (is_wide(d)) {
    RLKS_REQUIRE(co && params && dyn && mb && grad && workspace && M > 0, RLKS_ERR_ARG, "rlks_ppo_grad: bad argument");
    const WideWs w = wide_ws_layout(d->obs_dim, d->hidden, d->n_actions, M, (char*)workspace);
    RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_ppo_grad: workspace too small");
    (void)phases;
    return wide_grad(d, co, params, dyn, mb, M, grad, stats, w, (hipStream_t)stream);
  }
  if (is_sf(d)) {
    RLKS_REQUIRE(co && params && dyn && mb && grad && workspace, RLKS_ERR_ARG, "rlks_ppo_grad: null argument");
    return sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, phases, (hipStream_t)stream);
  }
  RLKS_REQUIRE(co && params && dyn && mb && grad && workspace, RLKS_ERR_ARG, "rlks_ppo_grad: null argument");
  RLKS_REQUIRE(M > 0 && M % GB == 0, RLKS_ERR_ARG, "rlks_ppo_grad: rows must be a positive multiple of 128");
  const int D = d->obs_dim, A = d->n_actions, H = HID;
  const Ws w = ws_layout(D, A, M, (char*)workspace);
  RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_ppo_grad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const Layout L = make_layout(D, H, A);
  const int stride = mb_stride(D, A);

  for (int net = 0; net < 2; ++net)
    if ((phases & RLKS_PHASE_FWD) || (phases & (net ? RLKS_PHASE_FWD_VF : RLKS_PHASE_FWD_PI))) {
      FwdArgs f{};
      f.P = net_ptrs_host(params, L, net);
      f.x = mb; f.x_stride = stride; f.M = M; f.D = D; f.A_pi = A;
      f.co = *co; f.dyn = dyn;
      const NetWs& n = w.n[net];
      f.dz2 = n.dz2; f.part_b2 = n.part_b2; f.part_w3 = n.part_w3; f.part_b3 = n.part_b3; f.part_stat = n.part_stat;
      if (int rc = launch_fwd_head(f, net, A, FWD_TRAIN, s)) return rc;
    }
  if (phases & RLKS_PHASE_DW2) {
    Dw2Args a{};
    a.x = mb; a.x_stride = stride; a.M = M; a.rows_per_split = M / w.splits;
    for (int net = 0; net < 2; ++net) {
      a.P[net] = net_ptrs_host(params, L, net);
      a.dz2[net] = w.n[net].dz2;
      a.part[net] = w.n[net].part_w2;
    }
    if (int rc = launch_dw2(a, D, w.splits, s)) return rc;
  }
  if (phases & RLKS_PHASE_DH1) {
    Dh1Args a{};
    a.x = mb; a.x_stride = stride; a.M = M;
    for (int net = 0; net < 2; ++net) {
      a.P[net] = net_ptrs_host(params, L, net);
      a.dz2[net] = w.n[net].dz2;
      a.part_w1[net] = w.n[net].part_w1;
      a.part_b1[net] = w.n[net].part_b1;
    }
    if (int rc = launch_dh1(a, D, s)) return rc;
  }
  if (!(phases & RLKS_PHASE_REDUCE)) return RLKS_OK;
  Reducer R;
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    const int64_t* o = L.off + 6 * net;
    const NetWs& n = w.n[net];
    R.add(n.part_w1, grad + o[0], nullptr, (int64_t)H * D, w.tiles, H * D);
    R.add(n.part_b1, grad + o[1], nullptr, H, w.tiles, H);
    R.add(n.part_w2, grad + o[2], nullptr, (int64_t)H * H, w.splits, H * H);
    R.add(n.part_b2, grad + o[3], nullptr, H, w.tiles, H);
    R.add(n.part_w3, grad + o[4], nullptr, (int64_t)An * H, w.tiles, An * H);
    if (net == 0) R.add(n.part_b3, grad + o[5], nullptr, An, w.tiles, An);
    else R.add(n.part_b3, grad + o[5], nullptr, 1, 2 * w.tiles, 1);  // every hi and lo, in f64
    if (stats) R.add(n.part_stat, nullptr, w.stat64 + 4 * net, 4, w.tiles, 4);
  }
  hipLaunchKernelGGL(k_reduce, dim3(R.blocks), dim3(256), 0, s, R.a);
  RLKS_LAUNCHED();
  if (stats) {
    hipLaunchKernelGGL(k_stats_finish, dim3(1), dim3(64), 0, s, stats, w.stat64, w.stat64 + 4, M);
    RLKS_LAUNCHED();
  }
  return RLKS_OK;
}

int rlks_sf_f1_fused(const rlks_mlp_desc* d) {
  if (!d || !is_sf(d) || is_wide(d)) return 0;
  return sf_f1_fused(d->n_actions) ? 1 : 0;
}

int rlks_ppo_grad(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                  const float* mb, int M, float* grad, double* stats, void* workspace, int64_t ws_bytes,
                  void* stream) {
  return rlks_ppo_grad_phases(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, stream);
}

int rlks_ppo_grad_profile(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                          const float* mb, int M, float* grad, double* stats, void* workspace, int64_t ws_bytes,
                          int reps, double* ms_out, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(is_sf(d) && !is_wide(d) && reps > 0 && ms_out && co && params && dyn && mb && grad && workspace,
               RLKS_ERR_ARG, "rlks_ppo_grad_profile: split-fp16 descriptor, reps > 0");
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t ev[2 * KEV_N];
  for (int i = 0; i < 2 * KEV_N; ++i)
    if (hipEventCreate(&ev[i]) != hipSuccess) return fail(RLKS_ERR_HIP, "rlks_ppo_grad_profile: event");
  for (int k = 0; k <= KEV_N; ++k) ms_out[k] = 0.0;
  // one untimed pass, then reps timed ones, each read back before its events are reused; a kernel
  // the pass does not launch (F1b under the fused F1) keeps its events unrecorded and reads 0
  int rc = sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, s);
  for (int r = 0; r < reps && rc == RLKS_OK; ++r) {
    g_kernel_events = ev;
    rc = sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, s);
    g_kernel_events = nullptr;
    if (rc) break;
    if (hipStreamSynchronize(s) != hipSuccess) { rc = fail(RLKS_ERR_HIP, "rlks_ppo_grad_profile: sync"); break; }
    for (int k = 0; k < KEV_N; ++k) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]) == hipSuccess) ms_out[k] += ms / reps;
      else (void)hipGetLastError();  // (an unrecorded pair: clear the error before the next pass's launch checks)
    }
  }
  g_kernel_events = nullptr;
  // the event bracket's own cost: the same start / stop pair around an empty kernel (one wave), read
  // like the others and subtracted from each kernel's figure (ms_out[KEV_N] reports it)
  double ovh = 0.0;
  for (int r = 0; r < reps && rc == RLKS_OK; ++r) {
    hipExtLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0u, s, ev[0], ev[1], 0u);
    if (hipStreamSynchronize(s) != hipSuccess) { rc = fail(RLKS_ERR_HIP, "rlks_ppo_grad_profile: sync"); break; }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) ovh += ms / reps;
  }
  for (int k = 0; k < KEV_N; ++k)
    if (ms_out[k] > 0.0) ms_out[k] = ms_out[k] > ovh ? ms_out[k] - ovh : 0.0;
  ms_out[KEV_N] = ovh;
  (void)hipGetLastError();  // (an unrecorded event's elapsed-time query)
  for (int i = 0; i < 2 * KEV_N; ++i) (void)hipEventDestroy(ev[i]);
  return rc;
}

static AdamCo adam_co(float lr, float beta1, float beta2, float eps, int step) {
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  return AdamCo{1.f - beta1, beta2, 1.f - beta2, (float)(lr / bc1), (float)std::sqrt(bc2), eps};
}

int rlks_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                   float eps, int step, void* stream) {
  RLKS_REQUIRE(p && g && m && v && n >= 0 && step >= 1, RLKS_ERR_ARG, "rlks_adam_step: bad argument");
  if (n == 0) return RLKS_OK;
  hipLaunchKernelGGL(k_adam, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     adam_co(lr, beta1, beta2, eps, step));
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_ppo_sgd_step(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, float* params, const float* dyn,
                      const float* mb, int M, float* grad, double* stats, float* adam_m, float* adam_v, int64_t n_params,
                      float lr, float beta1, float beta2, float eps, int step, int prev_fused, void* workspace,
                      int64_t ws_bytes, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(co && params && dyn && mb && grad && adam_m && adam_v && workspace && step >= 1, RLKS_ERR_ARG,
               "rlks_ppo_sgd_step: bad argument");
  if (!is_sf(d) || is_wide(d)) {  // unfused: gradient, then Adam
    if (int rc = rlks_ppo_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, stream)) return rc;
    return rlks_adam_step(params, grad, adam_m, adam_v, n_params, lr, beta1, beta2, eps, step, stream);
  }
  FusedAdam fa{params, adam_m, adam_v, adam_co(lr, beta1, beta2, eps, step), step, prev_fused ? 1 : 0};
  return sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, (hipStream_t)stream,
                 &fa);
}

// the next step's gather as extra reduce blocks (fused = true), or false: the caller gathers with
// rlks_ppo_gather_packed after the step (wide / fp32 paths, more than NEXT_GROUPS lane groups)
static int next_gather(const rlks_mlp_desc* d, const rlks_gather_next* x, NextGather& n, bool& fused) {
  RLKS_REQUIRE(x->packed_dev && x->mb_dev && x->rows >= 0 && x->T > 0 && x->N > 0, RLKS_ERR_ARG,
               "rlks_ppo_*_next: bad gather argument");
  RLKS_REQUIRE(rlks_packed_stride(d) > 0, RLKS_ERR_UNSUPPORTED, "rlks_ppo_*_next: records of 2, 4 or 8 clouds only");
  GatherArgs g;
  if (int rc = gather_args(d, x->T, x->N, x->perm_seed, x->epoch, x->groups, x->group0, x->row0, x->rows, x->mb_dev, g))
    return rc;
  fused = is_sf(d) && !is_wide(d) && x->groups <= NEXT_GROUPS;
  n = NextGather{};
  for (int k = 0; k < x->groups && k < NEXT_GROUPS; ++k) n.perm[k] = g.perm[k];
  n.row0g = g.row0g;
  n.rows = g.rows;
  n.rows_g = g.rows_g;
  n.Ng = g.Ng;
  n.N = x->N;
  n.mb = x->mb_dev;
  n.packed = x->packed_dev;
  return RLKS_OK;
}

static int gather_after(const rlks_mlp_desc* d, const rlks_gather_next* x, void* stream) {
  return rlks_ppo_gather_packed(d, x->packed_dev, x->T, x->N, x->perm_seed, x->epoch, x->groups, x->group0, x->row0,
                                x->rows, x->mb_dev, stream);
}

int rlks_ppo_sgd_step_next(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, float* params, const float* dyn,
                           const float* mb, int M, float* grad, double* stats, float* adam_m, float* adam_v,
                           int64_t n_params, float lr, float beta1, float beta2, float eps, int step, int prev_fused,
                           const rlks_gather_next* x, void* workspace, int64_t ws_bytes, void* stream) {
  if (!x)
    return rlks_ppo_sgd_step(d, co, params, dyn, mb, M, grad, stats, adam_m, adam_v, n_params, lr, beta1, beta2, eps,
                             step, prev_fused, workspace, ws_bytes, stream);
  if (int rc = check_desc(d)) return rc;
  NextGather n;
  bool fused;
  if (int rc = next_gather(d, x, n, fused)) return rc;
  if (!fused) {  // the two calls
    if (int rc = rlks_ppo_sgd_step(d, co, params, dyn, mb, M, grad, stats, adam_m, adam_v, n_params, lr, beta1, beta2,
                                   eps, step, prev_fused, workspace, ws_bytes, stream))
      return rc;
    return gather_after(d, x, stream);
  }
  RLKS_REQUIRE(co && params && dyn && mb && grad && adam_m && adam_v && workspace && step >= 1, RLKS_ERR_ARG,
               "rlks_ppo_sgd_step: bad argument");
  FusedAdam fa{params, adam_m, adam_v, adam_co(lr, beta1, beta2, eps, step), step, prev_fused ? 1 : 0};
  return sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, (hipStream_t)stream,
                 &fa, &n);
}

// The multi-rank form of rlks_ppo_sgd_step: the gradient (its prep reading the previous step's
// maxima when prev_fused), then, after the caller's all-reduce, Adam as a reduce over one partial
// (the summed gradient) that also leaves the new maxima and the step tag, so no SGD step needs the
// separate weight-max pass.  Same arithmetic as k_adam / the fused reduce: bit-identical parameters.
int rlks_ppo_grad_step(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                       const float* mb, int M, float* grad, double* stats, int step, int prev_fused, void* workspace,
                       int64_t ws_bytes, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(co && params && dyn && mb && grad && workspace && step >= 1, RLKS_ERR_ARG,
               "rlks_ppo_grad_step: bad argument");
  if (!is_sf(d) || is_wide(d))
    return rlks_ppo_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, stream);
  FusedAdam fa{nullptr, nullptr, nullptr, AdamCo{}, step, prev_fused ? 1 : 0, false};
  return sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, (hipStream_t)stream,
                 &fa);
}

int rlks_ppo_grad_step_next(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                            const float* mb, int M, float* grad, double* stats, int step, int prev_fused,
                            const rlks_gather_next* x, void* workspace, int64_t ws_bytes, void* stream) {
  if (!x)
    return rlks_ppo_grad_step(d, co, params, dyn, mb, M, grad, stats, step, prev_fused, workspace, ws_bytes, stream);
  if (int rc = check_desc(d)) return rc;
  NextGather n;
  bool fused;
  if (int rc = next_gather(d, x, n, fused)) return rc;
  if (!fused) {
    if (int rc = rlks_ppo_grad_step(d, co, params, dyn, mb, M, grad, stats, step, prev_fused, workspace, ws_bytes,
                                    stream))
      return rc;
    return gather_after(d, x, stream);
  }
  RLKS_REQUIRE(co && params && dyn && mb && grad && workspace && step >= 1, RLKS_ERR_ARG,
               "rlks_ppo_grad_step: bad argument");
  FusedAdam fa{nullptr, nullptr, nullptr, AdamCo{}, step, prev_fused ? 1 : 0, false};
  return sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, (hipStream_t)stream,
                 &fa, &n);
}

int rlks_ppo_grad_step_part(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                            const float* mb, int M, float* grad, double* stats, int step, int prev_fused, int part,
                            const rlks_gather_next* x, void* workspace, int64_t ws_bytes, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(part == 1 || part == 2, RLKS_ERR_ARG, "rlks_ppo_grad_step_part: part must be 1 or 2");
  RLKS_REQUIRE(co && params && dyn && mb && grad && workspace && step >= 1, RLKS_ERR_ARG,
               "rlks_ppo_grad_step_part: bad argument");
  if (!is_sf(d) || is_wide(d)) {  // no split form: everything in part 1
    if (part == 2) return x ? gather_after(d, x, stream) : RLKS_OK;
    return rlks_ppo_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, stream);
  }
  FusedAdam fa{nullptr, nullptr, nullptr, AdamCo{}, step, prev_fused ? 1 : 0, false};
  NextGather n;
  bool fused = false;
  if (x && part == 2)
    if (int rc = next_gather(d, x, n, fused)) return rc;
  if (int rc = sf_grad(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, (hipStream_t)stream,
                       &fa, fused ? &n : nullptr, part))
    return rc;
  return (x && part == 2 && !fused) ? gather_after(d, x, stream) : RLKS_OK;
}

int rlks_ppo_adam_apply(const rlks_mlp_desc* d, float* params, const float* grad, float* adam_m, float* adam_v,
                        int64_t n_params, float lr, float beta1, float beta2, float eps, int step, void* workspace,
                        int64_t ws_bytes, int rows, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(params && grad && adam_m && adam_v && workspace && step >= 1, RLKS_ERR_ARG,
               "rlks_ppo_adam_apply: bad argument");
  if (!is_sf(d) || is_wide(d))
    return rlks_adam_step(params, grad, adam_m, adam_v, n_params, lr, beta1, beta2, eps, step, stream);
  RLKS_REQUIRE(rows > 0 && rows % 256 == 0, RLKS_ERR_ARG, "rlks_ppo_adam_apply: rows as in rlks_ppo_grad_step");
  const int D = d->obs_dim, A = d->n_actions, H = HID;
  const SfWs w = sf_ws_layout(D, A, rows, (char*)workspace);
  RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_ppo_adam_apply: workspace too small");
  const Layout L = make_layout(D, H, A);
  RLKS_REQUIRE(n_params == L.padded, RLKS_ERR_ARG, "rlks_ppo_adam_apply: n_params must be the padded layout size");
  float* g = const_cast<float*>(grad);  // one partial, summed in place (each element read and written by one thread)
  Reducer R;
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    const int64_t* o = L.off + 6 * net;
    R.add(g + o[0], g + o[0], nullptr, 0, 1, H * D, 2 * net + 1);
    R.add(g + o[1], g + o[1], nullptr, 0, 1, H, 2 * net + 1);
    R.add(g + o[2], g + o[2], nullptr, 0, 1, H * H, 2 * net);
    R.add(g + o[3], g + o[3], nullptr, 0, 1, H);
    R.add(g + o[4], g + o[4], nullptr, 0, 1, An * H);
    R.add(g + o[5], g + o[5], nullptr, 0, 1, An);
  }
  for (int k = 0; k < 4; ++k)
    RLKS_REQUIRE(R.mnext[k] <= SF_PMAX, RLKS_ERR_UNSUPPORTED, "rlks_ppo_adam_apply: too many blocks per weight");
  R.a.p = params; R.a.m = adam_m; R.a.v = adam_v; R.a.grad = grad; R.a.co = adam_co(lr, beta1, beta2, eps, step);
  const int par = step & 1;
  for (int net = 0; net < 2; ++net) {
    R.a.slot[2 * net] = w.w[net].pmax + (par * 2 + 0) * SF_PMAX;
    R.a.slot[2 * net + 1] = w.w[net].pmax + (par * 2 + 1) * SF_PMAX;
  }
  R.a.tag[0] = w.w[0].tag + par;
  R.a.tag[1] = w.w[1].tag + par;
  R.a.tag_val = (unsigned)step + 1u;
  hipLaunchKernelGGL(k_reduce, dim3(R.blocks), dim3(256), 0, (hipStream_t)stream, R.a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_kl_update(float* dyn, const double* kc, float target, void* stream) {
  RLKS_REQUIRE(dyn && kc, RLKS_ERR_ARG, "rlks_kl_update: null argument");
  hipLaunchKernelGGL(k_kl_update, dim3(1), dim3(64), 0, (hipStream_t)stream, dyn, kc, target);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_rollout(rlks_env* env, const rlks_mlp_desc* d, const float* params, const rlks_rollout_bufs* b,
                 int explore, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(!is_wide(d), RLKS_ERR_UNSUPPORTED, "rlks_rollout: this MLP / env needs rlks_rollout_ws");
  RLKS_REQUIRE(env && params && b && b->T > 0 && b->N > 0, RLKS_ERR_ARG, "rlks_rollout: bad argument");
  rlks_env_cfg cfg;
  rlks_env_config(env, &cfg);
  RLKS_REQUIRE(cfg.n_envs == b->N && 3 * cfg.n_clouds == d->obs_dim && cfg.n_clouds == d->n_actions,
               RLKS_ERR_ARG, "rlks_rollout: env / policy / buffer shapes disagree");
  hipStream_t s = (hipStream_t)stream;
  if (cfg.nodes_per_cluster > 0) {
    RLKS_REQUIRE(cfg.autoreset, RLKS_ERR_ARG, "rlks_rollout: node-level rollout needs autoreset lanes");
    return node_rollout(env, d, params, b, explore, nullptr, s);
  }
  const int N = b->N, D = d->obs_dim, A = d->n_actions;
  const Layout L = make_layout(D, d->hidden, A);
  // per step: policy forward fused with sampling and the env step (one launch, pi net only)
  FwdArgs f{};
  f.P = net_ptrs_host(params, L, 0);
  f.x_stride = D; f.M = N; f.D = D; f.A_pi = A;
  f.env = view(env); f.tab_cost = env->d_cost; f.tab_lat = env->d_lat; f.explore = explore;
  for (int t = 0; t < b->T; ++t) {
    f.x = b->obs + (size_t)t * N * D;
    f.out = b->logits + (size_t)t * N * A;
    f.obs_next = b->obs + (size_t)(t + 1) * N * D;
    f.logp = b->logp + (size_t)t * N;
    f.actions = b->actions + (size_t)t * N;
    f.rewards = b->rewards + (size_t)t * N;
    f.dones = b->dones + (size_t)t * N;
    if (int rc = launch_fwd_head(f, 0, A, FWD_ROLLOUT, s)) return rc;
  }
  // values of every visited observation (incl. the bootstrap obs[T]) in one batched pass
  FwdArgs v{};
  v.P = net_ptrs_host(params, L, 1);
  v.x = b->obs; v.x_stride = D; v.M = (b->T + 1) * N; v.D = D; v.A_pi = A; v.out = b->values;
  return launch_fwd_head(v, 1, A, FWD_ONLY, s);
}

int rlks_rollout_ws(rlks_env* env, const rlks_mlp_desc* d, const float* params, const rlks_rollout_bufs* b,
                    int explore, void* workspace, int64_t ws_bytes, void* stream) {
  if (int rc = check_desc(d)) return rc;
  if (is_wide(d)) {
    RLKS_REQUIRE(env && params && b && b->T > 0 && b->N > 0 && workspace, RLKS_ERR_ARG, "rlks_rollout_ws: bad argument");
    rlks_env_cfg cfg;
    rlks_env_config(env, &cfg);
    RLKS_REQUIRE(cfg.n_envs == b->N && 3 * cfg.n_clouds == d->obs_dim && cfg.n_clouds == d->n_actions && cfg.autoreset,
                 RLKS_ERR_ARG, "rlks_rollout_ws: env / policy / buffer shapes disagree (autoreset lanes required)");
    const WideWs w = wide_ws_layout(d->obs_dim, d->hidden, d->n_actions, b->N, (char*)workspace);
    RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_rollout_ws: workspace too small");
    return wide_rollout(env, d, params, b, explore, w, (hipStream_t)stream);
  }
  if (!is_sf(d)) return rlks_rollout(env, d, params, b, explore, stream);
  RLKS_REQUIRE(env && params && b && b->T > 0 && b->N > 0 && workspace, RLKS_ERR_ARG, "rlks_rollout_ws: bad argument");
  rlks_env_cfg cfg;
  rlks_env_config(env, &cfg);
  RLKS_REQUIRE(cfg.n_envs == b->N && 3 * cfg.n_clouds == d->obs_dim && cfg.n_clouds == d->n_actions,
               RLKS_ERR_ARG, "rlks_rollout_ws: env / policy / buffer shapes disagree");
  const int N = b->N, D = d->obs_dim, A = d->n_actions;
  const SfWs w = sf_ws_layout(D, A, 0, (char*)workspace);
  RLKS_REQUIRE(ws_bytes >= w.weight_bytes, RLKS_ERR_ARG, "rlks_rollout_ws: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  if (cfg.nodes_per_cluster > 0) {
    RLKS_REQUIRE(cfg.autoreset, RLKS_ERR_ARG, "rlks_rollout_ws: node-level rollout needs autoreset lanes");
    return node_rollout(env, d, params, b, explore, &w, s);
  }
  // by the whole job's lane count: W ranks of N lanes and one rank of W N lanes (num_lane_groups = W)
  // run the same forward kernel, so their logits, and hence their sampled actions, agree bit for bit
  const int64_t job_lanes = b->global_lanes > 0 ? b->global_lanes : N;
  if (job_lanes > SF_ROLL_FUSED_MAX_LANES && cfg.autoreset) {
    // per step: the 16-row forward of both nets (k_sf_fwd16), then the fused sample + env step
    // (k_sample_step, auto-reset lanes); V(obs[T]) by one more forward
    if (int rc = sf_prep(d, w, params, s, true)) return rc;
    const Layout L = make_layout(D, HID, A);
    SfFwdArgs f{};
    for (int net = 0; net < 2; ++net) {
      const NetPtrs P = net_ptrs_host(params, L, net);
      f.n[net] = w.n[net];
      f.n[net].b2 = P.b2; f.n[net].w3 = P.w3; f.n[net].b3 = P.b3;
    }
    f.M = N; f.D = D;
    for (int t = 0; t <= b->T; ++t) {
      const size_t tN = (size_t)t * N;
      f.x = b->obs + tN * D;
      f.out[0] = t < b->T ? b->logits + tN * A : nullptr;
      f.out[1] = b->values + tN;
      if (int rc = launch_sf_fwd16(f, A, s)) return rc;
      if (t == b->T) break;
      if (int rc = rlks_env_sample_step(env, b->logits + tN * A, explore, b->actions + tN, b->logp + tN,
                                        b->obs + (tN + N) * D, b->rewards + tN, b->dones + tN, s))
        return rc;
    }
    return RLKS_OK;
  }
  if (int rc = sf_prep(d, w, params, s, true)) return rc;
  const Layout L = make_layout(D, HID, A);
  SfRollArgs a{};
  for (int net = 0; net < 2; ++net) {
    const NetPtrs P = net_ptrs_host(params, L, net);
    a.n[net] = SfRollNet{w.w[net].w1h, w.w[net].w1l, w.w[net].w2rh, w.w[net].w2rl, P.b2, P.w3, P.b3, w.w[net].sc};
  }
  a.M = N; a.D = D; a.A = A; a.T = b->T;
  a.env = view(env); a.tab_cost = env->d_cost; a.tab_lat = env->d_lat; a.explore = explore;
  // one launch: per step both nets' forward of obs[t] (logits[t], values[t]), sample, env step ->
  // obs[t + 1]; step T writes the bootstrap V(obs[T])
  a.x = b->obs;
  a.logits = b->logits;
  a.values = b->values;
  a.logp = b->logp;
  a.actions = b->actions;
  a.rewards = b->rewards;
  a.dones = b->dones;
  return launch_sf_roll(a, FWD_ROLLOUT, s);
}

}  // extern "C"
