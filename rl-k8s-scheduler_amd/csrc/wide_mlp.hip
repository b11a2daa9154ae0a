// wide_mlp.hip — the PPO policy/value MLP for widths the fused 256-unit kernels do not cover:
// config c5 (64 clusters x 1,024 nodes, obs 3 x 64 = 192, 64 actions, fcnet_hiddens
// [2048, 2048], "MFMA-bound update").  Every layer is a split-fp16 GEMM (gemm_sf16.hip, fp32-
// accurate) with the activation or its derivative fused into the epilogue; activations H1, H2 are
// materialised in HBM (M x 2048 fp32 each), which at this width is a small fraction of the GEMM
// time.  Same RLlib semantics as the fused path (mlp_fwd.hip / sgd_sf16.hip): FCNet tanh, separate
// value net, PPO clipped surrogate + KL + clipped value loss + entropy (train_ppo.py:9-31).
//
// Per net and SGD step (M minibatch rows; W1 [H][D], W2 [H][H], W3 [A][H] torch layouts):
//   H1 = tanh(X W1^T + b1)   H2 = tanh(H1 W2^T + b2)   out = H2 W3^T + b3          (NT GEMMs)
//   k_wide_loss_pi / _vf: dout [M][A] (+ per-block loss stats)
//   dW3 = dout^T H2 (TN)   db3 = colsum(dout) (value net: k_wide_vb3, exact row differences in f64)
//   dZ2 = (dout W3) * (1 - H2^2) (NN, fused)   dW2 = dZ2^T H1 (TN)   db2 = colsum(dZ2)
//   dZ1 = (dZ2 W2) * (1 - H1^2) (NN, fused)    dW1 = dZ1^T X  (TN)   db1 = colsum(dZ1)
// The three H x H GEMMs (Z2, dZ1, dW2) run on the pre-split kernel (gemm_ps.hip): H1 is written as
// fp16 planes at the fixed scale 2^14 by Z1's epilogue (|tanh| < 1), W2 and dZ2 are split into
// planes once (rlks split pass) after their max |x| is known; the others use the generic kernel.
// Operand scales: max |x| slots filled by rlks_absmax (X, weights) or by the producing GEMM's
// epilogue (H2, dZ2, dZ1), the loss kernel (dout).
#include "wide_mlp.h"

#include "gemm_sf16.h"

namespace rlks {

constexpr int LOSS_ROWS = 256;  // rows per loss block (stats partials)

using h8 = __attribute__((ext_vector_type(8))) _Float16;
enum { SL_X = 0, SL_W1, SL_W2, SL_W3, SL_H1, SL_H2, SL_DOUT, SL_DZ2, SL_DZ1, SL_DSUM, SL_N = 16 };  // SL_DSUM: max_m sum_a |dout|

WideWs wide_ws_layout(int D, int H, int A, int M, char* base) {
  WideWs w{};
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + o : nullptr;
    o += (bytes + 255) / 256 * 256;
    return p;
  };
  w.M = M;
  const int Mp = (M + 31) / 32 * 32;  // plane rows: the dW2 reduction runs over whole 32-row chunks
  w.blocks = (M + LOSS_ROWS - 1) / LOSS_ROWS;
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    WideNet& n = w.n[net];
    n.h1h = (_Float16*)take(2LL * Mp * H);
    n.h1l = (_Float16*)take(2LL * Mp * H);
    n.h2 = (float*)take(4LL * M * H);
    n.w2h = (_Float16*)take(2LL * H * H);
    n.w2l = (_Float16*)take(2LL * H * H);
    n.w1h = (_Float16*)take(2LL * H * D);
    n.w1l = (_Float16*)take(2LL * H * D);
    n.out = (float*)take(4LL * M * An);
    n.dout = (float*)take(4LL * M * An);
    n.slots = (unsigned*)take(4 * SL_N);
    n.part_stat = (float*)take(4LL * w.blocks * 4);
  }
  w.dzb = (float*)take(4LL * M * H);
  w.dzh = (_Float16*)take(2LL * Mp * H);
  w.dzl = (_Float16*)take(2LL * Mp * H);
  w.xh = (_Float16*)take(2LL * Mp * D);  // rows [M, Mp) zeroed by wide_grad (dW1's K runs over Mp)
  w.xl = (_Float16*)take(2LL * Mp * D);
  w.rew64 = (double*)take(8LL * M);
  {  // weight-gradient partials: dW3 [A][H], dW2 [H][H], dW1 [H][D] (K = M), column sums of M rows
    int64_t pf = (int64_t)2 * colsum_splits(M) * H;  // (hi, lo planes)
    pf = std::max(pf, (int64_t)gemm_splits(A, H, M) * A * H);
    pf = std::max(pf, (int64_t)gemm_ps_splits(H, H, Mp) * H * H);
    pf = std::max(pf, (int64_t)gemm_ps_splits(H, D, Mp) * H * D);
    pf = std::max(pf, (int64_t)gemm_splits(H, D, M) * H * D);
    pf = std::max(pf, (int64_t)2 * ((M + 511) / 512) * H);  // k_wide_dz2's db2 partials (DZ_ROWS x DZ_RT rows each; hi, lo)
    w.part = (float*)take(4 * pf);
  }
  w.stat_slots = (unsigned*)take(4 * 4);
  w.bytes = o;
  return w;
}

bool wide_needed(const rlks_mlp_desc* d) { return d->hidden != HID || d->n_actions > 8 || d->obs_dim + 1 > 32; }

// ----------------------------------------------------------------------------- kernels
// PPO loss per row (same math as sgd_sf16.hip's sf_loss, for up to 64 actions); dout -> HBM, per-block
// stats [policy loss, vf loss, kl, entropy], max |dout| -> slot.  Value net: one thread per row.
__global__ __launch_bounds__(LOSS_ROWS) void k_wide_loss_vf(const float* __restrict__ out, const float* __restrict__ x,
                                                          int stride, int M, int D, int A, rlks_ppo_coeffs co,
                                                          const float* __restrict__ dyn, float* __restrict__ dout,
                                                          float* __restrict__ part_stat, unsigned* __restrict__ dmax) {
  __shared__ float red[LOSS_ROWS / 64];
  __shared__ double redx[LOSS_ROWS / 64];
  const int m = blockIdx.x * LOSS_ROWS + threadIdx.x;
  float vl = 0.f, mx_d = 0.f;
  double ex = 0.0;
  if (m < M) {
    const VfRow v = vf_row(out[m], x[(size_t)m * stride + D + A + 1], co.vf_clip_param, co.vf_loss_coeff,
                           dyn[RLKS_DYN_INV_COUNT]);
    vl = v.sq;
    dout[m] = v.dl;
    mx_d = fabsf(v.dl);
    ex = v.ex;
  }
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float s = wave_sum(vl);
  const double sx = wave_sum(ex);
  if (l == 0) {
    red[w] = s;
    redx[w] = sx;
  }
  mx_d = wave_max(mx_d);
  if (l == 0) atomicMax(dmax, __float_as_uint(mx_d));
  __syncthreads();
  if (threadIdx.x < 2) {  // slot 1: the vf loss stat; slots 2, 3 (unused by the value net's stats): db3 hi, lo
    float t = 0.f;
    if (threadIdx.x == 1)
      for (int j = 0; j < LOSS_ROWS / 64; ++j) t += red[j];
    part_stat[(size_t)blockIdx.x * 4 + threadIdx.x] = t;
  } else if (threadIdx.x == 2) {
    double t = 0.0;
    for (int j = 0; j < LOSS_ROWS / 64; ++j) t += redx[j];
    vf_b3_part(t, co.vf_loss_coeff, dyn[RLKS_DYN_INV_COUNT], part_stat + (size_t)blockIdx.x * 4 + 2);
  }
}

// the value head's bias gradient: every block's (hi, lo) pair of k_wide_loss_vf summed in f64, fixed
// order (64 lanes over strided blocks, then the lanes)
__global__ __launch_bounds__(64) void k_wide_vb3(const float* __restrict__ part_stat, int blocks, float* __restrict__ out) {
  double t = 0.0;
  for (int b = threadIdx.x; b < blocks; b += 64)
    t += (double)part_stat[(size_t)b * 4 + 2] + (double)part_stat[(size_t)b * 4 + 3];
  t = wave_sum(t);
  if (threadIdx.x == 0) out[0] = (float)t;
}

// the policy net's loss with one wave per row and one lane per action (A <= 64; 16 waves per block of
// LOSS_ROWS rows, so four waves per SIMD): the logits and old
// logits of a row are one coalesced load each, the softmax sums wave reductions.  (One thread per row,
// looping over 64 actions with row-strided loads, took 0.29 ms per SGD step at c5: one wave per SIMD
// and 64 cache lines per load instruction.)  Same per-block stats layout as k_wide_loss_vf.
// The loss and dL/dlogits are evaluated in f64 from the fp32 logits and rounded once: every bias
// gradient downstream (db2 = colsum((dout W3)(1 - H2^2)), db1) is a sum over rows that cancels, and
// at the elements where it cancels most the fp32 loss arithmetic's few-ulp error per row (softmax,
// log-sum-exp, ratio) was the largest part of the result's error (tools/wide_b2_isolate.py,
// profiles/r05_precision).  ~a few hundred DP ops per row: noise beside the step's GEMMs.
constexpr int LOSS_PI_WAVES = 16;  // waves per policy-loss block: LOSS_ROWS / 16 rows each (4 waves per SIMD)
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__global__ __launch_bounds__(64 * LOSS_PI_WAVES) void k_wide_loss_pi(const float* __restrict__ out, const float* __restrict__ x,
                                                          int stride, int M, int D, int A, rlks_ppo_coeffs co,
                                                          const float* __restrict__ dyn, float* __restrict__ dout,
                                                          float* __restrict__ part_stat, unsigned* __restrict__ dmax,
                                                          unsigned* __restrict__ dsum) {
  constexpr int RPW = LOSS_ROWS / LOSS_PI_WAVES;  // rows per wave
  __shared__ double red[3][LOSS_PI_WAVES];
  __shared__ float redm[LOSS_PI_WAVES], reds[LOSS_PI_WAVES];
  float mx_s = 0.f;  // max over the wave's rows of sum_a |dout|: k_wide_dz2's split bound
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool on = l < A;
  const double inv_count = dyn[RLKS_DYN_INV_COUNT], klc = dyn[RLKS_DYN_KL_COEFF];
  const double adv_mean = dyn[RLKS_DYN_ADV_MEAN], adv_invstd = dyn[RLKS_DYN_ADV_INVSTD];
  const double lo_c = 1.0 - (double)co.clip_param, hi_c = 1.0 + (double)co.clip_param;
  const double ent_c = co.entropy_coeff;
  double st0 = 0.0, st2 = 0.0, st3 = 0.0;
  float mx_d = 0.f;
  for (int i = 0; i < RPW; ++i) {
    const int m = blockIdx.x * LOSS_ROWS + w * RPW + i;
    if (m >= M) break;
    const float* rec = x + (size_t)m * stride;
    const double lg = on ? (double)out[(size_t)m * A + l] : -INFINITY, lo = on ? (double)rec[D + l] : -INFINITY;
    const double adv = ((double)rec[D + A] - adv_mean) * adv_invstd;
    const double logp_old = rec[D + A + 2];
    const int act = (int)rec[D + A + 3];
    const double mx = wave_max_d(lg), mo = wave_max_d(lo);
    const double lse = mx + log(wave_sum(on ? exp(lg - mx) : 0.0)), lso = mo + log(wave_sum(on ? exp(lo - mo) : 0.0));
    const double lp = lg - lse, p = on ? exp(lp) : 0.0, lpo = lo - lso, po = on ? exp(lpo) : 0.0;
    const double kl = wave_sum(on ? po * (lpo - lp) : 0.0);
    const double ent = -wave_sum(on ? p * lp : 0.0);
    const double lpa = wave_sum(l == act ? lp : 0.0);
    const double ratio = exp(lpa - logp_old);
    const double rc = fmin(fmax(ratio, lo_c), hi_c);
    const double s1 = adv * ratio, s2 = adv * rc;
    // torch.min backward splits ties evenly; torch.clamp passes the gradient on [lo, hi]
    const double w1 = s1 < s2 ? 1.0 : (s1 == s2 ? 0.5 : 0.0);
    const double inr = (ratio >= lo_c && ratio <= hi_c) ? 1.0 : 0.0;
    const double dr = -adv * (w1 + (1.0 - w1) * inr) * ratio;
    float df = 0.f;
    if (on) {
      double d = dr * ((l == act ? 1.0 : 0.0) - p);
      d += klc * (p - po);
      d += ent_c * p * (lp + ent);
      df = (float)(d * inv_count);
      dout[(size_t)m * A + l] = df;
      mx_d = fmaxf(mx_d, fabsf(df));
    }
    mx_s = fmaxf(mx_s, wave_sum(fabsf(df)));
    st0 -= fmin(s1, s2);
    st2 += kl;
    st3 += ent;
  }
  mx_d = wave_max(mx_d);
  if (l == 0) {
    red[0][w] = st0;
    red[1][w] = st2;
    red[2][w] = st3;
    redm[w] = mx_d;
    reds[w] = mx_s;
  }
  __syncthreads();
  if (threadIdx.x == 64) {  // one atomic per block (single-address atomics serialise at their L2 channel)
    float m = 0.f, ms = 0.f;
    for (int j = 0; j < LOSS_PI_WAVES; ++j) {
      m = fmaxf(m, redm[j]);
      ms = fmaxf(ms, reds[j]);
    }
    atomicMax(dmax, __float_as_uint(m));
    atomicMax(dsum, __float_as_uint(ms));
  }
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    double s = 0.0;
    if (k != 1)
      for (int j = 0; j < LOSS_PI_WAVES; ++j) s += red[k == 0 ? 0 : k - 1][j];
    part_stat[(size_t)blockIdx.x * 4 + k] = (float)s;
  }
}

// stats[RLKS_STAT_*] from the per-block partials of both nets (fixed order, f64)
__global__ void k_wide_stats(const float* __restrict__ ps_pi, const float* __restrict__ ps_vf, int blocks, int rows,
                             double* __restrict__ stats) {
  const int i = threadIdx.x;
  if (i >= 4) return;
  const float* p = i == 1 ? ps_vf : ps_pi;
  double s = 0.0;
  for (int b = 0; b < blocks; ++b) s += (double)p[(size_t)b * 4 + i];
  stats[i] = s;
  if (i == 0) {
    stats[RLKS_STAT_ROWS] = (double)rows;
    stats[5] = stats[6] = stats[7] = 0.0;
  }
}

// TorchCategorical over A logits for every lane (Philox counter = lane / episode / step, as the
// fused rollout kernels): action and its log-probability
__global__ void k_wide_sample(EnvView v, const float* __restrict__ logits, int A, int explore,
                              int32_t* __restrict__ actions, float* __restrict__ logp) {
  const int m = v.lane0 + blockIdx.x * blockDim.x + threadIdx.x;  // (a lane range: node_rollout's halves)
  if (m >= v.lane_end) return;
  const float* lg = logits + (size_t)m * A;
  float mx = lg[0];
  int amax = 0;
  for (int a = 1; a < A; ++a)
    if (lg[a] > mx) { mx = lg[a]; amax = a; }
  float se = 0.f;
  for (int a = 0; a < A; ++a) se += expf(lg[a] - mx);
  int act = amax;
  if (explore) {
    const u32x4 x = philox4x32_10(u32x4{(uint32_t)(v.env_offset + m), (uint32_t)v.episode[m], (uint32_t)v.step[m],
                                        (uint32_t)RLKS_PURPOSE_ACTION << 16},
                                  v.k0, v.k1);
    const float u = (float)u53(x.x, x.y) * se;
    float c = 0.f;
    act = A - 1;
    for (int a = 0; a < A; ++a) {
      c += expf(lg[a] - mx);
      if (u < c) { act = a; break; }
    }
  }
  actions[m] = act;
  logp[m] = lg[act] - mx - logf(se);
}

// dZ2 = (dout W3) (1 - H2^2), K = the head's outputs (64 / 1): too short a reduction for the split
// GEMM's K pipeline (its tile prologue and epilogue were the whole 0.71 ms), so plain fp32 FMAs in k
// order on 64-row x 256-column tiles (8 per block): dout^T and W3 tiles in LDS (K chunks of 32), 8 x 8
// outputs per thread, H2 read and dZ2 written as float4 rows; max |dZ2| -> slot (one atomic per
// block); db2 as per-block column sums in f64 (a fixed order; hi + lo planes), summed by launch_split_reduce.
// 1 - H2^2 as one fma (a single rounding where H2 saturates)
constexpr int DZ_ROWS = 64, DZ_COLS = 256, DZ_K = 32, DZ_RT = 8;  // DZ_RT row tiles per block
__global__ __launch_bounds__(256) void k_wide_dz2(const float* __restrict__ dout, const float* __restrict__ w3,
                                                  const float* __restrict__ h2, _Float16* __restrict__ dzh,
                                                  _Float16* __restrict__ dzl, int M, int H, int K,
                                                  const unsigned* __restrict__ dsum_slot,
                                                  const unsigned* __restrict__ w3_slot, unsigned* __restrict__ cmax_slot,
                                                  float* __restrict__ part_db2) {
  // dZ2's planes scale from the bound |dZ2| <= max_m sum_a |dout[m][a]| max |W3| (|1 - H2^2| <= 1),
  // known before any dZ2 exists, so the planes are written here (no fp32 dZ2 round trip through HBM
  // and a split pass); the bound goes to cmax_slot for the GEMMs that read the planes (gemm_ps.hip
  // ps_exp: the same exponent)
  const float bnd = __uint_as_float(*dsum_slot) * __uint_as_float(*w3_slot);
  float ds;
  {
    int e = 0;
    if (bnd > 0.f && bnd <= 3.4e38f) {
      (void)frexpf(bnd, &e);
      e = min(max(15 - e, -120), 120);
    }
    ds = ldexpf(1.f, e);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *cmax_slot = __float_as_uint(bnd);
  __shared__ __attribute__((aligned(16))) float sA[DZ_K][DZ_ROWS + 4];  // dout^T chunk (padded: the transposing stores)
  __shared__ __attribute__((aligned(16))) float sB[DZ_K][DZ_COLS];      // W3 chunk; at the end the db2 sums
  const int tid = threadIdx.x, cg = tid & 31, rg = tid >> 5;
  const int n0 = blockIdx.x * DZ_COLS;
  int n = n0 + 8 * cg;  // this thread's 8 columns (H % 8 == 0: host check)
  if (!dcheck(n + 8 <= H || n0 + DZ_COLS > H, DC_WIDE_COL, n)) n = H - 8;
  double cs[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // db2: this thread's column sums (f64)
  for (int rt = 0; rt < DZ_RT; ++rt) {
    const int m0 = (blockIdx.y * DZ_RT + rt) * DZ_ROWS;
    if (m0 >= M) break;
    float acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
    for (int k0 = 0; k0 < K; k0 += DZ_K) {
      const int kn = min(DZ_K, K - k0);
      __syncthreads();
      for (int e = tid; e < DZ_K * DZ_ROWS; e += 256) {  // e = r * DZ_K + k: coalesced along k
        const int r = e / DZ_K, k = e - r * DZ_K, m = m0 + r;
        sA[k][r] = (k < kn && m < M) ? dout[(size_t)m * K + k0 + k] : 0.f;
      }
      for (int e = tid; e < DZ_K * DZ_COLS / 4; e += 256) {
        const int k = e / (DZ_COLS / 4), c4 = 4 * (e - k * (DZ_COLS / 4));
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kn && n0 + c4 < H) v = *reinterpret_cast<const float4*>(w3 + (size_t)(k0 + k) * H + n0 + c4);
        *reinterpret_cast<float4*>(&sB[k][c4]) = v;
      }
      __syncthreads();
      for (int k = 0; k < kn; ++k) {
        const float4 a0 = *reinterpret_cast<const float4*>(&sA[k][8 * rg]), a1 = *reinterpret_cast<const float4*>(&sA[k][8 * rg + 4]);
        const float4 b0 = *reinterpret_cast<const float4*>(&sB[k][8 * cg]), b1 = *reinterpret_cast<const float4*>(&sB[k][8 * cg + 4]);
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
      }
    }
    if (n < H) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + 8 * rg + i;
        if (m >= M) break;
        const float4* hp = reinterpret_cast<const float4*>(h2 + (size_t)m * H + n);
        const float4 g0 = hp[0], g1 = hp[1];
        const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        h8 hv, lv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = acc[i][j] * fmaf(-gv[j], gv[j], 1.f);
          cs[j] += (double)o;
          const _Float16 t = (_Float16)(o * ds);
          hv[j] = t;
          lv[j] = (_Float16)(o * ds - (float)t);
        }
        *reinterpret_cast<h8*>(dzh + (size_t)m * H + n) = hv;
        *reinterpret_cast<h8*>(dzl + (size_t)m * H + n) = lv;
      }
    }
  }
  // db2 partial of the block's rows: the 8 row groups' column sums combined in a fixed order
  __syncthreads();  // (every thread is past its last read of sB)
  double* sC = reinterpret_cast<double*>(&sB[0][0]);  // [8 rg][256] (16 KB of sB's 32)
#pragma unroll
  for (int j = 0; j < 8; ++j) sC[rg * DZ_COLS + 8 * cg + j] = cs[j];
  __syncthreads();
  if (n0 + tid < H) {  // the block's column sum as an exact-ish hi + lo pair: planes y and gridDim.y + y
    double t = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += sC[g * DZ_COLS + tid];
    const float hi = (float)t;
    part_db2[(size_t)blockIdx.y * H + n0 + tid] = hi;
    part_db2[(size_t)(gridDim.y + blockIdx.y) * H + n0 + tid] = (float)(t - (double)hi);
  }
}

// The value net's head out[m] = b3 + sum_n H2[m][n] W3[n] (one output: a GEMV, HBM-bound on H2's
// M x H floats), fp32 FMAs on the unsplit operands; one wave per row at a time, VH_RPW rows a wave,
// the lane partials added by a fixed-order wave reduction.  (As a split GEMM with N = 1 on 128-wide
// tiles it took ~250 µs at c5 for 0.5 GB.)
constexpr int VH_RPW = 8;
__global__ __launch_bounds__(256) void k_wide_vhead(const float* __restrict__ h2, const float* __restrict__ w3,
                                                    const float* __restrict__ b3, float* __restrict__ out, int M, int H) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool v4 = (H & 255) == 0;
  for (int i = 0; i < VH_RPW; ++i) {
    const int m = (blockIdx.x * 4 + w) * VH_RPW + i;
    if (m >= M) break;
    const float* r = h2 + (size_t)m * H;
    float acc = 0.f;
    if (v4) {
      for (int n = 4 * l; n < H; n += 256) {
        const float4 a = *reinterpret_cast<const float4*>(r + n), b = *reinterpret_cast<const float4*>(w3 + n);
        acc = fmaf(a.x, b.x, acc);
        acc = fmaf(a.y, b.y, acc);
        acc = fmaf(a.z, b.z, acc);
        acc = fmaf(a.w, b.w, acc);
      }
    } else {
      for (int n = l; n < H; n += 64) acc = fmaf(r[n], w3[n], acc);
    }
    acc = wave_sum_f(acc);
    if (l == 0) out[m] = b3[0] + acc;
  }
}

// The policy net's head out[m][a] = b3[a] + sum_n H2[m][n] W3[a][n] (A <= 32 NT actions, K = hidden):
// a split-fp16 GEMM with whole H2 rows streamed straight into the MFMA operands (VERDICT r05 item 6:
// the generic GEMM's 128-row tiles fetched 128-byte row pieces from 128 DRAM pages per chunk, 1.8 TB/s).
// One wave per 32 rows, v_mfma_f32_32x32x16_f16: A = 32 rows x 16 k of H2 (lane: row l & 31, k = 8
// (l >> 5) + 0..7: two float4 of its row), split at the fixed scale 2^14 (|tanh| < 1, like H1 in F1);
// B = W3^T (lane: action 32 t + (l & 31), the same 8 k) from L2, split at the W3 slot's power of two.
// Each k step is 3 MFMAs per action tile; H2 is read once (HBM-bound: 4 B x H per row).
constexpr int PH_KU = 4;  // H2 k steps of 16 in flight per wave (a ring)
__device__ __forceinline__ int ph_exp(float mx) {  // mx 2^e in [2^14, 2^15) (gemm_sf16.hip's operand scale)
  if (!(mx > 0.f) || !(mx <= 3.4e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  return min(max(15 - e, -120), 120);
}
template <int NT>
__global__ __launch_bounds__(256) void k_wide_phead(const float* __restrict__ h2, const float* __restrict__ w3,
                                                    const float* __restrict__ b3, const unsigned* __restrict__ w3max,
                                                    float* __restrict__ out, int M, int H, int A) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, r = l & 31, kg = l >> 5;
  const int m0 = (blockIdx.x * 4 + w) * 32;
  if (m0 >= M) return;
  const float* hrow = h2 + (size_t)min(m0 + r, M - 1) * H + 8 * kg;
  const int ew = ph_exp(__uint_as_float(*w3max));
  const float sw = ldexpf(1.f, ew);
  const float* wrow[NT];
  float wsc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int a = 32 * t + r;
    wrow[t] = w3 + (size_t)min(a, A - 1) * H + 8 * kg;
    wsc[t] = a < A ? sw : 0.f;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
  auto split8 = [](const float4& a, const float4& b, float sc, h8& hi, h8& lo) {
    const float x[8] = {a.x * sc, a.y * sc, a.z * sc, a.w * sc, b.x * sc, b.y * sc, b.z * sc, b.w * sc};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const _Float16 h = (_Float16)x[j];
      hi[j] = h;
      lo[j] = (_Float16)(x[j] - (float)h);
    }
  };
  // H2: a ring of PH_KU k steps in flight (the step u + PH_KU load is issued when step u is consumed;
  // past the end the address is clamped and the data unused); W3: one step ahead
  float4 xr[PH_KU][2], wc[NT][2];
#pragma unroll
  for (int u = 0; u < PH_KU; ++u) {
    xr[u][0] = *reinterpret_cast<const float4*>(hrow + 16 * u);
    xr[u][1] = *reinterpret_cast<const float4*>(hrow + 16 * u + 4);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    wc[t][0] = *reinterpret_cast<const float4*>(wrow[t]);
    wc[t][1] = *reinterpret_cast<const float4*>(wrow[t] + 4);
  }
  for (int k0 = 0; k0 < H; k0 += 16 * PH_KU) {
#pragma unroll
    for (int u = 0; u < PH_KU; ++u) {
      const float4 x0 = xr[u][0], x1 = xr[u][1];
      float4 w[NT][2];
#pragma unroll
      for (int t = 0; t < NT; ++t) { w[t][0] = wc[t][0]; w[t][1] = wc[t][1]; }
      const int kx = min(k0 + 16 * (u + PH_KU), H - 16), kw = min(k0 + 16 * (u + 1), H - 16);
      xr[u][0] = *reinterpret_cast<const float4*>(hrow + kx);
      xr[u][1] = *reinterpret_cast<const float4*>(hrow + kx + 4);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        wc[t][0] = *reinterpret_cast<const float4*>(wrow[t] + kw);
        wc[t][1] = *reinterpret_cast<const float4*>(wrow[t] + kw + 4);
      }
      __builtin_amdgcn_sched_barrier(0);
      h8 xh, xl;
      split8(x0, x1, 16384.f, xh, xl);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        h8 bh, bl;
        split8(w[t][0], w[t][1], wsc[t], bh, bl);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, bh, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bl, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bh, acc[t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const float un = ldexpf(1.f, -14 - ew);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int a = 32 * t + r;
    if (a >= A) continue;
    const float bb = b3[a];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int m = m0 + acc_row(q, l);
      if (m < M) out[(size_t)m * A + a] = fmaf(acc[t][q], un, bb);
    }
  }
}

// ----------------------------------------------------------------------------- host
namespace {

struct Net {
  const float *w1, *b1, *w2, *b2, *w3, *b3;
};

Net net_of(const float* params, const Layout& L, int net) {
  const NetPtrs P = net_ptrs_host(params, L, net);
  return Net{P.w1, P.b1, P.w2, P.b2, P.w3, P.b3};
}

int gemm(const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C, int ldc, int M, int N, int K,
         int epi, const float* bias, const float* aux, int ldaux, const unsigned* amax, const unsigned* bmax,
         unsigned* cmax, hipStream_t s, float* part = nullptr, _Float16* c_hi = nullptr, _Float16* c_lo = nullptr) {
  GemmArgs g{};
  g.c_hi = c_hi;
  g.c_lo = c_lo;
  if (part) {  // weight gradient (K = minibatch rows): split K over workgroup layers
    g.splits = gemm_splits(M, N, K);
    g.part = part;
  }
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.aux = aux;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldaux = ldaux;
  g.ta = ta; g.tb = tb; g.epi = epi; g.accumulate = 0;
  g.amax = amax; g.bmax = bmax; g.cmax = cmax;
  return launch_gemm_sf16(g, s);
}

// pre-split operand: planes (hi, lo), row stride ld, K-major or not, rows, scale slot (null: 2^fexp)
PsOperand ps_op(const _Float16* hi, const _Float16* lo, int ld, int kmajor, int rows, const unsigned* slot,
                int fexp = 0) {
  PsOperand o{};
  o.hi = hi; o.lo = lo; o.ld = ld; o.kmajor = kmajor; o.rows = rows; o.maxslot = slot; o.fexp = fexp;
  return o;
}
constexpr int H1_EXP = 14;  // H1 planes hold tanh x 2^14

// forward of net `net` over M rows of x (row stride ldx): H1 (planes), H2 and out in the workspace.
// xslot: X's max |x| slot; x_done: the other net's forward already filled it and (when X goes in
// planes) split X into xh / xl, identical for both nets (one absmax + split, not two)
int forward_net(const rlks_mlp_desc* d, const Net& P, const WideNet& n, const float* x, int ldx, int M, int net,
                _Float16* xh, _Float16* xl, unsigned* xslot, bool x_done, hipStream_t s) {
  const int D = d->obs_dim, H = d->hidden, An = net == 0 ? d->n_actions : 1;
  unsigned* sl = n.slots;
  if (!x_done)
    if (int rc = launch_absmax(x, M, D, ldx, xslot, s)) return rc;
  if (int rc = launch_absmax(P.w1, H, D, D, sl + SL_W1, s)) return rc;
  if (int rc = launch_absmax(P.w2, H, H, H, sl + SL_W2, s)) return rc;
  if (int rc = launch_absmax(P.w3, An, H, H, sl + SL_W3, s)) return rc;
  if (int rc = launch_split_planes(P.w2, H, H, H, sl + SL_W2, 0, n.w2h, n.w2l, H, s)) return rc;
  if (D % 32 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0) {
    // H1 = tanh(X W1^T + b1) on the pre-split GEMM (K = obs_dim, 192 at c5), written as planes
    if (!x_done)
      if (int rc = launch_split_planes(x, M, D, ldx, xslot, 0, xh, xl, D, s)) return rc;
    if (int rc = launch_split_planes(P.w1, H, D, D, sl + SL_W1, 0, n.w1h, n.w1l, D, s)) return rc;
    PsArgs a{};
    a.a = ps_op(xh, xl, D, 0, M, xslot);
    a.b = ps_op(n.w1h, n.w1l, D, 0, H, sl + SL_W1);
    a.M = M; a.N = H; a.K = D; a.epi = PS_TANH_BIAS_PLANES; a.c_hi = n.h1h; a.c_lo = n.h1l; a.ldc = H; a.bias = P.b1;
    if (int rc = launch_gemm_ps(a, s)) return rc;
  } else if (int rc = gemm(x, ldx, 0, P.w1, D, 1, nullptr, H, M, H, D, GEMM_TANH_BIAS_PLANES, P.b1, nullptr, 0, xslot,
                           sl + SL_W1, nullptr, s, nullptr, n.h1h, n.h1l)) {
    return rc;
  }
  {  // Z2 = H1 W2^T -> H2 = tanh(Z2 + b2)
    PsArgs a{};
    a.a = ps_op(n.h1h, n.h1l, H, 0, M, nullptr, H1_EXP);
    a.b = ps_op(n.w2h, n.w2l, H, 0, H, sl + SL_W2);
    a.M = M; a.N = H; a.K = H; a.epi = PS_TANH_BIAS; a.C = n.h2; a.ldc = H; a.bias = P.b2; a.cmax = sl + SL_H2;
    if (int rc = launch_gemm_ps(a, s)) return rc;
  }
  if (An == 1) {
    hipLaunchKernelGGL(k_wide_vhead, dim3(cdiv(M, 4 * VH_RPW)), dim3(256), 0, s, n.h2, P.w3, P.b3, n.out, M, H);
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
  if (An <= 64 && H % (16 * PH_KU) == 0 && !getenv("RLKS_WIDE_HEAD_GEMM")) {  // (RLKS_WIDE_HEAD_GEMM: the generic GEMM, A/B)
    if (An <= 32)
      hipLaunchKernelGGL(k_wide_phead<1>, dim3(cdiv(M, 128)), dim3(256), 0, s, n.h2, P.w3, P.b3, sl + SL_W3, n.out, M, H, An);
    else
      hipLaunchKernelGGL(k_wide_phead<2>, dim3(cdiv(M, 128)), dim3(256), 0, s, n.h2, P.w3, P.b3, sl + SL_W3, n.out, M, H, An);
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
  return gemm(n.h2, H, 0, P.w3, H, 1, n.out, An, M, An, H, GEMM_BIAS, P.b3, nullptr, 0, sl + SL_H2, sl + SL_W3,
              nullptr, s);
}

}  // namespace

int wide_forward(const rlks_mlp_desc* d, const float* params, const float* x, int ldx, int M, const WideWs& w,
                 float* logits, float* values, hipStream_t s) {
  const Layout L = make_layout(d->obs_dim, d->hidden, d->n_actions);
  RLKS_HIP(hipMemsetAsync(w.n[0].slots, 0, 4 * SL_N, s));  // net 0's X slot serves both nets
  for (int net = 0; net < 2; ++net) {
    float* dst = net == 0 ? logits : values;
    if (!dst) continue;
    const WideNet& n = w.n[net];
    if (net == 1) RLKS_HIP(hipMemsetAsync(n.slots, 0, 4 * SL_N, s));
    const bool x_done = net == 1 && logits;  // the policy net's forward split X already
    if (int rc = forward_net(d, net_of(params, L, net), n, x, ldx, M, net, w.xh, w.xl, w.n[0].slots + SL_X, x_done, s))
      return rc;
    const int An = net == 0 ? d->n_actions : 1;
    RLKS_HIP(hipMemcpyAsync(dst, n.out, sizeof(float) * M * An, hipMemcpyDeviceToDevice, s));
  }
  return RLKS_OK;
}

int wide_grad(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
              const float* mb, int M, float* grad, double* stats, const WideWs& w, hipStream_t s) {
  const int D = d->obs_dim, H = d->hidden, A = d->n_actions, stride = mb_stride(D, A);
  const Layout L = make_layout(D, H, A);
  const int Mp = (M + 31) / 32 * 32;
  if (Mp != M) {  // zero plane rows [M, Mp): the dW2 reduction over Mp rows then adds exact zeros
    const size_t off = (size_t)M * H, bytes = 2ull * (Mp - M) * H;
    for (_Float16* p : {w.n[0].h1h, w.n[0].h1l, w.n[1].h1h, w.n[1].h1l, w.dzh, w.dzl})
      RLKS_HIP(hipMemsetAsync(p + off, 0, bytes, s));
    for (_Float16* p : {w.xh, w.xl}) RLKS_HIP(hipMemsetAsync(p + (size_t)M * D, 0, 2ull * (Mp - M) * D, s));
  }
  const bool ps_x = D % 32 == 0 && stride % 4 == 0 && ((uintptr_t)mb & 15) == 0;  // X planes (forward_net)
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    const WideNet& n = w.n[net];
    const Net P = net_of(params, L, net);
    float* g = grad;
    const int64_t* o = L.off + 6 * net;
    unsigned* sl = n.slots;
    unsigned* xsl = w.n[0].slots + SL_X;  // X's scale: one slot for both nets
    if (net == 0) RLKS_HIP(hipMemsetAsync(sl, 0, 4 * SL_N, s));
    else RLKS_HIP(hipMemsetAsync(sl + SL_W1, 0, 4 * (SL_N - SL_W1), s));  // keep net 0's X slot (SL_X = 0)
    if (int rc = forward_net(d, P, n, mb, stride, M, net, w.xh, w.xl, xsl, net == 1, s)) return rc;
    if (net == 0)
      hipLaunchKernelGGL(k_wide_loss_pi, dim3(w.blocks), dim3(64 * LOSS_PI_WAVES), 0, s, n.out, mb, stride, M, D, A, *co, dyn,
                         n.dout, n.part_stat, sl + SL_DOUT, sl + SL_DSUM);
    else
      hipLaunchKernelGGL(k_wide_loss_vf, dim3(w.blocks), dim3(LOSS_ROWS), 0, s, n.out, mb, stride, M, D, A, *co, dyn,
                         n.dout, n.part_stat, sl + SL_DOUT);
    RLKS_LAUNCHED();
    // head: dW3 = dout^T H2 (value net: a dout-weighted column sum of H2, HBM-bound), db3 = colsum(dout)
    if (An == 1) {
      if (int rc = launch_colsum(n.h2, M, H, H, g + o[4], 0, w.part, s, n.dout)) return rc;
    } else if (int rc = gemm(n.dout, An, 1, n.h2, H, 0, g + o[4], H, An, H, M, GEMM_STORE, nullptr, nullptr, 0,
                             sl + SL_DOUT, sl + SL_H2, nullptr, s, w.part)) {
      return rc;
    }
    if (net == 0) {
      if (int rc = launch_colsum(n.dout, M, An, An, g + o[5], 0, w.part, s)) return rc;
    } else {
      hipLaunchKernelGGL(k_wide_vb3, dim3(1), dim3(64), 0, s, n.part_stat, w.blocks, g + o[5]);
      RLKS_LAUNCHED();
    }
    // dZ2 = (dout W3) (1 - H2^2); dW2 = dZ2^T H1; db2
    RLKS_REQUIRE(H % 8 == 0, RLKS_ERR_UNSUPPORTED, "wide path: hidden width must be a multiple of 8");
    const int dz_blocks = (int)cdiv(M, DZ_ROWS * DZ_RT);
    // (the value net's sum_a |dout| is |dout|: its max slot)
    hipLaunchKernelGGL(k_wide_dz2, dim3(cdiv(H, DZ_COLS), dz_blocks), dim3(256), 0, s, n.dout, P.w3, n.h2, w.dzh, w.dzl,
                       M, H, An, sl + (net == 0 ? SL_DSUM : SL_DOUT), sl + SL_W3, sl + SL_DZ2, w.part);
    RLKS_LAUNCHED();
    // db2 from the dZ2 kernel's per-block column sums (before dW2's split-K reuses the partial buffer)
    if (int rc = launch_split_reduce(w.part, 2 * dz_blocks, 1, H, g + o[3], H, 0, s)) return rc;  // hi + lo planes
    {  // dW2[n][k] = sum_m dZ2[m][n] H1[m][k]: both operands K-major planes, split over the rows
      PsArgs a{};
      a.a = ps_op(w.dzh, w.dzl, H, 1, H, sl + SL_DZ2);
      a.b = ps_op(n.h1h, n.h1l, H, 1, H, nullptr, H1_EXP);
      a.M = H; a.N = H; a.K = Mp; a.epi = PS_STORE; a.C = g + o[2]; a.ldc = H;
      a.splits = gemm_ps_splits(H, H, Mp);
      a.part = w.part;
      if (int rc = launch_gemm_ps(a, s)) return rc;
    }
    {  // dZ1[m][k] = (sum_n dZ2[m][n] W2[n][k]) (1 - H1^2): B = W2 planes read K-major
      PsArgs a{};
      a.a = ps_op(w.dzh, w.dzl, H, 0, M, sl + SL_DZ2);
      a.b = ps_op(n.w2h, n.w2l, H, 1, H, sl + SL_W2);
      a.M = M; a.N = H; a.K = H; a.epi = PS_DTANH; a.C = w.dzb; a.ldc = H;
      a.aux_hi = n.h1h; a.aux_lo = n.h1l; a.ldaux = H; a.cmax = sl + SL_DZ1;
      if (int rc = launch_gemm_ps(a, s)) return rc;
    }
    // dW1 = dZ1^T X; db1.  With X in planes (obs_dim a multiple of 32): dZ1 split into the dZ2 planes'
    // buffer (free once dZ1's GEMM has read it) and both read K-major by the pre-split GEMM
    if (ps_x) {
      if (int rc = launch_split_planes(w.dzb, M, H, H, sl + SL_DZ1, 0, w.dzh, w.dzl, H, s)) return rc;
      PsArgs a{};
      a.a = ps_op(w.dzh, w.dzl, H, 1, H, sl + SL_DZ1);
      a.b = ps_op(w.xh, w.xl, D, 1, D, w.n[0].slots + SL_X);
      a.M = H; a.N = D; a.K = Mp; a.epi = PS_STORE; a.C = g + o[0]; a.ldc = D;
      a.splits = gemm_ps_splits(H, D, Mp);
      a.part = w.part;
      if (int rc = launch_gemm_ps(a, s)) return rc;
    } else if (int rc = gemm(w.dzb, H, 1, mb, stride, 0, g + o[0], D, H, D, M, GEMM_STORE, nullptr, nullptr, 0,
                             sl + SL_DZ1, w.n[0].slots + SL_X, nullptr, s, w.part)) {
      return rc;
    }
    if (int rc = launch_colsum(w.dzb, M, H, H, g + o[1], 0, w.part, s)) return rc;
  }
  if (stats) {
    hipLaunchKernelGGL(k_wide_stats, dim3(1), dim3(64), 0, s, w.n[0].part_stat, w.n[1].part_stat, w.blocks, M, stats);
    RLKS_LAUNCHED();
  }
  return RLKS_OK;
}

int launch_sample(const EnvView& v, const float* logits, int A, int explore, int32_t* actions, float* logp,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_wide_sample, dim3(cdiv(v.lane_end - v.lane0, 256)), dim3(256), 0, s, v, logits, A, explore,
                     actions, logp);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int wide_rollout(rlks_env* env, const rlks_mlp_desc* d, const float* params, const rlks_rollout_bufs* b, int explore,
                 const WideWs& w, hipStream_t s) {
  const int N = b->N, D = d->obs_dim, A = d->n_actions;
  RLKS_REQUIRE(w.M >= N, RLKS_ERR_ARG, "rlks_rollout_ws: workspace rows < envs");
  const EnvView v = view(env);
  for (int t = 0; t < b->T; ++t) {
    const float* obs = b->obs + (size_t)t * N * D;
    if (int rc = wide_forward(d, params, obs, D, N, w, b->logits + (size_t)t * N * A, b->values + (size_t)t * N, s))
      return rc;
    if (int rc = launch_sample(v, b->logits + (size_t)t * N * A, A, explore, b->actions + (size_t)t * N,
                               b->logp + (size_t)t * N, s))
      return rc;
    if (int rc = rlks_env_step(env, b->actions + (size_t)t * N, b->obs + (size_t)(t + 1) * N * D, w.rew64,
                               b->rewards + (size_t)t * N, b->dones + (size_t)t * N, nullptr, nullptr, nullptr, nullptr,
                               s))
      return rc;
  }
  return wide_forward(d, params, b->obs + (size_t)b->T * N * D, D, N, w, nullptr, b->values + (size_t)b->T * N, s);
}

}  // namespace rlks
