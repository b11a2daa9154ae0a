// mlp.hip — K4: the policy / value MLP (RLlib FCNet, vf_share_layers=False) and the PPO update.
//
// Reference call sites: PPOConfig().framework("torch").training(train_batch_size=4000,
// sgd_minibatch_size=256, num_sgd_iter=10, lr=3e-4, gamma=0.99) (train_ppo.py:9-21); RLlib's
// defaults: fcnet_hiddens [256, 256], tanh, separate value net, clip 0.3, vf_clip 10, kl_coeff
// 0.2 / kl_target 0.01, entropy 0, Adam.  The restated loss (ppo_torch_policy.loss):
//   L = mean(-min(A*r, A*clip(r, 1-c, 1+c)) + vf_coeff*clamp((V-vt)^2, 0, vf_clip)
//            - ent_coeff*H) + kl_coeff*mean(KL(old || new)),   r = exp(logp - logp_old)
//
// Kernels per SGD step (all fp32; the 256x256 hidden products run on v_mfma_f32_32x32x2_f32,
// which is an exact f32 fma chain):
//   F1 k_fwd_head  rows x [H1 = tanh(X W1^T + b1) (VALU, K = D) -> Z2 = H1 W2^T (MFMA) -> H2 = tanh]
//                  -> head (VALU) -> loss -> dZ2 = (dlogits W3) * (1 - H2^2); writes dZ2 and
//                  per-tile partials of db2, dW3, db3, loss stats.  Forward-only for rollouts.
//   F2 k_dw2       dW2 = dZ2^T H1 (MFMA, split over rows; H1 recomputed from X, never stored)
//   F3 k_dh1       dH1 = dZ2 W2 (MFMA) -> dZ1 = dH1 * (1 - H1^2) -> partials of dW1 = dZ1^T X, db1
//   R  k_reduce    deterministic fixed-order sum of every partial into the flat gradient
//   k_adam         torch.optim.Adam
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "rlks_internal.h"

namespace rlks {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int MAXA = 8;   // max actions (clusters) handled by the fused head
constexpr int DMAX = 32;  // max obs dim handled by the VALU input layer
constexpr int BK = 32;    // reduction chunk

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row of accumulator register r for lane l (v_mfma_f32_32x32x* C/D map)
__device__ __forceinline__ int acc_row(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }

// ----------------------------------------------------------------------------- layout
struct Layout {
  int64_t off[RLKS_N_TENSORS];
  int64_t padded, real;
};

static Layout make_layout(int D, int H, int A) {
  const int64_t sz[RLKS_N_TENSORS] = {(int64_t)H * D, H, (int64_t)H * H, H, (int64_t)A * H, A,
                                      (int64_t)H * D, H, (int64_t)H * H, H, H, 1};
  Layout L{};
  int64_t o = 0;
  L.real = 0;
  for (int i = 0; i < RLKS_N_TENSORS; ++i) {
    L.off[i] = o;
    o += (sz[i] + 63) / 64 * 64;
    L.real += sz[i];
  }
  L.padded = o;
  return L;
}

struct NetPtrs {
  const float *w1, *b1, *w2, *b2, *w3, *b3;
};

__device__ __forceinline__ NetPtrs net_ptrs(const float* p, const int64_t* off, int net) {
  const int64_t* o = off + 6 * net;
  return NetPtrs{p + o[0], p + o[1], p + o[2], p + o[3], p + o[4], p + o[5]};
}

struct Offs {
  int64_t o[RLKS_N_TENSORS];
};

// ----------------------------------------------------------------------------- F1
struct FwdArgs {
  const float* params;
  Offs off;
  const float* x;    // row m at x + m * x_stride (obs first D floats)
  int x_stride;
  int M, D, A;
  // forward-only outputs
  float* logits;     // [M][A]
  float* values;     // [M]
  // training
  rlks_ppo_coeffs co;
  const float* dyn;
  float* dz2;        // [2][M][H]
  float* part_b2;    // [2][tiles][H]
  float* part_w3;    // [2][tiles][MAXA][H]  (vf uses a = 0)
  float* part_b3;    // [2][tiles][MAXA]
  float* part_stat;  // [2][tiles][4]
  int tiles;
};

// reduce 16 per-lane values (register r <-> accumulator row) over the 32 lanes of a half-wave;
// afterwards lane l holds the total of register ((l >> 1) & 15) (lanes l and l^1 agree)
__device__ __forceinline__ float half_wave_reduce16(const float (&v)[16], int l) {
  float v8[8], v4[4], v2[2];
  {
    const bool b = (l >> 4) & 1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float send = b ? v[j] : v[j + 8];
      const float keep = b ? v[j + 8] : v[j];
      v8[j] = keep + __shfl_xor(send, 16, 64);
    }
  }
  {
    const bool b = (l >> 3) & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float send = b ? v8[j] : v8[j + 4];
      const float keep = b ? v8[j + 4] : v8[j];
      v4[j] = keep + __shfl_xor(send, 8, 64);
    }
  }
  {
    const bool b = (l >> 2) & 1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float send = b ? v4[j] : v4[j + 2];
      const float keep = b ? v4[j + 2] : v4[j];
      v2[j] = keep + __shfl_xor(send, 4, 64);
    }
  }
  const bool b = (l >> 1) & 1;
  const float send = b ? v2[0] : v2[1];
  const float keep = b ? v2[1] : v2[0];
  float v1 = keep + __shfl_xor(send, 2, 64);
  v1 += __shfl_xor(v1, 1, 64);
  return v1;
}

template <int H, int WM, int WN, bool TRAIN>
__global__ __launch_bounds__(64 * WM * WN) void k_fwd_head(FwdArgs g) {
  constexpr int NT = H / (32 * WN);
  constexpr int BMr = 32 * WM;
  constexpr int NTHR = 64 * WM * WN;
  static_assert(NT >= 1 && NT * 32 * WN == H, "H must split into 32-column tiles per wave");

  static_assert(WM * H * (1 + MAXA) <= H * (BK + 1), "epilogue reduction must fit in the W2 chunk buffer");
  const int D = g.D, ds = g.D + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sB = lds;                             // [H][BK+1]   W2 chunk, [n][k]
  float* sA = sB + H * (BK + 1);               // [BK][BMr]   H1 chunk, [k][m]
  float* sHead = sA + BK * BMr;                // [WN][BMr][MAXA]
  float* sDl = sHead + WN * BMr * MAXA;        // [BMr][MAXA]
  float* sb1 = sDl + BMr * MAXA;               // [H]
  float* sX = sb1 + H;                         // [BMr][D+1]
  float* sW1 = sX + BMr * ds;                  // [H][D+1]

  const int net = blockIdx.y;
  const int A = net == 0 ? g.A : 1;
  const NetPtrs P = net_ptrs(g.params, g.off.o, net);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int row0 = blockIdx.x * BMr;

  // stage X rows, W1, b1
  for (int e = tid; e < BMr * D; e += NTHR) {
    const int m = e / D, d = e % D;
    sX[m * ds + d] = (row0 + m < g.M) ? g.x[(size_t)(row0 + m) * g.x_stride + d] : 0.f;
  }
  for (int e = tid; e < H * D; e += NTHR) sW1[(e / D) * ds + (e % D)] = P.w1[e];
  for (int e = tid; e < H; e += NTHR) sb1[e] = P.b1[e];

  f32x16 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nt][r] = 0.f;

  __syncthreads();
  for (int kc = 0; kc < H; kc += BK) {
    // H1 chunk: sA[k][m] = tanh(b1[k] + sum_d X[m][d] W1[k][d])
    for (int e = tid; e < BK * BMr; e += NTHR) {
      const int kk = e / BMr, m = e % BMr;
      const float* wr = sW1 + (kc + kk) * ds;
      const float* xr = sX + m * ds;
      float z = sb1[kc + kk];
      for (int d = 0; d < D; ++d) z = fmaf(xr[d], wr[d], z);
      sA[kk * BMr + m] = tanhf(z);
    }
    // W2 chunk: sB[n][k] = W2[n][kc + k]
    for (int e = tid; e < H * (BK / 4); e += NTHR) {
      const int n = e / (BK / 4), k4 = e % (BK / 4);
      const float4 v = *reinterpret_cast<const float4*>(P.w2 + (size_t)n * H + kc + 4 * k4);
      float* dst = sB + n * (BK + 1) + 4 * k4;
      dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
    }
    __syncthreads();
    const int h = l >> 5, li = l & 31;
#pragma unroll 4
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      const float a = sA[k * BMr + wm * 32 + li];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float b = sB[((wn * NT + nt) * 32 + li) * (BK + 1) + k];
        acc[nt] = mfma32(a, b, acc[nt]);
      }
    }
    __syncthreads();
  }

  // ---- epilogue: H2 = tanh(Z2 + b2); head partial dot products
  float w3r[NT][MAXA];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = (wn * NT + nt) * 32 + (l & 31);
    const float bb = P.b2[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nt][r] = tanhf(acc[nt][r] + bb);
#pragma unroll
    for (int a = 0; a < MAXA; ++a) w3r[nt][a] = (a < A) ? P.w3[(size_t)a * H + n] : 0.f;
  }
  for (int a = 0; a < A; ++a) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s = 0.f;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) s = fmaf(acc[nt][r], w3r[nt][a], s);
      v[r] = s;
    }
    const float tot = half_wave_reduce16(v, l);
    if ((l & 1) == 0) {
      const int row = wm * 32 + acc_row((l >> 1) & 15, l);
      sHead[(wn * BMr + row) * MAXA + a] = tot;
    }
  }
  __syncthreads();

  // ---- per-row head output, loss and dlogits (one thread per row)
  float st_pl = 0.f, st_vf = 0.f, st_kl = 0.f, st_ent = 0.f;
  if (tid < BMr) {
    const int m = row0 + tid;
    float out[MAXA];
    for (int a = 0; a < A; ++a) {
      float s = P.b3[a];
      for (int j = 0; j < WN; ++j) s += sHead[(j * BMr + tid) * MAXA + a];
      out[a] = s;
    }
    if (!TRAIN) {
      if (m < g.M) {
        if (net == 0) {
          if (g.logits)
            for (int a = 0; a < A; ++a) g.logits[(size_t)m * A + a] = out[a];
        } else if (g.values) {
          g.values[m] = out[0];
        }
      }
    } else {
      float dl[MAXA];
      for (int a = 0; a < MAXA; ++a) dl[a] = 0.f;
      if (m < g.M) {
        const float* rec = g.x + (size_t)m * g.x_stride;
        const float inv_count = g.dyn[RLKS_DYN_INV_COUNT];
        if (net == 0) {
          // record: [obs D | logits_old A | adv | vtarg | logp_old | action]
          const float* lo = rec + D;
          const float adv = (rec[D + A] - g.dyn[RLKS_DYN_ADV_MEAN]) * g.dyn[RLKS_DYN_ADV_INVSTD];
          const float logp_old = rec[D + A + 2];
          const int act = (int)rec[D + A + 3];
          float mx = out[0], mo = lo[0];
          for (int a = 1; a < A; ++a) { mx = fmaxf(mx, out[a]); mo = fmaxf(mo, lo[a]); }
          float se = 0.f, so = 0.f;
          for (int a = 0; a < A; ++a) { se += expf(out[a] - mx); so += expf(lo[a] - mo); }
          const float lse = mx + logf(se), lso = mo + logf(so);
          float p[MAXA], lp[MAXA];
          float kl = 0.f, ent = 0.f;
          for (int a = 0; a < A; ++a) {
            lp[a] = out[a] - lse;
            p[a] = expf(lp[a]);
            const float lpo = lo[a] - lso;
            kl += expf(lpo) * (lpo - lp[a]);
            ent -= p[a] * lp[a];
          }
          const float ratio = expf(lp[act] - logp_old);
          const float lo_c = 1.f - g.co.clip_param, hi_c = 1.f + g.co.clip_param;
          const float rc = fminf(fmaxf(ratio, lo_c), hi_c);
          const float s1 = adv * ratio, s2 = adv * rc;
          const float surr = fminf(s1, s2);
          // torch.min backward: ties split the gradient evenly; clamp passes on [lo, hi]
          const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
          const float w2 = 1.f - w1;
          const float inr = (ratio >= lo_c && ratio <= hi_c) ? 1.f : 0.f;
          const float dsurr_dr = adv * (w1 + w2 * inr);
          const float dr = -dsurr_dr * ratio;  // dL/dlogp(act)
          const float klc = g.dyn[RLKS_DYN_KL_COEFF];
          for (int a = 0; a < A; ++a) {
            const float po = expf(lo[a] - lso);
            float d = dr * ((a == act ? 1.f : 0.f) - p[a]);
            d += klc * (p[a] - po);
            d += g.co.entropy_coeff * p[a] * (lp[a] + ent);
            dl[a] = d * inv_count;
          }
          st_pl = -surr;
          st_kl = kl;
          st_ent = ent;
        } else {
          // value branch: clamp((V - vt)^2, 0, vf_clip); vtarg sits after the pi logits (A_pi)
          const float vt = rec[D + g.A + 1];
          const float diff = out[0] - vt;
          const float sq = diff * diff;
          st_vf = fminf(sq, g.co.vf_clip_param);
          dl[0] = (sq <= g.co.vf_clip_param) ? g.co.vf_loss_coeff * 2.f * diff * inv_count : 0.f;
        }
      }
      for (int a = 0; a < MAXA; ++a) sDl[tid * MAXA + a] = dl[a];
    }
  }
  if (!TRAIN) return;
  __syncthreads();

  // ---- dZ2 = (dlogits W3) * (1 - H2^2); partial db2 / dW3 over this tile's rows
  float* sRed = sB;  // reuse: [WM][H] db2, then [WM][MAXA][H] dW3 (W2 chunk no longer needed)
  float csum[NT], cw3[NT][MAXA];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    csum[nt] = 0.f;
#pragma unroll
    for (int a = 0; a < MAXA; ++a) cw3[nt][a] = 0.f;
  }
  float* dz2 = g.dz2 + (size_t)net * g.M * H;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = wm * 32 + acc_row(r, l);
    float dlr[MAXA];
#pragma unroll
    for (int a = 0; a < MAXA; ++a) dlr[a] = (a < A) ? sDl[row * MAXA + a] : 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float h2 = acc[nt][r];
      float dh = 0.f;
#pragma unroll
      for (int a = 0; a < MAXA; ++a) dh = fmaf(dlr[a], w3r[nt][a], dh);
      const float dz = dh * (1.f - h2 * h2);
      csum[nt] += dz;
#pragma unroll
      for (int a = 0; a < MAXA; ++a) cw3[nt][a] = fmaf(dlr[a], h2, cw3[nt][a]);
      if (row0 + row < g.M) dz2[(size_t)(row0 + row) * H + (wn * NT + nt) * 32 + (l & 31)] = dz;
    }
  }
  // combine the two half-waves (rows 4h + ...), then the WM waves sharing these columns
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    csum[nt] += __shfl_xor(csum[nt], 32, 64);
#pragma unroll
    for (int a = 0; a < MAXA; ++a) cw3[nt][a] += __shfl_xor(cw3[nt][a], 32, 64);
  }
  __syncthreads();  // sB reuse
  if (l < 32) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = (wn * NT + nt) * 32 + l;
      sRed[wm * H + n] = csum[nt];
      for (int a = 0; a < A; ++a) sRed[WM * H + (wm * MAXA + a) * H + n] = cw3[nt][a];
    }
  }
  __syncthreads();
  const int tile = blockIdx.x;
  for (int n = tid; n < H; n += NTHR) {
    float s = 0.f;
    for (int j = 0; j < WM; ++j) s += sRed[j * H + n];
    g.part_b2[((size_t)net * g.tiles + tile) * H + n] = s;
    for (int a = 0; a < A; ++a) {
      float t = 0.f;
      for (int j = 0; j < WM; ++j) t += sRed[WM * H + (j * MAXA + a) * H + n];
      g.part_w3[(((size_t)net * g.tiles + tile) * MAXA + a) * H + n] = t;
    }
  }
  // db3 and stats: one wave-reduction over the per-row values (rows live in threads < BMr <= 64)
  if (w == 0) {
    for (int a = 0; a < A; ++a) {
      const float s = wave_sum(l < BMr ? sDl[l * MAXA + a] : 0.f);
      if (l == 0) g.part_b3[((size_t)net * g.tiles + tile) * MAXA + a] = s;
    }
    const float a0 = wave_sum(st_pl), a1 = wave_sum(st_vf), a2 = wave_sum(st_kl), a3 = wave_sum(st_ent);
    if (l == 0) {
      float* ps = g.part_stat + ((size_t)net * g.tiles + tile) * 4;
      ps[0] = a0; ps[1] = a1; ps[2] = a2; ps[3] = a3;
    }
  }
}

template <int H, int WM, int WN>
static size_t fwd_lds_bytes(int D) {
  constexpr int BMr = 32 * WM;
  const size_t f = (size_t)H * (BK + 1) + BK * BMr + WN * BMr * MAXA + BMr * MAXA + H + (size_t)(BMr + H) * (D + 1);
  return f * sizeof(float);
}

// ----------------------------------------------------------------------------- F2: dW2
struct Dw2Args {
  const float* params;
  Offs off;
  const float* x;
  int x_stride;
  int M, D, H;
  int rows_per_split;
  const float* dz2;  // [2][M][H]
  float* part;       // [S][2][H][H]
  int splits;
};

constexpr int GB = 128;  // GEMM block tile (both dims), 4 waves of 64 x 64

template <int DD>
__global__ __launch_bounds__(256) void k_dw2(Dw2Args g) {
  constexpr int ds = DD + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sA = lds;                // [BK][GB]  dZ2 chunk [m][n]
  float* sB = sA + BK * GB;       // [BK][GB]  H1 chunk  [m][k]
  float* sb1 = sB + BK * GB;      // [GB]
  float* sX = sb1 + GB;           // [BK][DD+1]
  float* sW1 = sX + BK * ds;      // [GB][DD+1]

  const int H = g.H;
  const int tiles_k = H / GB;
  const int tn = blockIdx.x / tiles_k, tk = blockIdx.x % tiles_k;
  const int split = blockIdx.y, net = blockIdx.z;
  const int n0 = tn * GB, k0 = tk * GB;
  const NetPtrs P = net_ptrs(g.params, g.off.o, net);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int h = l >> 5, li = l & 31;
  const float* dz2 = g.dz2 + (size_t)net * g.M * H;

  for (int e = tid; e < GB * DD; e += 256) sW1[(e / DD) * ds + (e % DD)] = P.w1[(size_t)k0 * DD + e];
  for (int e = tid; e < GB; e += 256) sb1[e] = P.b1[k0 + e];

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int mbeg = split * g.rows_per_split;
  for (int mc = mbeg; mc < mbeg + g.rows_per_split; mc += BK) {
    for (int e = tid; e < BK * (GB / 4); e += 256) {
      const int row = e / (GB / 4), c4 = e % (GB / 4);
      *reinterpret_cast<float4*>(sA + row * GB + 4 * c4) =
          *reinterpret_cast<const float4*>(dz2 + (size_t)(mc + row) * H + n0 + 4 * c4);
    }
    for (int e = tid; e < BK * DD; e += 256) sX[(e / DD) * ds + (e % DD)] = g.x[(size_t)(mc + e / DD) * g.x_stride + (e % DD)];
    __syncthreads();
    // H1 recompute: sB[m][k] = tanh(b1[k] + X[m] . W1[k])
    for (int e = tid; e < BK * GB; e += 256) {
      const int row = e / GB, kk = e % GB;
      const float* wr = sW1 + kk * ds;
      const float* xr = sX + row * ds;
      float z = sb1[kk];
#pragma unroll
      for (int d = 0; d < DD; ++d) z = fmaf(xr[d], wr[d], z);
      sB[row * GB + kk] = tanhf(z);
    }
    __syncthreads();
#pragma unroll 4
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[k * GB + wm * 64 + i * 32 + li];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sB[k * GB + wn * 64 + j * 32 + li];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* out = g.part + ((size_t)split * 2 + net) * H * H;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wm * 64 + i * 32 + acc_row(r, l);
        const int k = k0 + wn * 64 + j * 32 + li;
        out[(size_t)n * H + k] = acc[i][j][r];
      }
}

static size_t dw2_lds_bytes(int D) { return ((size_t)2 * BK * GB + GB + (size_t)(BK + GB) * (D + 1)) * sizeof(float); }

// ----------------------------------------------------------------------------- F3: dH1 -> dW1, db1
struct Dh1Args {
  const float* params;
  Offs off;
  const float* x;
  int x_stride;
  int M, D, H;
  const float* dz2;  // [2][M][H]
  float* part_w1;    // [2][tiles][H][D]
  float* part_b1;    // [2][tiles][H]
  int tiles;
};

template <int DD>
__global__ __launch_bounds__(256) void k_dh1(Dh1Args g) {
  constexpr int ds = DD + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sA = lds;                    // [GB][BK+1]  dZ2 chunk [m][n]
  float* sB = sA + GB * (BK + 1);     // [BK][GB]    W2 chunk  [n][k]
  float* sb1 = sB + BK * GB;          // [GB]
  float* sX = sb1 + GB;               // [GB][DD+1]
  float* sW1 = sX + GB * ds;          // [GB][DD+1]
  float* sRed = sA;                   // epilogue reuse: [2][GB][DD+1]
  static_assert(2 * GB * ds <= GB * (BK + 1) + BK * GB, "dW1 reduction must fit in the staging buffers");

  const int H = g.H;
  const int tile = blockIdx.x, tk = blockIdx.y, net = blockIdx.z;
  const int m0 = tile * GB, k0 = tk * GB;
  const NetPtrs P = net_ptrs(g.params, g.off.o, net);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int h = l >> 5, li = l & 31;
  const float* dz2 = g.dz2 + (size_t)net * g.M * H;

  for (int e = tid; e < GB * DD; e += 256) {
    sX[(e / DD) * ds + (e % DD)] = g.x[(size_t)(m0 + e / DD) * g.x_stride + (e % DD)];
    sW1[(e / DD) * ds + (e % DD)] = P.w1[(size_t)k0 * DD + e];
  }
  for (int e = tid; e < GB; e += 256) sb1[e] = P.b1[k0 + e];

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (int nc = 0; nc < H; nc += BK) {
    for (int e = tid; e < GB * (BK / 4); e += 256) {
      const int row = e / (BK / 4), c4 = e % (BK / 4);
      const float4 v = *reinterpret_cast<const float4*>(dz2 + (size_t)(m0 + row) * H + nc + 4 * c4);
      float* dst = sA + row * (BK + 1) + 4 * c4;
      dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
    }
    for (int e = tid; e < BK * (GB / 4); e += 256) {
      const int row = e / (GB / 4), c4 = e % (GB / 4);
      *reinterpret_cast<float4*>(sB + row * GB + 4 * c4) =
          *reinterpret_cast<const float4*>(P.w2 + (size_t)(nc + row) * H + k0 + 4 * c4);
    }
    __syncthreads();
#pragma unroll 4
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[(wm * 64 + i * 32 + li) * (BK + 1) + k];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sB[k * GB + wn * 64 + j * 32 + li];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }

  // epilogue: dZ1 = dH1 * (1 - H1^2) with H1 recomputed; per-column sums over this tile's rows
  float pw[2][DD + 1];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int d = 0; d <= DD; ++d) pw[j][d] = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kk = wn * 64 + j * 32 + li;
    float wr[DD];
#pragma unroll
    for (int d = 0; d < DD; ++d) wr[d] = sW1[kk * ds + d];
    const float bb = sb1[kk];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = wm * 64 + i * 32 + acc_row(r, l);
        const float* xr = sX + mm * ds;
        float xv[DD];
#pragma unroll
        for (int d = 0; d < DD; ++d) xv[d] = xr[d];
        float z = bb;
#pragma unroll
        for (int d = 0; d < DD; ++d) z = fmaf(xv[d], wr[d], z);
        const float h1 = tanhf(z);
        const float dz = acc[i][j][r] * (1.f - h1 * h1);
        pw[j][DD] += dz;
#pragma unroll
        for (int d = 0; d < DD; ++d) pw[j][d] = fmaf(dz, xv[d], pw[j][d]);
      }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int d = 0; d <= DD; ++d) pw[j][d] += __shfl_xor(pw[j][d], 32, 64);
  if (l < 32) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kk = wn * 64 + j * 32 + l;
      float* dst = sRed + (wm * GB + kk) * ds;
#pragma unroll
      for (int d = 0; d <= DD; ++d) dst[d] = pw[j][d];
    }
  }
  __syncthreads();
  for (int e = tid; e < GB * ds; e += 256) {
    const int kk = e / ds, d = e % ds;
    const float s = sRed[kk * ds + d] + sRed[(GB + kk) * ds + d];
    if (d == DD)
      g.part_b1[((size_t)net * g.tiles + tile) * H + k0 + kk] = s;
    else
      g.part_w1[(((size_t)net * g.tiles + tile) * H + k0 + kk) * DD + d] = s;
  }
}

static size_t dh1_lds_bytes(int D) {
  return ((size_t)GB * (BK + 1) + BK * GB + GB + (size_t)2 * GB * (D + 1)) * sizeof(float);
}

// ----------------------------------------------------------------------------- R: reduce
// out[i] = sum_p part[p * pstride + i] for i < len, p < P, in fixed order (f64 accumulation)
struct RedTask {
  const float* part;
  float* out;
  int64_t pstride;
  int P, len;
  int blk0;  // first block of this task
};
constexpr int MAX_TASKS = 16;
struct RedArgs {
  RedTask t[MAX_TASKS];
  int ntasks;
};

__global__ __launch_bounds__(256) void k_reduce(RedArgs g) {
  __shared__ double sh[4][64];
  int ti = 0;
  while (ti + 1 < g.ntasks && (int)blockIdx.x >= g.t[ti + 1].blk0) ++ti;
  const RedTask& T = g.t[ti];
  const int i = ((int)blockIdx.x - T.blk0) * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  double s = 0.0;
  if (i < T.len)
    for (int p = grp; p < T.P; p += 4) s += (double)T.part[(int64_t)p * T.pstride + i];
  sh[grp][threadIdx.x & 63] = s;
  __syncthreads();
  if (grp == 0 && i < T.len) T.out[i] = (float)(sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x]);
}

__global__ void k_stats(const float* __restrict__ ps, int tiles, int rows, double* __restrict__ out) {
  __shared__ double sh[RLKS_STAT_SIZE][256];
  double s[4] = {0, 0, 0, 0};
  for (int i = threadIdx.x; i < 2 * tiles; i += blockDim.x)
    for (int c = 0; c < 4; ++c) s[c] += ps[(size_t)i * 4 + c];
  for (int c = 0; c < 4; ++c) sh[c][threadIdx.x] = s[c];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int c = 0; c < 4; ++c) sh[c][threadIdx.x] += sh[c][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[RLKS_STAT_POLICY_LOSS] = sh[0][0];
    out[RLKS_STAT_VF_LOSS] = sh[1][0];
    out[RLKS_STAT_KL] = sh[2][0];
    out[RLKS_STAT_ENTROPY] = sh[3][0];
    out[RLKS_STAT_ROWS] = (double)rows;
    out[5] = out[6] = out[7] = 0.0;
  }
}

// ----------------------------------------------------------------------------- Adam
// torch.optim.Adam (single-tensor path): exp_avg.lerp_(g, 1-b1); exp_avg_sq = b2*v + (1-b2)*g*g;
// p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, int64_t n, float w1, float b2, float omb2, float step_size,
                       float bc2_sqrt, float eps) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  const float mi = m[i] + w1 * (gi - m[i]);
  const float vi = b2 * v[i] + omb2 * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = p[i] - step_size * (mi / denom);
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
// Philox-keyed balanced Feistel bijection on [0, 2^(2*half)), cycle-walked into [0, S)
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

struct GatherArgs {
  rlks_rollout_bufs b;
  Perm perm;
  int64_t row0;
  int rows, D, A, stride;
  const float* dyn;
  float* mb;
};

__global__ void k_gather(GatherArgs g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.rows) return;
  const uint64_t s = perm_apply(g.perm, (uint64_t)(g.row0 + i));
  const int N = g.b.N;
  const int64_t t = (int64_t)(s / N), n = (int64_t)(s % N);
  const int64_t tn = t * N + n;
  float* rec = g.mb + (size_t)i * g.stride;
  const float* o = g.b.obs + tn * g.D;
  for (int d = 0; d < g.D; ++d) rec[d] = o[d];
  const float* lo = g.b.logits + tn * g.A;
  for (int a = 0; a < g.A; ++a) rec[g.D + a] = lo[a];
  rec[g.D + g.A] = g.b.adv[tn];
  rec[g.D + g.A + 1] = g.b.vtarg[tn];
  rec[g.D + g.A + 2] = g.b.logp[tn];
  rec[g.D + g.A + 3] = (float)g.b.actions[tn];
  for (int j = g.D + g.A + 4; j < g.stride; ++j) rec[j] = 0.f;
}

static Perm make_perm(uint64_t seed, int epoch, uint64_t S) {
  Perm P{};
  uint32_t bits = 2;
  while ((1ull << bits) < S) ++bits;
  if (bits & 1) ++bits;
  P.half = bits / 2;
  P.mask = (P.half >= 32) ? 0xffffffffu : ((1u << P.half) - 1u);
  P.S = S;
  // round keys: splitmix64 of (seed, epoch) — host side, cheap
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(epoch + 1));
  for (int r = 0; r < 4; ++r) {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    P.key[r] = (uint32_t)x;
  }
  return P;
}

static int mb_stride(int D, int A) { return (D + A + 4 + 3) / 4 * 4; }

// ----------------------------------------------------------------------------- host helpers
struct Ws {
  float* dz2;
  float* part_b2;
  float* part_w3;
  float* part_b3;
  float* part_stat;
  float* part_w2;
  float* part_w1;
  float* part_b1;
  int64_t bytes;
  int t1, t3, splits, rows_per_split;
};

static int pick_splits(int M, int H) {
  const int tiles = (H / GB) * (H / GB) * 2;
  int s = 1;
  while (s * 2 * tiles <= 1024 && (M / (s * 2)) % BK == 0 && M / (s * 2) >= 4 * BK) s *= 2;
  return s;
}

static Ws ws_layout(const rlks_mlp_desc* d, int M, char* base) {
  Ws w{};
  const int H = d->hidden, D = d->obs_dim;
  w.t1 = M / 64;
  w.t3 = M / GB;
  w.splits = pick_splits(M, H);
  w.rows_per_split = M / w.splits;
  int64_t o = 0;
  auto take = [&](float** p, int64_t n) {
    *p = base ? reinterpret_cast<float*>(base + o) : nullptr;
    o += (n * 4 + 255) / 256 * 256;
  };
  take(&w.dz2, 2LL * M * H);
  take(&w.part_b2, 2LL * w.t1 * H);
  take(&w.part_w3, 2LL * w.t1 * MAXA * H);
  take(&w.part_b3, 2LL * w.t1 * MAXA);
  take(&w.part_stat, 2LL * w.t1 * 4);
  take(&w.part_w2, (int64_t)w.splits * 2 * H * H);
  take(&w.part_w1, 2LL * w.t3 * H * D);
  take(&w.part_b1, 2LL * w.t3 * H);
  w.bytes = o;
  return w;
}

static int check_desc(const rlks_mlp_desc* d) {
  RLKS_REQUIRE(d, RLKS_ERR_ARG, "null mlp desc");
  RLKS_REQUIRE(d->obs_dim > 0 && d->obs_dim <= DMAX, RLKS_ERR_UNSUPPORTED, "obs_dim must be in [1, 32]");
  RLKS_REQUIRE(d->n_actions >= 1 && d->n_actions <= MAXA, RLKS_ERR_UNSUPPORTED, "n_actions must be in [1, 8]");
  RLKS_REQUIRE(d->hidden == 256, RLKS_ERR_UNSUPPORTED, "fused MLP kernels are built for hidden = 256");
  return RLKS_OK;
}

static Offs offs_of(const rlks_mlp_desc* d) {
  const Layout L = make_layout(d->obs_dim, d->hidden, d->n_actions);
  Offs o;
  for (int i = 0; i < RLKS_N_TENSORS; ++i) o.o[i] = L.off[i];
  return o;
}

template <int WM, int WN, bool TRAIN>
static int launch_fwd(const FwdArgs& a, int M, hipStream_t s) {
  constexpr int BMr = 32 * WM;
  const size_t lds = fwd_lds_bytes<256, WM, WN>(a.D);
  hipLaunchKernelGGL((k_fwd_head<256, WM, WN, TRAIN>), dim3(cdiv(M, BMr), 2), dim3(64 * WM * WN), lds, s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

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
  RLKS_REQUIRE(params && obs && n >= 0, RLKS_ERR_ARG, "rlks_policy_forward: bad argument");
  if (n == 0) return RLKS_OK;
  FwdArgs a{};
  a.params = params;
  a.off = offs_of(d);
  a.x = obs;
  a.x_stride = d->obs_dim;
  a.M = n;
  a.D = d->obs_dim;
  a.A = d->n_actions;
  a.logits = logits;
  a.values = values;
  hipStream_t s = (hipStream_t)stream;
  // small batches: 32-row tiles with the 4 waves split over columns (fills more CUs)
  if (n <= 64 * 1024) return launch_fwd<1, 4, false>(a, n, s);
  return launch_fwd<2, 2, false>(a, n, s);
}

int rlks_minibatch_stride(const rlks_mlp_desc* d) { return d ? mb_stride(d->obs_dim, d->n_actions) : 0; }

int rlks_ppo_gather(const rlks_mlp_desc* d, const rlks_rollout_bufs* b, uint64_t perm_seed, int epoch,
                    int64_t row0, int rows, const float* dyn, float* mb, void* stream) {
  RLKS_REQUIRE(d && b && mb && dyn && rows >= 0, RLKS_ERR_ARG, "rlks_ppo_gather: bad argument");
  const uint64_t S = (uint64_t)b->T * (uint64_t)b->N;
  RLKS_REQUIRE(row0 >= 0 && (uint64_t)(row0 + rows) <= S, RLKS_ERR_ARG, "rlks_ppo_gather: rows out of range");
  if (rows == 0) return RLKS_OK;
  GatherArgs g{};
  g.b = *b;
  g.perm = make_perm(perm_seed, epoch, S);
  g.row0 = row0;
  g.rows = rows;
  g.D = d->obs_dim;
  g.A = d->n_actions;
  g.stride = mb_stride(d->obs_dim, d->n_actions);
  g.dyn = dyn;
  g.mb = mb;
  hipLaunchKernelGGL(k_gather, dim3(cdiv(rows, 256)), dim3(256), 0, (hipStream_t)stream, g);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int rlks_ppo_workspace_bytes(const rlks_mlp_desc* d, int rows, int64_t* bytes) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(bytes && rows > 0 && rows % GB == 0, RLKS_ERR_ARG,
               "rlks_ppo_workspace_bytes: rows must be a positive multiple of 128");
  *bytes = ws_layout(d, rows, nullptr).bytes;
  return RLKS_OK;
}

int rlks_ppo_grad_phases(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                         const float* mb, int M, float* grad, double* stats, void* workspace, int64_t ws_bytes,
                         int phases, void* stream) {
  if (int rc = check_desc(d)) return rc;
  RLKS_REQUIRE(co && params && dyn && mb && grad && workspace, RLKS_ERR_ARG, "rlks_ppo_grad: null argument");
  RLKS_REQUIRE(M > 0 && M % GB == 0, RLKS_ERR_ARG, "rlks_ppo_grad: rows must be a positive multiple of 128");
  Ws w = ws_layout(d, M, (char*)workspace);
  RLKS_REQUIRE(ws_bytes >= w.bytes, RLKS_ERR_ARG, "rlks_ppo_grad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const Layout L = make_layout(d->obs_dim, d->hidden, d->n_actions);
  const Offs off = offs_of(d);
  const int H = d->hidden, D = d->obs_dim, A = d->n_actions;
  const int stride = mb_stride(D, A);

  FwdArgs f{};
  f.params = params; f.off = off; f.x = mb; f.x_stride = stride; f.M = M; f.D = D; f.A = A;
  f.co = *co; f.dyn = dyn; f.dz2 = w.dz2; f.part_b2 = w.part_b2; f.part_w3 = w.part_w3;
  f.part_b3 = w.part_b3; f.part_stat = w.part_stat; f.tiles = w.t1;
  if (phases & RLKS_PHASE_FWD)
    if (int rc = launch_fwd<2, 2, true>(f, M, s)) return rc;

  Dw2Args a2{};
  a2.params = params; a2.off = off; a2.x = mb; a2.x_stride = stride; a2.M = M; a2.D = D; a2.H = H;
  a2.rows_per_split = w.rows_per_split; a2.dz2 = w.dz2; a2.part = w.part_w2; a2.splits = w.splits;
  if (phases & RLKS_PHASE_DW2) switch (D) {
    case 6: hipLaunchKernelGGL(k_dw2<6>, dim3((H / GB) * (H / GB), w.splits, 2), dim3(256), dw2_lds_bytes(D), s, a2); break;
    case 24: hipLaunchKernelGGL(k_dw2<24>, dim3((H / GB) * (H / GB), w.splits, 2), dim3(256), dw2_lds_bytes(D), s, a2); break;
    default: return fail(RLKS_ERR_UNSUPPORTED, "rlks_ppo_grad: obs_dim must be 6 or 24");
  }
  RLKS_LAUNCHED();

  Dh1Args a3{};
  a3.params = params; a3.off = off; a3.x = mb; a3.x_stride = stride; a3.M = M; a3.D = D; a3.H = H;
  a3.dz2 = w.dz2; a3.part_w1 = w.part_w1; a3.part_b1 = w.part_b1; a3.tiles = w.t3;
  if (phases & RLKS_PHASE_DH1) switch (D) {
    case 6: hipLaunchKernelGGL(k_dh1<6>, dim3(w.t3, H / GB, 2), dim3(256), dh1_lds_bytes(D), s, a3); break;
    case 24: hipLaunchKernelGGL(k_dh1<24>, dim3(w.t3, H / GB, 2), dim3(256), dh1_lds_bytes(D), s, a3); break;
    default: return fail(RLKS_ERR_UNSUPPORTED, "rlks_ppo_grad: obs_dim must be 6 or 24");
  }
  RLKS_LAUNCHED();

  RedArgs r{};
  int blk = 0;
  auto add = [&](const float* part, float* out, int64_t pstride, int P, int len) {
    RedTask& t = r.t[r.ntasks++];
    t.part = part; t.out = out; t.pstride = pstride; t.P = P; t.len = len; t.blk0 = blk;
    blk += (int)cdiv(len, 64);
  };
  for (int net = 0; net < 2; ++net) {
    const int An = net == 0 ? A : 1;
    const int64_t* o = L.off + 6 * net;
    add(w.part_w1 + (size_t)net * w.t3 * H * D, grad + o[0], (int64_t)H * D, w.t3, H * D);
    add(w.part_b1 + (size_t)net * w.t3 * H, grad + o[1], H, w.t3, H);
    add(w.part_w2 + (size_t)net * H * H, grad + o[2], 2LL * H * H, w.splits, H * H);
    add(w.part_b2 + (size_t)net * w.t1 * H, grad + o[3], H, w.t1, H);
    // dW3 partials are [tile][MAXA][H]: the first An rows of each tile are the tensor [An][H]
    add(w.part_w3 + (size_t)net * w.t1 * MAXA * H, grad + o[4], (int64_t)MAXA * H, w.t1, An * H);
    add(w.part_b3 + (size_t)net * w.t1 * MAXA, grad + o[5], MAXA, w.t1, An);
  }
  if (!(phases & RLKS_PHASE_REDUCE)) return RLKS_OK;
  hipLaunchKernelGGL(k_reduce, dim3(blk), dim3(256), 0, s, r);
  RLKS_LAUNCHED();
  if (stats) {
    hipLaunchKernelGGL(k_stats, dim3(1), dim3(256), 0, s, w.part_stat, w.t1, M, stats);
    RLKS_LAUNCHED();
  }
  return RLKS_OK;
}

int rlks_ppo_grad(const rlks_mlp_desc* d, const rlks_ppo_coeffs* co, const float* params, const float* dyn,
                  const float* mb, int M, float* grad, double* stats, void* workspace, int64_t ws_bytes,
                  void* stream) {
  return rlks_ppo_grad_phases(d, co, params, dyn, mb, M, grad, stats, workspace, ws_bytes, RLKS_PHASE_ALL, stream);
}

int rlks_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                   float eps, int step, void* stream) {
  RLKS_REQUIRE(p && g && m && v && n >= 0 && step >= 1, RLKS_ERR_ARG, "rlks_adam_step: bad argument");
  if (n == 0) return RLKS_OK;
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)std::sqrt(bc2);
  hipLaunchKernelGGL(k_adam, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, 1.f - beta1,
                     beta2, 1.f - beta2, step_size, bc2_sqrt, eps);
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
  RLKS_REQUIRE(env && params && b && b->T > 0 && b->N > 0, RLKS_ERR_ARG, "rlks_rollout: bad argument");
  rlks_env_cfg cfg;
  rlks_env_config(env, &cfg);
  RLKS_REQUIRE(cfg.n_envs == b->N && 3 * cfg.n_clouds == d->obs_dim && cfg.n_clouds == d->n_actions,
               RLKS_ERR_ARG, "rlks_rollout: env / policy / buffer shapes disagree");
  const int N = b->N, D = d->obs_dim, A = d->n_actions;
  for (int t = 0; t < b->T; ++t) {
    float* obs_t = b->obs + (size_t)t * N * D;
    if (int rc = rlks_policy_forward(d, params, obs_t, N, b->logits + (size_t)t * N * A, b->values + (size_t)t * N,
                                     stream))
      return rc;
    if (int rc = rlks_env_sample_step(env, b->logits + (size_t)t * N * A, explore, b->actions + (size_t)t * N,
                                      b->logp + (size_t)t * N, b->obs + (size_t)(t + 1) * N * D,
                                      b->rewards + (size_t)t * N, b->dones + (size_t)t * N, stream))
      return rc;
  }
  return rlks_policy_forward(d, params, b->obs + (size_t)b->T * N * D, N, nullptr, b->values + (size_t)b->T * N,
                             stream);
}

}  // extern "C"
