// mlp_fwd.hip — F1: fused FCNet forward + head + PPO loss + dZ2 for one net (pi or vf).
//
// Per workgroup: BMr = 32*WM rows of the minibatch (or rollout obs), all HID = 256 hidden columns.
//   H1 = tanh(X W1^T + b1)      VALU (K = D = 6), computed chunk-wise straight into LDS
//   Z2 = H1 W2^T                v_mfma_f32_32x32x2_f32; W2 chunks staged through LDS, the next
//                               chunk's global loads in flight (registers) during the MFMAs
//   H2 = tanh(Z2 + b2)          in the accumulators
//   out = H2 W3^T + b3          VALU dot + half-wave butterfly reduce-scatter + LDS across waves
// Forward-only (rollout): write logits / values.  Training additionally:
//   pi: ratio, clipped surrogate, KL(old||new), entropy -> dlogits     (RLlib ppo_torch_policy.loss)
//   vf: clamp((V - vt)^2, 0, vf_clip) -> dV
//   dZ2 = (dout W3) * (1 - H2^2) -> HBM (the only activation that leaves the chip), and per-tile
//   partial sums of db2 = colsum dZ2, dW3 = dout^T H2, db3, loss stats (fixed-order reduction
//   later, so the gradient is bit-reproducible run to run).
#include "mlp_common.h"

namespace rlks {

template <int A_, int NET, int WM, int WN, int MODE, int DD>
__global__ __launch_bounds__(64 * WM * WN) void k_fwd_head(FwdArgs g) {
  constexpr bool TRAIN = MODE == FWD_TRAIN;
  static_assert(MODE != FWD_ROLLOUT || NET == 0, "rollout mode drives the policy net");
  constexpr int H = HID;
  constexpr int NT = H / (32 * WN);     // 32-column accumulator tiles per wave
  constexpr int BMr = 32 * WM;          // rows per workgroup
  constexpr int NTHR = 64 * WM * WN;
  constexpr int F4 = H * BK / 4 / NTHR; // float4 of the W2 chunk per thread
  static_assert(NT * 32 * WN == H && F4 * 4 * NTHR == H * BK, "tile split");
  static_assert(WM * H * (1 + A_) <= 2 * H * (BK + 1), "epilogue reduction must fit in the staging buffers");
  static_assert(BMr <= 128, "loss rows are handled by the first two waves");

  constexpr int D = DD, ds = DD + 1;
  constexpr int SB = H * (BK + 1), SA = BK * BMr;
  constexpr int HPT = SA / NTHR;         // H1 elements per thread per chunk
  static_assert(HPT * NTHR == SA && (BK / 2) % HPT == 0, "H1 chunk split over the MFMA steps");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sB = lds;                       // [2][H][BK+1]  W2 chunks [n][k] (double buffer)
  float* sA = sB + 2 * SB;               // [2][BK][BMr]  H1 chunks [k][m] (double buffer)
  float* sHead = sA + 2 * SA;            // [WN][BMr][A_]
  float* sDl = sHead + WN * BMr * A_;    // [BMr][A_]
  float* sStat = sDl + BMr * A_;         // [2][A_ + 4]
  float* sb1 = sStat + 2 * (A_ + 4);     // [H]
  float* sX = sb1 + H;                   // [BMr][D+1]
  float* sW1 = sX + BMr * ds;            // [H][D+1]
  double* sTab = reinterpret_cast<double*>(sW1 + ((H * ds + 1) & ~1));  // rollout: [2][T][C] tables
  __shared__ double sVx[2];             // value net: waves 0, 1's f64 sums of v - vt (vf_row)

  const NetPtrs& P = g.P;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int h = l >> 5, li = l & 31;
  const int row0 = blockIdx.x * BMr;

  for (int e = tid; e < BMr * D; e += NTHR) {
    const int m = e / D, d = e - m * D;
    sX[m * ds + d] = (row0 + m < g.M) ? g.x[(size_t)(row0 + m) * g.x_stride + d] : 0.f;
  }
  for (int e = tid; e < H * D; e += NTHR) sW1[(e / D) * ds + (e % D)] = P.w1[e];
  for (int e = tid; e < H; e += NTHR) sb1[e] = P.b1[e];
  if (MODE == FWD_ROLLOUT)
    for (int e = tid; e < g.env.T * g.env.C; e += NTHR) {
      sTab[e] = g.tab_cost[e];
      sTab[g.env.T * g.env.C + e] = g.tab_lat[e];
    }

  float4 pre[F4];
#define F1_LOAD_W2(kc)                                                                     \
  _Pragma("unroll") for (int j = 0; j < F4; ++j) {                                         \
    const int e_ = tid + j * NTHR;                                                         \
    pre[j] = *reinterpret_cast<const float4*>(P.w2 + (size_t)(e_ >> 3) * H + (kc) + 4 * (e_ & 7)); \
  }
#define F1_STORE_W2(buf)                                                                   \
  _Pragma("unroll") for (int j = 0; j < F4; ++j) {                                         \
    const int e_ = tid + j * NTHR;                                                         \
    float* dst_ = sB + (buf) * SB + (e_ >> 3) * (BK + 1) + 4 * (e_ & 7);                   \
    dst_[0] = pre[j].x; dst_[1] = pre[j].y; dst_[2] = pre[j].z; dst_[3] = pre[j].w;        \
  }
  // one H1 element of chunk kc: sA[buf][k][m] = tanh(b1[k] + X[m] . W1[k])
#define F1_H1(kc, buf, idx)                                                                \
  {                                                                                        \
    const int e_ = tid + (idx) * NTHR, kk_ = e_ / BMr, m_ = e_ - kk_ * BMr;                 \
    const float* wr_ = sW1 + ((kc) + kk_) * ds;                                            \
    const float* xr_ = sX + m_ * ds;                                                       \
    float z_ = sb1[(kc) + kk_];                                                            \
    _Pragma("unroll") for (int d_ = 0; d_ < D; ++d_) z_ = fmaf(xr_[d_], wr_[d_], z_);    \
    sA[(buf) * SA + kk_ * BMr + m_] = fast_tanh(z_);                                       \
  }

  F1_LOAD_W2(0);
  f32x16 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nt][r] = 0.f;
  __syncthreads();  // sX / sW1 / sb1 staged
  F1_STORE_W2(0);
#pragma unroll
  for (int i = 0; i < HPT; ++i) F1_H1(0, 0, i);
  F1_LOAD_W2(BK);
  __syncthreads();

  // chunk c: MFMAs on buffer c&1 while this thread computes its H1 share of chunk c+1 into the
  // other buffer between them and parks W2 chunk c+1 / issues the loads of chunk c+2: one
  // barrier per chunk, the tanh work overlapping the matrix pipe.
  constexpr int NC = H / BK, SPH = (BK / 2) / HPT;  // chunks; MFMA steps per H1 element
  for (int c = 0; c < NC - 1; ++c) {
    const int cur = c & 1, nxt = cur ^ 1;
    F1_STORE_W2(nxt);
    if (c + 2 < NC) { F1_LOAD_W2((c + 2) * BK); }
    const float* a_src = sA + cur * SA + wm * 32 + li;
    const float* b_src = sB + cur * SB + (wn * NT * 32 + li) * (BK + 1);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      const float a = a_src[k * BMr];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma32(a, b_src[nt * 32 * (BK + 1) + k], acc[nt]);
      if (s % SPH == 0) F1_H1((c + 1) * BK, nxt, s / SPH);
    }
    __syncthreads();
  }
  {
    const float* a_src = sA + ((NC - 1) & 1) * SA + wm * 32 + li;
    const float* b_src = sB + ((NC - 1) & 1) * SB + (wn * NT * 32 + li) * (BK + 1);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      const float a = a_src[k * BMr];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma32(a, b_src[nt * 32 * (BK + 1) + k], acc[nt]);
    }
    __syncthreads();
  }
#undef F1_LOAD_W2
#undef F1_STORE_W2
#undef F1_H1

  // ---- H2 = tanh(Z2 + b2); head partial dot products over this wave's columns
  float w3r[NT][A_];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = (wn * NT + nt) * 32 + li;
    const float bb = P.b2[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nt][r] = fast_tanh(acc[nt][r] + bb);
#pragma unroll
    for (int a = 0; a < A_; ++a) w3r[nt][a] = P.w3[(size_t)a * H + n];
  }
#pragma unroll
  for (int a = 0; a < A_; ++a) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s = 0.f;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) s = fmaf(acc[nt][r], w3r[nt][a], s);
      v[r] = s;
    }
    const float tot = half_wave_reduce16(v, l);
    if ((l & 1) == 0) sHead[(wn * BMr + wm * 32 + acc_row((l >> 1) & 15, l)) * A_ + a] = tot;
  }
  __syncthreads();

  // ---- per-row output, loss and dout (one thread per row)
  float st_pl = 0.f, st_vf = 0.f, st_kl = 0.f, st_ent = 0.f;
  double vex = 0.0;  // value net: the row's exact v - vt (vf_row)
  if (tid < BMr) {
    const int m = row0 + tid;
    float out[A_];
#pragma unroll
    for (int a = 0; a < A_; ++a) {
      float s = P.b3[a];
#pragma unroll
      for (int j = 0; j < WN; ++j) s += sHead[(j * BMr + tid) * A_ + a];
      out[a] = s;
    }
    if (MODE == FWD_ONLY) {
      if (m < g.M)
#pragma unroll
        for (int a = 0; a < A_; ++a) g.out[(size_t)m * A_ + a] = out[a];
    } else if (MODE == FWD_ROLLOUT) {
      if (m < g.M) {
        // TorchCategorical: sample (Philox, counter = lane/episode/step) or argmax (explore=False)
        float mx = out[0];
        int amax = 0;
#pragma unroll
        for (int a = 1; a < A_; ++a)
          if (out[a] > mx) { mx = out[a]; amax = a; }
        float e[A_], se = 0.f;
#pragma unroll
        for (int a = 0; a < A_; ++a) { e[a] = expf(out[a] - mx); se += e[a]; }
        int act = amax;
        const EnvView& v = g.env;
        if (g.explore) {
          const u32x4 x = philox4x32_10(u32x4{(uint32_t)(v.env_offset + m), (uint32_t)v.episode[m],
                                              (uint32_t)v.step[m], (uint32_t)RLKS_PURPOSE_ACTION << 16},
                                        v.k0, v.k1);
          const float u = (float)u53(x.x, x.y) * se;
          float c = 0.f;
          act = A_ - 1;
          bool found = false;
#pragma unroll
          for (int a = 0; a < A_; ++a) {
            c += e[a];
            if (!found && u < c) { act = a; found = true; }
          }
        }
        float la = out[0];
#pragma unroll
        for (int a = 0; a < A_; ++a) {
          g.out[(size_t)m * A_ + a] = out[a];
          la = (a == act) ? out[a] : la;
        }
        g.actions[m] = act;
        g.logp[m] = la - mx - logf(se);
        const StepOut r = step_lane(v, sTab, m, act, g.obs_next + (size_t)m * D, nullptr);
        g.rewards[m] = (float)r.reward;
        g.dones[m] = (uint8_t)r.done;
      }
    } else {
      float dl[A_];
#pragma unroll
      for (int a = 0; a < A_; ++a) dl[a] = 0.f;
      if (m < g.M) {
        const float* rec = g.x + (size_t)m * g.x_stride;
        const float inv_count = g.dyn[RLKS_DYN_INV_COUNT];
        const int Ap = g.A_pi;
        if (NET == 0) {
          const float* lo = rec + D;
          const float adv = (rec[D + Ap] - g.dyn[RLKS_DYN_ADV_MEAN]) * g.dyn[RLKS_DYN_ADV_INVSTD];
          const float logp_old = rec[D + Ap + 2];
          const int act = (int)rec[D + Ap + 3];
          float mx = out[0], mo = lo[0];
#pragma unroll
          for (int a = 1; a < A_; ++a) { mx = fmaxf(mx, out[a]); mo = fmaxf(mo, lo[a]); }
          float se = 0.f, so = 0.f;
#pragma unroll
          for (int a = 0; a < A_; ++a) { se += expf(out[a] - mx); so += expf(lo[a] - mo); }
          const float lse = mx + logf(se), lso = mo + logf(so);
          float p[A_], lp[A_], po[A_];
          float kl = 0.f, ent = 0.f, lpa = 0.f;
#pragma unroll
          for (int a = 0; a < A_; ++a) {
            lp[a] = out[a] - lse;
            p[a] = expf(lp[a]);
            const float lpo = lo[a] - lso;
            po[a] = expf(lpo);
            kl += po[a] * (lpo - lp[a]);
            ent -= p[a] * lp[a];
            lpa = (a == act) ? lp[a] : lpa;
          }
          const float ratio = expf(lpa - logp_old);
          const float lo_c = 1.f - g.co.clip_param, hi_c = 1.f + g.co.clip_param;
          const float rc = fminf(fmaxf(ratio, lo_c), hi_c);
          const float s1 = adv * ratio, s2 = adv * rc;
          // torch.min backward splits ties evenly; torch.clamp passes the gradient on [lo, hi]
          const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
          const float inr = (ratio >= lo_c && ratio <= hi_c) ? 1.f : 0.f;
          const float dr = -adv * (w1 + (1.f - w1) * inr) * ratio;  // dL / dlogp(act)
          const float klc = g.dyn[RLKS_DYN_KL_COEFF];
#pragma unroll
          for (int a = 0; a < A_; ++a) {
            float d = dr * ((a == act ? 1.f : 0.f) - p[a]);
            d += klc * (p[a] - po[a]);
            d += g.co.entropy_coeff * p[a] * (lp[a] + ent);
            dl[a] = d * inv_count;
          }
          st_pl = -fminf(s1, s2);
          st_kl = kl;
          st_ent = ent;
        } else {
          const VfRow v = vf_row(out[0], rec[D + Ap + 1], g.co.vf_clip_param, g.co.vf_loss_coeff, inv_count);
          st_vf = v.sq;
          dl[0] = v.dl;
          vex = v.ex;
        }
      }
#pragma unroll
      for (int a = 0; a < A_; ++a) sDl[tid * A_ + a] = dl[a];
    }
  }
  if (!TRAIN) return;
  __syncthreads();

  // ---- dZ2 = (dout W3) * (1 - H2^2); column partials of db2 and dW3 over this tile's rows
  float csum[NT], cw3[NT][A_];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    csum[nt] = 0.f;
#pragma unroll
    for (int a = 0; a < A_; ++a) cw3[nt][a] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = wm * 32 + acc_row(r, l);
    float dlr[A_];
#pragma unroll
    for (int a = 0; a < A_; ++a) dlr[a] = sDl[row * A_ + a];
    float* dst = g.dz2 + (size_t)(row0 + row) * H + wn * NT * 32 + li;  // M % BMr == 0 in training
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float h2 = acc[nt][r];
      float dh = 0.f;
#pragma unroll
      for (int a = 0; a < A_; ++a) {
        dh = fmaf(dlr[a], w3r[nt][a], dh);
        cw3[nt][a] = fmaf(dlr[a], h2, cw3[nt][a]);
      }
      const float dz = dh * (1.f - h2 * h2);
      csum[nt] += dz;
      dst[nt * 32] = dz;
    }
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    csum[nt] += __shfl_xor(csum[nt], 32, 64);
#pragma unroll
    for (int a = 0; a < A_; ++a) cw3[nt][a] += __shfl_xor(cw3[nt][a], 32, 64);
  }
  float* sRed = sB;  // [WM][H] db2, then [WM][A_][H] dW3 (over the dead W2 chunk buffers)
  if (l < 32) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = (wn * NT + nt) * 32 + l;
      sRed[wm * H + n] = csum[nt];
#pragma unroll
      for (int a = 0; a < A_; ++a) sRed[WM * H + (wm * A_ + a) * H + n] = cw3[nt][a];
    }
  }
  // db3 and loss stats: rows live in threads < BMr (waves 0, 1)
  if (w < 2) {
    float v[A_ + 4];
#pragma unroll
    for (int a = 0; a < A_; ++a) v[a] = (tid < BMr) ? sDl[tid * A_ + a] : 0.f;
    v[A_] = st_pl; v[A_ + 1] = st_vf; v[A_ + 2] = st_kl; v[A_ + 3] = st_ent;
#pragma unroll
    for (int c = 0; c < A_ + 4; ++c) {
      const float s = wave_sum(v[c]);
      if (l == 0) sStat[w * (A_ + 4) + c] = s;
    }
    if (NET == 1) {
      const double sx = wave_sum(vex);
      if (l == 0) sVx[w] = sx;
    }
  }
  __syncthreads();
  const int tile = blockIdx.x;
  for (int n = tid; n < H; n += NTHR) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < WM; ++j) s += sRed[j * H + n];
    g.part_b2[(size_t)tile * H + n] = s;
#pragma unroll
    for (int a = 0; a < A_; ++a) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < WM; ++j) t += sRed[WM * H + (j * A_ + a) * H + n];
      g.part_w3[((size_t)tile * A_ + a) * H + n] = t;
    }
  }
  if (tid < A_ + 4) {
    const float s = sStat[tid] + sStat[A_ + 4 + tid];
    if (tid >= A_) g.part_stat[(size_t)tile * 4 + tid - A_] = s;
    else if (NET == 0) g.part_b3[(size_t)tile * A_ + tid] = s;
    else vf_b3_part(sVx[0] + sVx[1], g.co.vf_loss_coeff, g.dyn[RLKS_DYN_INV_COUNT], g.part_b3 + (size_t)tile * 2);
  }
}

template <int WM, int WN>
static size_t fwd_lds_bytes(int A_, int D, int table_doubles) {
  constexpr int BMr = 32 * WM;
  const size_t f = (size_t)2 * HID * (BK + 1) + 2 * BK * BMr + WN * BMr * A_ + BMr * A_ + 2 * (A_ + 4) + HID +
                   (size_t)BMr * (D + 1) + (((size_t)HID * (D + 1) + 1) & ~(size_t)1);
  return f * sizeof(float) + (size_t)table_doubles * sizeof(double);
}

template <int A_, int NET, int WM, int WN, int MODE, int DD>
static int launch_cfg(const FwdArgs& a, hipStream_t s) {
  constexpr int BMr = 32 * WM;
  const size_t lds = fwd_lds_bytes<WM, WN>(A_, DD, MODE == FWD_ROLLOUT ? 2 * a.env.T * a.env.C : 0);
  hipLaunchKernelGGL((k_fwd_head<A_, NET, WM, WN, MODE, DD>), dim3(cdiv(a.M, BMr)), dim3(64 * WM * WN), lds, s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

template <int A_, int NET, int DD>
static int launch_net(const FwdArgs& a, int mode, hipStream_t s) {
  if (mode == FWD_TRAIN) return launch_cfg<A_, NET, 4, 2, FWD_TRAIN, DD>(a, s);
  // small batches (rollouts of a few thousand lanes) use 32-row tiles with the 4 waves split
  // over columns so that more CUs get work; large batches use 128-row tiles
  const bool small = a.M <= 32 * 1024;
  if (mode == FWD_ROLLOUT) {
    if constexpr (NET == 0) {
      return small ? launch_cfg<A_, 0, 1, 4, FWD_ROLLOUT, DD>(a, s) : launch_cfg<A_, 0, 4, 2, FWD_ROLLOUT, DD>(a, s);
    }
    return fail(RLKS_ERR_ARG, "rollout mode drives the policy net");
  }
  return small ? launch_cfg<A_, NET, 1, 4, FWD_ONLY, DD>(a, s) : launch_cfg<A_, NET, 4, 2, FWD_ONLY, DD>(a, s);
}

// obs_dim = 3 x clusters (cost, latency, utilisation per cluster): C = 2, 4, 8 -> D = 6, 12, 24
int launch_fwd_head(const FwdArgs& a, int net, int A, int mode, hipStream_t s) {
  if (a.D != 3 * A) return fail(RLKS_ERR_UNSUPPORTED, "fused MLP kernels expect obs_dim = 3 x n_actions");
  switch (A) {
    case 2: return net ? launch_net<1, 1, 6>(a, mode, s) : launch_net<2, 0, 6>(a, mode, s);
    case 4: return net ? launch_net<1, 1, 12>(a, mode, s) : launch_net<4, 0, 12>(a, mode, s);
    case 8: return net ? launch_net<1, 1, 24>(a, mode, s) : launch_net<8, 0, 24>(a, mode, s);
    default: return fail(RLKS_ERR_UNSUPPORTED, "fused policy head is built for 2, 4 or 8 actions");
  }
}

}  // namespace rlks
