// rollout_sf16.hip — one rollout step of the c2 hot path on split-fp16 MFMA: both nets' forward
// (pi logits and vf values of the step's observations), TorchCategorical sampling (Philox) and the
// env step, in one launch per step.  With the values computed here, the rollout needs no separate
// value pass (only V(obs[T]) for the bootstrap, FWD_ONLY mode).
//
// Reference: the env step is K8sMultiCloudEnv.step (k8s_multi_cloud_env.py:115-144) via
// env_device.h:step_lane; the policy is RLlib's FCNet [256, 256] tanh with a separate value net
// (train_ppo.py:12), action sampling = compute_single_action(explore=True) (eval_ppo.py:27),
// argmax for explore=False (final_evaluation.py:48).
//
// Workgroup = 32 rows (envs) x 8 waves: waves 0-3 run the policy net, 4-7 the value net; wave q of a
// net owns hidden units [64q, 64q + 64) of layer 2.
//   phase 1: wave q computes H1^T k-tiles 2q, 2q+1 of its net (Z1^T = W1a Xa^T, tanh) and parks
//            them in LDS as split B fragments (lane-contiguous 16-byte slots, conflict-free);
//   phase 2: Z2^T = W2 H1^T for its two n-tiles (A fragments straight from L2-resident w2p);
//   phase 3: H2^T = tanh(.), head partial sums over its 64 units (in registers + one xor-32 shuffle)
//            -> LDS; wave 0 / wave 4 finish logits / values for the 32 rows, wave 0 samples and
//            steps the env lanes.
// The latency of one step is what matters at c2 (4,096 lanes = 128 workgroups); the split products
// are fp32-accurate as in sgd_sf16.hip.
#include "sgd_sf16.h"

namespace rlks {

using h8 = __attribute__((ext_vector_type(8))) _Float16;

namespace {

__device__ __forceinline__ f32x16 mma(h8 a, h8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void split1(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}
__device__ __forceinline__ int sf_exp(float mx) {
  if (!(mx > 0.f) || !(mx <= 3.4e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  return min(max(15 - e, -120), 120);
}
__device__ __forceinline__ float tanh_abs(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.885390081777927f);
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

}  // namespace

#ifdef RLKS_STAMPS
// diagnostic build only (tools/stamps.py --roll): [workgroup][wave 0 / wave 4][phase] clocks of step 0
__device__ unsigned long long g_roll_stamps[256][2][8];
#define RL_STAMP(i) \
  if (t == 0 && (w == 0 || w == 4) && l == 0 && blockIdx.x < 256 && MODE == FWD_ROLLOUT) \
  g_roll_stamps[blockIdx.x][w >> 2][i] = __builtin_amdgcn_s_memtime()
#else
#define RL_STAMP(i)
#endif

// FWD_ROLLOUT: the whole rollout in one launch.  A workgroup's 32 env lanes depend on nothing
// outside the workgroup, so it loops over the T steps itself: weights, tables and W1a fragments are
// staged once, each step's observations stay in LDS for the next step (and go to HBM for the
// update), and step T is the bootstrap value pass.  FWD_ONLY: one forward of M rows.
template <int A_, int KD, int MODE>
__global__ __launch_bounds__(512) void k_sf_roll(SfRollArgs g) {
  constexpr int KS = KD / 16;
  constexpr float H1S = 16384.f;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  h8* sH = reinterpret_cast<h8*>(lds);                       // [2 net][8 kt][2 s][2 hi/lo][64]
  float* sPart = reinterpret_cast<float*>(sH + 2 * 8 * 2 * 2 * 64);  // [2 net][4 q][A_][32]
  float* sBW = sPart + 2 * 4 * A_ * 32;                               // [2 net][b2 | w3 (A_ rows)][HID]
  float* sObs = sBW + 2 * (1 + A_) * HID;                             // [32][KD] this step's observations
  double* sTab = reinterpret_cast<double*>(sObs + 32 * KD);           // rollout: [2][T][C]

  // wave index made scalar (readfirstlane) so that weight addresses are SGPR bases + one lane offset
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), r = l & 31, h = l >> 5;
  const int net = w >> 2, q = w & 3;
  const int D = g.D, M = g.M;
  const int row0 = blockIdx.x * 32;
  const int m = row0 + r;
  const bool valid = m < M;
  const SfRollNet& N = g.n[net];
  const int steps = MODE == FWD_ROLLOUT ? g.T : 0;

  // ---- once: b2 / W3 of both nets and the tables in LDS; this wave's W1a fragments in registers
  for (int e = tid; e < 2 * (1 + A_) * HID; e += 512) {
    const int nn = e / ((1 + A_) * HID), rem = e - nn * (1 + A_) * HID;
    const SfRollNet& Q = g.n[nn];
    const int An_ = nn == 0 ? A_ : 1;
    sBW[e] = rem < HID ? Q.b2[rem] : (rem - HID < An_ * HID ? Q.w3[rem - HID] : 0.f);
  }
  if (MODE == FWD_ROLLOUT)
    for (int e = tid; e < g.env.T * g.env.C; e += 512) {
      sTab[e] = g.tab_cost[e];
      sTab[g.env.T * g.env.C + e] = g.tab_lat[e];
    }
  for (int e = tid; e < 32 * KD; e += 512) {  // observations of step 0: Xa = [X | 1 | 0]
    const int rr = e / KD, d = e - rr * KD;
    sObs[e] = (row0 + rr < M && d < D) ? g.x[(size_t)(row0 + rr) * D + d] : (d == D ? 1.f : 0.f);
  }
  h8 w1f[2][KS][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 32 * (2 * q + i) + r;
      w1f[i][ks][0] = *reinterpret_cast<const h8*>(N.w1h + k * KD + 16 * ks + 8 * h);
      w1f[i][ks][1] = *reinterpret_cast<const h8*>(N.w1l + k * KD + 16 * ks + 8 * h);
    }
  const float inv_w1 = N.sc[1], inv_z2 = N.sc[3] / H1S;
  __syncthreads();

  h8 fa[8][2][2][2];  // [kt][s][i][hi/lo]: this wave's W2 fragments (w2r: 1-KB coalesced loads)
  const _Float16* w2rh = N.w2rh + (size_t)q * 8 * 2 * 2 * 64 * 8;
  const _Float16* w2rl = N.w2rl + (size_t)q * 8 * 2 * 2 * 64 * 8;
  auto load_a = [&](int kt) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = (((kt * 2 + s) * 2 + i) * 64 + l) * 8;
        fa[kt][s][i][0] = *reinterpret_cast<const h8*>(w2rh + o);
        fa[kt][s][i][1] = *reinterpret_cast<const h8*>(w2rl + o);
      }
  };

  for (int t = 0; t <= steps; ++t) {
    RL_STAMP(0);
    // Xa fragments (lane row m = r, d = 16 ks + 8 h + j) with a per-tile power-of-two scale
    float xv[KS * 8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[ks * 8 + j] = sObs[r * KD + 16 * ks + 8 * h + j];
    float xm = 0.f;
#pragma unroll
    for (int i = 0; i < KS * 8; ++i) xm = fmaxf(xm, fabsf(xv[i]));
    const float sx = ldexpf(1.f, sf_exp(wave_max(xm)));
    h8 xh[KS], xl[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        _Float16 a, b;
        split1(xv[ks * 8 + j] * sx, a, b);
        xh[ks][j] = a;
        xl[ks][j] = b;
      }
    const float inv_z1 = inv_w1 / sx;
    RL_STAMP(1);

    // ---- phase 1: H1^T k-tiles 2q, 2q+1 of this net -> LDS as split B fragments
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kt = 2 * q + i;
      f32x16 z;
#pragma unroll
      for (int e = 0; e < 16; ++e) z[e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        z = mma(w1f[i][ks][1], xh[ks], z);
        z = mma(w1f[i][ks][0], xl[ks], z);
        z = mma(w1f[i][ks][0], xh[ks], z);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        h8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          _Float16 a, b;
          split1(tanh_abs(z[8 * s + j] * inv_z1) * H1S, a, b);
          bh[j] = a;
          bl[j] = b;
        }
        sH[(((net * 8 + kt) * 2 + s) * 2 + 0) * 64 + l] = bh;
        sH[(((net * 8 + kt) * 2 + s) * 2 + 1) * 64 + l] = bl;
      }
    }
    __syncthreads();
    RL_STAMP(2);
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) load_a(kt);  // two k-tiles ahead

    // ---- phase 2: Z2^T rows n = 32 (2q + i) + ., B fragments from LDS
    f32x16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const h8 bh = sH[(((net * 8 + kt) * 2 + s) * 2 + 0) * 64 + l];
        const h8 bl = sH[(((net * 8 + kt) * 2 + s) * 2 + 1) * 64 + l];
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i] = mma(fa[kt][s][i][1], bh, acc[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i] = mma(fa[kt][s][i][0], bl, acc[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i] = mma(fa[kt][s][i][0], bh, acc[i]);
      }
      if (kt < 6) load_a(kt + 2);
    }
    RL_STAMP(3);

    // ---- phase 3: H2^T = tanh(Z2^T + b2); head partials over this wave's 64 units
    const int An = net == 0 ? A_ : 1;
    const float* bw = sBW + net * (1 + A_) * HID;
    float out[A_];
#pragma unroll
    for (int a = 0; a < A_; ++a) out[a] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = 32 * (2 * q + i) + acc_row(e, l);
        const float h2 = tanh_abs(fmaf(acc[i][e], inv_z2, bw[n]));
#pragma unroll
        for (int a = 0; a < A_; ++a)
          if (a < An) out[a] = fmaf(h2, bw[HID + a * HID + n], out[a]);
      }
#pragma unroll
    for (int a = 0; a < A_; ++a) {
      out[a] += __shfl_xor(out[a], 32, 64);
      if (h == 0 && a < An) sPart[((net * 4 + q) * A_ + a) * 32 + r] = out[a];
    }
    __syncthreads();
    RL_STAMP(4);

    const size_t tN = (size_t)t * M;
    if (w == 4 && h == 0 && valid && g.values) {  // V(obs[t]) of the 32 rows
      const float v = N.b3[0] + ((sPart[((4 + 0) * A_) * 32 + r] + sPart[((4 + 1) * A_) * 32 + r]) +
                                 (sPart[((4 + 2) * A_) * 32 + r] + sPart[((4 + 3) * A_) * 32 + r]));
      g.values[tN + m] = v;
    }
    if (w == 0 && h == 0 && valid && (MODE == FWD_ONLY || t < steps)) {
      float lg[A_];
#pragma unroll
      for (int a = 0; a < A_; ++a)
        lg[a] = g.n[0].b3[a] + ((sPart[(0 * A_ + a) * 32 + r] + sPart[(1 * A_ + a) * 32 + r]) +
                                (sPart[(2 * A_ + a) * 32 + r] + sPart[(3 * A_ + a) * 32 + r]));
      if (g.logits)
#pragma unroll
        for (int a = 0; a < A_; ++a) g.logits[(tN + m) * A_ + a] = lg[a];
      if (MODE == FWD_ROLLOUT) {
        // TorchCategorical: sample (Philox, counter = lane / episode / step) or argmax (explore = 0)
        float mx = lg[0];
        int amax = 0;
#pragma unroll
        for (int a = 1; a < A_; ++a)
          if (lg[a] > mx) { mx = lg[a]; amax = a; }
        float ex[A_], se = 0.f;
#pragma unroll
        for (int a = 0; a < A_; ++a) { ex[a] = expf(lg[a] - mx); se += ex[a]; }
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
            c += ex[a];
            if (!found && u < c) { act = a; found = true; }
          }
        }
        float la = lg[0];
#pragma unroll
        for (int a = 0; a < A_; ++a) la = (a == act) ? lg[a] : la;
        g.actions[tN + m] = act;
        g.logp[tN + m] = la - mx - logf(se);
        // next observation straight into this lane's LDS row, then to obs[t + 1] in HBM
        float* o = sObs + r * KD;
        const StepOut so = step_lane(v, sTab, m, act, o, nullptr);
        float* og = g.x + ((size_t)(t + 1) * M + m) * D;
        for (int d = 0; d < D; ++d) og[d] = o[d];
        g.rewards[tN + m] = (float)so.reward;
        g.dones[tN + m] = (uint8_t)so.done;
      }
    }
    RL_STAMP(5);
    __syncthreads();  // sObs of step t + 1 complete; sH / sPart free
  }
}

#ifdef RLKS_STAMPS
extern "C" int rlks_dbg_roll_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_roll_stamps), sizeof(g_roll_stamps)) == hipSuccess ? 0 : 1;
}
#endif

template <int A_, int KD>
static int launch_roll_a(const SfRollArgs& a, int mode, hipStream_t s) {
  const size_t lds = (size_t)2 * 8 * 2 * 2 * 64 * 16 + (size_t)2 * 4 * A_ * 32 * sizeof(float) +
                     (size_t)2 * (1 + A_) * HID * sizeof(float) + (size_t)32 * KD * sizeof(float) +
                     (mode == FWD_ROLLOUT ? (size_t)2 * a.env.T * a.env.C * sizeof(double) : 0);
  const dim3 grid(cdiv(a.M, 32));
  if (mode == FWD_ROLLOUT) hipLaunchKernelGGL((k_sf_roll<A_, KD, FWD_ROLLOUT>), grid, dim3(512), lds, s, a);
  else hipLaunchKernelGGL((k_sf_roll<A_, KD, FWD_ONLY>), grid, dim3(512), lds, s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int launch_sf_roll(const SfRollArgs& a, int mode, hipStream_t s) {
  RLKS_REQUIRE(a.D == 3 * a.A, RLKS_ERR_UNSUPPORTED, "split-fp16 rollout expects obs_dim = 3 x n_actions");
  switch (a.A) {
    case 2: return launch_roll_a<2, 16>(a, mode, s);
    case 4: return launch_roll_a<4, 16>(a, mode, s);
    case 8: return launch_roll_a<8, 32>(a, mode, s);
    default: return fail(RLKS_ERR_UNSUPPORTED, "split-fp16 rollout is built for 2, 4 or 8 actions");
  }
}

}  // namespace rlks
