// sgd_sf16.hip — the PPO SGD step (K4) on split-fp16 MFMA: fp32-accurate products at 16x the
// fp32 matrix rate.
//
// Every GEMM operand x is carried as a pair of fp16 values (hi, lo) of x * 2^e, with 2^e a power
// of two chosen from max|x| so that the scaled values sit in [2^14, 2^15): hi = fp16(x 2^e),
// lo = fp16(x 2^e - hi), |x 2^e - hi - lo| <= 2^-22 |x 2^e|.  A product a.b is accumulated by three
// v_mfma_f32_32x32x16_f16 (lo.hi + hi.lo + hi.hi, fp32 accumulate); the dropped lo.lo term is
// <= 2^-22 |a b|.  Measured on MI355X (tools/micro/sf16_layout.hip, K = 256): 1.9e-7 relative
// error vs fp64, against 2.8e-7 for an fp32 fmaf chain.  Three f16 MFMAs cost 96 cycles per
// 32x32x16 block, where the same work on v_mfma_f32_32x32x2_f32 takes 512.
//
// Orientation.  An MFMA accumulator tile X (columns on lanes, rows in registers) is the next
// MFMA's B operand without data movement when the next product sums over X's rows (Y = A X), or
// its A operand (Z = X^T B); the other operand is then read in X's row order perm(s, h, j)
// (cdna_hip_programming.md §3).  Weights are pre-split by k_sf_prep into those orders, so:
//   F1 (k_sf_fwdbwd, one wave per 32-row tile, hidden units in registers, rows on lanes)
//     Z1^T = W1a Xa^T          Xa = [X | 1]: b1 folded into W1a's column D
//     Z2^T = W2 H1^T           B = H1^T straight from the tanh'd accumulator
//     H2^T, head (in-register sums over hidden units), PPO loss -> dlogits, dZ2^T
//     dW3 (half-wave reduce), db3, stats; dZ2^T -> HBM for F2; per-tile max|dZ2| -> atomicMax
//     dH1 = dZ2 W2             A = dZ2^T accumulator (transposes to rows-in-registers)
//     Z1 = Xa W1a^T, dZ1 = dH1 (1 - H1^2)
//     dW1a^T = Xa^T dZ1        B = dZ1 accumulator; row D of dW1a is db1
//   F2 (k_sf_dw2): dW2 = dZ2^T H1 over the rows, H1 recomputed (rows in registers) as the B
//     operand, dZ2^T tiles staged through registers into LDS pre-split with the global max|dZ2|
//     scale; db2 from the same loads.  Row splits write fp32 partials, summed in a fixed order by k_reduce.
//
// Reference semantics: RLlib FCNet [256, 256] tanh, vf_share_layers=False, PPO loss as in
// mlp_fwd.hip (train_ppo.py:9-31; RLlib third-party).
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "sgd_sf16.h"

namespace rlks {


using h8 = __attribute__((ext_vector_type(8))) _Float16;
using h4 = __attribute__((ext_vector_type(4))) _Float16;
using v4u = __attribute__((ext_vector_type(4))) unsigned;  // 16-byte staging register (a vector, not HIP's uint4 struct, so it stays in VGPRs)

constexpr int SF_ROWS = 256;        // minibatch rows must be a multiple of this
constexpr float SF_H1_SCALE = 16384.f;  // tanh outputs (|h| < 1) scaled by 2^14

__device__ __forceinline__ int sf_perm(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }
// P16: element p = 8g + j of a 16x16x32 k-fragment taken from two stacked accumulator tiles
__device__ __forceinline__ int p16(int p) { return 16 * ((p >> 2) & 1) + 4 * (p >> 3) + (p & 3); }

__device__ __forceinline__ f32x16 mma(h8 a, h8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// (ah + al)(bh + bl) - al bl, small terms first
__device__ __forceinline__ f32x16 mma3(h8 ah, h8 al, h8 bh, h8 bl, f32x16 c) {
  c = mma(al, bh, c);
  c = mma(ah, bl, c);
  return mma(ah, bh, c);
}
template <int P>
__device__ __forceinline__ f32x16 mmaP(h8 ah, h8 al, h8 bh, h8 bl, f32x16 c) {
  if constexpr (P == 1) return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  else return mma3(ah, al, bh, bl, c);
}

__device__ __forceinline__ void split1(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}
// the same for a pair, packed: hi = f16(x) by v_cvt_pk_f16_f32 (round to nearest even), lo = f16(x -
// hi) by v_fma_mix{lo,hi}_f16, which forms x - hi exactly and rounds once: the same bits as split1's
// cvt / cvt back / sub / cvt, in 3 instructions a pair instead of ~6 (tools/micro/mix_split.hip
// compares the two on 4M random pairs on the GPU: identical)
typedef _Float16 hf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(float x0, float x1, unsigned& hi, unsigned& lo) {
  const hf2 h = {(_Float16)x0, (_Float16)x1};
  hi = __builtin_bit_cast(unsigned, h);
  unsigned l;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(x0), "v"(hi), "v"(x1));
  lo = l;
}
// 8 values -> (hi, lo) fragments
__device__ __forceinline__ void split8v(const float (&x)[8], h8& hi, h8& lo) {
  v4u h, l;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned a, b;
    split2(x[2 * q], x[2 * q + 1], a, b);
    h[q] = a;
    l[q] = b;
  }
  hi = __builtin_bit_cast(h8, h);
  lo = __builtin_bit_cast(h8, l);
}
// elements [o, o + 8) of v, times s
template <int N>
__device__ __forceinline__ void split8(const float (&v)[N], int o, float s, h8& hi, h8& lo) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = v[o + j] * s;
  split8v(x, hi, lo);
}
__device__ __forceinline__ void split16(const f32x16& v, int o, float s, h8& hi, h8& lo) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = v[o + j] * s;
  split8v(x, hi, lo);
}

// exponent e with mx 2^e in [2^14, 2^15); 0 for mx = 0 / non-finite
__device__ __forceinline__ int sf_exp(float mx) {
  if (!(mx > 0.f) || !(mx <= 3.4e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  return min(max(15 - e, -120), 120);
}
__device__ __forceinline__ float pow2(int e) { return ldexpf(1.f, e); }

// 1 - 2 / (exp(2x) + 1): 5 VALU ops (2 transcendental); absolute error ~1e-7, which is what the
// split products see (|h| < 1 carried at a fixed 2^14 scale)
constexpr float SF_2LOG2E = 2.885390081777927f;  // 2 log2(e): exp(2x) = exp2(x SF_2LOG2E)
__device__ __forceinline__ float tanh_abs(float x) {
  const float e = __builtin_amdgcn_exp2f(x * SF_2LOG2E);
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}
// r = 1 / (exp(2x) + 1) given kx = x SF_2LOG2E (callers fold SF_2LOG2E into the scale they already
// multiply by): tanh x = 1 - 2 r, 1 - tanh^2 x = 4 r (1 - r).  4 VALU ops instead of 6 with the
// separate scale multiply.
__device__ __forceinline__ float tanh_r(float kx) { return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(kx) + 1.f); }

// interleave the scheduling region: NM x (1 MFMA, NV VALU) (cdna_hip_programming.md T19); an
// MFMA leaves 24 of its 32 issue cycles for independent vector work of the same wave
template <int NM, int NV>
__device__ __forceinline__ void sched_interleave() {
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
  }
}

// Xa = [X | 1 | 0] element d of a row: a load from a clamped column and an arithmetic select (X is
// finite), so the load is unconditional and a row's loads issue back to back instead of as one
// exec-masked load -> wait per element
__device__ __forceinline__ float xa_elem(const float* __restrict__ xr, int d, int D) {
  const float v = xr[d < D ? d : D - 1];
  return fmaf(v, d < D ? 1.f : 0.f, d == D ? 1.f : 0.f);
}

// elements [base, base + 8) of Xa = [X | 1 | 0] for a record row xr of S floats (S a multiple of 4,
// S >= D + 4, 16-byte aligned rows): two 16-byte loads and arithmetic selects.  A block that starts
// past S - 8 lies entirely beyond the obs (base >= D + 1 for the record shapes used) and loads
// the row's last 8 floats in its place so that no load leaves the row.
__device__ __forceinline__ void xa_row8(const float* __restrict__ xr, int base, int D, int S, float (&o)[8]) {
  using v4f = __attribute__((ext_vector_type(4))) float;
  const int pb = base < S - 8 ? base : S - 8;
  const v4f a = *reinterpret_cast<const v4f*>(xr + pb), b = *reinterpret_cast<const v4f*>(xr + pb + 4);
  const float t[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int d = base + j;
    o[j] = fmaf(t[j], (d < D && pb == base) ? 1.f : 0.f, d == D ? 1.f : 0.f);
  }
}


// ----------------------------------------------------------------------------- weight prep
// W1a = [W1 | b1] -> w1h/w1l [HID][KD]; W2 -> w2p (A operand of Z2^T = W2 H1^T: row n, k in perm
// order per 32-block) and w2t (B operand of dH1 = dZ2 W2: row k, n in perm order per 32-block),
// each with its own power-of-two scale from max |w|.
// pass 1: per-block max |w| (16 blocks over W2, 16 over W1a) -> pmax[net][32]
__global__ __launch_bounds__(256) void k_sf_wmax(SfPrepArgs g) {
  __shared__ float red[256];
  const SfNetW& N = g.n[blockIdx.x];
  const int b = blockIdx.y, tid = threadIdx.x, D = g.D;
  float mx = 0.f;
  if (b < 16) {
    for (int e = b * 4096 + tid; e < (b + 1) * 4096; e += 256) mx = fmaxf(mx, fabsf(N.w2[e]));
  } else {
    const int n = HID * (D + 1), per = (n + 15) / 16, e0 = (b - 16) * per, e1 = min(n, e0 + per);
    for (int e = e0 + tid; e < e1; e += 256) {
      const int k = e / (D + 1), d = e - k * (D + 1);
      mx = fmaxf(mx, fabsf(d < D ? N.w1[k * D + d] : N.b1[k]));
    }
  }
  red[tid] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
    __syncthreads();
  }
  if (tid == 0) N.pmax[(g.parity * 2 + (b < 16 ? 0 : 1)) * SF_PMAX + (b & 15)] = red[0];
}

// pass 2: grid (2 nets, 64 blocks) x 256 threads, 4 elements of W2 (both orders) per thread and
// the W1a split in the first blocks
__global__ __launch_bounds__(256) void k_sf_split(SfPrepArgs g) {
  const SfNetW& N = g.n[blockIdx.x];
  const int D = g.D, KD = g.KD, tid = threadIdx.x;
  // the weights this thread splits, loaded before the scale is known: their latency overlaps the
  // maxima's
  const int base = blockIdx.y * 1024;
  float vp[4], vt[4], vr[4], v1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = base + j * 256 + tid;
    const int row = i >> 8, c = i & 255, blk = c >> 5, rem = c & 31;
    const int src = 32 * blk + p16(rem);  // F1's P16 fragment order (k_sf_fwd / k_sf_bwd)
    vp[j] = N.w2[row * HID + src];  // w2p[n = row][k perm]
    vt[j] = N.w2[src * HID + row];  // w2t[k = row][n perm]
    vr[j] = 0.f;
    if (g.write_roll) {  // rollout copy: i = ((((q 8 + kt) 2 + s) 2 + ii) 64 + lane) 8 + jj -> w2p[n][32kt+16s+8h+jj]
      const int jj = i & 7, lane = (i >> 3) & 63, ii = (i >> 9) & 1, ss = (i >> 10) & 1, kt = (i >> 11) & 7,
                q = i >> 14;
      const int n = 32 * (2 * q + ii) + (lane & 31);
      vr[j] = N.w2[n * HID + 32 * kt + sf_perm(ss, lane >> 5, jj)];
    }
    v1[j] = 0.f;
    if (i < HID * KD) {
      const int k = i / KD, d = i - k * KD;
      v1[j] = d < D ? N.w1[k * D + d] : (d == D ? N.b1[k] : 0.f);
    }
  }
  float m2 = 0.f, m1 = 0.f;
  if (g.skip_wmax && N.tag[g.parity] != g.expect_tag) {  // stale slots: this block scans the weights
    __shared__ float red[2][256];
    for (int e = tid; e < HID * HID; e += 256) m2 = fmaxf(m2, fabsf(N.w2[e]));
    for (int e = tid; e < HID * (D + 1); e += 256) {
      const int k = e / (D + 1), d = e - k * (D + 1);
      m1 = fmaxf(m1, fabsf(d < D ? N.w1[k * D + d] : N.b1[k]));
    }
    red[0][tid] = m2;
    red[1][tid] = m1;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (tid < o) {
        red[0][tid] = fmaxf(red[0][tid], red[0][tid + o]);
        red[1][tid] = fmaxf(red[1][tid], red[1][tid + o]);
      }
      __syncthreads();
    }
    m2 = red[0][0];
    m1 = red[1][0];
  } else if (!g.skip_wmax) {  // k_sf_wmax's 16 block maxima per kind
    const float* pm = N.pmax + g.parity * 2 * SF_PMAX;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      m2 = fmaxf(m2, pm[i]);
      m1 = fmaxf(m1, pm[SF_PMAX + i]);
    }
  } else {  // the fused reduce's per-block maxima (unused entries are zero): every wave reduces all
            // of them itself (no barrier, so the weight loads above stay in flight)
    const float4* pm = reinterpret_cast<const float4*>(N.pmax + g.parity * 2 * SF_PMAX);
    const int l = tid & 63;
#pragma unroll
    for (int q = 0; q < SF_PMAX / 256; ++q) {
      const float4 a = pm[q * 64 + l], c = pm[SF_PMAX / 4 + q * 64 + l];
      m2 = fmaxf(m2, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
      m1 = fmaxf(m1, fmaxf(fmaxf(c.x, c.y), fmaxf(c.z, c.w)));
    }
    m2 = wave_max(m2);
    m1 = wave_max(m1);
  }
  const int e1 = sf_exp(m1), e2 = sf_exp(m2);
  const float s1 = pow2(e1), s2 = pow2(e2);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = base + j * 256 + tid;
    _Float16 a, b;
    split1(vp[j] * s2, a, b);
    N.w2ph[i] = a;
    N.w2pl[i] = b;
    split1(vt[j] * s2, a, b);
    N.w2th[i] = a;
    N.w2tl[i] = b;
    if (g.write_roll) {
      split1(vr[j] * s2, a, b);
      N.w2rh[i] = a;
      N.w2rl[i] = b;
    }
    if (i < HID * KD) {
      split1(v1[j] * s1, a, b);
      N.w1h[i] = a;
      N.w1l[i] = b;
    }
  }
  if (blockIdx.y == 0 && tid == 0) {
    N.sc[0] = s1; N.sc[1] = 1.f / s1; N.sc[4] = (float)e1;
    N.sc[2] = s2; N.sc[3] = 1.f / s2; N.sc[5] = (float)e2;
  }
  // the other parity's entries: the coming fused reduce writes some of them.  The rollout's prep
  // (write_roll) has slots of its own and leaves the SGD steps' parity state (entries and tags) alone.
  if (blockIdx.y == 0 && !g.write_roll) {
    float4* z = reinterpret_cast<float4*>(N.pmax + (g.parity ^ 1) * 2 * SF_PMAX);
    for (int i = tid; i < 2 * SF_PMAX / 4; i += 256) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid == 0) N.tag[g.parity ^ 1] = 0u;
  }
}

// the record fields the PPO loss of one row reads: pi: old logits, advantage, old log-prob, action;
// vf: the value target (record layout [obs D | logits_old A_pi | adv | vtarg | logp_old | action])
template <int A_>
struct RecTail {
  float lo[A_];
  float adv, vt, lpo, act;
};
template <int A_, int NET>
__device__ __forceinline__ void load_tail(const SfArgs& g, int row, RecTail<A_>& r) {
  const float* rec = g.x + (size_t)row * g.x_stride + g.D;
  const int Ap = g.A_pi;
  if (NET == 0) {
#pragma unroll
    for (int a = 0; a < A_; ++a) r.lo[a] = rec[a];
    r.adv = rec[Ap];
    r.lpo = rec[Ap + 2];
    r.act = rec[Ap + 3];
    r.vt = 0.f;
  } else {
#pragma unroll
    for (int a = 0; a < A_; ++a) r.lo[a] = 0.f;
    r.adv = r.lpo = r.act = 0.f;
    r.vt = rec[Ap + 1];
  }
}

// the device-resident loss scalars of the step (advantage moments, KL coefficient, 1 / rows): read
// once per kernel, not at every loss evaluation
struct LossDyn {
  float inv_count, adv_mean, adv_invstd, klc;
};
__device__ __forceinline__ LossDyn load_dyn(const SfArgs& g) {
  return {g.dyn[RLKS_DYN_INV_COUNT], g.dyn[RLKS_DYN_ADV_MEAN], g.dyn[RLKS_DYN_ADV_INVSTD], g.dyn[RLKS_DYN_KL_COEFF]};
}

// PPO loss of one row (RLlib ppo_torch_policy semantics): d loss / d logits (pi) or
// d loss / d value (vf), scaled by 1 / global rows, and the row's [policy loss, vf loss, kl,
// entropy] terms
template <int A_, int NET>
__device__ __forceinline__ void sf_loss_t(const SfArgs& g, const LossDyn& dy, const float (&out)[A_],
                                          const RecTail<A_>& r, float (&dl)[A_], float (&st)[4], double& vex) {
  const float inv_count = dy.inv_count;
  st[0] = st[1] = st[2] = st[3] = 0.f;
  vex = 0.0;
  if (NET == 0) {
    const float* lo = r.lo;
    const float adv = (r.adv - dy.adv_mean) * dy.adv_invstd;
    const float logp_old = r.lpo;
    const int act = (int)r.act;
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
    const float dr = -adv * (w1 + (1.f - w1) * inr) * ratio;
    const float klc = dy.klc;
#pragma unroll
    for (int a = 0; a < A_; ++a) {
      float d = dr * ((a == act ? 1.f : 0.f) - p[a]);
      d += klc * (p[a] - po[a]);
      d += g.co.entropy_coeff * p[a] * (lp[a] + ent);
      dl[a] = d * inv_count;
    }
    st[0] = -fminf(s1, s2);
    st[2] = kl;
    st[3] = ent;
  } else {
    const VfRow v = vf_row(out[0], r.vt, g.co.vf_clip_param, g.co.vf_loss_coeff, inv_count);
    st[1] = v.sq;
    dl[0] = v.dl;
    vex = v.ex;
  }
}
template <int A_, int NET>
__device__ __forceinline__ void sf_loss(const SfArgs& g, const float (&out)[A_], int row, float (&dl)[A_],
                                        float (&st)[4], double& vex) {
  RecTail<A_> r;
  load_tail<A_, NET>(g, row, r);
  sf_loss_t<A_, NET>(g, load_dyn(g), out, r, dl, st, vex);
}


#ifdef RLKS_STAMPS
// diagnostic build only (make -C csrc stamps, tools/stamps.py): F1a (k_sf_fwd) phase clocks of
// lane 0 of every wave, [net][tile][phase]; slot 7 = HW_ID | XCC_ID << 32
__device__ unsigned long long g_fa_stamps[2][8192][8];
#define FA_STAMP(i) \
  if (l == 0 && tile < 8192) g_fa_stamps[NET][tile][i] = __builtin_amdgcn_s_memtime()

#define FA_HWID()                                                                                   \
  if (l == 0 && tile < 8192)                                                                        \
  g_fa_stamps[NET][tile][7] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |       \
                              ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32)
#else
#define FA_STAMP(i)
#define FA_HWID()
#endif

// ----------------------------------------------------------------------------- F1 (16-row tiles)
// One wave per 16-row tile on v_mfma_f32_16x16x32_f16, eight waves per workgroup (128 rows), two
// workgroups per CU: the per-wave state is the 256 x 16 accumulator block (64 registers), so a
// kernel fits 128 registers and every SIMD interleaves four waves (the 32-row tiles of round 2
// needed 256 registers, two waves per SIMD, and waited on their own dependency chains).
//
// Fragments (lane l, c = l & 15, g = l >> 4): A[row c][k = 8g + j], B[k = 8g + j][col c] (j < 8),
// C[row 4g + i][col c] (i < 4).  A 32-row block held as two accumulator tiles gives a lane the rows
// 4g + i and 16 + 4g + i: as the next product's B (or A) operand, element j of its k-fragment is
// row P16(8g + j) = 16 (j >> 2) + 4g + (j & 3) of the block.  The prep writes W2 with each 32-block
// of columns in that order (k_sf_split), so
//   F1a (k_sf_fwd): Z1^T = W1a Xa^T (two tiles) -> tanh -> split = B of Z2^T = W2 H1^T (A = w2p:
//     rows n, columns k in P16 order); H2^T, head, PPO loss, dW3 / db3 / stats (workgroup sums),
//     dZ2^T = (dl W3)(1 - H2^2) -> HBM in the lane's own order, the tile's max |dZ2|;
//   F1b (k_sf_bwd): dH1 = dZ2 W2 (A = dZ2 read back by the same lane that wrote it, B = w2t: rows
//     k, columns n in P16 order); Z1 = Xa W1a^T in dH1's layout -> dZ1 = dH1 (1 - H1^2) ->
//     dW1a^T = Xa^T dZ1 on v_mfma_f32_16x16x16_f16 (B = the dZ1 tile as it stands: K = its rows m).
using f4 = __attribute__((ext_vector_type(4))) float;
using v4f = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f4 mm16(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mm16x3(h8 ah, h8 al, h8 bh, h8 bl, f4 c) {
  c = mm16(al, bh, c);
  c = mm16(ah, bl, c);
  return mm16(ah, bh, c);
}
__device__ __forceinline__ f4 mk16(h4 a, h4 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }
// P products per split-fp16 product: 3 (lo hi + hi lo + hi hi: fp32-accurate, the default) or 1 (hi hi:
// the fp16 throughput mode, RLKS_PRECISION_F16 -- fp16 operands, fp32 accumulation)
template <int P>
__device__ __forceinline__ f4 mmP(h8 ah, h8 al, h8 bh, h8 bl, f4 c) {
  if constexpr (P == 1) return mm16(ah, bh, c);
  else return mm16x3(ah, al, bh, bl, c);
}
__device__ __forceinline__ f4 mk16x3(h4 ah, h4 al, h4 bh, h4 bl, f4 c) {
  c = mk16(al, bh, c);
  c = mk16(ah, bl, c);
  return mk16(ah, bh, c);
}
__device__ __forceinline__ f4 f4zero() { return f4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// half-chunk image: 128 rows x 32 halves (64-byte rows), hi and lo; 16-byte piece q of row r at
// slot q ^ SW16(r), which makes the A / B fragment reads (ds_read_b128: rows 16j + c, piece g)
// conflict-free in each of the instruction's four 16-lane groups
constexpr int H16 = 4096;  // halves per [128][32] image
__device__ __forceinline__ int sw16(int r) { return 2 * ((r >> 2) & 1); }

// LDS-DMA of rows [r0, r0 + 128), columns [col, col + 32) of a [256][256] split weight: 2 x 512
// 16-byte slots (hi, lo) = 16 blocks of 64 lanes, wave w of W moves blocks (16 / W) w + i
template <int W>
__device__ __forceinline__ void hc_dma(const _Float16* hi, const _Float16* lo, int r0, int col, _Float16* buf, int w,
                                       int l) {
#pragma unroll
  for (int i = 0; i < 16 / W; ++i) {
    const int blk = (16 / W) * w + i, arr = blk >> 3, sig = (blk & 7) * 64 + l;
    const int r = sig >> 2, q = (sig & 3) ^ sw16(r);
    const _Float16* src = (arr ? lo : hi) + (r0 + r) * HID + col + 8 * q;
    _Float16* dst = buf + arr * H16 + (blk & 7) * 512;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}
// (hi, lo) fragment of image row 16 j + c, piece g
__device__ __forceinline__ void hc_frag(const _Float16* buf, int j, int c, int g, h8& fh, h8& fl) {
  const int off = (16 * j + c) * 32 + 8 * (g ^ sw16(c));
  fh = *reinterpret_cast<const h8*>(buf + off);
  fl = *reinterpret_cast<const h8*>(buf + H16 + off);
}

// W1a = [W1 | b1] (hi, lo) in LDS: [2][HID k][KD] halves; at KD = 32 the 16-byte pieces of a row
// are swizzled like the weight images (conflict-free); at KD = 16 the plain 32-byte rows already are
template <int KD>
__device__ __forceinline__ int w1_off(int k, int q) {
  return k * KD + 8 * (KD == 32 ? (q ^ sw16(k)) : q);
}
template <int KD, int NTHR>
__device__ __forceinline__ void w1_stage(const SfNet& N, _Float16* sW1, int tid) {
  for (int p = tid; p < 2 * HID * KD / 8; p += NTHR) {
    const int arr = p / (HID * KD / 8), e = p - arr * (HID * KD / 8), k = e / (KD / 8), q = e - k * (KD / 8);
    const v4u v = *reinterpret_cast<const v4u*>((arr ? N.w1l : N.w1h) + k * KD + 8 * q);
    *reinterpret_cast<v4u*>(sW1 + arr * HID * KD + w1_off<KD>(k, q)) = v;
  }
}
// the same copy as w1_stage through the LDS DMA (global_load_lds, 1 KB per wave instruction): no
// register round trip, so it is in flight beside the W2 chunk and the X rows (F1a's prologue)
template <int KD, int W>
__device__ __forceinline__ void w1_dma(const SfNet& N, _Float16* sW1, int w, int l) {
  constexpr int PER_PLANE = HID * KD / 8 / 64;  // wave instructions per plane
  static_assert((2 * PER_PLANE) % W == 0, "W1a planes split evenly over the waves");
#pragma unroll
  for (int i = 0; i < 2 * PER_PLANE / W; ++i) {
    const int blk = (2 * PER_PLANE / W) * w + i, arr = blk / PER_PLANE, j = blk - arr * PER_PLANE;
    const int pc = 64 * j + l, k = pc / (KD / 8), qs = pc - k * (KD / 8);
    const int q = KD == 32 ? (qs ^ sw16(k)) : qs;
    const _Float16* src = (arr ? N.w1l : N.w1h) + k * KD + 8 * q;
    _Float16* dst = sW1 + arr * HID * KD + j * 512;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}
// W1a fragment of rows k = 16 kt + c, columns d = 8g + j: lanes with 8g >= KD read a duplicate
// piece (finite; the Xa fragment is zero there)
template <int KD>
__device__ __forceinline__ void w1_frag(const _Float16* sW1, int kt, int c, int g, h8& fh, h8& fl) {
  const int off = w1_off<KD>(16 * kt + c, g & (KD / 8 - 1));
  fh = *reinterpret_cast<const h8*>(sW1 + off);
  fl = *reinterpret_cast<const h8*>(sW1 + HID * KD + off);
}

// sum over the four 16-lane rows of a wave (lanes c, c + 16, c + 32, c + 48): every lane gets the
// same bits
__device__ __forceinline__ float sum_rows4(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
// reduce-scatter of 16 per-lane values over the 16 lanes of a row: lane c of the row ends with the
// row total of v[c] (DPP row_ror:8, row_half_mirror, quad_perm xor 2, xor 1; 43 VALU)
__device__ __forceinline__ float row_reduce16(const float (&v)[16], int l) {
  float u[8], w[4], x[2];
  const bool b3 = (l >> 3) & 1, b2 = (l >> 2) & 1, b1 = (l >> 1) & 1, b0 = l & 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = (b3 ? v[i + 8] : v[i]) + dpp<0x128>(b3 ? v[i] : v[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (b2 ? u[i + 4] : u[i]) + dpp<0x141>(b2 ? u[i] : u[i + 4]);
#pragma unroll
  for (int i = 0; i < 2; ++i) x[i] = (b1 ? w[i + 2] : w[i]) + dpp<0x4E>(b1 ? w[i] : w[i + 2]);
  return (b0 ? x[1] : x[0]) + dpp<0xB1>(b0 ? x[0] : x[1]);
}
// sum over the 16 lanes of a row (every lane of the row gets it)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0x128>(v);
  v += dpp<0x141>(v);
  v += dpp<0x4E>(v);
  return v + dpp<0xB1>(v);
}

// Xa = [X | 1 | 0] fragment of a 16-row tile: lane (g, c) holds row row0 + c, columns 8g .. 8g + 7,
// scaled by the wave's power of two (returned: its exponent) times sgn (the tile's sign, below) and split
__device__ __forceinline__ int x_split(const float (&xv)[8], h8& xh, h8& xl, float sgn) {
  float xm = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) xm = fmaxf(xm, fabsf(xv[j]));
  const int ex = sf_exp(wave_max(xm));
  split8(xv, 0, sgn * pow2(ex), xh, xl);
  return ex;
}
__device__ __forceinline__ int x_frag(const SfArgs& a, int row0, int c, int g, h8& xh, h8& xl, float sgn = 1.f) {
  float xv[8];
  xa_row8(a.x + (size_t)(row0 + c) * a.x_stride, 8 * g, a.D, a.x_stride, xv);
  float xm = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) xm = fmaxf(xm, fabsf(xv[j]));
  const int ex = sf_exp(wave_max(xm));
  split8(xv, 0, sgn * pow2(ex), xh, xl);
  return ex;
}

// Rounding-bias cancellation.  The f16 MFMAs' fp32 accumulation is not sign-symmetric: averaged over
// many dot products its error leans negative (tools/micro/mfma_round.hip: mean signed error -1e-10 of
// sum |a b| over K = 256, ~2 % of the typical error).  A bias gradient sums such errors over all the
// rows of a minibatch coherently (65,536 of them at c4), where fp32's rounding errors average out:
// db1 came out ~7x less accurate than an fp32 evaluation at the median (tools/f1b_isolate.py,
// profiles/r05_precision).  So every 16-row tile runs its products on operands of sign sgn = -1 for
// odd tiles (+1 even): the error of an odd tile's products leans the other way and undoing the sign
// afterwards is exact (powers of two and signs fold into the scales that are applied anyway):
//   F1a: Xa and H1 of the tile enter their MFMAs negated (k_z1, k_z2 undo it), and its dZ2 is handed
//     to F1b / F2 negated;
//   F1b: dH1 = dZ2 W2 and dW1a = Xa^T dZ1 then come out negated, undone by u1; Z1's recompute as F1a;
//   F2: its row splits alternate the same way over whole workgroups (each split's partial of dW2 is
//     one accumulator chain; odd splits run on negated H1 and negate the partial back).
__device__ __forceinline__ float tile_sign(int tile) { return (tile & 1) ? -1.f : 1.f; }

// LDS of F1a: the loop region (two half-chunk buffers + W1a) doubles as the epilogue's workgroup
// slots (dW3 [W][A][HID], then [W][A + 4] db3 / stats); b2 and W3 follow it
template <int A_, int KD, int W>
constexpr int f1a_region_bytes() {
  constexpr int loop = 4 * H16 * 2 + 2 * HID * KD * 2;
  constexpr int ep = W * A_ * HID * 4 + W * (A_ + 4) * 4;
  return ((loop > ep ? loop : ep) + 15) / 16 * 16;
}
template <int A_, int KD, int W>
constexpr int f1a_lds_bytes() {
  return f1a_region_bytes<A_, KD, W>() + (HID + A_ * HID) * 4;
}
template <int KD>
constexpr int f1b_lds_bytes() {
  return 4 * H16 * 2 + 2 * HID * KD * 2;
}

// The policy head is evaluated relative to its last action: the PPO loss depends on the logits only
// through their log-softmax, so every row's logit gradients sum to zero (sum_a dL/dz_a = 0) and
//   z_a - z_{A-1} = (W3[a] - W3[A-1]) H2 + b3[a] - b3[A-1]        (a < A - 1; z_{A-1} - z_{A-1} = 0)
//   dZ2 = sum_{a < A-1} dl_a (W3[a] - W3[A-1]) (1 - H2^2)
//   dW3[A-1] = -sum_{a < A-1} dW3[a]
// which is the same loss and gradient with A - 1 head rows instead of A (at 2 actions: half of the
// head, of dZ2's products and of the dW3 reduce-scatter, the epilogue's largest part).  AH: head rows.
template <int A_, int NET, int KD, int W, int P>
__device__ __forceinline__ int f1a_body(const SfArgs& g, int grp) {
  constexpr int NTHR = 64 * W;
  constexpr int AH = NET == 0 ? A_ - 1 : 1;
  const SfNet& N = g.n[NET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sCh = reinterpret_cast<_Float16*>(lds);  // [2 buf][2 hi/lo][128][32]
  _Float16* sW1 = sCh + 4 * H16;                      // [2 hi/lo][HID][KD]
  float* sSlot = lds;                                 // epilogue (after the loop's last barrier)
  float* sB2 = lds + f1a_region_bytes<A_, KD, W>() / 4;
  float* sW3 = sB2 + HID;

  // w wave-uniform (readfirstlane): tile bases stay in SGPRs, stores use a 32-bit lane offset
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), c = l & 15, gq = l >> 4;
  // Prologue: every global load of the first group goes out before any result is used (the W2
  // half-chunk and W1a planes by LDS DMA, the tile's X rows, b2 and W3 into registers), so the
  // workgroup waits for one memory round trip instead of four in a row
  int tile = grp * W + w;
  if (!dcheck(tile < g.M / 16, DC_SGD_TILE, tile)) tile = g.M / 16 - 1;
  const int row0 = tile * 16;
  FA_STAMP(0);
  FA_HWID();
  hc_dma<W>(N.w2ph, N.w2pl, 0, 0, sCh, w, l);
  w1_dma<KD, W>(N, sW1, w, l);
  float xv[8];
  xa_row8(g.x + (size_t)(row0 + c) * g.x_stride, 8 * gq, g.D, g.x_stride, xv);
  __shared__ float s_w3m[W];  // per wave: max |W3 row| entry it staged (the dZ2 scale bound below)
  __shared__ double s_vx[W];  // value net: per wave, the f64 sum of its rows' v - vt (vf_row)
  {
    constexpr int NW3 = (AH * HID + NTHR - 1) / NTHR;
    const float b2v = tid < HID ? N.b2[tid] : 0.f;
    float w3v[NW3], w3l[NW3];
#pragma unroll
    for (int j = 0; j < NW3; ++j) {
      const int i = tid + j * NTHR;
      w3v[j] = i < AH * HID ? N.w3[i] : 0.f;
      w3l[j] = (NET == 0 && i < AH * HID) ? N.w3[(A_ - 1) * HID + (i & (HID - 1))] : 0.f;
    }
    if (tid < HID) sB2[tid] = b2v * SF_2LOG2E;  // H2 = tanh(Z2 + b2): exp2 argument
    float m3 = 0.f;
#pragma unroll
    for (int j = 0; j < NW3; ++j) {
      const int i = tid + j * NTHR;
      if (i < AH * HID) {
        const float v = w3v[j] - w3l[j];
        sW3[i] = v;
        m3 = fmaxf(m3, fabsf(v));
      }
    }
    m3 = wave_max(m3);
    if (l == 0) s_w3m[w] = m3;
  }
  h8 xh, xl;
  const float sgn = tile_sign(tile);
  const int ex = x_split(xv, xh, xl, sgn);
  if ((NET == 0 || g.net0 == 1) && 8 * gq < KD) {  // the rows' Xa split for F2: by the policy net (both
                                                    // nets split the same rows alike), or the value net alone
    _Float16* xo = g.xsp + (size_t)(row0 + c) * KD + 8 * gq;
    *reinterpret_cast<h8*>(xo) = xh;
    *reinterpret_cast<h8*>(xo + (size_t)g.M * KD) = xl;
  }
  const float k_z1 = sgn * N.sc[1] * pow2(-ex) * SF_2LOG2E;  // Z1 accumulator -> 2 log2(e) Z1
  const float h1s = sgn * SF_H1_SCALE;                        // H1 enters Z2's products as sgn 2^14 H1
  vm_drain();
  __syncthreads();
  FA_STAMP(1);

  // ---- Z2^T = W2 H1^T: 16 steps (k-tile t, n-half ph) of 8 n-tiles x 3 MFMAs over double-
  // buffered half-chunks; H1^T of k-tile t (two Z1^T tiles, tanh, split) at the start of its first step
  f4 acc[16];
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) acc[nt] = f4zero();
  h8 bh, bl;
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      const int st = 2 * t + ph;  // reads buffer ph; the next half-chunk -> buffer ph ^ 1
      if (st < 15) hc_dma<W>(N.w2ph, N.w2pl, 128 * (ph ^ 1), 32 * (t + ph), sCh + (ph ^ 1) * 2 * H16, w, l);
      if (ph == 0) {
        f4 z[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          h8 wh, wl;
          w1_frag<KD>(sW1, 2 * t + b, c, gq, wh, wl);
          z[b] = mmP<P>(wh, wl, xh, xl, f4zero());
        }
        float hv[8];  // 2^14 tanh = 2^14 - 2^15 r (the split's fixed H1 scale folded in)
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = fmaf(-2.f * h1s, tanh_r(z[j >> 2][j & 3] * k_z1), h1s);
        split8(hv, 0, 1.f, bh, bl);
      }
      // fragments one n-tile ahead of their MFMAs, fenced so that only two sets are live
      const _Float16* buf = sCh + ph * 2 * H16;
      h8 ch, cl;
      hc_frag(buf, 0, c, gq, ch, cl);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        h8 nh, nl;
        if (j < 7) hc_frag(buf, j + 1, c, gq, nh, nl);
        __builtin_amdgcn_sched_barrier(0);
        acc[8 * ph + j] = mmP<P>(ch, cl, bh, bl, acc[8 * ph + j]);
        __builtin_amdgcn_sched_barrier(0);
        if (j < 7) { ch = nh; cl = nl; }
      }
      vm_drain();
      __syncthreads();
    }
    if (t == 0) FA_STAMP(2);
  }
  FA_STAMP(3);

  // ---- H2^T = tanh(Z2^T + b2) (lane: rows n = 16 nt + 4g + i of column m = c); head
  // out[a] = b3 + sum_n W3[a][n] H2[n] (partial over the lane's 64 n, then over the four rows)
  const float k_z2 = sgn * N.sc[3] / SF_H1_SCALE * SF_2LOG2E;
  float out[A_];  // NET 0: z_a - z_{A-1}; out[A-1] = 0
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] = 0.f;
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) {
    const int n0 = 16 * nt + 4 * gq;
    const float4 bb = *reinterpret_cast<const float4*>(sB2 + n0);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float r = tanh_r(fmaf(acc[nt][i], k_z2, bv[i]));  // H2 = 1 - 2 r; r is kept for 1 - H2^2 = 4 r (1 - r)
      hv[i] = fmaf(-2.f, r, 1.f);
      acc[nt][i] = r;
    }
#pragma unroll
    for (int a = 0; a < AH; ++a) {
      const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
      out[a] = fmaf(hv[0], t.x, out[a]);
      out[a] = fmaf(hv[1], t.y, out[a]);
      out[a] = fmaf(hv[2], t.z, out[a]);
      out[a] = fmaf(hv[3], t.w, out[a]);
    }
    if constexpr (A_ > 4) asm volatile("" ::: "memory");  // keep the W3 reads per n-tile (8 actions: spills)
  }
#pragma unroll
  for (int a = 0; a < AH; ++a) out[a] = sum_rows4(out[a]) + (NET == 0 ? N.b3[a] - N.b3[A_ - 1] : N.b3[a]);
  // the dZ2 pass below re-reads W3 from LDS rather than keeping the head's 16 A float4 alive
  // through the dW3 reductions (the compiler would otherwise reuse them and spill)
  asm volatile("" ::: "memory");
  FA_STAMP(4);
  float dl[A_];
  float st[4];
  double vex;
  sf_loss<A_, NET>(g, out, row0 + c, dl, st, vex);

  // ---- dW3[a][n] over the tile's rows: reduce-scatter over the 16 lanes of a row (lane c ends
  // with n = 64G + 16 (c >> 2) + 4g + (c & 3) of group G), one slot per wave
  constexpr int SLOT_B3 = W * AH * HID;
#pragma unroll
  for (int a = 0; a < AH; ++a)
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = fmaf(-2.f * dl[a], acc[4 * G + (k >> 2)][k & 3], dl[a]);  // dl H2
      sSlot[(w * AH + a) * HID + 64 * G + 16 * (c >> 2) + 4 * gq + (c & 3)] = row_reduce16(v, l);
    }
  {  // db3 and the loss stats: row sums (the four rows of the wave hold the same 16 rows m)
    float sv[A_ + 4];
#pragma unroll
    for (int a = 0; a < A_; ++a) sv[a] = dl[a];
#pragma unroll
    for (int i = 0; i < 4; ++i) sv[A_ + i] = st[i];
#pragma unroll
    for (int i = 0; i < A_ + 4; ++i) sv[i] = row_sum16(sv[i]);
    if (l == 0)
#pragma unroll
      for (int i = 0; i < A_ + 4; ++i) sSlot[SLOT_B3 + w * (A_ + 4) + i] = sv[i];
    if constexpr (NET == 1) {  // the value head's bias: exact row differences summed in f64 (vf_row)
      const double vx = row_sum16d(vex);
      if (l == 0) s_vx[w] = vx;
    }
  }
  FA_STAMP(5);

  // ---- dZ2^T = (dl W3) (1 - H2^2) 2^edz, in place of H2 in the accumulators, then -> HBM split at
  // that scale: [tile][s = nt >> 1][hi, lo][lane][4 (nt & 1) + i], i.e. each lane's eight values of an
  // n-step are the A fragment F1b's same lane reads (pre-split: neither F1b nor F2 splits it again).
  // The tile's exponent edz comes from the bound |dZ2| <= sum_a |dl_a| max |W3| (|1 - H2^2| <= 1): a
  // wave max of one value per lane instead of one over the 64 products, and the power of two is folded
  // into dl (exactly), so the products come out scaled.  The bound can sit a few binades above the
  // tile's largest element; the split keeps all 22 bits of every element down to 2^-17 of the scale.
  float w3m = s_w3m[0];
#pragma unroll
  for (int ww = 1; ww < W; ++ww) w3m = fmaxf(w3m, s_w3m[ww]);
  float bnd = 0.f;
#pragma unroll
  for (int a = 0; a < AH; ++a) bnd += fabsf(dl[a]);
  bnd = wave_max(bnd * w3m);
  const int edz = bnd > 0.f ? sf_exp(bnd) : 120;  // an all-zero tile: the largest exponent (F2 takes the min)
  {
    const float sdz = sgn * pow2(edz + 2);  // (handed over with the tile's sign; x4: 1 - H2^2 = 4 r (1 - r))
#pragma unroll
    for (int a = 0; a < AH; ++a) dl[a] *= sdz;
  }
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) {
    const int n0 = 16 * nt + 4 * gq;
    float gs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < AH; ++a) {
      const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
      gs[0] = fmaf(dl[a], t.x, gs[0]);
      gs[1] = fmaf(dl[a], t.y, gs[1]);
      gs[2] = fmaf(dl[a], t.z, gs[2]);
      gs[3] = fmaf(dl[a], t.w, gs[3]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float r = acc[nt][i];
      acc[nt][i] = gs[i] * fmaf(-r, r, r);  // (no cancellation where H2 saturates, unlike 1 - H2^2)
    }
    if constexpr (A_ > 4) asm volatile("" ::: "memory");
  }
  {
    _Float16* dst = N.dz2s + (size_t)tile * (16 * HID * 2) + l * 8;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      h8 hi, lo;
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = acc[2 * st + (j >> 2)][j & 3];
      split8v(x, hi, lo);
      *reinterpret_cast<h8*>(dst + st * 1024) = hi;
      *reinterpret_cast<h8*>(dst + st * 1024 + 512) = lo;
    }
  }
  if (l == 0) {
    N.tile_edz[tile] = edz;
    N.tile_ex[tile] = ex;
  }
  FA_STAMP(6);
  // ---- workgroup sums (fixed wave order) -> this block's partials
  __syncthreads();
  const int blk = grp;
  for (int e = tid; e < A_ * HID; e += NTHR) {
    const int a = e >> 8, n = e & (HID - 1);
    float s = 0.f;
    if (a < AH) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) s += sSlot[(ww * AH + a) * HID + n];
    } else {  // the policy's last action: dW3[A-1] = -sum_{a < A-1} dW3[a]
#pragma unroll
      for (int b = 0; b < AH; ++b) {
        float sb = 0.f;
#pragma unroll
        for (int ww = 0; ww < W; ++ww) sb += sSlot[(ww * AH + b) * HID + n];
        s += sb;
      }
      s = -s;
    }
    N.part_w3[(size_t)blk * A_ * HID + e] = s;
  }
  if (tid < A_ + 4) {
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) s += sSlot[SLOT_B3 + ww * (A_ + 4) + tid];
    if (tid >= A_) N.part_stat[(size_t)blk * 4 + tid - A_] = s;
    else if (NET == 0) N.part_b3[(size_t)blk * A_ + tid] = s;
    else {  // [blk][hi, lo]
      double vx = 0.0;
#pragma unroll
      for (int ww = 0; ww < W; ++ww) vx += s_vx[ww];
      vf_b3_part(vx, g.co.vf_loss_coeff, load_dyn(g).inv_count, N.part_b3 + (size_t)blk * 2);
    }
  }
  return edz;  // (wave-uniform: the fused F1 hands it to f1b_body in a register)
}

// workgroup -> (net, tile group) for F1a / F1b launched as one row of G x nets workgroups.  Both
// nets in one launch: blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one), so the
// nets alternate in runs of 8 -- each XCD, and so each CU, gets workgroups of both nets, whose
// different epilogue lengths keep a CU's co-resident workgroups from running their epilogues in
// phase (the policy net's is longer).  G not a multiple of 8, or !MIX: net-major.  Measured
// (profiles/r05_mix): c4 F1a 72.7 -> 69.9 µs, F1b 62.4 -> 58.2; at 8 actions F1b 76.5 -> 71.3 but
// F1a 91.8 -> 101.7, so F1a keeps the net-major order above 4 actions.
template <int W, bool MIX>
__device__ __forceinline__ int2 f1_net_group(const SfArgs& g) {
  const int G = g.M / (16 * W), b = blockIdx.x;
  if ((int)gridDim.x <= G) return make_int2(0, b);
  if (MIX && (G & 7) == 0) return make_int2((b >> 3) & 1, ((b >> 4) << 3) | (b & 7));
  return make_int2(b / G, b % G);
}

template <int A_, int KD, int W, int P>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_sf_fwd(SfArgs g) {
  const int2 ng = f1_net_group<W, (A_ <= 4)>(g);
  if (ng.x + g.net0 == 0) f1a_body<A_, 0, KD, W, P>(g, ng.y);
  else f1a_body<1, 1, KD, W, P>(g, ng.y);
}

int sf_f1_parts(int M, bool fused) { return M / (16 * (fused ? SF_F1F_W : SF_F1_W)); }
// F1a + F1b as one kernel (k_sf_f1) for a whole gradient by default at up to 4 actions (16 columns of
// Xa): with F2 = k_sf_dw2r and the no-SLP build it is the faster form there (c4 +1.3-2.1%, three same-box
// alternations, profiles/r06_fusedab); at 8 actions the two kernels stay (c3 -0.2 to -3.9% fused).
// RLKS_F1_FUSED=1 / RLKS_F1_SPLIT=1 force either form (A/B runs, the tests' references).
bool sf_f1_fused(int A) {
  if (getenv("RLKS_F1_FUSED")) return true;
  if (getenv("RLKS_F1_SPLIT")) return false;
  return A <= 4;
}

// FUSED (k_sf_f1: right after f1a_body in the same workgroup): the tile's dZ2 exponent arrives in a
// register (edz_in), and the W1a planes F1a staged are still in LDS when its epilogue slots stopped
// short of them (W1_KEPT)
template <int NET, int KD, int ND, int W, int P, bool FUSED = false, bool W1_KEPT = false>
__device__ __forceinline__ void f1b_body(const SfArgs& g, int grp, int edz_in = 0) {  // ND = obs_dim + 1 (rows d of dW1a^T)
  constexpr int NTHR = 64 * W;
  constexpr int DT = KD / 16;                      // 16-row d-tiles of dW1a^T
  constexpr int SLOT = W * 16 * 16 * DT;           // floats per k-tile: [W][16 k][16 DT d]
  constexpr int KPR = (4 * H16 * 2 / 4) / SLOT;    // k-tiles per flush round (the half-chunk buffers)
  static_assert(KPR >= 1 && 16 % KPR == 0, "dW1 epilogue slots");
  const SfNet& N = g.n[NET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sCh = reinterpret_cast<_Float16*>(lds);  // [2 buf][2 hi/lo][128][32]
  _Float16* sW1 = sCh + 4 * H16;                      // [2 hi/lo][HID][KD]
  float* sEp = lds;                                   // epilogue slots (the chunk buffers)

  // w wave-uniform (readfirstlane): tile bases stay in SGPRs, stores use a 32-bit lane offset.  FUSED:
  // the lane index through an opaque copy, so that the compiler derives F1b's lane offsets afresh
  // instead of keeping F1a's alive across its epilogue (which spilled)
  int tid = threadIdx.x;
  if constexpr (FUSED) asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(tid));
  const int l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), c = l & 15, gq = l >> 4;
  int tile = grp * W + w;
  if (!dcheck(tile < g.M / 16, DC_SGD_TILE, tile)) tile = g.M / 16 - 1;
  const int row0 = tile * 16, blk = grp;
  const int D = g.D, stride = g.x_stride;

  hc_dma<W>(N.w2th, N.w2tl, 0, 0, sCh, w, l);
  if constexpr (!W1_KEPT) w1_stage<KD, NTHR>(N, sW1, tid);
  const int edz = FUSED ? edz_in : N.tile_edz[tile];
  const _Float16* dzp = N.dz2s + (size_t)tile * (16 * HID * 2) + l * 8;  // split by F1a at 2^edz
  h8 dh = *reinterpret_cast<const h8*>(dzp), dl = *reinterpret_cast<const h8*>(dzp + 512);
  vm_drain();
  __syncthreads();

  // ---- dH1 = dZ2 W2: 16 steps (n-step s, k-half ph) of 8 k-tiles x 3 MFMAs; the (pre-split) dZ2
  // fragment of n-step s taken at its first step and the next one loaded
  f4 acc[16];
#pragma unroll
  for (int kt = 0; kt < 16; ++kt) acc[kt] = f4zero();
  h8 ah, al;
  for (int s = 0; s < 8; ++s) {
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      const int st = 2 * s + ph;
      if (st < 15) hc_dma<W>(N.w2th, N.w2tl, 128 * (ph ^ 1), 32 * (s + ph), sCh + (ph ^ 1) * 2 * H16, w, l);
      if (ph == 0) {
        ah = dh;
        al = dl;
        if (s < 7) {
          dh = *reinterpret_cast<const h8*>(dzp + (s + 1) * 1024);
          dl = *reinterpret_cast<const h8*>(dzp + (s + 1) * 1024 + 512);
        }
      }
      const _Float16* buf = sCh + ph * 2 * H16;
      h8 ch, cl;
      hc_frag(buf, 0, c, gq, ch, cl);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        h8 nh, nl;
        if (j < 7) hc_frag(buf, j + 1, c, gq, nh, nl);
        __builtin_amdgcn_sched_barrier(0);
        acc[8 * ph + j] = mmP<P>(ah, al, ch, cl, acc[8 * ph + j]);
        __builtin_amdgcn_sched_barrier(0);
        if (j < 7) { ch = nh; cl = nl; }
      }
      vm_drain();
      __syncthreads();
    }
  }

  // ---- dZ1 = dH1 (1 - H1^2) (lane: rows m = 4g + i, column k = 16 kt + c), in place of dH1 over
  // all k-tiles first, so that it enters the split at the tile's own power of two (round 3 split it
  // at 2^(e_dz + e_w2 - 23) from the bound |dH1 2^(e_dz + e_w2)| <= 256 2^15 2^15: typical tiles then
  // sat 2^8-2^12 below it and their lo halves fell into fp16 subnormals, dW1 / db1 ~5x less accurate
  // per element than fp32); then dW1a^T = Xa^T dZ1 per k-tile
  h8 xh, xl;
  const float sgn = tile_sign(tile);
  const int ex = x_frag(g, row0, c, gq, xh, xl, sgn);
  const float sx = pow2(ex), k_z1 = sgn * N.sc[1] / sx * SF_2LOG2E;
  // 1 - H1^2 = 4 r (1 - r): the 4 joins the unscaling power of two
  float zmx = 0.f;
  const _Float16* w1b = sW1 + w1_off<KD>(c, gq & (KD / 8 - 1));  // row c; rows 16 kt + c at immediates
#pragma unroll
  for (int kt = 0; kt < 16; ++kt) {
    const _Float16* q = w1b + kt * 16 * KD;
    const h8 wh = *reinterpret_cast<const h8*>(q), wl = *reinterpret_cast<const h8*>(q + HID * KD);
    const f4 z = mmP<P>(xh, xl, wh, wl, f4zero());  // Z1 rows m = 4g + i, column k = 16 kt + c
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float r = tanh_r(z[i] * k_z1);
      acc[kt][i] *= fmaf(-r, r, r);
      zmx = fmaxf(zmx, fabsf(acc[kt][i]));
    }
  }
  const int ez = sf_exp(wave_max(zmx));
  const float sz1 = pow2(ez), u1 = sgn * pow2(2 - ex - edz - (int)N.sc[5] - ez);  // (sgn: F1a's tile sign)
  h4 xth[DT], xtl[DT];  // Xa^T (16x16x16 A operand): rows d = 16 dt + c, columns m = 4g + j
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      _Float16 a, b;
      split1(xa_elem(g.x + (size_t)(row0 + 4 * gq + j) * stride, 16 * dt + c, D) * sx, a, b);
      xth[dt][j] = a;
      xtl[dt][j] = b;
    }
  // dZ1's lo half carried at 2^11 (its own accumulator, unscaled at the end): an element far below
  // the tile's max keeps a normal fp16 lo (a plain lo half turns subnormal 2^18 below the max)
  const float u1l = u1 * (1.f / 2048.f);
#pragma unroll
  for (int kt = 0; kt < 16; ++kt) {
    h4 zh, zl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = acc[kt][i] * sz1;
      const _Float16 a = (_Float16)x;
      zh[i] = a;
      zl[i] = (_Float16)((x - (float)a) * 2048.f);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const f4 dh = P == 1 ? mk16(xth[dt], zh, f4zero())
                           : mk16(xtl[dt], zh, mk16(xth[dt], zh, f4zero()));  // rows d = 16 dt + 4g + i, column k
      const f4 dl2 = P == 1 ? f4zero() : mk16(xth[dt], zl, f4zero());
      const float4 v = {fmaf(dl2[0], u1l, dh[0] * u1), fmaf(dl2[1], u1l, dh[1] * u1), fmaf(dl2[2], u1l, dh[2] * u1),
                        fmaf(dl2[3], u1l, dh[3] * u1)};
      // row k = c of the wave's slot: 16-byte quad gq at gq ^ ((c >> 1) & 3), so that the 8 lanes of a
      // ds_write_b128 group (c = 0..7) cover all 32 banks (unswizzled: 4-way conflicts; profiles/r03s
      // F1b 11% of CU cycles in LDS bank conflicts)
      *reinterpret_cast<float4*>(sEp + (kt % KPR) * SLOT + (w * 16 + c) * 16 * DT + 16 * dt + 4 * (gq ^ ((c >> 1) & 3))) = v;
    }
    if (kt % KPR == KPR - 1) {  // (k-tile, k, d) elements; ND a compile-time constant (no runtime division)
      __syncthreads();
      const int kt0 = kt + 1 - KPR;
      for (int e = tid; e < KPR * 16 * ND; e += NTHR) {
        const int jj = e / (16 * ND), e2 = e - jj * 16 * ND, kk = e2 / ND, d = e2 - kk * ND;
        const int k = 16 * (kt0 + jj) + kk;
        float sum = 0.f;
        const int dq = (d & ~15) + 4 * (((d >> 2) & 3) ^ ((kk >> 1) & 3)) + (d & 3);  // the stores' quad swizzle
#pragma unroll
        for (int ww = 0; ww < W; ++ww) sum += sEp[jj * SLOT + (ww * 16 + kk) * 16 * DT + dq];
        if (d < ND - 1) N.part_w1[((size_t)blk * HID + k) * (ND - 1) + d] = sum;
        else N.part_b1[(size_t)blk * HID + k] = sum;
      }
      if (kt < 15) __syncthreads();
    }
  }
}

template <int KD, int ND, int W, int P>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_sf_bwd(SfArgs g) {
  const int2 ng = f1_net_group<W, true>(g);
  if (ng.x + g.net0 == 0) f1b_body<0, KD, ND, W, P>(g, ng.y);
  else f1b_body<1, KD, ND, W, P>(g, ng.y);
}

// F1 fused (the default up to 4 actions, sf_f1_fused): F1a then F1b on the same 16-row tiles in one
// workgroup.  The dZ2 hand-off is still written for F2, but F1b reads each lane's own fragments back
// right after they were written (from the XCD's L2, not HBM), the tile exponent stays in a register,
// the W1a planes stay in LDS (up to 4 actions), and there is one launch boundary less per SGD step.
// Launched with 16-wave workgroups, one per CU (SF_F1F_W): with two 8-wave workgroups per CU in
// different phases a few policy tiles a step came out different from run to run (cause not isolated).
// Measured no faster than the two kernels on round 6's first trees (126-128 µs against 126 µs for the
// pair at c4); faster end to end with k_sf_dw2r and the no-SLP build (profiles/r06_fusedab).
template <int A_, int KD, int W>
constexpr bool f1_w1_kept() {  // F1a's epilogue slots end before the W1a planes (sW1 = 4 H16 halves in)
  return W * (A_ - 1 > 1 ? A_ - 1 : 1) * HID * 4 + W * (A_ + 4) * 4 <= 4 * H16 * 2;
}
template <int A_, int KD, int W>
constexpr int f1_lds_bytes() {
  return f1a_lds_bytes<A_, KD, W>() > f1b_lds_bytes<KD>() ? f1a_lds_bytes<A_, KD, W>() : f1b_lds_bytes<KD>();
}
template <int A_, int KD, int W, int P>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_sf_f1(SfArgs g) {
  const int2 ng = f1_net_group<W, (A_ <= 4)>(g);
  // F1b's loads of the X rows are the ones F1a made: an opaque copy of the row pointer keeps the
  // compiler from carrying F1a's values across the epilogue in registers (which spilled)
  SfArgs g2 = g;
  if (ng.x + g.net0 == 0) {
    const int edz = f1a_body<A_, 0, KD, W, P>(g, ng.y);
    __syncthreads();  // epilogue slots read; the dZ2 stores complete (the fence waits for them)
    asm volatile("" : "+s"(g2.x));
    f1b_body<0, KD, 3 * A_ + 1, W, P, true, f1_w1_kept<A_, KD, W>()>(g2, ng.y, edz);
  } else {
    const int edz = f1a_body<1, 1, KD, W, P>(g, ng.y);
    __syncthreads();
    asm volatile("" : "+s"(g2.x));
    f1b_body<1, KD, 3 * A_ + 1, W, P, true, f1_w1_kept<1, KD, W>()>(g2, ng.y, edz);
  }
}

// ----------------------------------------------------------------------------- F2
// dW2 = dZ2^T H1 over a row range as a tiled split-fp16 GEMM: C [256 n][256 k] per workgroup (512
// threads, 8 waves of 64 n x 128 k = 2 x 4 v_mfma_f32_32x32x16_f16 tiles: 128 accumulator registers,
// two waves per SIMD), K = the rows, in chunks of 32, double-buffered in LDS:
//   A = dZ2^T chunk: F1a's fp32 dZ2 (two 16-row tiles in its lane order), loaded into registers one
//     chunk ahead, split with the step's max |dZ2| scale; db2 from the same loads;
//   B = H1 chunk, produced by the workgroup: wave w forms Z1 = Xa W1a^T for the chunk's 32 rows and
//     hidden units k = 32 w + 0..31 (v_mfma_f32_16x16x16_f16, X scaled by F1a's per-tile exponent),
//     tanh, split at 2^14.
// Chunk c + 1's operands are produced after chunk c's MFMAs are issued, in the same basic block (the
// scheduler interleaves the two), into the other buffer; one barrier per chunk.  Round 2's F2 (eight
// waves of 256 n x 32 k, H1 in registers) read every A fragment -> wait -> MFMA: 30% MFMA-busy
// (profiles/r03c).  A 1,024-thread version of this kernel (64 x 64 per wave) spilled at its
// 128-register budget, and each spill reload waited for the prefetches (vmcnt counts in issue order).
typedef __fp16 hf4_t __attribute__((vector_size(8)));
// ds_read_b64_tr_b16 (T10): per 16-lane group, 4 rows x 16 columns of 16-bit elements, lane i of
// the group gets column i (row q in element q); EXEC must be all ones
__device__ __forceinline__ h4 tr_read(const _Float16* p) {
  const hf4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) hf4_t*)(p));
  return __builtin_bit_cast(h4, v);
}
#ifdef RLKS_STAMPS
// diagnostic build only (tools/stamps.py): F2 phase cycles of lane 0 of every wave,
// [net][split][wave][prologue, MFMA issue, production, barrier waits, epilogue, start]
__device__ unsigned long long g_f2_stamps[2][128][16][6];
#define F2_NOW() __builtin_amdgcn_s_memtime()
#endif
constexpr int F2_THREADS = 512;
// LDS images (halves), per buffer: A = dZ2 chunk [plane hi, lo][32 m][F2_AROW] (n contiguous, rows
// padded by 32 halves: the transposed fragment reads of 4 rows x 32 columns land on 4 disjoint
// 16-bank windows; 8-byte quads XOR 2 ((m >> 2) & 3) within each 32-column block for the stores), B = H1 chunk [plane][s 2][256 k][16] (16-byte piece h of row k
// at slot h ^ ((k >> 3) & 1): conflict-free ds_read_b128).  Unswizzled along n, s and k-blocks, every
// fragment address is one per-lane base plus immediates.
constexpr int F2_AROW = HID + 32;
constexpr int F2_APLANE = 32 * F2_AROW;
constexpr int F2_BPLANE = 2 * HID * 16;
constexpr int F2_BUF = 2 * F2_APLANE + 2 * F2_BPLANE;
constexpr int F2_MAX_TILES = 2 * 256;  // 16-row tiles per F2 workgroup (tiles_per_split <= 256 chunks)

// grid (splits, 2 nets) x 512 threads; split z covers 32-row chunks [z tps, (z + 1) tps).
// dZ2 arrives split by F1a, each 16-row tile T at its own scale 2^e_T; the H1 rows of tile T are
// split at 2^(14 + E - e_T), E = min over the workgroup's tiles, so that every product carries
// 2^(14 + E) (unscaled at the end).  Production of chunk c + 1 (copy of its dZ2 pieces into the A
// image, db2, and H1: wave w forms hidden units k = 32 w + 0..31) is shared by all eight waves and
// placed ping-pong: per chunk c, phase 1 = {waves 0-3: MFMAs of c, 4-7: production}, phase 2 =
// {0-3: production, 4-7: MFMAs of c}, a barrier after each, so that each SIMD's VALU work runs
// beside its partner wave's MFMAs.
template <int KD, int P>
__global__ __launch_bounds__(F2_THREADS) void k_sf_dw2(SfArgs g) {
  const SfNet& N = g.n[blockIdx.y];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sm = reinterpret_cast<_Float16*>(lds);  // [2 buf][F2_BUF]
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = l & 15, gq = l >> 4, wm = w >> 1, wn = w & 1, r = l & 31, h = l >> 5;
  const bool first = w < 4;  // waves 0-3: MFMAs in phase 1; 4-7: in phase 2
  const int D = g.D, stride = g.x_stride;
  int t0 = blockIdx.x * g.tiles_per_split, t1 = t0 + g.tiles_per_split;
  if (!dcheck(t1 <= g.M / 32, DC_SGD_TILE, t1)) t0 = t1 = 0;
  const int nk = t1 - t0;

  // F1a's X and dZ2 exponents of the workgroup's 16-row tiles -> LDS (read per chunk from there, not
  // by a global load among the prefetches); E = min e_T (F1a stores 120 for an all-zero tile)
  int* sEx = reinterpret_cast<int*>(sm + 2 * F2_BUF);  // [2 (t1 - t0)] X exponents, then dZ2 exponents
  int* sEd = sEx + F2_MAX_TILES;
  int emin = 120;
  for (int i = tid; i < 2 * nk; i += F2_THREADS) {
    sEx[i] = N.tile_ex[2 * t0 + i];
    const int e = N.tile_edz[2 * t0 + i];
    sEd[i] = e;
    emin = min(emin, e);
  }
  __shared__ float s_emin[F2_THREADS / 64];
  emin = (int)-wave_max((float)-emin);
  if (l == 0) s_emin[w] = (float)emin;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < F2_THREADS / 64; ++i) emin = min(emin, (int)s_emin[i]);
  const int E = __builtin_amdgcn_readfirstlane(emin);
  // this split's sign (tile_sign: odd splits run their products on -H1 and negate the partial back)
  const float ssgn = tile_sign(blockIdx.x);
  const float unscale = ssgn * pow2(-14 - E);

  // per-lane fragment bases (halves within a buffer):
  //   A (transposed reads): lane 4 q + p of its 16-lane group addresses row 4 h + q (+ 16 s, + 8 for
  //   the second read), columns 64 wm + 32 i + 16 ((l >> 4) & 1) + 4 p; K order of k-step s: rows
  //   16 s + 8 (j >> 2) + 4 h + (j & 3) (the MFMA accumulator row order the B image follows)
  //   B: column k = 128 wn + 32 j + r, piece h
  //   (A image quads XOR-swizzled by 2 ((m >> 2) & 3): the 4 rows of a transposed read share one XOR,
  //   and the dZ2 stores of 16 consecutive rows spread over all banks; profiles/r03k: 20% of CU cycles
  //   were LDS bank conflicts without it)
  const int aq = (4 * ((l >> 4) & 1) + (l & 3)) ^ (2 * h);  // quad within the 8-quad block, rows 4 h + q
  const int abase = (4 * h + ((l & 15) >> 2)) * F2_AROW + 4 * aq + 64 * wm;
  const int abase8 = (4 * h + ((l & 15) >> 2) + 8) * F2_AROW + 4 * (aq ^ 4) + 64 * wm;  // rows + 8
  const int bbase = 2 * F2_APLANE + (128 * wn + r) * 16 + 8 * (h ^ ((r >> 3) & 1));
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  auto mfma_chunk = [&](const _Float16* b) {  // A fragments of both i, then B one j at a time (24 registers)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      h8 ah[2], al[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const _Float16* pa = b + abase + s * 16 * F2_AROW + 32 * i;
        const _Float16* pa8 = b + abase8 + s * 16 * F2_AROW + 32 * i;
        const h4 a0 = tr_read(pa), a1 = tr_read(pa8);
        const h4 c0 = tr_read(pa + F2_APLANE), c1 = tr_read(pa8 + F2_APLANE);
        ah[i] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
        al[i] = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const _Float16* pb = b + bbase + s * HID * 16 + 32 * 16 * j;
        const h8 bh = *reinterpret_cast<const h8*>(pb), bl = *reinterpret_cast<const h8*>(pb + F2_BPLANE);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mmaP<P>(ah[i], al[i], bh, bl, acc[i][j]);
      }
    }
  };

  // ---- dZ2 pieces: wave w takes n-step w of both 16-row tiles T2 and both planes (hi, lo): piece
  // i = 2 T2 + plane of lane l holds halves j at row m = 16 T2 + c, columns n = 32 w + 16 (j >> 2) +
  // 4 gq + (j & 3) (F1a's layout, loaded one chunk ahead).  (Buffer loads: an SGPR resource, the
  // chunk offset in an SGPR and one 32-bit lane offset, instead of a 64-bit address pair per load,
  // which cost the registers that made this kernel spill.)
  const __amdgpu_buffer_rsrc_t dz_rsrc = __builtin_amdgcn_make_buffer_rsrc(N.dz2s, (short)0, 0x7fffffff, 0x00020000);
  const int dz_lane = 2 * (w * 1024 + l * 8);  // bytes
  h8 dp[4];
  auto load_dz = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dp[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(
                                         dz_rsrc, dz_lane, t * (32 * HID * 4) + (i >> 1) * (16 * HID * 4) + (i & 1) * 1024, 0));
  };
  float db2[8] = {};  // dZ2 of this lane's columns, summed over its rows
  auto store_dz = [&](_Float16* img, float s0, float s1) {  // s0, s1: 2^-e of the two tiles (0: not counted)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float sc = (i >> 1) ? s1 : s0;
#pragma unroll
      for (int j = 0; j < 8; ++j) db2[j] = fmaf((float)dp[i][j], sc, db2[j]);
      // quads 8 w + gq and 8 w + gq + 4 of row m = 16 T2 + c, XOR 2 ((m >> 2) & 3)
      const int off = (i & 1) * F2_APLANE + (16 * (i >> 1) + c) * F2_AROW + 32 * w;
      const int sw = 2 * ((c >> 2) & 3);
      *reinterpret_cast<h4*>(img + off + 4 * (gq ^ sw)) = __builtin_shufflevector(dp[i], dp[i], 0, 1, 2, 3);
      *reinterpret_cast<h4*>(img + off + 4 * ((gq + 4) ^ sw)) = __builtin_shufflevector(dp[i], dp[i], 4, 5, 6, 7);
    }
  };

  // ---- H1 of a chunk as one 32 x 32 block per wave: Z1 (rows m of the chunk, hidden units k =
  // 32 w + (l & 31)) = Xa W1a^T on v_mfma_f32_32x32x8_f16, K = 8 columns of Xa = [X | 1 | 0] per MFMA
  // (D + 1 = 7 at 2 actions: one K step, no padding), three products; B = W1a rows k (loaded once),
  // A = the chunk's X rows (one 16-byte piece per lane and K step, loaded a chunk ahead, the selects
  // at use); F1a's X and dZ2 exponents of its two 16-row tiles, loaded a chunk ahead
  constexpr int KB = KD / 8;
  const int kh = 32 * w + r;  // this lane's hidden unit
  // (at KD = 32 the fragments are reloaded at every production, ahead of the dZ2 pieces: kept for
  // the whole kernel they make it spill)
  h4 wh[KB], wl[KB];
  auto load_w1 = [&]() {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      wh[kb] = *reinterpret_cast<const h4*>(N.w1h + kh * KD + 8 * kb + 4 * h);
      wl[kb] = *reinterpret_cast<const h4*>(N.w1l + kh * KD + 8 * kb + 4 * h);
    }
  };
  if constexpr (KB <= 2) load_w1();
  const float inv_w1 = N.sc[1];
  v4f xr[KB];
  int2 xe, de;
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x), (short)0, 0x7fffffff, 0x00020000);
  auto load_x = [&](int t) {
    xe = *reinterpret_cast<const int2*>(sEx + 2 * (t - t0));
    de = *reinterpret_cast<const int2*>(sEd + 2 * (t - t0));
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int base = 8 * kb + 4 * h, pb = base < stride - 4 ? base : stride - 4;
      xr[kb] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(x_rsrc, 4 * (r * stride + pb), 4 * t * 32 * stride, 0));
    }
  };
  // Z1 row m = acc_row(q) -> B image k-step m >> 4, position 8 h + 4 (q >> 2 & 1) + (q & 3) (bits 2 and 3
  // of m swapped), hidden unit kh (16-byte piece h at slot h ^ ((kh >> 3) & 1))
  const int hoff = 2 * F2_APLANE + kh * 16 + 8 * (h ^ ((kh >> 3) & 1));
  auto store_h1 = [&](_Float16* img) {
    // X scale of the chunk from F1a's per-tile exponents (the larger max: the smaller exponent)
    const int ex = min(xe.x, xe.y);
    const float sx = ssgn * pow2(ex), k_z1 = ssgn * inv_w1 * pow2(-ex) * SF_2LOG2E;
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int base = 8 * kb + 4 * h;
      const bool inrow = base < stride - 4;
      h4 xh, xl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = base + j;
        _Float16 a, b;
        split1(fmaf(xr[kb][j], (d < D && inrow) ? sx : 0.f, d == D ? sx : 0.f), a, b);
        xh[j] = a;
        xl[j] = b;
      }
      if constexpr (P != 1) {
        z = __builtin_amdgcn_mfma_f32_32x32x8f16(xl, wh[kb], z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x8f16(xh, wl[kb], z, 0, 0, 0);
      }
      z = __builtin_amdgcn_mfma_f32_32x32x8f16(xh, wh[kb], z, 0, 0, 0);
    }
    // rows of tile 2t + (q >> 3): H1 split at 2^(14 + E - e_T) (<= 2^14)
    // (the chunk's odd tile arrives negated from F1a: -hs1 undoes it)
    const float hs0 = ssgn * pow2(14 + E - de.x), hs1 = -ssgn * pow2(14 + E - de.y);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float hs = i < 2 ? hs0 : hs1;
      float x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = fmaf(-2.f * hs, tanh_r(z[4 * i + j] * k_z1), hs);
      unsigned a0, b0, a1, b1;
      split2(x[0], x[1], a0, b0);
      split2(x[2], x[3], a1, b1);
      const h4 hh = __builtin_bit_cast(h4, make_uint2(a0, a1)), hl = __builtin_bit_cast(h4, make_uint2(b0, b1));
      const int off = hoff + (i >> 1) * HID * 16 + 4 * (i & 1);
      *reinterpret_cast<h4*>(img + off) = hh;
      *reinterpret_cast<h4*>(img + off + F2_BPLANE) = hl;
    }
  };
  // production of the loaded chunk into img; counted: add its dZ2 to db2
  auto produce = [&](_Float16* img, bool counted) {
    if constexpr (KB > 2) load_w1();
    const float s0 = counted ? pow2(-de.x) : 0.f, s1 = counted ? -pow2(-de.y) : 0.f;  // (odd tile: negated)
    store_dz(img, s0, s1);
    store_h1(img);
  };
  // barrier without __syncthreads()'s fence (which would wait for the prefetches in flight: s_waitcnt
  // vmcnt(0)); the LDS stores need only lgkmcnt(0).  Scheduling barriers on both sides: the scheduler
  // otherwise moves each phase's VALU into the other phase (e.g. the X split into the MFMA phase,
  // where it waits for the X loads).
  auto phase_barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

#ifdef RLKS_STAMPS
  unsigned long long ts0 = F2_NOW(), tph[5] = {0ull, 0ull, 0ull, 0ull, 0ull}, tq = ts0;
#define F2_STAMP(i) { const unsigned long long tn = F2_NOW(); tph[i] += tn - tq; tq = tn; }
#else
#define F2_STAMP(i)
#endif
  if (nk > 0) {
    load_dz(t0);
    load_x(t0);
    produce(sm, true);
    load_dz(min(t0 + 1, t1 - 1));
    load_x(min(t0 + 1, t1 - 1));
  }
  __syncthreads();
  F2_STAMP(0);
  if constexpr (KD > 16) {
    // KD = 32 (8 actions): one loop for both halves, [MFMAs of chunk ci | barrier | production of chunk
    // ci + 1 + off | barrier], the second half (off = 1) one phase behind after a production of chunk 1
    // of its own, so that each SIMD still pairs one wave's MFMAs with its partner's production.  (With a
    // loop per half the two compiled to different code and the second half's production ran at half the
    // first half's speed, profiles/r05_f2; here this form also avoids that instance's 10 spilled
    // registers: c3 F2 86.5 -> 84.8 µs.  At KD = 16 the two loops stay: c4 66-68 vs 69-71 µs.)  The
    // production runs at the last chunks too, redoing one into the idle buffer uncounted.
    const int off = first ? 0 : 1;
    if (!first) {
      produce(sm + F2_BUF, 1 < nk);
      load_x(min(t0 + 2, t1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      load_dz(min(t0 + 2, t1 - 1));
      F2_STAMP(2);
      phase_barrier();
      F2_STAMP(3);
    }
    for (int ci = 0; ci < nk; ++ci) {
      mfma_chunk(sm + (ci & 1) * F2_BUF);
      F2_STAMP(1);
      phase_barrier();
      F2_STAMP(3);
      const int cn = ci + 1 + off;  // the chunk this production makes
      produce(sm + (cn & 1) * F2_BUF, cn < nk);
      load_x(min(t0 + cn + 1, t1 - 1));  // (before the dZ2 pieces: a spill reload for these
      __builtin_amdgcn_sched_barrier(0);  // addresses would otherwise wait for them)
      load_dz(min(t0 + cn + 1, t1 - 1));
      F2_STAMP(2);
      phase_barrier();
      F2_STAMP(3);
    }
    if (first) {  // the second half's extra phase
      phase_barrier();
      F2_STAMP(3);
    }
  } else if (first) {
    // (one loop per half, so that the phases' state stays in registers; the production runs at the last
    // chunk too, redoing it into the idle buffer uncounted: unconditional, so that the compiler keeps
    // the prefetches where they are)
    for (int ci = 0; ci < nk; ++ci) {
      mfma_chunk(sm + (ci & 1) * F2_BUF);
      F2_STAMP(1);
      phase_barrier();
      F2_STAMP(3);
      produce(sm + ((ci + 1) & 1) * F2_BUF, ci + 1 < nk);
      load_x(min(t0 + ci + 2, t1 - 1));  // (before the dZ2 pieces: a spill reload for these
      __builtin_amdgcn_sched_barrier(0);  // addresses would otherwise wait for them)
      load_dz(min(t0 + ci + 2, t1 - 1));
      F2_STAMP(2);
      phase_barrier();
      F2_STAMP(3);
    }
  } else {
    for (int ci = 0; ci < nk; ++ci) {
      produce(sm + ((ci + 1) & 1) * F2_BUF, ci + 1 < nk);
      load_x(min(t0 + ci + 2, t1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      load_dz(min(t0 + ci + 2, t1 - 1));
      F2_STAMP(2);
      phase_barrier();
      F2_STAMP(3);
      mfma_chunk(sm + (ci & 1) * F2_BUF);
      F2_STAMP(1);
      phase_barrier();
      F2_STAMP(3);
    }
  }
#undef F2_STAMP

  float* out = N.part_w2 + (size_t)blockIdx.x * SF_W2_PSTRIDE;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q)
        out[(size_t)(64 * wm + 32 * i + acc_row(q, l)) * HID + 128 * wn + 32 * j + r] = acc[i][j][q] * unscale;
  // db2: sum over the 16 lanes c of the same n
#pragma unroll
  for (int j = 0; j < 8; ++j) db2[j] = row_sum16(db2[j]);
  if (c == 0)
#pragma unroll
    for (int j = 0; j < 8; ++j) N.part_b2[(size_t)blockIdx.x * HID + 32 * w + 16 * (j >> 2) + 4 * gq + (j & 3)] = db2[j];
#ifdef RLKS_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tph[4] = F2_NOW() - tq;
  if (l == 0 && blockIdx.x < 128) {
    unsigned long long* o = g_f2_stamps[blockIdx.y][blockIdx.x][w];
    for (int i = 0; i < 5; ++i) o[i] = tph[i];
    o[5] = ts0;
  }
#endif
}

// F2 with H1 in registers (round 6): dW2^T = H1^T dZ2 over the workgroup's rows, eight waves of 32
// hidden units k x 256 outputs n (8 v_mfma_f32_32x32x16_f16 tiles, 128 accumulator registers, two
// waves per SIMD).  Wave w's A operand is H1 of its own hidden units k = 32 w + (l & 31), taken from
// its Z1 = Xa W1a^T accumulator as it stands: the accumulator's rows acc_row(8 s + j) are the K order
// perm(s, h, j) in which k_sf_dw2's transposed reads deliver the dZ2 chunk, so that image is this
// kernel's B operand unchanged.  No H1 image and no ping-pong between wave halves (k_sf_dw2's phases,
// bound by their pairing): every wave issues its MFMAs of chunk c beside its own
// production of chunk c + 1 (its share of the dZ2 image, its H1), one barrier per chunk.  Each wave
// holds 4 consecutive k of one n per accumulator quad, so the partials are written in [k / 4][n][4]
// order (16-byte stores, 512 contiguous bytes per half-wave); the reduce maps them back
// (RedTask::kq).
constexpr int F2R_ABUF = 2 * F2_APLANE;
#ifndef F2R_DIAG
#define F2R_DIAG 0  // (timing-only diagnostic builds, wrong gradients: 1 no partial stores, 2 no MFMAs, 3 no production)
#endif  // halves per buffer: the dZ2 image's hi and lo planes
template <int KD, int P>
__global__ __launch_bounds__(F2_THREADS) void k_sf_dw2r(SfArgs g) {
  const SfNet& N = g.n[blockIdx.y];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sm = reinterpret_cast<_Float16*>(lds);  // [2 buf][F2R_ABUF]
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = l & 15, gq = l >> 4, r = l & 31, h = l >> 5;
  int t0 = blockIdx.x * g.tiles_per_split, t1 = t0 + g.tiles_per_split;
  if (!dcheck(t1 <= g.M / 32, DC_SGD_TILE, t1)) t0 = t1 = 0;
  const int nk = t1 - t0;

  // F1a's X and dZ2 exponents of the workgroup's 16-row tiles -> LDS; E = min e_T (as k_sf_dw2)
  int* sEx = reinterpret_cast<int*>(sm + 2 * F2R_ABUF);
  int* sEd = sEx + F2_MAX_TILES;
  int emin = 120;
  for (int i = tid; i < 2 * nk; i += F2_THREADS) {
    sEx[i] = N.tile_ex[2 * t0 + i];
    const int e = N.tile_edz[2 * t0 + i];
    sEd[i] = e;
    emin = min(emin, e);
  }
  __shared__ float s_emin[F2_THREADS / 64];
  emin = (int)-wave_max((float)-emin);
  if (l == 0) s_emin[w] = (float)emin;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < F2_THREADS / 64; ++i) emin = min(emin, (int)s_emin[i]);
  const int E = __builtin_amdgcn_readfirstlane(emin);
  const float ssgn = tile_sign(blockIdx.x);  // odd splits: products on -H1, partial negated back
  const float unscale = ssgn * pow2(-14 - E);

  // B fragments (k_sf_dw2's A reads): output block n = 32 ob + r, K order of k-step s as above
  const int aq = (4 * ((l >> 4) & 1) + (l & 3)) ^ (2 * h);
  const int bbase = (4 * h + ((l & 15) >> 2)) * F2_AROW + 4 * aq;
  const int bbase8 = (4 * h + ((l & 15) >> 2) + 8) * F2_AROW + 4 * (aq ^ 4);
  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
  auto mfma_chunk = [&](const _Float16* b, const h8 (&hh)[2], const h8 (&hl)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) {
        const _Float16* pb = b + bbase + s * 16 * F2_AROW + 32 * ob;
        const _Float16* pb8 = b + bbase8 + s * 16 * F2_AROW + 32 * ob;
        const h4 a0 = tr_read(pb), a1 = tr_read(pb8);
        const h4 c0 = tr_read(pb + F2_APLANE), c1 = tr_read(pb8 + F2_APLANE);
        const h8 bh = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
        const h8 bl = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7);
        acc[ob] = mmaP<P>(hh[s], hl[s], bh, bl, acc[ob]);
      }
  };

  // dZ2 pieces (k_sf_dw2's load_dz / store_dz: wave w moves n-step w of the chunk's two tiles)
  const __amdgpu_buffer_rsrc_t dz_rsrc = __builtin_amdgcn_make_buffer_rsrc(N.dz2s, (short)0, 0x7fffffff, 0x00020000);
  const int dz_lane = 2 * (w * 1024 + l * 8);
  h8 dp[4];
  auto load_dz = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dp[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(
                                         dz_rsrc, dz_lane, t * (32 * HID * 4) + (i >> 1) * (16 * HID * 4) + (i & 1) * 1024, 0));
  };
  float db2[8] = {};
  auto store_dz = [&](_Float16* img, float s0, float s1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float sc = (i >> 1) ? s1 : s0;
#pragma unroll
      for (int j = 0; j < 8; ++j) db2[j] = fmaf((float)dp[i][j], sc, db2[j]);
      const int off = (i & 1) * F2_APLANE + (16 * (i >> 1) + c) * F2_AROW + 32 * w;
      const int sw = 2 * ((c >> 2) & 3);
      *reinterpret_cast<h4*>(img + off + 4 * (gq ^ sw)) = __builtin_shufflevector(dp[i], dp[i], 0, 1, 2, 3);
      *reinterpret_cast<h4*>(img + off + 4 * ((gq + 4) ^ sw)) = __builtin_shufflevector(dp[i], dp[i], 4, 5, 6, 7);
    }
  };

  // H1 of the chunk for this wave's hidden units kh = 32 w + r: Z1 = Xa W1a^T on
  // v_mfma_f32_32x32x8_f16 (as k_sf_dw2), tanh, split into the two k-steps' A fragments
  constexpr int KB = KD / 8;
  const int kh = 32 * w + r;
  h4 wh[KB], wl[KB];
  auto load_w1 = [&]() {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      wh[kb] = *reinterpret_cast<const h4*>(N.w1h + kh * KD + 8 * kb + 4 * h);
      wl[kb] = *reinterpret_cast<const h4*>(N.w1l + kh * KD + 8 * kb + 4 * h);
    }
  };
  if constexpr (KB <= 2) load_w1();
  const float inv_w1 = N.sc[1];
  // the chunk's Xa rows as F1a split them (SfArgs::xsp: tile 2t + s at 2^e_T and sign (-1)^s): lane row
  // r, columns 8 kb + 4 h + 0..3, the Z1 MFMA's A fragment as loaded (no split here)
  h4 xrh[KB], xrl[KB];
  int2 xe, de;
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(g.xsp, (short)0, 0x7fffffff, 0x00020000);
  const int xlo = 2 * g.M * KD;  // bytes from the hi plane to the lo plane
  auto load_x = [&](int t) {
    xe = *reinterpret_cast<const int2*>(sEx + 2 * (t - t0));
    de = *reinterpret_cast<const int2*>(sEd + 2 * (t - t0));
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int off = 2 * (r * KD + 8 * kb + 4 * h);
      xrh[kb] = __builtin_bit_cast(h4, __builtin_amdgcn_raw_buffer_load_b64(x_rsrc, off, 2 * t * 32 * KD, 0));
      xrl[kb] = __builtin_bit_cast(h4, __builtin_amdgcn_raw_buffer_load_b64(x_rsrc, off + xlo, 2 * t * 32 * KD, 0));
    }
  };
  auto make_h1 = [&](h8 (&hh)[2], h8 (&hl)[2]) {
    if constexpr (KB > 2) load_w1();
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if constexpr (P != 1) {
        z = __builtin_amdgcn_mfma_f32_32x32x8f16(xrl[kb], wh[kb], z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x8f16(xrh[kb], wl[kb], z, 0, 0, 0);
      }
      z = __builtin_amdgcn_mfma_f32_32x32x8f16(xrh[kb], wh[kb], z, 0, 0, 0);
    }
    // k-step s = rows of tile 2t + s: Z1 unscaled by that tile's X exponent and sign; H1 at
    // 2^(14 + E - e_T) (the odd tile's dZ2 arrives negated: -hs1), times this split's sign
    const float kz0 = inv_w1 * pow2(-xe.x) * SF_2LOG2E, kz1 = -inv_w1 * pow2(-xe.y) * SF_2LOG2E;
    const float hs0 = ssgn * pow2(14 + E - de.x), hs1 = -ssgn * pow2(14 + E - de.y);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float hs = s ? hs1 : hs0, kz = s ? kz1 : kz0;
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = fmaf(-2.f * hs, tanh_r(z[8 * s + j] * kz), hs);
      split8v(x, hh[s], hl[s]);
    }
  };
  auto barrier = [&]() {  // (k_sf_dw2's phase barrier: LDS stores drained, prefetches left in flight)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  h8 hh[2], hl[2];
  if (nk > 0) {
    load_dz(t0);
    load_x(t0);
    store_dz(sm, pow2(-de.x), -pow2(-de.y));
    make_h1(hh, hl);
    load_x(min(t0 + 1, t1 - 1));
    load_dz(min(t0 + 1, t1 - 1));
  }
  __syncthreads();
  // (An interleave of 1 MFMA with 4-6 VALU and LDS reads by sched_group_barrier: 50 -> 51 us at c4;
  // the opposite orders below before the -fno-slp-vectorize build: 50 -> 60 us, 13 registers spilled;
  // the next chunk's Z1 MFMAs issued ahead of the chunk's 48 (and interleaved 1 : 5 with the VALU):
  // within noise; nontemporal partial stores: the reduce 9.4 -> 12.5 us; profiles/r06_f2regs/sched,
  // order, zfirst, nt.)
  // At 16 columns of Xa (2 and 4 actions) waves 4-7 produce before their MFMAs and waves 0-3 after, so
  // that each SIMD pairs one wave's production with the other's MFMAs (c4 F2 50.0 -> 47.6 µs, same box,
  // profiles/r06_order); at KD = 32 that form spills 23 registers and is slower (c3 F2 60 -> 63 µs), so
  // both halves keep the one order there.
  if (KD == 16 && w >= 4) {
    for (int ci = 0; ci < nk; ++ci) {
      const bool counted = ci + 1 < nk;
      const float s0 = counted ? pow2(-de.x) : 0.f, s1 = counted ? -pow2(-de.y) : 0.f;
      h8 nh[2], nl[2];
      store_dz(sm + ((ci + 1) & 1) * F2R_ABUF, s0, s1);
      make_h1(nh, nl);
      load_x(min(t0 + ci + 2, t1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      load_dz(min(t0 + ci + 2, t1 - 1));
#if F2R_DIAG != 2
      mfma_chunk(sm + (ci & 1) * F2R_ABUF, hh, hl);
#endif
      barrier();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        hh[s] = nh[s];
        hl[s] = nl[s];
      }
    }
  } else
  for (int ci = 0; ci < nk; ++ci) {
#if F2R_DIAG != 2
    mfma_chunk(sm + (ci & 1) * F2R_ABUF, hh, hl);
#endif
    // chunk ci + 1 (past the end: the last chunk again, into the idle buffer, uncounted -- unconditional,
    // so that this production shares the MFMAs' basic block)
    const bool counted = ci + 1 < nk;
    const float s0 = counted ? pow2(-de.x) : 0.f, s1 = counted ? -pow2(-de.y) : 0.f;
    h8 nh[2], nl[2];
#if F2R_DIAG != 3
    store_dz(sm + ((ci + 1) & 1) * F2R_ABUF, s0, s1);
    make_h1(nh, nl);
#else
    nh[0] = hh[1]; nh[1] = hh[0]; nl[0] = hl[1]; nl[1] = hl[0];
#endif
    load_x(min(t0 + ci + 2, t1 - 1));
    __builtin_amdgcn_sched_barrier(0);
    load_dz(min(t0 + ci + 2, t1 - 1));
    barrier();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      hh[s] = nh[s];
      hl[s] = nl[s];
    }
  }

  // partials [k / 4][n][4]: accumulator quad t of tile ob = k 32 w + 8 t + 4 h + 0..3, n = 32 ob + r
  float* out = N.part_w2 + (size_t)blockIdx.x * SF_W2_PSTRIDE;
#pragma unroll
  for (int ob = 0; ob < 8; ++ob)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const v4f v = {acc[ob][4 * t] * unscale, acc[ob][4 * t + 1] * unscale, acc[ob][4 * t + 2] * unscale,
                     acc[ob][4 * t + 3] * unscale};
#if F2R_DIAG != 1
      *reinterpret_cast<v4f*>(out + ((size_t)(8 * w + 2 * t + h) * HID + 32 * ob + r) * 4) = v;
#else
      if (v[0] == 1.2345f) out[0] = v[1];  // (keeps the accumulators live)
#endif
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) db2[j] = row_sum16(db2[j]);
  if (c == 0)
#pragma unroll
    for (int j = 0; j < 8; ++j) N.part_b2[(size_t)blockIdx.x * HID + 32 * w + 16 * (j >> 2) + 4 * gq + (j & 3)] = db2[j];
}


// ----------------------------------------------------------------------------- forward only
// Rollout forward of both nets on 16-row tiles (the F1a schedule above without the loss and the
// backward epilogue): logits [M][A] of the policy net and values [M] of the value net for M
// observation rows of stride D.  The node-level rollout (ppo.hip node_rollout) runs it once per step
// and for the bootstrap; k_sf_roll's 32-row tiles needed 256 registers per wave (2 waves per SIMD),
// here a wave holds one 16 x 256 accumulator block and four waves share a SIMD.
// Rows past M (the last tile of a ragged M) are computed on row M - 1 and not stored.
__device__ __forceinline__ int x_frag_rows(const float* __restrict__ x, int row, int D, int g, h8& xh, h8& xl) {
  const float* xr = x + (size_t)row * D;
  float xv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) xv[j] = xa_elem(xr, 8 * g + j, D);
  float xm = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) xm = fmaxf(xm, fabsf(xv[j]));
  const int ex = sf_exp(wave_max(xm));
  split8(xv, 0, pow2(ex), xh, xl);
  return ex;
}

template <int A_, int KD, int W>
constexpr int fwd16_lds_bytes() {
  return 4 * H16 * 2 + 2 * HID * KD * 2 + (HID + A_ * HID) * 4;
}

template <int A_, int NET, int KD, int W>
__device__ __forceinline__ void fwd16_body(const SfFwdArgs& g) {
  constexpr int NTHR = 64 * W;
  const SfNet& N = g.n[NET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sCh = reinterpret_cast<_Float16*>(lds);  // [2 buf][2 hi/lo][128][32]
  _Float16* sW1 = sCh + 4 * H16;                      // [2 hi/lo][HID][KD]
  float* sB2 = lds + (4 * H16 * 2 + 2 * HID * KD * 2) / 4;
  float* sW3 = sB2 + HID;

  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), c = l & 15, gq = l >> 4;
  const int row0 = (blockIdx.x * W + w) * 16;
  const int row = min(row0 + c, g.M - 1);

  hc_dma<W>(N.w2ph, N.w2pl, 0, 0, sCh, w, l);
  for (int i = tid; i < HID; i += NTHR) sB2[i] = N.b2[i] * SF_2LOG2E;
  for (int i = tid; i < A_ * HID; i += NTHR) sW3[i] = N.w3[i];
  w1_stage<KD, NTHR>(N, sW1, tid);
  h8 xh, xl;
  const int ex = x_frag_rows(g.x, row, g.D, gq, xh, xl);
  const float k_z1 = N.sc[1] * pow2(-ex) * SF_2LOG2E;
  vm_drain();
  __syncthreads();

  f4 acc[16];
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) acc[nt] = f4zero();
  h8 bh, bl;
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      const int st = 2 * t + ph;
      if (st < 15) hc_dma<W>(N.w2ph, N.w2pl, 128 * (ph ^ 1), 32 * (t + ph), sCh + (ph ^ 1) * 2 * H16, w, l);
      if (ph == 0) {
        f4 z[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          h8 wh, wl;
          w1_frag<KD>(sW1, 2 * t + b, c, gq, wh, wl);
          z[b] = mm16x3(wh, wl, xh, xl, f4zero());
        }
        float hv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = fmaf(-2.f * SF_H1_SCALE, tanh_r(z[j >> 2][j & 3] * k_z1), SF_H1_SCALE);
        split8(hv, 0, 1.f, bh, bl);
      }
      const _Float16* buf = sCh + ph * 2 * H16;
      h8 ch, cl;
      hc_frag(buf, 0, c, gq, ch, cl);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        h8 nh, nl;
        if (j < 7) hc_frag(buf, j + 1, c, gq, nh, nl);
        __builtin_amdgcn_sched_barrier(0);
        acc[8 * ph + j] = mm16x3(ch, cl, bh, bl, acc[8 * ph + j]);
        __builtin_amdgcn_sched_barrier(0);
        if (j < 7) { ch = nh; cl = nl; }
      }
      vm_drain();
      __syncthreads();
    }
  }

  const float k_z2 = N.sc[3] / SF_H1_SCALE * SF_2LOG2E;
  float out[A_];
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] = 0.f;
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) {
    const int n0 = 16 * nt + 4 * gq;
    const float4 bb = *reinterpret_cast<const float4*>(sB2 + n0);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) hv[i] = fmaf(-2.f, tanh_r(fmaf(acc[nt][i], k_z2, bv[i])), 1.f);
#pragma unroll
    for (int a = 0; a < A_; ++a) {
      const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
      out[a] = fmaf(hv[0], t.x, out[a]);
      out[a] = fmaf(hv[1], t.y, out[a]);
      out[a] = fmaf(hv[2], t.z, out[a]);
      out[a] = fmaf(hv[3], t.w, out[a]);
    }
  }
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] = sum_rows4(out[a]) + N.b3[a];
  // every row group holds the row's outputs: group gq stores actions gq, gq + 4, ...
  float* dst = g.out[NET];
  if (dst && row0 + c < g.M)
#pragma unroll
    for (int a = 0; a < A_; ++a)
      if ((a & 3) == gq) dst[(size_t)(row0 + c) * A_ + a] = out[a];
}

template <int A_, int KD, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_sf_fwd16(SfFwdArgs g) {
  if (blockIdx.y + g.net0 == 0) fwd16_body<A_, 0, KD, W>(g);
  else fwd16_body<1, 1, KD, W>(g);
}

// ----------------------------------------------------------------------------- launchers
#ifdef RLKS_STAMPS
extern "C" int rlks_dbg_fa_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fa_stamps), sizeof(g_fa_stamps)) == hipSuccess ? 0 : 1;
}
extern "C" int rlks_dbg_f2_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_f2_stamps), sizeof(g_f2_stamps)) == hipSuccess ? 0 : 1;
}
#endif

hipEvent_t* g_kernel_events = nullptr;

int launch_sf_prep(const SfPrepArgs& a, hipStream_t s) {
  if (!a.skip_wmax) {
    hipLaunchKernelGGL(k_sf_wmax, dim3(2, 32), dim3(256), 0, s, a);
    RLKS_LAUNCHED();
  }
  if (a.write_roll) hipLaunchKernelGGL(k_sf_split, dim3(2, 64), dim3(256), 0, s, a);
  else launch_timed(KEV_SPLIT, k_sf_split, dim3(2, 64), dim3(256), 0, s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

template <int A_, int KD, int P>
static int launch_f1_net_p(SfArgs a, int net0, int nets, hipStream_t s, int halves) {
  constexpr int W = SF_F1_W;
  a.net0 = net0;
  const dim3 grid(a.M / (16 * W) * nets);  // (f1_net_group)
  if (halves == SF_F1_FUSED) {  // one fused kernel
    constexpr int WF = SF_F1F_W;
    launch_timed(KEV_F1A, k_sf_f1<A_, KD, WF, P>, dim3(a.M / (16 * WF) * nets), dim3(64 * WF), f1_lds_bytes<A_, KD, WF>(),
                 s, a);
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
  if (halves & 1) {  // pi's LDS (A_ >= 1) covers the value net's
    launch_timed(KEV_F1A, k_sf_fwd<A_, KD, W, P>, grid, dim3(64 * W), f1a_lds_bytes<A_, KD, W>(), s, a);
    RLKS_LAUNCHED();
  }
  if (halves & 2) {
    launch_timed(KEV_F1B, k_sf_bwd<KD, 3 * A_ + 1, W, P>, grid, dim3(64 * W), f1b_lds_bytes<KD>(), s, a);
    RLKS_LAUNCHED();
  }
  return RLKS_OK;
}
template <int A_, int KD>
static int launch_f1_net(const SfArgs& a, int net0, int nets, hipStream_t s, int halves) {
  return a.products == 1 ? launch_f1_net_p<A_, KD, 1>(a, net0, nets, s, halves)
                         : launch_f1_net_p<A_, KD, 3>(a, net0, nets, s, halves);
}

// obs_dim = 3 x clusters: C = 2, 4, 8 -> D = 6, 12, 24 (D + 1 <= 8, 16, 32)
int sf_kd(int D) { return D + 1 <= 16 ? 16 : 32; }

int launch_sf_f1(const SfArgs& a, int net0, int nets, int A, hipStream_t s, int halves) {
  RLKS_REQUIRE(a.M % SF_ROWS == 0, RLKS_ERR_ARG, "split-fp16 SGD step: rows must be a multiple of 256");
  RLKS_REQUIRE(a.D == 3 * A, RLKS_ERR_UNSUPPORTED, "split-fp16 SGD step expects obs_dim = 3 x n_actions");
  switch (A) {
    case 2: return launch_f1_net<2, 16>(a, net0, nets, s, halves);
    case 4: return launch_f1_net<4, 16>(a, net0, nets, s, halves);
    case 8: return launch_f1_net<8, 32>(a, net0, nets, s, halves);
    default: return fail(RLKS_ERR_UNSUPPORTED, "split-fp16 head is built for 2, 4 or 8 actions");
  }
}

bool sf_f2_regs() {
  const char* e = getenv("RLKS_F2_IMAGE");  // (read per call: tests switch it within a process)
  return !(e && e[0] == '1');
}

int launch_sf_dw2(const SfArgs& a, int splits, hipStream_t s) {
  RLKS_REQUIRE(a.tiles_per_split <= F2_MAX_TILES / 2, RLKS_ERR_ARG, "split-fp16 F2: too many row chunks per split");
  if (sf_f2_regs()) {
    const size_t lds = (size_t)2 * F2R_ABUF * sizeof(_Float16) + 2 * F2_MAX_TILES * sizeof(int);  // 76 KB
    const bool p1 = a.products == 1;
    if (sf_kd(a.D) == 16) {
      if (p1) launch_timed(KEV_F2, k_sf_dw2r<16, 1>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
      else launch_timed(KEV_F2, k_sf_dw2r<16, 3>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
    } else {
      if (p1) launch_timed(KEV_F2, k_sf_dw2r<32, 1>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
      else launch_timed(KEV_F2, k_sf_dw2r<32, 3>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
    }
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
  const size_t lds = (size_t)2 * F2_BUF * sizeof(_Float16) + 2 * F2_MAX_TILES * sizeof(int);  // 140 KB
  const bool p1 = a.products == 1;
  if (sf_kd(a.D) == 16) {
    if (p1) launch_timed(KEV_F2, k_sf_dw2<16, 1>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
    else launch_timed(KEV_F2, k_sf_dw2<16, 3>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
  } else {
    if (p1) launch_timed(KEV_F2, k_sf_dw2<32, 1>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
    else launch_timed(KEV_F2, k_sf_dw2<32, 3>, dim3(splits, 2), dim3(F2_THREADS), lds, s, a);
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}


template <int A_, int KD>
static int launch_fwd16_t(const SfFwdArgs& a, int net0, int nets, hipStream_t s) {
  constexpr int W = SF_FWD_W;
  SfFwdArgs b = a;
  b.net0 = net0;
  hipLaunchKernelGGL((k_sf_fwd16<A_, KD, W>), dim3((a.M + 16 * W - 1) / (16 * W), nets), dim3(64 * W),
                     (fwd16_lds_bytes<A_, KD, W>()), s, b);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int launch_sf_fwd16(const SfFwdArgs& a, int A, hipStream_t s) {
  RLKS_REQUIRE(a.M > 0 && a.D > 0 && a.D + 1 <= 32, RLKS_ERR_UNSUPPORTED, "split-fp16 forward: obs_dim in [1, 31]");
  const int net0 = a.out[0] ? 0 : 1, nets = (a.out[0] ? 1 : 0) + (a.out[1] ? 1 : 0);
  if (nets == 0) return RLKS_OK;
  if (nets == 1 && net0 == 0) return fail(RLKS_ERR_ARG, "split-fp16 forward: the policy net alone is not a launch shape");
  const bool k16 = sf_kd(a.D) == 16;
  switch (A) {
    case 2: return k16 ? launch_fwd16_t<2, 16>(a, net0, nets, s) : launch_fwd16_t<2, 32>(a, net0, nets, s);
    case 4: return k16 ? launch_fwd16_t<4, 16>(a, net0, nets, s) : launch_fwd16_t<4, 32>(a, net0, nets, s);
    case 8: return k16 ? launch_fwd16_t<8, 16>(a, net0, nets, s) : launch_fwd16_t<8, 32>(a, net0, nets, s);
    default: return fail(RLKS_ERR_UNSUPPORTED, "split-fp16 forward is built for 2, 4 or 8 actions");
  }
}

}  // namespace rlks
