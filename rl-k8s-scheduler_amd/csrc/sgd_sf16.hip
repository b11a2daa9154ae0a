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

#ifndef RLKS_F1B_ONEPASS
#define RLKS_F1B_ONEPASS 1
#endif
#ifndef RLKS_F2_PHASES
#define RLKS_F2_PHASES 1
#endif
constexpr int SF_ROWS = 256;        // minibatch rows must be a multiple of this
constexpr int SF_CH = 8192;         // halves per staged chunk (per hi / lo array)
constexpr float SF_H1_SCALE = 16384.f;  // tanh outputs (|h| < 1) scaled by 2^14
// max |dZ2| of an SGD step as SF_DZ_SLOTS partial maxima, one 64-byte line apart: F1a waves update
// the slot of (tile mod SF_DZ_SLOTS), F2 takes the max over them.  One address for all 4,096 tile
// atomics serialised at its L2 channel and cost F1a ~12 us of 93 (profiles/r02d/f1a_atomic_xp).
__device__ __forceinline__ unsigned* dz_slot(unsigned* base, int tile) {
  return base + (tile & (SF_DZ_SLOTS - 1)) * SF_DZ_STRIDE;
}

__device__ __forceinline__ int sf_perm(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }

__device__ __forceinline__ f32x16 mma(h8 a, h8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// (ah + al)(bh + bl) - al bl, small terms first
__device__ __forceinline__ f32x16 mma3(h8 ah, h8 al, h8 bh, h8 bl, f32x16 c) {
  c = mma(al, bh, c);
  c = mma(ah, bl, c);
  return mma(ah, bh, c);
}

__device__ __forceinline__ void split1(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}
// elements [o, o + 8) of v, times s
template <int N>
__device__ __forceinline__ void split8(const float (&v)[N], int o, float s, h8& hi, h8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    _Float16 a, b;
    split1(v[o + j] * s, a, b);
    hi[j] = a;
    lo[j] = b;
  }
}
__device__ __forceinline__ void split16(const f32x16& v, int o, float s, h8& hi, h8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    _Float16 a, b;
    split1(v[o + j] * s, a, b);
    hi[j] = a;
    lo[j] = b;
  }
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
__device__ __forceinline__ float tanh_abs(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.885390081777927f);
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

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
    const int src = 32 * blk + sf_perm(rem >> 4, (rem >> 3) & 1, rem & 7);
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
    for (int i = 0; i < SF_DZ_SLOTS; ++i) N.dzmax[i * SF_DZ_STRIDE] = 0u;
  }
  if (blockIdx.y == 0) {  // the other parity's entries: the coming fused reduce writes some of them
    float4* z = reinterpret_cast<float4*>(N.pmax + (g.parity ^ 1) * 2 * SF_PMAX);
    for (int i = tid; i < 2 * SF_PMAX / 4; i += 256) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (blockIdx.y == 0 && tid == 0) N.tag[g.parity ^ 1] = 0u;
}

// ----------------------------------------------------------------------------- F1
// Weight chunks staged through registers: a wave loads its share of chunk c + 1 at the start of
// a step (global_load_dwordx4 into 32 / W x 16 B per lane) and writes it to the idle LDS buffer at
// the end.  (LDS-DMA, global_load_lds, would save the registers, but while one is in flight the
// compiler waits for every outstanding LDS read, lgkmcnt(0), before any LDS result is used, which
// serialises the fragment pipeline below.)  Chunk c < 8: w2p columns [32c, 32c+32) of all 256
// rows (Z2 loop, k-tile c); c >= 8: w2t columns [32(c-8), +32) of all 256 rows (dH1 loop, n-tile
// c - 8).  Both are [256 rows][32 halves] images with 16-byte pieces XOR-swizzled by
// (row >> 2) & 3, read by sf_frag.  A chunk is 2 x 1024 slots of 16 B (hi, lo) = 32 blocks of 64;
// wave w of W moves blocks (32/W) w + i.
template <int W>
__device__ __forceinline__ void chunk_load(const SfNet& N, int c, int w, int l, v4u (&v)[32 / W]) {
  const bool p = c < 8;
  const int col = 32 * (p ? c : c - 8);
#pragma unroll
  for (int i = 0; i < 32 / W; ++i) {
    const int blk = (32 / W) * w + i, arr = blk >> 4, sig = (blk & 15) * 64 + l;
    const int row = sig >> 2, pc = (sig & 3) ^ ((row >> 2) & 3);
    const _Float16* src = (p ? (arr ? N.w2pl : N.w2ph) : (arr ? N.w2tl : N.w2th)) + row * HID + col + 8 * pc;
    v[i] = *reinterpret_cast<const v4u*>(src);
  }
}
template <int W>
__device__ __forceinline__ void chunk_store(_Float16* buf, int w, int l, const v4u (&v)[32 / W]) {
#pragma unroll
  for (int i = 0; i < 32 / W; ++i) {
    const int blk = (32 / W) * w + i, arr = blk >> 4;
    *reinterpret_cast<v4u*>(buf + arr * SF_CH + ((blk & 15) * 64 + l) * 8) = v[i];
  }
}
// the (hi, lo) fragments of one 32-row block of a chunk for both k-steps s: lane (r, h) of row
// `row` gets halves [16 s + 8 h, +8) of its 32
__device__ __forceinline__ void sf_frag(const _Float16* buf, int row, int h, h8 (&f)[2][2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int off = row * 32 + 8 * ((2 * s + h) ^ ((row >> 2) & 3));
    f[s][0] = *reinterpret_cast<const h8*>(buf + off);
    f[s][1] = *reinterpret_cast<const h8*>(buf + SF_CH + off);
  }
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// PPO loss of one row (RLlib ppo_torch_policy semantics): d loss / d logits (pi) or
// d loss / d value (vf), scaled by 1 / global rows, and the row's [policy loss, vf loss, kl,
// entropy] terms
template <int A_, int NET>
__device__ __forceinline__ void sf_loss(const SfArgs& g, const float (&out)[A_], int row, float (&dl)[A_],
                                        float (&st)[4]) {
  const int D = g.D;
  const float* rec = g.x + (size_t)row * g.x_stride;
  const float inv_count = g.dyn[RLKS_DYN_INV_COUNT];
  const int Ap = g.A_pi;
  st[0] = st[1] = st[2] = st[3] = 0.f;
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
    const float dr = -adv * (w1 + (1.f - w1) * inr) * ratio;
    const float klc = g.dyn[RLKS_DYN_KL_COEFF];
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
    const float diff = out[0] - rec[D + Ap + 1];
    const float sq = diff * diff;
    st[1] = fminf(sq, g.co.vf_clip_param);
    dl[0] = (sq <= g.co.vf_clip_param) ? g.co.vf_loss_coeff * 2.f * diff * inv_count : 0.f;
  }
}

#ifdef RLKS_STAMPS
// diagnostic build only (tools/stamps.sh): per-wave phase clocks of F1, [net][tile][phase]
__device__ unsigned long long g_sf_stamps[2][4096][8];
#define SF_STAMP(i) \
  if (l == 0 && tile < 4096) g_sf_stamps[NET][tile][i] = __builtin_amdgcn_s_memtime()
// loop-internal clocks: Z2 chunk 3 (top, after the MFMA steps, after the barrier) and dH1 n-tile 3
__device__ unsigned long long g_sf_stamps2[2][4096][8];
#define SF_STAMP2(i) \
  if (l == 0 && tile < 4096) g_sf_stamps2[NET][tile][i] = __builtin_amdgcn_s_memtime()
// F1a (k_sf_fwd) phase clocks [net][tile][phase]; slot 7 = HW_ID | XCC_ID << 32
__device__ unsigned long long g_fa_stamps[2][4096][8];
#define FA_STAMP(i) \
  if (l == 0 && tile < 4096) g_fa_stamps[NET][tile][i] = __builtin_amdgcn_s_memtime()
#define FA_HWID()                                                                                   \
  if (l == 0 && tile < 4096)                                                                        \
  g_fa_stamps[NET][tile][7] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |       \
                              ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32)
#else
#define SF_STAMP(i)
#define SF_STAMP2(i)
#define FA_STAMP(i)
#define FA_HWID()
#endif

// W waves per workgroup, one 32-row tile each; one wave per SIMD (waves_per_eu 1) so that every
// wave has the full 512-register file: dZ2^T stays split in registers through the dH1 loop and
// the LDS fragments of the next MFMA step are in flight during the current one.
template <int A_, int NET, int KD, int NG, int W>
__device__ __forceinline__ void sf_fwdbwd_body(const SfArgs& g) {
  constexpr int NTHR = 64 * W;
  constexpr int KS = KD / 16;   // k-steps of the first layer
  // NG: accumulator row groups (8 rows each) holding the rows d <= D of dW1a^T.  Each k-tile's
  // dW1a^T block goes to an LDS slot (the epilogue reuses the chunk buffers) and is summed over the
  // W waves there, so no accumulator outlives its k-tile.
  constexpr int DWR = 8 * NG;   // LDS rows per dW1a^T column
  const SfNet& N = g.n[NET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sCh = reinterpret_cast<_Float16*>(lds);  // [2 buf][2 hi/lo][SF_CH]  (64 KB)
  float* sB2 = lds + 2 * SF_CH;                      // [HID]
  float* sW3 = sB2 + HID;                            // [A_][HID]
  _Float16* sW1 = reinterpret_cast<_Float16*>(sW3 + A_ * HID);  // [2 hi/lo][HID k][KD] (swizzled)
  h8* sXT = reinterpret_cast<h8*>(sW1 + 2 * HID * KD);          // [W][2 s][2 hi/lo][64 lanes]

  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int D = g.D, stride = g.x_stride;
  const int tile = blockIdx.x * W + w, row0 = tile * 32;
  SF_STAMP(0);

  {
    v4u cv[32 / W];
    chunk_load<W>(N, 0, w, l, cv);
    chunk_store<W>(sCh, w, l, cv);
  }
  for (int i = tid; i < HID; i += NTHR) sB2[i] = N.b2[i];
  for (int i = tid; i < A_ * HID; i += NTHR) sW3[i] = N.w3[i];

  // ---- this wave's rows: Xa = [X | 1 | 0] fragments, lane row m = r, d = 16ks + 8h + j
  float xv[KS * 8];
  const float* xr = g.x + (size_t)(row0 + r) * stride;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 16 * ks + 8 * h + j;
      xv[ks * 8 + j] = xa_elem(xr, d, D);
    }
  float xm = 0.f;
#pragma unroll
  for (int i = 0; i < KS * 8; ++i) xm = fmaxf(xm, fabsf(xv[i]));
  const int ex = sf_exp(wave_max(xm));
  const float sx = pow2(ex);
  h8 xh[KS], xl[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) split8(xv, ks * 8, sx, xh[ks], xl[ks]);
  const float inv_w1 = N.sc[1], inv_w2 = N.sc[3];
  const int e_w2 = (int)N.sc[5];
  const float inv_z1 = inv_w1 / sx;  // Z1 accumulators carry s_x s_w1

  // W1a (hi, lo) in LDS: row k of KD halves, 16-byte pieces XOR-swizzled by (k >> 3) so that the
  // fragment reads of 16 consecutive rows are conflict-free
  for (int p = tid; p < 2 * HID * KD / 8; p += NTHR) {
    const int arr = p / (HID * KD / 8), q = p - arr * (HID * KD / 8), k = q / (KD / 8), pc = q - k * (KD / 8);
    const uint4 v = *reinterpret_cast<const uint4*>((arr ? N.w1l : N.w1h) + k * KD + 8 * pc);
    *reinterpret_cast<uint4*>(sW1 + arr * HID * KD + k * KD + 8 * (pc ^ ((k >> 3) & 1))) = v;
  }
  h8 wh[KS], wl[KS];
  auto w1_frag = [&](int kt) {
    const int k = 32 * kt + r;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int off = k * KD + 8 * ((2 * ks + h) ^ ((k >> 3) & 1));
      wh[ks] = *reinterpret_cast<const h8*>(sW1 + off);
      wl[ks] = *reinterpret_cast<const h8*>(sW1 + HID * KD + off);
    }
  };
  vm_drain();
  __syncthreads();
  SF_STAMP(1);

  // ---- Z2^T = W2 H1^T over 8 k-tiles; H1^T tile kt recomputed from Xa just before its use
  f32x16 acc[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[nt][q] = 0.f;
  // H1^T tile kt (rows k = 32 kt + perm) as split B fragments; software-pipelined one k-tile
  // ahead so that its MFMA + tanh + split overlap the current tile's 48 MFMAs
  auto h1t_tile = [&](int kt, h8 (&bh)[2], h8 (&bl)[2]) {
    w1_frag(kt);
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) z = mma3(wh[ks], wl[ks], xh[ks], xl[ks], z);
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = tanh_abs(z[q] * inv_z1);
    split16(z, 0, SF_H1_SCALE, bh[0], bl[0]);
    split16(z, 8, SF_H1_SCALE, bh[1], bl[1]);
  };
  h8 bh[2], bl[2];
  h1t_tile(0, bh, bl);
  for (int c = 0; c < 8; ++c) {
    const _Float16* buf = sCh + (c & 1) * 2 * SF_CH;
    v4u cv[32 / W];
    chunk_load<W>(N, c + 1, w, l, cv);
    // n-tile steps fenced by sched_barrier: step nt issues the LDS reads of n-tile nt + 1's W2
    // fragments, then n-tile nt's six MFMAs, so every read has a whole step (192 MFMA cycles) to
    // land and only two fragment sets are live (the register budget goes to the accumulators).
    // The next k-tile's H1^T (kn = c + 1; the last is discarded) is computed in the MFMA shadows.
    if (c == 3) SF_STAMP2(0);
    const int kn = c + 1 < 8 ? c + 1 : 7;
    h8 fc[2][2], fn[2][2], nbh[2], nbl[2];
    f32x16 z;
    sf_frag(buf, r, h, fc);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      if (nt < 7) sf_frag(buf, 32 * (nt + 1) + r, h, fn);
      if (nt == 0) w1_frag(kn);
#ifndef RLKS_Z2_NOFENCE
      __builtin_amdgcn_sched_barrier(0);  // the reads issue before this step's MFMAs
#endif
      if (nt == 1) {
#pragma unroll
        for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) z = mma3(wh[ks], wl[ks], xh[ks], xl[ks], z);
      }
      if (nt >= 2 && nt < 6) {
#pragma unroll
        for (int q = 4 * (nt - 2); q < 4 * (nt - 1); ++q) z[q] = tanh_abs(z[q] * inv_z1);
      }
      if (nt == 6) {
        split16(z, 0, SF_H1_SCALE, nbh[0], nbl[0]);
        split16(z, 8, SF_H1_SCALE, nbh[1], nbl[1]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        acc[nt] = mma(fc[s][1], bh[s], acc[nt]);
        acc[nt] = mma(fc[s][0], bl[s], acc[nt]);
        acc[nt] = mma(fc[s][0], bh[s], acc[nt]);
      }
#ifndef RLKS_Z2_NOFENCE
      __builtin_amdgcn_sched_barrier(0);
#endif
      if (nt < 7)
#pragma unroll
        for (int s = 0; s < 2; ++s) { fc[s][0] = fn[s][0]; fc[s][1] = fn[s][1]; }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) { bh[s] = nbh[s]; bl[s] = nbl[s]; }
    if (c == 3) SF_STAMP2(1);
    chunk_store<W>(sCh + ((c + 1) & 1) * 2 * SF_CH, w, l, cv);
    if (c == 3) SF_STAMP2(2);
    __syncthreads();
    if (c == 3) SF_STAMP2(3);
  }

  SF_STAMP(2);
  // Xa^T values for dW1a^T = Xa^T dZ1 (lane row d = r, m = perm(s, h, j)), loaded before the
  // head so that their latency hides behind it; split after dZ2
  float xtv[16];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = sf_perm(s, h, j);
      xtv[s * 8 + j] = xa_elem(g.x + (size_t)(row0 + m) * stride, r, D);
    }
  // ---- H2^T = tanh(Z2^T + b2), head out[a] = b3 + sum_n W3[a][n] H2[n]
  const float inv_z2 = inv_w2 / SF_H1_SCALE;
  float out[A_];
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] = 0.f;
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int n0 = 32 * nt + 8 * gq + 4 * h;
      const float4 bb = *reinterpret_cast<const float4*>(sB2 + n0);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
      float wv[A_][4];
#pragma unroll
      for (int a = 0; a < A_; ++a) {
        const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
        wv[a][0] = t.x; wv[a][1] = t.y; wv[a][2] = t.z; wv[a][3] = t.w;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 4 * gq + i;
        const float h2 = tanh_abs(fmaf(acc[nt][q], inv_z2, bv[i]));
        acc[nt][q] = h2;
#pragma unroll
        for (int a = 0; a < A_; ++a) out[a] = fmaf(h2, wv[a][i], out[a]);
      }
    }
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] += __shfl_xor(out[a], 32, 64) + N.b3[a];

  // ---- PPO loss for row m = row0 + r (both half-waves compute it; stats from h = 0)
  float dl[A_];
  float stv[4];
  sf_loss<A_, NET>(g, out, row0 + r, dl, stv);
  const float st_pl = stv[0], st_vf = stv[1], st_kl = stv[2], st_ent = stv[3];

  SF_STAMP(3);
  // ---- per-tile partials straight to HBM: dW3[a][n] = sum_m dl[m][a] H2[m][n] (half-wave
  // reduce), db3, loss stats
#pragma unroll
  for (int a = 0; a < A_; ++a)
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = dl[a] * acc[nt][q];
      const float t = half_wave_reduce16(v, l);
      if ((l & 1) == 0) N.part_w3[((size_t)tile * A_ + a) * HID + 32 * nt + acc_row((l >> 1) & 15, l)] = t;
    }
  {
    float sv[A_ + 4];
#pragma unroll
    for (int a = 0; a < A_; ++a) sv[a] = h ? 0.f : dl[a];
    sv[A_] = h ? 0.f : st_pl; sv[A_ + 1] = h ? 0.f : st_vf; sv[A_ + 2] = h ? 0.f : st_kl; sv[A_ + 3] = h ? 0.f : st_ent;
#pragma unroll
    for (int i = 0; i < A_ + 4; ++i) {
      const float t = wave_sum_f(sv[i]);
      if (l == 0) {
        if (i < A_) N.part_b3[(size_t)tile * A_ + i] = t;
        else N.part_stat[(size_t)tile * 4 + i - A_] = t;
      }
    }
  }

  SF_STAMP(4);
  // ---- dZ2^T = (dl W3) (1 - H2^2): to HBM (F2), tile max |dZ2| (this wave's split + F2's scale)
  float dmx = 0.f;
  {
    // one base per n-tile, so every store of the n-tile takes an immediate offset (< 4 KB)
    float* dst0 = N.dz2t + (size_t)tile * HID * 32 + 4 * h * 32 + r;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        float* dst = dst0 + (size_t)nt * 32 * 32 + (size_t)8 * gq * 32;
        const int n0 = 32 * nt + 8 * gq + 4 * h;
        float wv[A_][4];
#pragma unroll
        for (int a = 0; a < A_; ++a) {
          const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
          wv[a][0] = t.x; wv[a][1] = t.y; wv[a][2] = t.z; wv[a][3] = t.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 4 * gq + i;
          float gsum = 0.f;
#pragma unroll
          for (int a = 0; a < A_; ++a) gsum = fmaf(dl[a], wv[a][i], gsum);
          const float h2 = acc[nt][q];
          const float dz = gsum * (1.f - h2 * h2);
          acc[nt][q] = dz;
          dmx = fmaxf(dmx, fabsf(dz));
          dst[i * 32] = dz;
        }
      }
  }
  dmx = wave_max(dmx);
  if (l == 0) atomicMax(dz_slot(N.dzmax, tile), __float_as_uint(dmx));
  const int edz = sf_exp(dmx);
  const float sdz = pow2(edz);
  {
    h8 a, b;
    split8(xtv, 0, sx, a, b);
    sXT[(w * 4 + 0) * 64 + l] = a;
    sXT[(w * 4 + 1) * 64 + l] = b;
    split8(xtv, 8, sx, a, b);
    sXT[(w * 4 + 2) * 64 + l] = a;
    sXT[(w * 4 + 3) * 64 + l] = b;
  }
  SF_STAMP(5);
  // ---- dH1 = dZ2 W2, n-tile outer: chunk 8 + nt holds W2's n-tile nt (w2t columns) for every
  // k-tile, the n-tile's dZ2^T accumulator is split into the A fragments just before its MFMAs,
  // and all eight dH1 k-tile accumulators stay live (AGPRs) until the last n-tile.  Fragment
  // reads run one k-tile step ahead of the MFMAs (sched_barrier fences), so only two fragment sets
  // and one n-tile's dZ2 split are live instead of the whole split dZ2^T.
  f32x16 dh[8];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int q = 0; q < 16; ++q) dh[kt][q] = 0.f;
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    const int c = 8 + nt;
    const _Float16* buf = sCh + (c & 1) * 2 * SF_CH;
    v4u cv[32 / W];
    if (nt == 3) SF_STAMP2(4);
    if (nt < 7) chunk_load<W>(N, c + 1, w, l, cv);
    h8 ah[2], al[2], fc[2][2], fn[2][2];
    split16(acc[nt], 0, sdz, ah[0], al[0]);
    split16(acc[nt], 8, sdz, ah[1], al[1]);
    sf_frag(buf, r, h, fc);
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      if (kt < 7) sf_frag(buf, 32 * (kt + 1) + r, h, fn);
      __builtin_amdgcn_sched_barrier(0);  // the reads issue before this step's MFMAs
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        dh[kt] = mma(al[s], fc[s][0], dh[kt]);
        dh[kt] = mma(ah[s], fc[s][1], dh[kt]);
        dh[kt] = mma(ah[s], fc[s][0], dh[kt]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kt < 7)
#pragma unroll
        for (int s = 0; s < 2; ++s) { fc[s][0] = fn[s][0]; fc[s][1] = fn[s][1]; }
    }
    if (nt == 3) SF_STAMP2(5);
    if (nt < 7) chunk_store<W>(sCh + ((c + 1) & 1) * 2 * SF_CH, w, l, cv);
    if (nt == 3) SF_STAMP2(6);
    __syncthreads();
    if (nt == 3) SF_STAMP2(7);
  }
  SF_STAMP(6);
  // ---- dZ1 = dH1 (1 - H1^2) -> dW1a^T = Xa^T dZ1 per k-tile; dZ1 enters the split at
  // 2^(e_dz + e_w2 - 23): |dH1 2^(e_dz + e_w2)| <= 256 2^15 2^15.  Each wave's dW1a^T blocks go to
  // LDS slots in the (now idle) chunk buffers, KPR k-tiles per round, and the workgroup sums them
  // over the W waves in a fixed order after one barrier per round.
  constexpr int SLOT = W * 32 * DWR;                       // floats per k-tile
  constexpr int KPR = (2 * SF_CH) / SLOT >= 8 ? 8 : (2 * SF_CH) / SLOT;  // 64 KB of chunk buffers
  static_assert(KPR >= 1 && 8 % KPR == 0, "dW1 epilogue slots");
  float* sEp = reinterpret_cast<float*>(sCh);
  const int blk = blockIdx.x;
  auto dw1_flush = [&](int kt0) {  // k-tiles kt0 .. kt0 + KPR - 1: (k, d) elements, fixed wave order
    const int nd = D + 1;
    for (int e = tid; e < KPR * 32 * nd; e += NTHR) {
      const int j = e / (32 * nd), e2 = e - j * 32 * nd, kk = e2 / nd, d = e2 - kk * nd, k = 32 * (kt0 + j) + kk;
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < W; ++ww) s += sEp[j * SLOT + (ww * 32 + kk) * DWR + d];
      if (d < D) N.part_w1[((size_t)blk * HID + k) * D + d] = s;
      else N.part_b1[(size_t)blk * HID + k] = s;
    }
  };
  const float sz1 = pow2(-23);
  const float u1 = pow2(23 - ex - edz - e_w2);
  // derivative (1 - H1^2) of k-tile kt, rows m in registers (Z1 = Xa W1a^T)
  auto h1_der = [&](int kt, f32x16& der) {
    w1_frag(kt);
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) z = mma3(xh[ks], xl[ks], wh[ks], wl[ks], z);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float h1 = tanh_abs(z[q] * inv_z1);
      der[q] = 1.f - h1 * h1;
    }
  };
  // dZ1 -> split -> dW1a^T of k-tile kt into this wave's part of slot kt mod KPR
  auto dw1_tile = [&](int kt, const f32x16& dhk, const f32x16& der) {
    f32x16 dz;
#pragma unroll
    for (int q = 0; q < 16; ++q) dz[q] = dhk[q] * der[q];
    h8 zh[2], zl[2];
    split16(dz, 0, sz1, zh[0], zl[0]);
    split16(dz, 8, sz1, zh[1], zl[1]);
    f32x16 wacc, wacc2;
#pragma unroll
    for (int q = 0; q < 16; ++q) { wacc[q] = 0.f; wacc2[q] = 0.f; }
    const h8 x0h = sXT[(w * 4 + 0) * 64 + l], x0l = sXT[(w * 4 + 1) * 64 + l];
    const h8 x1h = sXT[(w * 4 + 2) * 64 + l], x1l = sXT[(w * 4 + 3) * 64 + l];
    wacc = mma(x0l, zh[0], wacc);
    wacc2 = mma(x1l, zh[1], wacc2);
    wacc = mma(x0h, zl[0], wacc);
    wacc2 = mma(x1h, zl[1], wacc2);
    wacc = mma(x0h, zh[0], wacc);
    wacc2 = mma(x1h, zh[1], wacc2);
#pragma unroll
    for (int q = 0; q < 16; ++q) wacc[q] += wacc2[q];
    // rows d = 8g + 4h + 0..3 of column k: 16-byte stores
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      float4 v = {wacc[4 * gq] * u1, wacc[4 * gq + 1] * u1, wacc[4 * gq + 2] * u1, wacc[4 * gq + 3] * u1};
      *reinterpret_cast<float4*>(sEp + (kt % KPR) * SLOT + (w * 32 + r) * DWR + 8 * gq + 4 * h) = v;
    }
  };
  // software-pipelined: the next k-tile's derivative (MFMAs + tanh) overlaps this one's dW1a
  f32x16 der;
  h1_der(0, der);
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    f32x16 nder;
    if (kt < 7) h1_der(kt + 1, nder);
    dw1_tile(kt, dh[kt], der);
    if (kt % KPR == KPR - 1) {
      __syncthreads();
      dw1_flush(kt + 1 - KPR);
      if (kt < 7) __syncthreads();  // slots free for the next round
    }
    if (kt < 7) der = nder;
  }
  SF_STAMP(7);
}

// ----------------------------------------------------------------------------- split F1
// The fused F1 needs ~460 registers (the Z2^T / dZ2^T accumulators plus the eight dH1 k-tile
// accumulators), so it runs one wave per SIMD and its ~9k VALU instructions per tile (tanh and
// splits, head, dW3, dZ2, dZ1) cannot hide behind another wave's MFMAs.  Split at the dZ2 hand-off
// (which F2 needs in HBM anyway), each half fits 256 registers and ~50-80 KB of LDS, so two
// independent workgroups share every CU and each SIMD interleaves two waves in different phases:
//   F1a (k_sf_fwd): Z1, Z2^T = W2 H1^T, head, loss, dW3 / db3 / stats, dZ2^T -> HBM, tile scale;
//   F1b (k_sf_bwd): dH1 = dZ2 W2 (dZ2^T n-tiles from HBM, W2 chunks per k-half), dZ1, dW1a.
// W2 chunks are single-buffered: a step computes from LDS while its successor is loaded into
// registers, then barrier / store / barrier.
// Half-chunk of the Z2 loop: w2p rows n in [128 p, +128), columns [32 c, +32) -> [128][32] image;
// of the dH1 loop: w2t rows k in [128 p, +128), columns [32 nt, +32).  1024 slots of 16 B (hi,
// lo): 16 blocks of 64 lanes, wave w of W moves blocks (16 / W) w + i.
template <int W>
__device__ __forceinline__ void half_load(const _Float16* hi, const _Float16* lo, int p, int col, int w, int l,
                                          v4u (&v)[16 / W]) {
#pragma unroll
  for (int i = 0; i < 16 / W; ++i) {
    const int blk = (16 / W) * w + i, arr = blk >> 3, sig = (blk & 7) * 64 + l;
    const int row = sig >> 2, pc = (sig & 3) ^ ((row >> 2) & 3);
    v[i] = *reinterpret_cast<const v4u*>((arr ? lo : hi) + (128 * p + row) * HID + col + 8 * pc);
  }
}
template <int W>
__device__ __forceinline__ void half_store(_Float16* buf, int w, int l, const v4u (&v)[16 / W]) {
  constexpr int HALF = SF_CH / 2;  // halves per [128][32] image
#pragma unroll
  for (int i = 0; i < 16 / W; ++i) {
    const int blk = (16 / W) * w + i, arr = blk >> 3;
    *reinterpret_cast<v4u*>(buf + arr * HALF + ((blk & 7) * 64 + l) * 8) = v[i];
  }
}
// the same half-chunk by LDS-DMA (no staging registers; the split kernels run two waves per SIMD,
// which hide the LDS waits the DMA brings with it)
template <int W>
__device__ __forceinline__ void half_dma(const _Float16* hi, const _Float16* lo, int p, int col, _Float16* buf, int w,
                                         int l) {
  constexpr int HALF = SF_CH / 2;
#pragma unroll
  for (int i = 0; i < 16 / W; ++i) {
    const int blk = (16 / W) * w + i, arr = blk >> 3, sig = (blk & 7) * 64 + l;
    const int row = sig >> 2, pc = (sig & 3) ^ ((row >> 2) & 3);
    const _Float16* src = (arr ? lo : hi) + (128 * p + row) * HID + col + 8 * pc;
    _Float16* dst = buf + arr * HALF + (blk & 7) * 64 * 8;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}
__device__ __forceinline__ void half_frag(const _Float16* buf, int row, int h, h8 (&f)[2][2]) {
  constexpr int HALF = SF_CH / 2;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int off = row * 32 + 8 * ((2 * s + h) ^ ((row >> 2) & 3));
    f[s][0] = *reinterpret_cast<const h8*>(buf + off);
    f[s][1] = *reinterpret_cast<const h8*>(buf + HALF + off);
  }
}

template <int A_, int NET, int KD, int W>
__device__ __forceinline__ void sf_fwd_body(const SfArgs& g) {
  constexpr int NTHR = 64 * W;
  constexpr int KS = KD / 16;
  const SfNet& N = g.n[NET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sCh = reinterpret_cast<_Float16*>(lds);             // [2 buf][2 hi/lo][128][32] (32 KB)
  float* sB2 = lds + SF_CH;                                     // [HID]
  float* sW3 = sB2 + HID;                                       // [A_][HID]
  _Float16* sW1 = reinterpret_cast<_Float16*>(sW3 + A_ * HID);  // [2 hi/lo][HID k][KD] (swizzled)

  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int D = g.D, stride = g.x_stride;
  const int tile = blockIdx.x * W + w, row0 = tile * 32;
  FA_STAMP(0);
  FA_HWID();

  half_dma<W>(N.w2ph, N.w2pl, 0, 0, sCh, w, l);
  for (int i = tid; i < HID; i += NTHR) sB2[i] = N.b2[i];
  for (int i = tid; i < A_ * HID; i += NTHR) sW3[i] = N.w3[i];
  float xv[KS * 8];
  const float* xr = g.x + (size_t)(row0 + r) * stride;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[ks * 8 + j] = xa_elem(xr, 16 * ks + 8 * h + j, D);
  float xm = 0.f;
#pragma unroll
  for (int i = 0; i < KS * 8; ++i) xm = fmaxf(xm, fabsf(xv[i]));
  const float sx = pow2(sf_exp(wave_max(xm)));
  h8 xh[KS], xl[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) split8(xv, ks * 8, sx, xh[ks], xl[ks]);
  const float inv_z1 = N.sc[1] / sx;
  for (int p = tid; p < 2 * HID * KD / 8; p += NTHR) {
    const int arr = p / (HID * KD / 8), q = p - arr * (HID * KD / 8), k = q / (KD / 8), pc = q - k * (KD / 8);
    const v4u v = *reinterpret_cast<const v4u*>((arr ? N.w1l : N.w1h) + k * KD + 8 * pc);
    *reinterpret_cast<v4u*>(sW1 + arr * HID * KD + k * KD + 8 * (pc ^ ((k >> 3) & 1))) = v;
  }
  h8 wh[KS], wl[KS];
  auto w1_frag = [&](int kt) {
    const int k = 32 * kt + r;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int off = k * KD + 8 * ((2 * ks + h) ^ ((k >> 3) & 1));
      wh[ks] = *reinterpret_cast<const h8*>(sW1 + off);
      wl[ks] = *reinterpret_cast<const h8*>(sW1 + HID * KD + off);
    }
  };
  auto h1t = [&](int kt, h8 (&bh)[2], h8 (&bl)[2]) {
    w1_frag(kt);
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) z = mma3(wh[ks], wl[ks], xh[ks], xl[ks], z);
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = tanh_abs(z[q] * inv_z1);
    split16(z, 0, SF_H1_SCALE, bh[0], bl[0]);
    split16(z, 8, SF_H1_SCALE, bh[1], bl[1]);
  };
  vm_drain();
  __syncthreads();
  FA_STAMP(1);

  // ---- Z2^T = W2 H1^T: 16 steps (k-tile c, n-half p) of 24 MFMAs over double-buffered
  // half-chunks; H1^T of k-tile c is computed at the start of its first step
  f32x16 acc[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[nt][q] = 0.f;
  h8 bh[2], bl[2];
  for (int c = 0; c < 8; ++c) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {  // step 2c + p reads buffer p; the next half-chunk -> buffer p ^ 1
      if (!(c == 7 && p == 1)) half_dma<W>(N.w2ph, N.w2pl, p ^ 1, 32 * (c + p), sCh + (p ^ 1) * SF_CH, w, l);
      if (p == 0) h1t(c, bh, bl);
      const _Float16* buf = sCh + p * SF_CH;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h8 fc[2][2];
        half_frag(buf, 32 * j + r, h, fc);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          acc[4 * p + j] = mma(fc[s][1], bh[s], acc[4 * p + j]);
          acc[4 * p + j] = mma(fc[s][0], bl[s], acc[4 * p + j]);
          acc[4 * p + j] = mma(fc[s][0], bh[s], acc[4 * p + j]);
        }
      }
      vm_drain();
      __syncthreads();
    }
    if (c == 0) FA_STAMP(2);
  }
  FA_STAMP(3);

  // ---- H2^T = tanh(Z2^T + b2), head out[a] = b3 + sum_n W3[a][n] H2[n]
  const float inv_z2 = N.sc[3] / SF_H1_SCALE;
  float out[A_];
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] = 0.f;
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int n0 = 32 * nt + 8 * gq + 4 * h;
      const float4 bb = *reinterpret_cast<const float4*>(sB2 + n0);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
      float h2v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 4 * gq + i;
        h2v[i] = tanh_abs(fmaf(acc[nt][q], inv_z2, bv[i]));
        acc[nt][q] = h2v[i];
      }
      // one action's W3 quad at a time (4 registers live instead of 4 A): the same fma order per
      // out[a] as element-major
#pragma unroll
      for (int a = 0; a < A_; ++a) {
        const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
        out[a] = fmaf(h2v[0], t.x, out[a]);
        out[a] = fmaf(h2v[1], t.y, out[a]);
        out[a] = fmaf(h2v[2], t.z, out[a]);
        out[a] = fmaf(h2v[3], t.w, out[a]);
      }
    }
#pragma unroll
  for (int a = 0; a < A_; ++a) out[a] += __shfl_xor(out[a], 32, 64) + N.b3[a];
  FA_STAMP(4);
  float dl[A_];
  float st[4];
  sf_loss<A_, NET>(g, out, row0 + r, dl, st);
  // ---- dW3 (half-wave reduce), db3, loss stats
#pragma unroll
  for (int a = 0; a < A_; ++a)
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = dl[a] * acc[nt][q];
      const float t = half_wave_reduce16(v, l);
      if ((l & 1) == 0) N.part_w3[((size_t)tile * A_ + a) * HID + 32 * nt + acc_row((l >> 1) & 15, l)] = t;
    }
  {
    float sv[A_ + 4];
#pragma unroll
    for (int a = 0; a < A_; ++a) sv[a] = h ? 0.f : dl[a];
#pragma unroll
    for (int i = 0; i < 4; ++i) sv[A_ + i] = h ? 0.f : st[i];
    float tv[A_ + 4];
#pragma unroll
    for (int i = 0; i < A_ + 4; ++i) tv[i] = wave_sum_f(sv[i]);  // independent chains, interleaved
    if (l == 0) {
#pragma unroll
      for (int i = 0; i < A_ + 4; ++i) {
        if (i < A_) N.part_b3[(size_t)tile * A_ + i] = tv[i];
        else N.part_stat[(size_t)tile * 4 + i - A_] = tv[i];
      }
    }
  }
  FA_STAMP(5);
  // ---- dZ2^T = (dl W3) (1 - H2^2) -> HBM; the tile's split exponent for F1b, max for F2
  float dmx = 0.f;
  {
    // one base per n-tile, so every store of the n-tile takes an immediate offset (< 4 KB)
    float* dst0 = N.dz2t + (size_t)tile * HID * 32 + 4 * h * 32 + r;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        float* dst = dst0 + (size_t)nt * 32 * 32 + (size_t)8 * gq * 32;
        const int n0 = 32 * nt + 8 * gq + 4 * h;
        float gs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < A_; ++a) {
          const float4 t = *reinterpret_cast<const float4*>(sW3 + a * HID + n0);
          gs[0] = fmaf(dl[a], t.x, gs[0]);
          gs[1] = fmaf(dl[a], t.y, gs[1]);
          gs[2] = fmaf(dl[a], t.z, gs[2]);
          gs[3] = fmaf(dl[a], t.w, gs[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 4 * gq + i;
          const float gsum = gs[i];
          const float h2 = acc[nt][q];
          const float dz = gsum * (1.f - h2 * h2);
          dmx = fmaxf(dmx, fabsf(dz));
          dst[i * 32] = dz;
        }
      }
  }
  dmx = wave_max(dmx);
  if (l == 0) {
    atomicMax(dz_slot(N.dzmax, tile), __float_as_uint(dmx));
    N.tile_edz[tile] = sf_exp(dmx);
  }
  FA_STAMP(6);
}

template <int A_, int KD, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_sf_fwd(SfArgs g) {
  if (blockIdx.y + g.net0 == 0) sf_fwd_body<A_, 0, KD, W>(g);
  else sf_fwd_body<1, 1, KD, W>(g);
}

template <int NET, int KD, int NG, int W>
__device__ __forceinline__ void sf_bwd_body(const SfArgs& g) {
  constexpr int NTHR = 64 * W;
  constexpr int KS = KD / 16;
  constexpr int DWR = 8 * NG;
  constexpr int SLOT = W * 32 * DWR;                           // floats per k-tile of dW1a^T partials
  constexpr int KPR = SF_CH / SLOT >= 4 ? 4 : SF_CH / SLOT;   // k-tiles per flush round (32-KB buffers)
  static_assert(KPR >= 1 && 4 % KPR == 0, "dW1 epilogue slots");
  const SfNet& N = g.n[NET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sCh = reinterpret_cast<_Float16*>(lds);             // [2 buf][2 hi/lo][128][32] (32 KB)
  _Float16* sW1 = reinterpret_cast<_Float16*>(lds + SF_CH);    // [2 hi/lo][HID k][KD] (swizzled)
  h8* sXT = reinterpret_cast<h8*>(sW1 + 2 * HID * KD);          // [W][2 s][2 hi/lo][64 lanes]
  float* sEp = lds;                                             // epilogue slots (the chunk buffers)

  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int D = g.D, stride = g.x_stride;
  const int tile = blockIdx.x * W + w, row0 = tile * 32, blk = blockIdx.x;

#if !RLKS_F1B_ONEPASS
  half_dma<W>(N.w2th, N.w2tl, 0, 0, sCh, w, l);
#endif
  float xv[KS * 8];
  const float* xr = g.x + (size_t)(row0 + r) * stride;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[ks * 8 + j] = xa_elem(xr, 16 * ks + 8 * h + j, D);
  float xm = 0.f;
#pragma unroll
  for (int i = 0; i < KS * 8; ++i) xm = fmaxf(xm, fabsf(xv[i]));
  const int ex = sf_exp(wave_max(xm));
  const float sx = pow2(ex);
  h8 xh[KS], xl[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) split8(xv, ks * 8, sx, xh[ks], xl[ks]);
  const float inv_z1 = N.sc[1] / sx;
  {  // Xa^T for dW1a^T = Xa^T dZ1 (lane row d = r, m = perm(s, h, j))
    float xtv[16];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) xtv[s * 8 + j] = xa_elem(g.x + (size_t)(row0 + sf_perm(s, h, j)) * stride, r, D);
    h8 a, b;
    split8(xtv, 0, sx, a, b);
    sXT[(w * 4 + 0) * 64 + l] = a;
    sXT[(w * 4 + 1) * 64 + l] = b;
    split8(xtv, 8, sx, a, b);
    sXT[(w * 4 + 2) * 64 + l] = a;
    sXT[(w * 4 + 3) * 64 + l] = b;
  }
  for (int p = tid; p < 2 * HID * KD / 8; p += NTHR) {
    const int arr = p / (HID * KD / 8), q = p - arr * (HID * KD / 8), k = q / (KD / 8), pc = q - k * (KD / 8);
    const v4u v = *reinterpret_cast<const v4u*>((arr ? N.w1l : N.w1h) + k * KD + 8 * pc);
    *reinterpret_cast<v4u*>(sW1 + arr * HID * KD + k * KD + 8 * (pc ^ ((k >> 3) & 1))) = v;
  }
  h8 wh[KS], wl[KS];
  auto w1_frag = [&](int kt) {
    const int k = 32 * kt + r;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int off = k * KD + 8 * ((2 * ks + h) ^ ((k >> 3) & 1));
      wh[ks] = *reinterpret_cast<const h8*>(sW1 + off);
      wl[ks] = *reinterpret_cast<const h8*>(sW1 + HID * KD + off);
    }
  };
  const int edz = N.tile_edz[tile];
  const float sdz = pow2(edz);
  const float sz1 = pow2(-23);
  const float u1 = pow2(23 - ex - edz - (int)N.sc[5]);
  // dZ2^T n-tile nt of this wave's rows in accumulator form (register q <-> row n = acc_row(q, l)):
  // one base address and constant offsets
  const float* dzsrc = N.dz2t + (size_t)tile * HID * 32 + 4 * h * 32 + r;
  auto dz_load = [&](int nt, float (&v)[16]) {
    const float* b = dzsrc + (size_t)nt * 32 * 32;
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = b[((q & 3) + 8 * (q >> 2)) * 32];
  };
  vm_drain();
  __syncthreads();

#if RLKS_F1B_ONEPASS
  // ---- one pass: the eight dH1 k-tile accumulators (AGPRs) over the 8 n-tiles; chunk nt = W2's
  // w2t columns [32 nt, +32) of all 256 rows k ([256][32] hi / lo image), single-buffered through
  // registers: a step computes from LDS while the next chunk and dZ2^T n-tile load into registers,
  // then barrier / store / barrier.  Each dZ2^T element is read and split once.
  {
    f32x16 dh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) dh[j][q] = 0.f;
    v4u stg[32 / W];
    float dzc[16], dzn[16];
    chunk_load<W>(N, 8, w, l, stg);
    dz_load(0, dzc);
    vm_drain();
    chunk_store<W>(sCh, w, l, stg);
    __syncthreads();
    for (int nt = 0; nt < 8; ++nt) {
      if (nt < 7) {
        chunk_load<W>(N, 9 + nt, w, l, stg);
        dz_load(nt + 1, dzn);
      }
      h8 ah[2], al[2];
      split8(dzc, 0, sdz, ah[0], al[0]);
      split8(dzc, 8, sdz, ah[1], al[1]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        h8 fc[2][2];
        sf_frag(sCh, 32 * j + r, h, fc);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dh[j] = mma(al[s], fc[s][0], dh[j]);
          dh[j] = mma(ah[s], fc[s][1], dh[j]);
          dh[j] = mma(ah[s], fc[s][0], dh[j]);
        }
      }
      __syncthreads();
      if (nt < 7) {
        vm_drain();
        chunk_store<W>(sCh, w, l, stg);
#pragma unroll
        for (int q = 0; q < 16; ++q) dzc[q] = dzn[q];
      }
      __syncthreads();
    }
    // ---- dZ1 = dH1 (1 - H1^2) -> dW1a^T of the 8 k-tiles; sums over the W waves in the chunk
    // buffer (free now), KPR k-tiles per round
    constexpr int KT0 = 0, NKT = 8;
#pragma unroll
    for (int j = 0; j < NKT; ++j) {
      const int kt = KT0 + j;
      w1_frag(kt);
      f32x16 z;
#pragma unroll
      for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) z = mma3(xh[ks], xl[ks], wh[ks], wl[ks], z);
      f32x16 dz;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float h1 = tanh_abs(z[q] * inv_z1);
        dz[q] = dh[j][q] * (1.f - h1 * h1);
      }
      h8 zh[2], zl[2];
      split16(dz, 0, sz1, zh[0], zl[0]);
      split16(dz, 8, sz1, zh[1], zl[1]);
      f32x16 wacc, wacc2;
#pragma unroll
      for (int q = 0; q < 16; ++q) { wacc[q] = 0.f; wacc2[q] = 0.f; }
      const h8 x0h = sXT[(w * 4 + 0) * 64 + l], x0l = sXT[(w * 4 + 1) * 64 + l];
      const h8 x1h = sXT[(w * 4 + 2) * 64 + l], x1l = sXT[(w * 4 + 3) * 64 + l];
      wacc = mma(x0l, zh[0], wacc);
      wacc2 = mma(x1l, zh[1], wacc2);
      wacc = mma(x0h, zl[0], wacc);
      wacc2 = mma(x1h, zl[1], wacc2);
      wacc = mma(x0h, zh[0], wacc);
      wacc2 = mma(x1h, zh[1], wacc2);
#pragma unroll
      for (int q = 0; q < 16; ++q) wacc[q] += wacc2[q];
#pragma unroll
      for (int gq = 0; gq < NG; ++gq) {
        float4 v = {wacc[4 * gq] * u1, wacc[4 * gq + 1] * u1, wacc[4 * gq + 2] * u1, wacc[4 * gq + 3] * u1};
        *reinterpret_cast<float4*>(sEp + (j % KPR) * SLOT + (w * 32 + r) * DWR + 8 * gq + 4 * h) = v;
      }
      if (j % KPR == KPR - 1) {
        __syncthreads();
        const int nd = D + 1, kt0 = kt + 1 - KPR;
        for (int e = tid; e < KPR * 32 * nd; e += NTHR) {
          const int jj = e / (32 * nd), e2 = e - jj * 32 * nd, kk = e2 / nd, d = e2 - kk * nd;
          const int k = 32 * (kt0 + jj) + kk;
          float sum = 0.f;
#pragma unroll
          for (int ww = 0; ww < W; ++ww) sum += sEp[jj * SLOT + (ww * 32 + kk) * DWR + d];
          if (d < D) N.part_w1[((size_t)blk * HID + k) * D + d] = sum;
          else N.part_b1[(size_t)blk * HID + k] = sum;
        }
        __syncthreads();
      }
    }
  }
#else
  // ---- two passes over the k-halves p: dH1 k-tiles 4p .. 4p+3 accumulate over the 8 n-tiles
  // (24 MFMAs per n-tile step; half-chunks double-buffered), then their dZ1 and dW1a^T
#pragma unroll 1
  for (int p = 0; p < 2; ++p) {
    f32x16 dh[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) dh[j][q] = 0.f;
    float dzc[16], dzn[16];
    dz_load(0, dzc);
    for (int nt = 0; nt < 8; ++nt) {
      if (nt < 7) {
        half_dma<W>(N.w2th, N.w2tl, p, 32 * (nt + 1), sCh + ((nt + 1) & 1) * SF_CH, w, l);
        dz_load(nt + 1, dzn);
      }
      const _Float16* buf = sCh + (nt & 1) * SF_CH;
      h8 ah[2], al[2];
      split8(dzc, 0, sdz, ah[0], al[0]);
      split8(dzc, 8, sdz, ah[1], al[1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h8 fc[2][2];
        half_frag(buf, 32 * j + r, h, fc);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dh[j] = mma(al[s], fc[s][0], dh[j]);
          dh[j] = mma(ah[s], fc[s][1], dh[j]);
          dh[j] = mma(ah[s], fc[s][0], dh[j]);
        }
      }
      vm_drain();
      __syncthreads();
      if (nt < 7)
#pragma unroll
        for (int q = 0; q < 16; ++q) dzc[q] = dzn[q];
    }
    // ---- dZ1 = dH1 (1 - H1^2) -> dW1a^T of k-tiles 4p + j; sums over the W waves in the chunk
    // buffers (free now), KPR k-tiles per round
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kt = 4 * p + j;
      w1_frag(kt);
      f32x16 z;
#pragma unroll
      for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) z = mma3(xh[ks], xl[ks], wh[ks], wl[ks], z);
      f32x16 dz;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float h1 = tanh_abs(z[q] * inv_z1);
        dz[q] = dh[j][q] * (1.f - h1 * h1);
      }
      h8 zh[2], zl[2];
      split16(dz, 0, sz1, zh[0], zl[0]);
      split16(dz, 8, sz1, zh[1], zl[1]);
      f32x16 wacc, wacc2;
#pragma unroll
      for (int q = 0; q < 16; ++q) { wacc[q] = 0.f; wacc2[q] = 0.f; }
      const h8 x0h = sXT[(w * 4 + 0) * 64 + l], x0l = sXT[(w * 4 + 1) * 64 + l];
      const h8 x1h = sXT[(w * 4 + 2) * 64 + l], x1l = sXT[(w * 4 + 3) * 64 + l];
      wacc = mma(x0l, zh[0], wacc);
      wacc2 = mma(x1l, zh[1], wacc2);
      wacc = mma(x0h, zl[0], wacc);
      wacc2 = mma(x1h, zl[1], wacc2);
      wacc = mma(x0h, zh[0], wacc);
      wacc2 = mma(x1h, zh[1], wacc2);
#pragma unroll
      for (int q = 0; q < 16; ++q) wacc[q] += wacc2[q];
#pragma unroll
      for (int gq = 0; gq < NG; ++gq) {
        float4 v = {wacc[4 * gq] * u1, wacc[4 * gq + 1] * u1, wacc[4 * gq + 2] * u1, wacc[4 * gq + 3] * u1};
        *reinterpret_cast<float4*>(sEp + (j % KPR) * SLOT + (w * 32 + r) * DWR + 8 * gq + 4 * h) = v;
      }
      if (j % KPR == KPR - 1) {
        __syncthreads();
        const int nd = D + 1, kt0 = kt + 1 - KPR;
        for (int e = tid; e < KPR * 32 * nd; e += NTHR) {
          const int jj = e / (32 * nd), e2 = e - jj * 32 * nd, kk = e2 / nd, d = e2 - kk * nd;
          const int k = 32 * (kt0 + jj) + kk;
          float sum = 0.f;
#pragma unroll
          for (int ww = 0; ww < W; ++ww) sum += sEp[jj * SLOT + (ww * 32 + kk) * DWR + d];
          if (d < D) N.part_w1[((size_t)blk * HID + k) * D + d] = sum;
          else N.part_b1[(size_t)blk * HID + k] = sum;
        }
        __syncthreads();
      }
    }
    if (p == 0) {  // the second pass's first half-chunk (the buffers held the epilogue slots)
      half_dma<W>(N.w2th, N.w2tl, 1, 0, sCh, w, l);
      vm_drain();
      __syncthreads();
    }
  }

#endif
}

template <int KD, int NG, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_sf_bwd(SfArgs g) {
  if (blockIdx.y + g.net0 == 0) sf_bwd_body<0, KD, NG, W>(g);
  else sf_bwd_body<1, KD, NG, W>(g);
}

// both nets in one grid (blockIdx.y + net0): the hardware backfills CUs across the two nets
// instead of draining between two launches
template <int A_, int KD, int NG, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_sf_fwdbwd(SfArgs g) {
  if (blockIdx.y + g.net0 == 0) sf_fwdbwd_body<A_, 0, KD, NG, W>(g);
  else sf_fwdbwd_body<1, 1, KD, NG, W>(g);
}

// ----------------------------------------------------------------------------- F2
// grid (splits, 2 nets), 512 threads; wave w owns dW2 columns k = 32w + r, all 256 rows n.
template <int KD>
__global__ __launch_bounds__(512) void k_sf_dw2(SfArgs g) {
  constexpr int KS = KD / 16;
  const int net = blockIdx.y;
  const SfNet& N = g.n[net];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sA = reinterpret_cast<_Float16*>(lds);  // [2 buf][2 hi/lo][HID n][32 m perm]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int D = g.D, stride = g.x_stride;
  const int t0 = blockIdx.x * g.tiles_per_split, t1 = t0 + g.tiles_per_split;

  static_assert(SF_DZ_SLOTS == 64, "one max slot per lane");
  // sg / unscale: from the step's max |dZ2|, read after the first tile's loads are in flight
  float sg = 0.f, unscale = 0.f;
  const float inv_w1 = N.sc[1];

  h8 wh[KS], wl[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    wh[ks] = *reinterpret_cast<const h8*>(N.w1h + (32 * w + r) * KD + 16 * ks + 8 * h);
    wl[ks] = *reinterpret_cast<const h8*>(N.w1l + (32 * w + r) * KD + 16 * ks + 8 * h);
  }

  float db2[4] = {0.f, 0.f, 0.f, 0.f};
  // dZ2^T tile t (32 KB) staged through registers: thread tid loads float4 f = tid + 512 i
  // (row n = f >> 3, rows m 4 (f & 7) .. +3) one tile ahead, and splits it into an MFMA buffer at
  // the end of the step.  (LDS-DMA would make the compiler wait for every outstanding LDS read,
  // lgkmcnt(0), before each fragment's use while a DMA is in flight.)
  using v4f = __attribute__((ext_vector_type(4))) float;
  v4f dv[4];
  auto load = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dv[i] = *reinterpret_cast<const v4f*>(N.dz2t + (size_t)t * HID * 32 + (size_t)(tid + 512 * i) * 4);
  };
  auto store = [&](int buf) {
    _Float16* b = sA + buf * 2 * SF_CH;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 512 * i, n = f >> 3, c = f & 7;
      const v4f v = dv[i];
      db2[i] += (v[0] + v[1]) + (v[2] + v[3]);
      h4 hi, lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        _Float16 a, bb;
        split1(v[j] * sg, a, bb);
        hi[j] = a;
        lo[j] = bb;
      }
      const int pc = 2 * (c >> 2) + (c & 1);
      const int off = n * 32 + 8 * (pc ^ ((n >> 2) & 3)) + 4 * ((c >> 1) & 1);
      *reinterpret_cast<h4*>(b + off) = hi;
      *reinterpret_cast<h4*>(b + SF_CH + off) = lo;
    }
  };

  f32x16 acc[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[nt][q] = 0.f;

  // X rows of the next tile are loaded one step ahead (their latency hides behind the MFMAs)
  float xnext[KD == 16 ? KS * 8 : 1];
  auto load_x = [&](int t) {
    if constexpr (KD != 16) return;
    const float* xr = g.x + (size_t)(t * 32 + r) * stride;
    // exec-masked loads of the obs columns (measured faster here than xa_row8's vector loads)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 8 * h + j;
      xnext[j] = d < D ? xr[d] : (d == D ? 1.f : 0.f);
    }
  };
  // H1 tile (rows m in registers, columns k = 32w + r on lanes) of tile tc's X rows, as the B
  // operand.  Obs 6 / 12 (KD 16): the rows were loaded a step ahead into xnext, and tile tn's are
  // loaded now; obs 24 (KD 32): loaded here (the prefetch registers would spill)
  constexpr bool XPRE = KD == 16;
  auto h1 = [&](int tc, int tn, h8 (&bh)[2], h8 (&bl)[2]) {
    float xv[KS * 8];
    if constexpr (XPRE) {
#pragma unroll
      for (int i = 0; i < KS * 8; ++i) xv[i] = xnext[i];
      load_x(tn);
    } else {
      const float* xr = g.x + (size_t)(tc * 32 + r) * stride;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float v[8];
        xa_row8(xr, 16 * ks + 8 * h, D, stride, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[ks * 8 + j] = v[j];
      }
    }
    float xm = 0.f;
#pragma unroll
    for (int i = 0; i < KS * 8; ++i) xm = fmaxf(xm, fabsf(xv[i]));
    const float sx = pow2(sf_exp(wave_max(xm)));
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      h8 a, b;
      split8(xv, ks * 8, sx, a, b);
      z = mma3(a, b, wh[ks], wl[ks], z);
    }
    const float inv_z1 = inv_w1 / sx;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = tanh_abs(z[q] * inv_z1);
    split16(z, 0, SF_H1_SCALE, bh[0], bl[0]);
    split16(z, 8, SF_H1_SCALE, bh[1], bl[1]);
  };

  // Software pipeline: step t runs tile t's 48 MFMAs and, in their shadow, splits tile t + 1's
  // dZ2^T (loaded during step t - 1) into the other LDS buffer, loads tile t + 2's and computes
  // tile t + 1's H1.  The VALU work of a step thus overlaps the same wave's MFMAs instead of
  // following them: both waves of a SIMD meet at every barrier, so they cannot hide each
  // other's VALU phases.
  h8 bh[2], bl[2];
  load(t0);
  {  // lane i of every wave loads F1a's max slot i; one wave-wide max
    const float mxg = wave_max(__uint_as_float(N.dzmax[(threadIdx.x & 63) * SF_DZ_STRIDE]));
    sg = pow2(sf_exp(mxg));
    unscale = 1.f / (sg * SF_H1_SCALE);
  }
  store(0);
  if (t0 + 1 < t1) load(t0 + 1);
  if constexpr (XPRE) load_x(t0);
  h1(t0, t0 + 1 < t1 ? t0 + 1 : t0, bh, bl);
  __syncthreads();
  // Waves 4-7 share SIMDs with waves 0-3 (wave i runs on SIMD i mod 4) and run the same step
  // with the VALU blocks moved (H1 first, the tile split late): the two waves of a SIMD are then
  // in complementary phases between barriers, and one's VALU issues under the other's MFMAs.
  auto step = [&](auto PH, int t) {
    constexpr int ph = decltype(PH)::value;
    constexpr int NT_STORE = ph ? 5 : 1, NT_LOAD = ph ? 6 : 3, NT_H1 = ph ? -1 : 4;
    const int buf = (t - t0) & 1;
    const bool more = t + 1 < t1;
    const _Float16* b = sA + buf * 2 * SF_CH;
    h8 nbh[2], nbl[2];
    const int th = t + 2 < t1 ? t + 2 : t + 1 < t1 ? t + 1 : t;
    const int tc = t + 1 < t1 ? t + 1 : t;
    if (NT_H1 < 0) h1(tc, th, nbh, nbl);  // tile t + 1's H1
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int n = 32 * nt + r;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int off = n * 32 + 8 * ((2 * s + h) ^ ((n >> 2) & 3));
        const h8 ah = *reinterpret_cast<const h8*>(b + off);
        const h8 al = *reinterpret_cast<const h8*>(b + SF_CH + off);
        acc[nt] = mma3(ah, al, bh[s], bl[s], acc[nt]);
      }
      if (nt == NT_STORE && more) store(buf ^ 1);              // tile t + 1 -> other buffer
      if (nt == NT_LOAD && t + 2 < t1) load(t + 2);            // tile t + 2 -> registers
      if (nt == NT_H1) h1(tc, th, nbh, nbl);                   // tile t + 1's H1
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) { bh[s] = nbh[s]; bl[s] = nbl[s]; }
    __syncthreads();
  };
#if RLKS_F2_PHASES
  if (KD == 16 && (w & 4))
    for (int t = t0; t < t1; ++t) step(std::integral_constant<int, 1>{}, t);
  else
#endif
    for (int t = t0; t < t1; ++t) step(std::integral_constant<int, 0>{}, t);
  float* out = N.part_w2 + (size_t)blockIdx.x * SF_W2_PSTRIDE;
#ifdef RLKS_F2_NOSTORE  // timing experiment only: the partials are not written
  if (acc[0][0] != 12345.f) return;
#endif
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int q = 0; q < 16; ++q) out[(size_t)(32 * nt + acc_row(q, l)) * HID + 32 * w + r] = acc[nt][q] * unscale;
  // db2: the 8 threads tid & ~7 .. | 7 hold row n = (tid + 512 i) >> 3
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = db2[i];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    if ((tid & 7) == 0) N.part_b2[(size_t)blockIdx.x * HID + ((tid + 512 * i) >> 3)] = v;
  }
}

// ----------------------------------------------------------------------------- launchers
#ifdef RLKS_STAMPS
extern "C" int rlks_dbg_sf_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sf_stamps), sizeof(g_sf_stamps)) == hipSuccess ? 0 : 1;
}
extern "C" int rlks_dbg_sf_stamps2(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sf_stamps2), sizeof(g_sf_stamps2)) == hipSuccess ? 0 : 1;
}
extern "C" int rlks_dbg_fa_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fa_stamps), sizeof(g_fa_stamps)) == hipSuccess ? 0 : 1;
}
#endif

size_t sf_f1_lds_bytes(int A_, int NG, int KD, int W) {
  return (size_t)2 * 2 * SF_CH * sizeof(_Float16) + (size_t)(HID + A_ * HID) * sizeof(float) +
         (size_t)2 * HID * KD * sizeof(_Float16) + (size_t)W * 4 * 64 * 16;
}

// F1 as two kernels (F1a k_sf_fwd + F1b k_sf_bwd, two workgroups per CU) or the fused one-wave-
// per-SIMD kernel: RLKS_F1_SPLIT=0 / 1 overrides the default
bool sf_f1_split() {
  static const int v = [] {
    const char* e = getenv("RLKS_F1_SPLIT");
    return e ? atoi(e) : RLKS_F1_SPLIT_DEFAULT;
  }();
  return v != 0;
}

int launch_sf_prep(const SfPrepArgs& a, hipStream_t s) {
  if (!a.skip_wmax) {
    hipLaunchKernelGGL(k_sf_wmax, dim3(2, 32), dim3(256), 0, s, a);
    RLKS_LAUNCHED();
  }
  hipLaunchKernelGGL(k_sf_split, dim3(2, 64), dim3(256), 0, s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

template <int A_, int KD, int NG>
static int launch_f1_net(SfArgs a, int net0, int nets, hipStream_t s, int halves) {
  constexpr int W = SF_F1_W;
  a.net0 = net0;
  const dim3 grid(a.M / (32 * W), nets);
  if (sf_f1_split()) {
    const size_t lds_a = (size_t)2 * SF_CH * sizeof(_Float16) + (size_t)(1 + A_) * HID * sizeof(float) +
                         (size_t)2 * HID * KD * sizeof(_Float16);
    const size_t lds_b = (size_t)2 * SF_CH * sizeof(_Float16) + (size_t)2 * HID * KD * sizeof(_Float16) +
                         (size_t)W * 4 * 64 * 16;
    if (halves & 1) {
      hipLaunchKernelGGL((k_sf_fwd<A_, KD, W>), grid, dim3(64 * W), lds_a, s, a);
      RLKS_LAUNCHED();
    }
    if (halves & 2) {
      hipLaunchKernelGGL((k_sf_bwd<KD, NG, W>), grid, dim3(64 * W), lds_b, s, a);
      RLKS_LAUNCHED();
    }
    return RLKS_OK;
  }
  hipLaunchKernelGGL((k_sf_fwdbwd<A_, KD, NG, W>), grid, dim3(64 * W), sf_f1_lds_bytes(A_, NG, KD, W), s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

// obs_dim = 3 x clusters: C = 2, 4, 8 -> D = 6, 12, 24 (D + 1 <= 8, 16, 32)
int sf_kd(int D) { return D + 1 <= 16 ? 16 : 32; }

int launch_sf_f1(const SfArgs& a, int net0, int nets, int A, hipStream_t s, int halves) {
  RLKS_REQUIRE(a.M % SF_ROWS == 0, RLKS_ERR_ARG, "split-fp16 SGD step: rows must be a multiple of 256");
  RLKS_REQUIRE(a.D == 3 * A, RLKS_ERR_UNSUPPORTED, "split-fp16 SGD step expects obs_dim = 3 x n_actions");
  switch (A) {
    case 2: return launch_f1_net<2, 16, 1>(a, net0, nets, s, halves);
    case 4: return launch_f1_net<4, 16, 2>(a, net0, nets, s, halves);
    case 8: return launch_f1_net<8, 32, 4>(a, net0, nets, s, halves);
    default: return fail(RLKS_ERR_UNSUPPORTED, "split-fp16 head is built for 2, 4 or 8 actions");
  }
}

int launch_sf_dw2(const SfArgs& a, int splits, hipStream_t s) {
  const size_t lds = (size_t)2 * 2 * SF_CH * sizeof(_Float16);
  if (sf_kd(a.D) == 16) hipLaunchKernelGGL(k_sf_dw2<16>, dim3(splits, 2), dim3(512), lds, s, a);
  else hipLaunchKernelGGL(k_sf_dw2<32>, dim3(splits, 2), dim3(512), lds, s, a);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

}  // namespace rlks
