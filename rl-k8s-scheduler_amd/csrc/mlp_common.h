// mlp_common.h — shared pieces of the policy/value MLP kernels (K4): flat parameter layout,
// fp32 MFMA helpers, the fast tanh and the argument blocks of the SGD-step kernels.
//
// Reference: RLlib's default torch FCNet behind PPOConfig().framework("torch")
// (train_ppo.py:12): pi = D -> 256 tanh -> 256 tanh -> A, vf = D -> 256 tanh -> 256 tanh -> 1,
// vf_share_layers=False.  RLlib is third-party (absent here); see DESIGN.md §3.
#pragma once

#include <hip/hip_runtime.h>

#include "env_device.h"
#include "rlks_internal.h"

namespace rlks {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int HID = 256;   // hidden width the fused kernels are built for (fcnet_hiddens [256, 256])
constexpr int MAXA = 8;    // max actions (clusters)
constexpr int DMAX = 32;   // max obs dim of the VALU input layer
constexpr int BK = 32;     // reduction chunk staged in LDS
constexpr int GB = 128;    // F2/F3 block tile (4 waves of 64 x 64)

// v_mfma_f32_32x32x2_f32: exact f32 fma chain in k order (cdna_hip_programming.md §3)
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row of accumulator register r for lane l (v_mfma_f32_32x32x* C/D map; col = l & 31)
__device__ __forceinline__ int acc_row(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }

// tanh in ~14 VALU ops (ocml tanhf is ~35): odd minimax polynomial for |x| < 0.6, else
// 1 - 2 / (exp(2|x|) + 1) with v_exp_f32 / v_rcp_f32.  Max relative error 1.8e-7 (~3 ulp) over
// all of fp32, measured against float64 tanh (tools/fit_tanh.py); far inside the 1e-5 parity bar.
__device__ __forceinline__ float fast_tanh(float x) {
  const float ax = fabsf(x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.885390081777927f);
  const float big = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  const float x2 = x * x;
  float p = -0.006104227155447006f;
  p = fmaf(p, x2, 0.020971255376935005f);
  p = fmaf(p, x2, -0.05383438989520073f);
  p = fmaf(p, x2, 0.1333249807357788f);
  p = fmaf(p, x2, -0.33333319425582886f);
  const float small = fmaf(x * x2, p, x);
  return ax < 0.6f ? small : __builtin_copysignf(big, x);
}

// reduce 16 per-lane values (register r <-> accumulator row) over the 32 lanes of a half-wave;
// afterwards lane l holds the total of register ((l >> 1) & 15) (lanes l and l^1 agree).
// Reduce-scatter without LDS: v_permlane16_swap pairs rows 0/1 (and 2/3) of the wave, then
// DPP row_ror:8, row_half_mirror and two quad_perms finish within each row of 16 lanes
// (38 VALU, no ds_bpermute round trips).
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float half_wave_reduce16(const float (&v)[16], int l) {
  float u[8], w[4], x[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
    u[i] = __uint_as_float(p[0]) + __uint_as_float(p[1]);  // even rows: v[i], odd rows: v[i + 8]
  }
  const bool b3 = (l >> 3) & 1, b2 = (l >> 2) & 1, b1 = (l >> 1) & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (b3 ? u[i + 4] : u[i]) + dpp<0x128>(b3 ? u[i] : u[i + 4]);  // row_ror:8
#pragma unroll
  for (int i = 0; i < 2; ++i) x[i] = (b2 ? w[i + 2] : w[i]) + dpp<0x141>(b2 ? w[i] : w[i + 2]);  // half_mirror
  const float y = (b1 ? x[1] : x[0]) + dpp<0x4E>(b1 ? x[0] : x[1]);                             // quad [2,3,0,1]
  return y + dpp<0xB1>(y);                                                                         // quad [1,0,3,2]
}

// wave-wide reductions as a butterfly over lane bits 0..5 in VALU cross-lane ops (DPP quad_perm,
// row_half_mirror, row_ror:8, v_permlane16/32_swap) instead of __shfl_xor's ds_bpermute round trips
// through the LDS pipe (each a dependent lgkmcnt wait: ~40 of them per F1a epilogue).  Every step
// adds a lane's value to its partner's (a + b on one lane, b + a on the other), so all lanes end
// with the same bits.
template <typename Op>
__device__ __forceinline__ float wave_reduce(float v, Op op) {
  v = op(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]: lane ^ 1
  v = op(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]: lane ^ 2
  v = op(v, dpp<0x141>(v));  // row_half_mirror: the other quad of the 8
  v = op(v, dpp<0x128>(v));  // row_ror:8: lane ^ 8
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = op(__uint_as_float(p[0]), __uint_as_float(p[1]));  // rows 0 + 1, 2 + 3
  p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(p[0]), __uint_as_float(p[1]));  // rows 0-1 + rows 2-3
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float a, float b) { return fmaxf(a, b); });
}
__device__ __forceinline__ float wave_sum_f(float v) {
  return wave_reduce(v, [](float a, float b) { return a + b; });
}
// row_sum16 over doubles (each 32-bit half moved by the same DPP step)
template <int CTRL>
__device__ __forceinline__ double dppd(double x) {
  const unsigned long long u = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double row_sum16d(double v) {  // over the 16 lanes of a row
  v += dppd<0x128>(v);
  v += dppd<0x141>(v);
  v += dppd<0x4E>(v);
  return v + dppd<0xB1>(v);
}

// RLlib's value loss of one row, clamp((v - vt)^2, 0, vf_clip) (as oracle.py:ppo_loss_grad restates it):
// dl = dL/dv already over the row count, the clamped square (the vf_loss stat), and ex = v - vt
// exactly (the fp32 difference plus its rounding error, Knuth's TwoSum) where the row is inside the
// clamp, else 0.  The value head's bias gradient is 2 vf_coeff / count times the sum of ex over the
// rows: a single sum over the minibatch whose rows cancel to ~1/sqrt(rows) of their magnitudes, so the
// fp32 rounding of each row's difference (half an ulp of |v - vt|, the same size as the terms' error
// that a float32 evaluation makes) would dominate its relative error; summed exactly in f64 it is
// left with the forward's own error of v (profiles/r05_precision).
struct VfRow {
  float dl, sq;
  double ex;
};
__device__ __forceinline__ VfRow vf_row(float v, float vt, float vf_clip, float vf_coeff, float inv_count) {
  const float diff = v - vt;
  const float bv = diff - v;
  const float err = (v - (diff - bv)) + (-vt - bv);
  const float sq = diff * diff;
  const bool in = sq <= vf_clip;
  return {in ? vf_coeff * 2.f * diff * inv_count : 0.f, fminf(sq, vf_clip), in ? (double)diff + (double)err : 0.0};
}
// the bias gradient's per-block partial from a block's f64 sum of ex, as an exact hi + lo pair of
// floats (both summed by the f64 reduce)
__device__ __forceinline__ void vf_b3_part(double sum_ex, float vf_coeff, float inv_count, float* part2) {
  const double t = sum_ex * (2.0 * (double)vf_coeff * (double)inv_count);
  const float hi = (float)t;
  part2[0] = hi;
  part2[1] = (float)(t - (double)hi);
}

// ----------------------------------------------------------------------------- layout
struct Layout {
  int64_t off[RLKS_N_TENSORS];
  int64_t padded, real;
};

// storage order (include/rlks.h): both nets' first layers, then pi's and vf's W2 / b2 / W3 / b3, so
// that the overlapped all-reduce's two gradient buckets are two contiguous ranges
// (rlks_ppo_grad_step_part)
constexpr int LAYOUT_ORDER[RLKS_N_TENSORS] = {0, 1, 6, 7, 2, 3, 4, 5, 8, 9, 10, 11};
inline Layout make_layout(int D, int H, int A) {
  const int64_t sz[RLKS_N_TENSORS] = {(int64_t)H * D, H, (int64_t)H * H, H, (int64_t)A * H, A,
                                      (int64_t)H * D, H, (int64_t)H * H, H, H, 1};
  Layout L{};
  int64_t o = 0;
  for (int j = 0; j < RLKS_N_TENSORS; ++j) {
    const int i = LAYOUT_ORDER[j];
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

inline NetPtrs net_ptrs_host(const float* p, const Layout& L, int net) {
  const int64_t* o = L.off + 6 * net;
  return NetPtrs{p + o[0], p + o[1], p + o[2], p + o[3], p + o[4], p + o[5]};
}

// packed minibatch record: [obs D | logits_old A | adv | vtarg | logp_old | action | pad]
inline int mb_stride(int D, int A) { return (D + A + 4 + 3) / 4 * 4; }

// ----------------------------------------------------------------------------- F1 arguments
struct FwdArgs {
  NetPtrs P;          // this net's tensors
  const float* x;     // row m at x + m * x_stride (obs = first D floats)
  int x_stride;
  int M, D, A_pi;     // A_pi: pi action count (record layout)
  float* out;         // forward-only: logits [M][A] (pi) or values [M] (vf)
  rlks_ppo_coeffs co;
  const float* dyn;
  float* dz2;         // this net's [M][HID]
  float* part_b2;     // [tiles][HID]
  float* part_w3;     // [tiles][A_][HID]
  float* part_b3;     // [tiles][A_]
  float* part_stat;   // [tiles][4]
  // rollout mode: sample an action from the logits and step the env lane (row m = lane m)
  EnvView env;
  const double* tab_cost;  // [T][C]
  const double* tab_lat;   // [T][C]
  int explore;
  float* obs_next;         // [M][D]
  float* logp;             // [M]
  int32_t* actions;        // [M]
  float* rewards;          // [M]
  uint8_t* dones;          // [M]
};

// ----------------------------------------------------------------------------- F2 / F3 arguments
// one launch covers both nets: blockIdx.z selects pi (0) or vf (1)
struct Dw2Args {
  NetPtrs P[2];
  const float* x;
  int x_stride;
  int M, rows_per_split;
  const float* dz2[2];  // per net [M][HID]
  float* part[2];       // per net [S][HID][HID]
};

struct Dh1Args {
  NetPtrs P[2];
  const float* x;
  int x_stride;
  int M;
  const float* dz2[2];  // per net [M][HID]
  float* part_w1[2];    // per net [tiles][HID][D]
  float* part_b1[2];    // per net [tiles][HID]
};

// host launchers (mlp_fwd.hip / mlp_bwd.hip)
enum { FWD_ONLY = 0, FWD_TRAIN = 1, FWD_ROLLOUT = 2 };
int launch_fwd_head(const FwdArgs& a, int net, int A, int mode, hipStream_t s);
int launch_dw2(const Dw2Args& a, int D, int splits, hipStream_t s);
int launch_dh1(const Dh1Args& a, int D, hipStream_t s);

}  // namespace rlks
