// gemm_sf16.hip — generic split-fp16 GEMM with fused epilogues, for the wide policy MLP of config
// c5 (fcnet_hiddens [2048, 2048], obs 3 x 64 clusters, 64 actions: SURVEY §8d "MFMA-bound update").
//
//   C[M x N] = epi( op(A)[M x K] . op(B)[K x N] )
//   op(A) = A (A stored [M][lda]) or A^T (TA: stored [K][lda]); op(B) = B (stored [K][ldb]) or B^T
//   (TB: stored [N][ldb]); all fp32 in HBM.
//   epi: store | tanh(acc + bias[n]) | acc + bias[n] | acc * (1 - G[m][n]^2)  (G = stored tanh output)
//   optionally the max |C| of the tile goes to an atomicMax slot (the next GEMM's operand scale).
//
// Arithmetic as in sgd_sf16.hip: operands split into fp16 hi/lo of x 2^e on their way into LDS, with
// 2^e from a per-operand max|x| slot (uint bits of a non-negative float, written by the producer's
// epilogue or by rlks_absmax); three v_mfma_f32_32x32x16_f16 per product; fp32-accurate.
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (2 x 2 waves of 64 x 64 = 2 x 2 MFMA 32x32
// tiles), K in chunks of 32 double-buffered in LDS as [row][32 k] halves with 16-byte pieces
// XOR-swizzled by (row >> 2) & 3 (conflict-free ds_read_b128 fragment loads).  Global loads are
// float4 along the contiguous dimension; operands whose contiguous dimension is not K are
// transposed by the LDS store.  M, N and K are masked (zero fill / masked stores).
#include "gemm_sf16.h"

namespace rlks {

using h8 = __attribute__((ext_vector_type(8))) _Float16;
using h4 = __attribute__((ext_vector_type(4))) _Float16;

namespace {

constexpr int GT = 128;  // output tile
constexpr int GKC = 32;  // K chunk
constexpr int GCH = GT * GKC;  // halves per operand chunk (per hi / lo)

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
// half offset of (row, k) in a [GT][GKC] chunk with swizzled 8-half pieces
__device__ __forceinline__ int coff(int row, int k) {
  return row * GKC + 8 * ((k >> 3) ^ ((row >> 2) & 3)) + (k & 7);
}

// stage one operand chunk: rows [r0, r0 + 128) of op(X) ([rows][K]) and k in [k0, k0 + 32).
// T = false: X stored [rows][ld] (k contiguous); T = true: X stored [K][ld] (rows contiguous).
template <bool T>
struct Stager {
  float4 v[4];
  // vec: ld % 4 == 0 and X 16-byte aligned (float4 loads), else four scalar loads
  __device__ __forceinline__ void load(const float* X, int ld, int rows, int K, int r0, int k0, int tid, bool vec) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      int row, k;
      if (!T) { row = f >> 3; k = 4 * (f & 7); }     // 128 rows x 8 float4
      else { k = f >> 5; row = 4 * (f & 31); }       // 32 k x 32 float4
      const int gr = r0 + row, gk = k0 + k;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!T) {
        if (gr < rows) {
          const float* p = X + (size_t)gr * ld + gk;
          if (vec && gk + 3 < K) x = *reinterpret_cast<const float4*>(p);
          else {
            if (gk < K) x.x = p[0];
            if (gk + 1 < K) x.y = p[1];
            if (gk + 2 < K) x.z = p[2];
            if (gk + 3 < K) x.w = p[3];
          }
        }
      } else {
        if (gk < K) {
          const float* p = X + (size_t)gk * ld + gr;
          if (vec && gr + 3 < rows) x = *reinterpret_cast<const float4*>(p);
          else {
            if (gr < rows) x.x = p[0];
            if (gr + 1 < rows) x.y = p[1];
            if (gr + 2 < rows) x.z = p[2];
            if (gr + 3 < rows) x.w = p[3];
          }
        }
      }
      v[i] = x;
    }
  }
  __device__ __forceinline__ void store(_Float16* buf, float s, int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      const float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      if (!T) {
        const int row = f >> 3, k = 4 * (f & 7);
        h4 hi, lo;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          _Float16 a, b;
          split1(e[j] * s, a, b);
          hi[j] = a;
          lo[j] = b;
        }
        *reinterpret_cast<h4*>(buf + coff(row, k)) = hi;
        *reinterpret_cast<h4*>(buf + GCH + coff(row, k)) = lo;
      } else {
        const int k = f >> 5, row = 4 * (f & 31);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          _Float16 a, b;
          split1(e[j] * s, a, b);
          buf[coff(row + j, k)] = a;
          buf[GCH + coff(row + j, k)] = b;
        }
      }
    }
  }
};

}  // namespace

template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(256) void k_gemm_sf16(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sm = reinterpret_cast<_Float16*>(lds);  // [2 buf][A hi, A lo, B hi, B lo][GCH]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int n0 = blockIdx.x * GT, m0 = blockIdx.y * GT;
  const int ea = sf_exp(__uint_as_float(*g.amax)), eb = sf_exp(__uint_as_float(*g.bmax));
  const float sa = ldexpf(1.f, ea), sb = ldexpf(1.f, eb), unscale = ldexpf(1.f, -ea - eb);

  Stager<TA> SA;
  Stager<!TB> SB;  // B is staged as rows n: B stored [N][K] (TB) has k contiguous
  const bool va = (g.lda & 3) == 0 && ((uintptr_t)g.A & 15) == 0;
  const bool vb = (g.ldb & 3) == 0 && ((uintptr_t)g.B & 15) == 0;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk = (g.K + GKC - 1) / GKC;
  SA.load(g.A, g.lda, g.M, g.K, m0, 0, tid, va);
  SB.load(g.B, g.ldb, g.N, g.K, n0, 0, tid, vb);
  SA.store(sm, sa, tid);
  SB.store(sm + 2 * GCH, sb, tid);
  if (nk > 1) {
    SA.load(g.A, g.lda, g.M, g.K, m0, GKC, tid, va);
    SB.load(g.B, g.ldb, g.N, g.K, n0, GKC, tid, vb);
  }
  __syncthreads();
  for (int c = 0; c < nk; ++c) {
    const _Float16* buf = sm + (c & 1) * 4 * GCH;
    h8 fa[2][2][2], fb[2][2][2];  // [tile][s][hi/lo]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ra = wm * 64 + 32 * i + r, rb = wn * 64 + 32 * i + r, k = 16 * s + 8 * h;
        fa[i][s][0] = *reinterpret_cast<const h8*>(buf + coff(ra, k));
        fa[i][s][1] = *reinterpret_cast<const h8*>(buf + GCH + coff(ra, k));
        fb[i][s][0] = *reinterpret_cast<const h8*>(buf + 2 * GCH + coff(rb, k));
        fb[i][s][1] = *reinterpret_cast<const h8*>(buf + 3 * GCH + coff(rb, k));
      }
    if (c + 1 < nk) {  // park chunk c + 1 in the other buffer, fetch chunk c + 2
      _Float16* nb = sm + ((c + 1) & 1) * 4 * GCH;
      SA.store(nb, sa, tid);
      SB.store(nb + 2 * GCH, sb, tid);
      if (c + 2 < nk) {
        SA.load(g.A, g.lda, g.M, g.K, m0, (c + 2) * GKC, tid, va);
        SB.load(g.B, g.ldb, g.N, g.K, n0, (c + 2) * GKC, tid, vb);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(fa[i][s][1], fb[j][s][0], acc[i][j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(fa[i][s][0], fb[j][s][1], acc[i][j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(fa[i][s][0], fb[j][s][0], acc[i][j]);
    }
    __syncthreads();
  }

  // epilogue: C rows m = m0 + wm 64 + 32 i + acc_row(q), column n = n0 + wn 64 + 32 j + r
  float cmax = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + 32 * j + r;
    const bool nok = n < g.N;
    const float bias = (EPI == GEMM_TANH_BIAS || EPI == GEMM_BIAS) && nok ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm * 64 + 32 * i + acc_row(q, l);
        if (!nok || m >= g.M) continue;
        float v = acc[i][j][q] * unscale;
        if (EPI == GEMM_TANH_BIAS) v = tanh_abs(v + bias);
        if (EPI == GEMM_BIAS) v += bias;
        if (EPI == GEMM_DTANH) {
          const float gg = g.aux[(size_t)m * g.ldaux + n];
          v *= 1.f - gg * gg;
        }
        if (g.accumulate) v += g.C[(size_t)m * g.ldc + n];
        g.C[(size_t)m * g.ldc + n] = v;
        cmax = fmaxf(cmax, fabsf(v));
      }
  }
  if (g.cmax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cmax = fmaxf(cmax, __shfl_xor(cmax, o, 64));
    if (l == 0) atomicMax(g.cmax, __float_as_uint(cmax));
  }
}

// max |x| over a strided [rows][cols] fp32 matrix -> atomicMax slot (slot zeroed by the caller)
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ x, int rows, int cols, int ld,
                                                unsigned* __restrict__ slot) {
  float mx = 0.f;
  const size_t n = (size_t)rows * cols;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const size_t rr = i / cols, cc = i - rr * cols;
    mx = fmaxf(mx, fabsf(x[rr * ld + cc]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(slot, __float_as_uint(mx));
}

// column sums of a [rows][cols] matrix: out[c] (+)= sum_r x[r][c]; one thread per column, f64
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ x, int rows, int cols, int ld,
                                                float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  double s = 0.0;
  for (int rr = 0; rr < rows; ++rr) s += (double)x[(size_t)rr * ld + c];
  out[c] = accumulate ? out[c] + (float)s : (float)s;
}

template <bool TA, bool TB>
static int launch_t(const GemmArgs& a, hipStream_t s) {
  const dim3 grid(cdiv(a.N, GT), cdiv(a.M, GT));
  const size_t lds = (size_t)2 * 4 * GCH * sizeof(_Float16);
  switch (a.epi) {
    case GEMM_STORE: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_STORE>), grid, dim3(256), lds, s, a); break;
    case GEMM_TANH_BIAS: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_TANH_BIAS>), grid, dim3(256), lds, s, a); break;
    case GEMM_BIAS: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_BIAS>), grid, dim3(256), lds, s, a); break;
    case GEMM_DTANH: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_DTANH>), grid, dim3(256), lds, s, a); break;
    default: return fail(RLKS_ERR_ARG, "gemm: unknown epilogue");
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int launch_gemm_sf16(const GemmArgs& a, hipStream_t s) {
  RLKS_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0 && a.A && a.B && a.C && a.amax && a.bmax, RLKS_ERR_ARG, "gemm: bad argument");
  if (!a.ta && !a.tb) return launch_t<false, false>(a, s);
  if (!a.ta && a.tb) return launch_t<false, true>(a, s);
  if (a.ta && !a.tb) return launch_t<true, false>(a, s);
  return launch_t<true, true>(a, s);
}

int launch_absmax(const float* x, int rows, int cols, int ld, unsigned* slot, hipStream_t s) {
  const size_t n = (size_t)rows * cols;
  const unsigned blocks = (unsigned)std::min<size_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(k_absmax, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, x, rows, cols, ld, slot);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int launch_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(k_colsum, dim3(cdiv(cols, 256)), dim3(256), 0, s, x, rows, cols, ld, out, accumulate);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

}  // namespace rlks

using namespace rlks;

extern "C" int rlks_gemm_sf16(const rlks_gemm_desc* d, void* stream) {
  RLKS_REQUIRE(d, RLKS_ERR_ARG, "rlks_gemm_sf16: null desc");
  GemmArgs a{};
  a.A = d->a; a.B = d->b; a.C = d->c; a.bias = d->bias; a.aux = d->aux;
  a.M = d->m; a.N = d->n; a.K = d->k; a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc; a.ldaux = d->ldaux;
  a.ta = d->trans_a; a.tb = d->trans_b; a.epi = d->epilogue; a.accumulate = d->accumulate;
  a.amax = d->a_max; a.bmax = d->b_max; a.cmax = d->c_max;
  return launch_gemm_sf16(a, (hipStream_t)stream);
}

extern "C" int rlks_absmax(const float* x, int rows, int cols, int ld, unsigned* slot, void* stream) {
  RLKS_REQUIRE(x && slot && rows >= 0 && cols >= 0 && ld >= cols, RLKS_ERR_ARG, "rlks_absmax: bad argument");
  if (rows == 0 || cols == 0) return RLKS_OK;
  return launch_absmax(x, rows, cols, ld, slot, (hipStream_t)stream);
}
