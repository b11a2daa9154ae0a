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
  // interior chunk: four unmasked float4 loads, issued back to back (the masked path compiles to a
  // load -> wait per element, which serialises the loads' latency)
  __device__ __forceinline__ void load_full(const float* X, int ld, int r0, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      const size_t off = !T ? (size_t)(r0 + (f >> 3)) * ld + k0 + 4 * (f & 7)
                            : (size_t)(k0 + 4 * (tid >> 5) + i) * ld + r0 + 4 * (tid & 31);
      v[i] = *reinterpret_cast<const float4*>(X + off);
    }
  }
  // vec: ld % 4 == 0 and X 16-byte aligned (float4 loads), else four scalar loads
  __device__ __forceinline__ void load(const float* X, int ld, int rows, int K, int r0, int k0, int tid, bool vec) {
    if (vec && r0 + GT <= rows && k0 + GKC <= K) {
      load_full(X, ld, r0, k0, tid);
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      int row, k;
      if (!T) { row = f >> 3; k = 4 * (f & 7); }     // 128 rows x 8 float4
      else { k = 4 * (tid >> 5) + i; row = 4 * (tid & 31); }  // 4 k x 4 rows per thread (i = k)
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
      }
    }
    if (T) {  // register transpose: row j of the thread's 4 x 4 block is 4 consecutive k -> one h4
      const int k = 4 * (tid >> 5), row = 4 * (tid & 31);
      const float e[4][4] = {{v[0].x, v[0].y, v[0].z, v[0].w}, {v[1].x, v[1].y, v[1].z, v[1].w},
                             {v[2].x, v[2].y, v[2].z, v[2].w}, {v[3].x, v[3].y, v[3].z, v[3].w}};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h4 hi, lo;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          _Float16 a, b;
          split1(e[i][j] * s, a, b);
          hi[i] = a;
          lo[i] = b;
        }
        *reinterpret_cast<h4*>(buf + coff(row + j, k)) = hi;
        *reinterpret_cast<h4*>(buf + GCH + coff(row + j, k)) = lo;
      }
    }
  }
};

}  // namespace

template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_gemm_sf16(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sm = reinterpret_cast<_Float16*>(lds);  // [2 buf][A hi, A lo, B hi, B lo][GCH]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int n0 = blockIdx.x * GT, m0 = blockIdx.y * GT;
  const int ea = sf_exp(__uint_as_float(*g.amax)), eb = sf_exp(__uint_as_float(*g.bmax));
  // rounding-bias cancellation in the dZ1 GEMM (gemm_ps.hip, sgd_sf16.hip tile_sign): A enters
  // negated in odd row blocks / split layers, and the result is negated back
  const float sg = (EPI == GEMM_DTANH && ((blockIdx.y + blockIdx.z) & 1)) ? -1.f : 1.f;
  const float sa = sg * ldexpf(1.f, ea), sb = ldexpf(1.f, eb), unscale = sg * ldexpf(1.f, -ea - eb);

  // register ring of two chunks per operand: while chunk c is multiplied, chunks c + 1 (parked in
  // LDS at the start of iteration c) and c + 2 / c + 3 are in flight, so a load has two MFMA
  // blocks to arrive instead of one
  Stager<TA> SA0, SA1;
  Stager<!TB> SB0, SB1;  // B is staged as rows n: B stored [N][K] (TB) has k contiguous
  const bool va = (g.lda & 3) == 0 && ((uintptr_t)g.A & 15) == 0;
  const bool vb = (g.ldb & 3) == 0 && ((uintptr_t)g.B & 15) == 0;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  // this workgroup's K range (split-K: layer z of `splits`, each kper long, a multiple of GKC)
  const int kper = g.splits > 1 ? (((g.K + g.splits - 1) / g.splits + GKC - 1) / GKC) * GKC : g.K;
  const int kb = blockIdx.z * kper, ke = min(g.K, kb + kper);
  const int nk = ke > kb ? (ke - kb + GKC - 1) / GKC : 0;
  SA0.load(g.A, g.lda, g.M, ke, m0, kb, tid, va);
  SB0.load(g.B, g.ldb, g.N, ke, n0, kb, tid, vb);
  SA0.store(sm, sa, tid);
  SB0.store(sm + 2 * GCH, sb, tid);
  if (nk > 1) {
    SA1.load(g.A, g.lda, g.M, ke, m0, kb + GKC, tid, va);
    SB1.load(g.B, g.ldb, g.N, ke, n0, kb + GKC, tid, vb);
  }
  if (nk > 2) {
    SA0.load(g.A, g.lda, g.M, ke, m0, kb + 2 * GKC, tid, va);
    SB0.load(g.B, g.ldb, g.N, ke, n0, kb + 2 * GKC, tid, vb);
  }
  __syncthreads();
  // iteration c: fragments of chunk c (LDS buffer c & 1); chunk c + 1 from ring slot RA / RB into
  // the other buffer; that slot then fetches chunk c + 3; the MFMAs of chunk c
#define GEMM_ITER(c, RA, RB, STEADY)                                                                \
  {                                                                                                 \
    const _Float16* buf = sm + ((c) & 1) * 4 * GCH;                                                 \
    h8 fa[2][2][2], fb[2][2][2];                                                                    \
    _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                   \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                 \
      const int ra = wm * 64 + 32 * i + r, rb = wn * 64 + 32 * i + r, k = 16 * s + 8 * h;           \
      fa[i][s][0] = *reinterpret_cast<const h8*>(buf + coff(ra, k));                                \
      fa[i][s][1] = *reinterpret_cast<const h8*>(buf + GCH + coff(ra, k));                          \
      fb[i][s][0] = *reinterpret_cast<const h8*>(buf + 2 * GCH + coff(rb, k));                      \
      fb[i][s][1] = *reinterpret_cast<const h8*>(buf + 3 * GCH + coff(rb, k));                      \
    }                                                                                               \
    if (STEADY || (c) + 1 < nk) {                                                                   \
      _Float16* nb = sm + (((c) + 1) & 1) * 4 * GCH;                                                \
      RA.store(nb, sa, tid);                                                                        \
      RB.store(nb + 2 * GCH, sb, tid);                                                              \
      if (STEADY) {                                                                                 \
        RA.load_full(g.A, g.lda, m0, kb + ((c) + 3) * GKC, tid);                                    \
        RB.load_full(g.B, g.ldb, n0, kb + ((c) + 3) * GKC, tid);                                    \
      } else if ((c) + 3 < nk) {                                                                    \
        RA.load(g.A, g.lda, g.M, ke, m0, kb + ((c) + 3) * GKC, tid, va);                            \
        RB.load(g.B, g.ldb, g.N, ke, n0, kb + ((c) + 3) * GKC, tid, vb);                            \
      }                                                                                             \
    }                                                                                               \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                 \
      _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                 \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[i][j] = mma(fa[i][s][1], fb[j][s][0], acc[i][j]); \
      _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                 \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[i][j] = mma(fa[i][s][0], fb[j][s][1], acc[i][j]); \
      _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                 \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[i][j] = mma(fa[i][s][0], fb[j][s][0], acc[i][j]); \
    }                                                                                               \
    __syncthreads();                                                                                \
  }
  // steady state (interior tile, every operand chunk whole): branch-free bodies with unmasked loads;
  // then the general masked iterations for the last chunks (or the whole range of an edge tile)
  int c = 0;
  if (va && vb && m0 + GT <= g.M && n0 + GT <= g.N && kb + nk * GKC <= ke) {
    for (; c + 4 < nk; c += 2) {
      GEMM_ITER(c, SA1, SB1, true)  // chunk c + 1 (odd) lives in slot 1
      GEMM_ITER(c + 1, SA0, SB0, true)
    }
  }
  for (; c < nk; c += 2) {
    GEMM_ITER(c, SA1, SB1, false)
    if (c + 1 < nk) GEMM_ITER(c + 1, SA0, SB0, false)
  }
#undef GEMM_ITER

  // epilogue: C rows m = m0 + wm 64 + 32 i + acc_row(q), column n = n0 + wn 64 + 32 j + r
  const bool split = g.splits > 1;
  float* const Cout = split ? g.part + (size_t)blockIdx.z * g.M * g.N : g.C;
  const int ldc = split ? g.N : g.ldc;
  float cmax = 0.f;
  // the wave's 64 x 64 block from uniform base pointers and 32-bit per-lane offsets (gemm_ps.hip)
  const int mw = m0 + wm * 64, nw = n0 + wn * 64;
  float* const cw = Cout + (size_t)mw * ldc + nw;
  const float* const cin = g.C + (size_t)mw * g.ldc + nw;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nl = 32 * j + r, n = nw + nl;
    const bool nok = n < g.N;
    const float bias = (EPI == GEMM_TANH_BIAS || EPI == GEMM_BIAS || EPI == GEMM_TANH_BIAS_PLANES) && nok ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ml = 32 * i + acc_row(q, l), m = mw + ml;
        if (!nok || m >= g.M) continue;
        float v = acc[i][j][q] * unscale;
        if (EPI == GEMM_TANH_BIAS_PLANES) {  // H1 for the pre-split GEMMs: fp16 planes at 2^14
          const float hs = tanh_abs(v + bias) * 16384.f;
          const _Float16 a = (_Float16)hs;
          g.c_hi[(size_t)m * g.ldc + n] = a;
          g.c_lo[(size_t)m * g.ldc + n] = (_Float16)(hs - (float)a);
          continue;
        }
        if (EPI == GEMM_TANH_BIAS) v = tanh_abs(v + bias);
        if (EPI == GEMM_BIAS) v += bias;
        if (EPI == GEMM_DTANH) {
          const float gg = g.aux[(size_t)m * g.ldaux + n];
          v *= 1.f - gg * gg;
        }
        if (g.accumulate && !split) v += cin[ml * g.ldc + nl];
        cw[ml * ldc + nl] = v;
        cmax = fmaxf(cmax, fabsf(v));
      }
  }
  if (g.cmax && !split) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cmax = fmaxf(cmax, __shfl_xor(cmax, o, 64));
    if (l == 0) atomicMax(g.cmax, __float_as_uint(cmax));
  }
}

// max |x| over a strided [rows][cols] fp32 matrix -> atomicMax slot (slot zeroed by the caller).
// Contiguous matrices (ld == cols, 16-B aligned, n % 4 == 0) are swept as one float4 stream;
// strided ones row by row (block-stride rows, thread-stride columns): no per-element division.
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ x, int rows, int cols, int ld,
                                                unsigned* __restrict__ slot, int flat4) {
  float mx = 0.f;
  if (flat4) {  // float4 pieces: of the whole array (ld == cols) or of each row (flat4 == 2: ld, cols % 4 == 0)
    const int c4 = cols / 4;
    const size_t n4 = (size_t)rows * c4;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
      size_t e = i;
      if (flat4 == 2) {
        const size_t rr = i / c4;
        e = rr * (ld / 4) + (i - rr * c4);
      }
      const float4 v = reinterpret_cast<const float4*>(x)[e];
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    for (int rr = blockIdx.x; rr < rows; rr += gridDim.x)
      for (int cc = threadIdx.x; cc < cols; cc += 256) mx = fmaxf(mx, fabsf(x[(size_t)rr * ld + cc]));
  }
  // one atomic per block (single-address atomics serialise at their L2 channel)
  __shared__ float red[4];
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(slot, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// column sums of a [rows][cols] matrix over the row range of layer blockIdx.y (rows_per rows):
// out[y * cols + c] (or, with one layer, out[c] (+)=) = sum_r x[r][c]; one thread per column, f64.
// Several layers: each layer's f64 sum as hi (plane y) + lo (plane gridDim.y + y), both reduced
// With weights wt (one per row): sum_r wt[r] x[r][c], each product formed in f64 (a column-weighted
// sum: the value head's dW3 = dout^T H2 at one output, memory-bound, wide_mlp.hip).
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ x, int rows, int cols, int ld, int rows_per,
                                                float* __restrict__ out, int accumulate, const float* __restrict__ wt) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  double s = 0.0;
  int rr = r0;
  // 8 independent loads in flight per thread, summed in row order (same result as the plain loop)
  for (; rr + 8 <= r1; rr += 8) {
    float v[8], u[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = x[(size_t)(rr + j) * ld + c];
      u[j] = wt ? wt[rr + j] : 1.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (double)u[j] * (double)v[j];
  }
  for (; rr < r1; ++rr) s += (double)(wt ? wt[rr] : 1.f) * (double)x[(size_t)rr * ld + c];
  if (gridDim.y > 1) {
    const float hi = (float)s;
    out[(size_t)blockIdx.y * cols + c] = hi;
    out[(size_t)(gridDim.y + blockIdx.y) * cols + c] = (float)(s - (double)hi);
  }
  else out[c] = accumulate ? out[c] + (float)s : (float)s;
}

// out[i] (+)= sum_z part[z][i] in a fixed order (f64): the second pass of split-K / split colsum;
// out is [rows][ld] with n = rows * cols elements per layer
__global__ __launch_bounds__(256) void k_split_reduce(const float* __restrict__ part, int splits, int rows, int cols,
                                                      float* __restrict__ out, int ld, int accumulate) {
  const size_t n = (size_t)rows * cols;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    double s = 0.0;
    for (int z = 0; z < splits; ++z) s += (double)part[(size_t)z * n + i];
    float* o = out + i;
    if (ld != cols) {  // strided destination (no division for the common contiguous case)
      const size_t rr = i / cols, cc = i - rr * cols;
      o = out + rr * ld + cc;
    }
    *o = accumulate ? *o + (float)s : (float)s;
  }
}

// the same for few outputs over many layers (bias column sums: 2,048 columns x 256 hi / lo layers at
// c5, where one thread per output left 8 workgroups summing 256 values each): 32 outputs x 8 layer
// groups per workgroup, each group summing its layers z = zg, zg + 8, ... in order, the 8 group sums
// then added in order (a fixed order: deterministic)
constexpr int SR_COLS = 32, SR_ZG = 8;
__global__ __launch_bounds__(SR_COLS * SR_ZG) void k_split_reduce_narrow(const float* __restrict__ part, int splits, int n,
                                                                         float* __restrict__ out, int accumulate) {
  __shared__ double red[SR_ZG][SR_COLS];
  const int c = threadIdx.x % SR_COLS, zg = threadIdx.x / SR_COLS;
  const int i = blockIdx.x * SR_COLS + c;
  double t = 0.0;
  if (i < n)
    for (int z = zg; z < splits; z += SR_ZG) t += (double)part[(size_t)z * n + i];
  red[zg][c] = t;
  __syncthreads();
  if (zg == 0 && i < n) {
#pragma unroll
    for (int g = 1; g < SR_ZG; ++g) t += red[g][c];
    out[i] = accumulate ? out[i] + (float)t : (float)t;
  }
}

int launch_split_reduce(const float* part, int splits, int rows, int cols, float* out, int ld, int accumulate,
                        hipStream_t s) {
  const size_t n = (size_t)rows * cols;
  if (ld == cols && n <= 16384 && splits >= 2 * SR_ZG) {
    hipLaunchKernelGGL(k_split_reduce_narrow, dim3((unsigned)cdiv((int64_t)n, SR_COLS)), dim3(SR_COLS * SR_ZG), 0, s,
                       part, splits, (int)n, out, accumulate);
    RLKS_LAUNCHED();
    return RLKS_OK;
  }
  const unsigned blocks = (unsigned)std::min<size_t>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(k_split_reduce, dim3(blocks), dim3(256), 0, s, part, splits, rows, cols, out, ld, accumulate);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

template <bool TA, bool TB>
static int launch_t(const GemmArgs& a, hipStream_t s) {
  const dim3 grid(cdiv(a.N, GT), cdiv(a.M, GT), a.splits > 1 ? a.splits : 1);
  const size_t lds = (size_t)2 * 4 * GCH * sizeof(_Float16);
  switch (a.epi) {
    case GEMM_STORE: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_STORE>), grid, dim3(256), lds, s, a); break;
    case GEMM_TANH_BIAS: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_TANH_BIAS>), grid, dim3(256), lds, s, a); break;
    case GEMM_BIAS: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_BIAS>), grid, dim3(256), lds, s, a); break;
    case GEMM_DTANH: hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_DTANH>), grid, dim3(256), lds, s, a); break;
    case GEMM_TANH_BIAS_PLANES:
      hipLaunchKernelGGL((k_gemm_sf16<TA, TB, GEMM_TANH_BIAS_PLANES>), grid, dim3(256), lds, s, a);
      break;
    default: return fail(RLKS_ERR_ARG, "gemm: unknown epilogue");
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}

static int launch_any(const GemmArgs& a, hipStream_t s) {
  if (!a.ta && !a.tb) return launch_t<false, false>(a, s);
  if (!a.ta && a.tb) return launch_t<false, true>(a, s);
  if (a.ta && !a.tb) return launch_t<true, false>(a, s);
  return launch_t<true, true>(a, s);
}

int gemm_splits(int M, int N, int K) {
  const int tiles = cdiv(M, GT) * cdiv(N, GT);
  int sp = std::max(1, 2048 / tiles);          // >= 2048 workgroups: 8 per CU
  sp = std::min(sp, std::max(1, K / 512));     // >= 16 K chunks per workgroup
  return std::min(sp, 64);
}

int launch_gemm_sf16(const GemmArgs& a, hipStream_t s) {
  RLKS_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0 && a.A && a.B && a.amax && a.bmax &&
                   (a.epi == GEMM_TANH_BIAS_PLANES ? (a.c_hi && a.c_lo) : a.C != nullptr),
               RLKS_ERR_ARG, "gemm: bad argument");
  if (a.splits <= 1) return launch_any(a, s);
  RLKS_REQUIRE(a.part && a.epi == GEMM_STORE, RLKS_ERR_ARG, "gemm: split-K needs a partial buffer and GEMM_STORE");
  // layers beyond the last non-empty K range would write zero partials: trim them
  const int kper = ((cdiv(a.K, a.splits) + GKC - 1) / GKC) * GKC;
  GemmArgs b = a;
  b.splits = cdiv(a.K, kper);
  if (int rc = launch_any(b, s)) return rc;
  return launch_split_reduce(a.part, b.splits, a.M, a.N, a.C, a.ldc, a.accumulate, s);
}

int launch_absmax(const float* x, int rows, int cols, int ld, unsigned* slot, hipStream_t s) {
  const size_t n = (size_t)rows * cols;
  const bool al = ((uintptr_t)x & 15) == 0;
  const int flat4 = (ld == cols && n % 4 == 0 && al) ? 1 : (ld % 4 == 0 && cols % 4 == 0 && al) ? 2 : 0;
  const size_t units = flat4 ? (n / 4 + 255) / 256 : (size_t)rows;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(2048, units));
  hipLaunchKernelGGL(k_absmax, dim3(blocks), dim3(256), 0, s, x, rows, cols, ld, slot, flat4);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int colsum_splits(int rows) { return std::min(128, std::max(1, rows / 512)); }

int launch_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate, float* part,
                  hipStream_t s, const float* wt) {
  const int sp = part ? colsum_splits(rows) : 1;
  const int rows_per = cdiv(rows, sp);
  hipLaunchKernelGGL(k_colsum, dim3(cdiv(cols, 256), sp), dim3(256), 0, s, x, rows, cols, ld, rows_per,
                     sp > 1 ? part : out, accumulate, wt);
  RLKS_LAUNCHED();
  if (sp == 1) return RLKS_OK;
  return launch_split_reduce(part, 2 * sp, 1, cols, out, cols, accumulate, s);
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
