// gemm_ps.hip — split-fp16 GEMM over PRE-SPLIT operands: fp16 hi / lo planes of x 2^e in HBM, staged
// into LDS by DMA (global_load_lds_dwordx4), no split arithmetic in the loop.  The wide policy MLP's
// three big GEMMs per net (config c5, fcnet_hiddens [2048, 2048]: SURVEY §8d "MFMA-bound update"):
//   Z2  = H1 W2^T          A = H1 planes [M][H] (K contiguous), B = W2 planes [H][H] (K contiguous)
//   dZ1 = (dZ2 W2)(1-H1^2) A = dZ2 planes [M][H],               B = W2 planes read K-major
//   dW2 = dZ2^T H1         A = dZ2 planes read K-major,         B = H1 planes read K-major (split-K)
// The generic kernel (gemm_sf16.hip) loads fp32 and splits on the way into LDS; its register ring
// could not keep two chunks in flight.  Here the operands arrive split, so a chunk is
// pure DMA issued one chunk ahead, and the loop is fragment reads + MFMAs.
//
// Tile 256 x 256 per 1024-thread workgroup (16 waves, 4 x 4 of 64 x 64 = 2 x 2 v_mfma_f32_32x32x16_f16
// tiles each, 64 accumulator registers: four waves per SIMD), K in chunks of 32 double-buffered in
// LDS (2 x 64 KB).  Operand images per chunk and plane:
//   K-contiguous ("N"): [256 rows][32 k], 16-byte piece q of row r at slot q ^ ((r >> 2) & 3): the
//     32x32x16 fragment reads (ds_read_b128, rows 32b + r, piece 2s + h) are conflict-free;
//   K-major ("T", stored [K][rows]): [32 k][256 rows], 16-byte piece p of k-row k at slot
//     p ^ 4 (k & 3), read by ds_read_b64_tr_b16 (4 k-rows x 16 rows per 16-lane group, one 8-byte
//     quad per lane, quads XOR 8 (k & 3)): conflict-free in each 32-lane half.
// Reference semantics: RLlib FCNet tanh layers (train_ppo.py:12; RLlib third-party).
#include "gemm_sf16.h"

namespace rlks {

using h8 = __attribute__((ext_vector_type(8))) _Float16;
using h4 = __attribute__((ext_vector_type(4))) _Float16;
using v4u = __attribute__((ext_vector_type(4))) unsigned;

namespace {

constexpr int PT = 256;          // output tile (rows and columns)
constexpr int PK = 32;           // K chunk
constexpr int PCH = PT * PK;     // halves per operand plane chunk
constexpr int PNT = 1024;        // threads per workgroup

__device__ __forceinline__ f32x16 mma(h8 a, h8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ int ps_exp(float mx) {
  if (!(mx > 0.f) || !(mx <= 3.4e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  return min(max(15 - e, -120), 120);
}
__device__ __forceinline__ int op_exp(const PsOperand& o) { return o.maxslot ? ps_exp(__uint_as_float(*o.maxslot)) : o.fexp; }

typedef __fp16 hf4_t __attribute__((vector_size(8)));
__device__ __forceinline__ h4 tr_read(const _Float16* p) {
  return __builtin_bit_cast(h4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) hf4_t*)(p)));
}

// DMA of one plane chunk (rows [r0, r0 + 256), k [k0, k0 + 32)) into its LDS image; each of the 16
// waves moves one 1 KB piece (64 lanes x 16 bytes).  Rows past the operand's extent are clamped to its
// last row / last 8-row piece (their results are never stored).
template <bool KM>
__device__ __forceinline__ void dma_plane(const _Float16* plane, int ld, int rows, int r0, int k0, _Float16* img, int w,
                                          int l) {
  const int sig = w * 64 + l;
  const _Float16* src;
  if (!KM) {
    const int r = sig >> 2, q = (sig & 3) ^ ((r >> 2) & 3);
    int kk = k0 + 8 * q;
    if (!dcheck(kk + 8 <= ld, DC_GEMM_K, kk)) kk = ld - 8;
    src = plane + (size_t)min(r0 + r, rows - 1) * ld + kk;
  } else {
    const int k = sig >> 5, p = (sig & 31) ^ (4 * (k & 3));
    int c = min(r0 + 8 * p, rows - 8);
    if (!dcheck(c >= 0 && c + 8 <= ld, DC_GEMM_K, c)) c = 0;
    src = plane + (size_t)(k0 + k) * ld + c;
  }
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(img + w * 512), 16, 0, 0);
}

// (hi, lo) fragment of the 32-row block at image row rb, k-step s (lane: row rb + r, k 16 s + 8 h + j)
template <bool KM>
__device__ __forceinline__ void frag(const _Float16* img, int rb, int s, int l, h8& fh, h8& fl) {
  if (!KM) {
    const int r = l & 31, h = l >> 5, row = rb + r;
    const int off = row * PK + 8 * ((2 * s + h) ^ ((row >> 2) & 3));
    fh = *reinterpret_cast<const h8*>(img + off);
    fl = *reinterpret_cast<const h8*>(img + PCH + off);
  } else {
    const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    const int kb = 16 * s + 8 * (g >> 1), quad = ((rb + 16 * (g & 1)) >> 2) + p;
    const int o0 = (kb + q) * PT + 4 * (quad ^ (8 * q)), o1 = o0 + 4 * PT;
    fh = __builtin_shufflevector(tr_read(img + o0), tr_read(img + o1), 0, 1, 2, 3, 4, 5, 6, 7);
    fl = __builtin_shufflevector(tr_read(img + PCH + o0), tr_read(img + PCH + o1), 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace

template <bool AK, bool BK, int EPI>
__global__ __launch_bounds__(PNT) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_gemm_ps(PsArgs g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  _Float16* sm = reinterpret_cast<_Float16*>(lds);  // [2 buf][A hi, A lo, B hi, B lo][PCH]
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), r = l & 31;
  const int wm = w >> 2, wn = w & 3;
  // XCD-aware tile order (no split-K): workgroups are dealt round-robin over the 8 XCDs in dispatch
  // order (x fastest), so dispatch slot b runs on XCD b % 8.  Give XCD j the tiles [j T/8, (j + 1) T/8)
  // in row-major order (n fastest): an XCD's concurrent workgroups then cover a few M row blocks with
  // all their N tiles, and each A row block (the large operand: M x K planes, 512 MB at c5) comes from
  // HBM once into that XCD's L2 instead of once per N tile into every XCD.
  int bx = blockIdx.x, by = blockIdx.y;
  if (gridDim.z == 1 && ((gridDim.x * gridDim.y) & 7) == 0) {
    const int T = gridDim.x * gridDim.y, b = blockIdx.y * gridDim.x + blockIdx.x;
    const int t = (b & 7) * (T >> 3) + (b >> 3);
    bx = t % gridDim.x;
    by = t / gridDim.x;
  }
  const int n0 = bx * PT, m0 = by * PT;
  const int ea = op_exp(g.a), eb = op_exp(g.b);
  // rounding-bias cancellation (sgd_sf16.hip tile_sign) in the dZ1 GEMM: workgroups alternate the
  // sign of their A fragments by row block, and unscale negates the result back, so the slight
  // negative lean of the MFMA accumulation does not add up coherently in db1 = colsum(dZ1).  Only
  // here: without it pi.b1 sat at 4.4x fp32 (p50, 4096 rows); on every GEMM it cost 3-4.5% of their
  // time for no measurable gain (profiles/r05_precision)
  const bool neg = EPI == PS_DTANH && ((by + (int)blockIdx.z) & 1) != 0;
  const unsigned nmask = neg ? 0x80008000u : 0u;
  const float unscale = (neg ? -1.f : 1.f) * ldexpf(1.f, -ea - eb);
  // this workgroup's K range (split-K: layer z)
  const int kper = g.splits > 1 ? ((g.K + g.splits - 1) / g.splits + PK - 1) / PK * PK : g.K;
  const int kb = blockIdx.z * kper, ke = min(g.K, kb + kper);
  const int nk = ke > kb ? (ke - kb) / PK : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  auto dma = [&](int c) {  // chunk c -> buffer c & 1: waves 0-15 each move one 1 KB piece per plane
    _Float16* b = sm + (c & 1) * 4 * PCH;
    const int k0 = kb + c * PK;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      dma_plane<AK>(pl ? g.a.lo : g.a.hi, g.a.ld, g.a.rows, m0, k0, b + pl * PCH, w, l);
      dma_plane<BK>(pl ? g.b.lo : g.b.hi, g.b.ld, g.b.rows, n0, k0, b + (2 + pl) * PCH, w, l);
    }
  };
  if (nk > 0) dma(0);
  for (int c = 0; c < nk; ++c) {
    vm_drain();       // this wave's pieces of chunk c have landed
    __syncthreads();  // ... and every wave's; buffer (c + 1) & 1 is no longer read
    if (c + 1 < nk) dma(c + 1);
    const _Float16* b = sm + (c & 1) * 4 * PCH;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      h8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        frag<AK>(b, wm * 64 + 32 * i, s, l, ah[i], al[i]);
        ah[i] = __builtin_bit_cast(h8, __builtin_bit_cast(v4u, ah[i]) ^ nmask);
        al[i] = __builtin_bit_cast(h8, __builtin_bit_cast(v4u, al[i]) ^ nmask);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) frag<BK>(b + 2 * PCH, wn * 64 + 32 * j, s, l, bh[j], bl[j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(al[i], bh[j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(ah[i], bl[j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(ah[i], bh[j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);  // one k-step's fragments live at a time (128 registers)
    }
  }

  // epilogue: C rows m = m0 + 64 wm + 32 i + acc_row(q), column n = n0 + 64 wn + 32 j + r
  const bool split = g.splits > 1;
  float* const Cout = split ? g.part + (size_t)blockIdx.z * g.M * g.N : g.C;
  const int ldc = split ? g.N : g.ldc;
  float cmax = 0.f;
  // the wave's 64 x 64 block from uniform base pointers (SGPRs) and 32-bit per-lane offsets: with a
  // 64-bit address per element the unrolled epilogue spilled (10-16 registers); -1.3% on the c5
  // gradient (profiles/r05_gemm).  Without the bounds branches it hoisted its loads and spilled more
  const int mw = m0 + wm * 64, nw = n0 + wn * 64;
  float* const cw = Cout + (size_t)mw * ldc + nw;
  _Float16* const hw = EPI == PS_TANH_BIAS_PLANES ? g.c_hi + (size_t)mw * ldc + nw : nullptr;
  _Float16* const lw = EPI == PS_TANH_BIAS_PLANES ? g.c_lo + (size_t)mw * ldc + nw : nullptr;
  const _Float16* const ahw = EPI == PS_DTANH ? g.aux_hi + (size_t)mw * g.ldaux + nw : nullptr;
  const _Float16* const alw = EPI == PS_DTANH ? g.aux_lo + (size_t)mw * g.ldaux + nw : nullptr;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nl = 32 * j + r, n = nw + nl;
    const bool nok = n < g.N;
    const float bias = (EPI == PS_TANH_BIAS || EPI == PS_TANH_BIAS_PLANES) && nok ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int qb = 0; qb < 16; qb += 8) {
        // dZ1: the batch's 8 aux (hi, lo) pairs loaded up front from clamped (always in-bounds)
        // addresses, so that their latencies overlap instead of each load waiting behind its
        // element's bounds branch (219 of dZ1's 1,900 µs at c5, profiles/r05_gemm)
        _Float16 gh[8], gl[8];
        if (EPI == PS_DTANH) {
          const int nc = min(n, g.N - 1) - nw;
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int mc = min(mw + 32 * i + acc_row(qb + t, l), g.M - 1) - mw;
            gh[t] = ahw[mc * g.ldaux + nc];
            gl[t] = alw[mc * g.ldaux + nc];
          }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int ml = 32 * i + acc_row(qb + t, l);  // C row mw + ml, column n
          if (!nok || mw + ml >= g.M) continue;
          const int off = ml * ldc + nl;
          float v = acc[i][j][qb + t] * unscale;
          if (EPI == PS_TANH_BIAS || EPI == PS_TANH_BIAS_PLANES)
            v = fmaf(-2.f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f((v + bias) * 2.885390081777927f) + 1.f), 1.f);
          if (EPI == PS_TANH_BIAS_PLANES) {  // H1 for the pre-split GEMMs: fp16 planes at 2^14
            const float hs = v * 16384.f;
            const _Float16 hh = (_Float16)hs;
            hw[off] = hh;
            lw[off] = (_Float16)(hs - (float)hh);
            continue;
          }
          if (EPI == PS_DTANH) {  // G = (hi + lo) 2^-14 from the aux planes
            const float gg = ((float)gh[t] + (float)gl[t]) * (1.f / 16384.f);
            v *= 1.f - gg * gg;
          }
          cw[off] = v;
          cmax = fmaxf(cmax, fabsf(v));
        }
        if (EPI == PS_DTANH) __builtin_amdgcn_sched_barrier(0);  // one batch's loads in flight at a time
      }
  }
  if (g.cmax && !split) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cmax = fmaxf(cmax, __shfl_xor(cmax, o, 64));
    if (l == 0) atomicMax(g.cmax, __float_as_uint(cmax));
  }
}

// planes of x 2^e (e from the max slot, or the fixed exponent when slot is null): hi = fp16(x 2^e),
// lo = fp16(x 2^e - hi); x [rows][ld] fp32 -> planes [rows][ldp]; one thread per 4 consecutive columns
__global__ __launch_bounds__(256) void k_split_planes(const float* __restrict__ x, int rows, int cols, int ld,
                                                      const unsigned* __restrict__ maxslot, int fexp,
                                                      _Float16* __restrict__ hi, _Float16* __restrict__ lo, int ldp) {
  const int e = maxslot ? ps_exp(__uint_as_float(*maxslot)) : fexp;
  const float s = ldexpf(1.f, e);
  const int cq = cols / 4;
  const size_t n = (size_t)rows * cq;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const size_t rr = i / cq;
    const int c4 = (int)(i - rr * cq) * 4;
    const float4 v = *reinterpret_cast<const float4*>(x + rr * ld + c4);
    const float e4[4] = {v.x, v.y, v.z, v.w};
    h4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const _Float16 t = (_Float16)(e4[j] * s);
      a[j] = t;
      b[j] = (_Float16)(e4[j] * s - (float)t);
    }
    *reinterpret_cast<h4*>(hi + rr * ldp + c4) = a;
    *reinterpret_cast<h4*>(lo + rr * ldp + c4) = b;
  }
}

template <bool AK, bool BK>
static int launch_ps_t(const PsArgs& a, hipStream_t s) {
  const dim3 grid(cdiv(a.N, PT), cdiv(a.M, PT), a.splits > 1 ? a.splits : 1);
  const size_t lds = (size_t)2 * 4 * PCH * sizeof(_Float16);
  switch (a.epi) {
    case PS_STORE: hipLaunchKernelGGL((k_gemm_ps<AK, BK, PS_STORE>), grid, dim3(PNT), lds, s, a); break;
    case PS_TANH_BIAS: hipLaunchKernelGGL((k_gemm_ps<AK, BK, PS_TANH_BIAS>), grid, dim3(PNT), lds, s, a); break;
    case PS_DTANH: hipLaunchKernelGGL((k_gemm_ps<AK, BK, PS_DTANH>), grid, dim3(PNT), lds, s, a); break;
    case PS_TANH_BIAS_PLANES:
      hipLaunchKernelGGL((k_gemm_ps<AK, BK, PS_TANH_BIAS_PLANES>), grid, dim3(PNT), lds, s, a);
      break;
    default: return fail(RLKS_ERR_ARG, "gemm_ps: unknown epilogue");
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int launch_gemm_ps(const PsArgs& a, hipStream_t s) {
  RLKS_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0 && a.K % PK == 0 &&
                   (a.epi == PS_TANH_BIAS_PLANES ? (a.c_hi && a.c_lo) : a.C != nullptr),
               RLKS_ERR_ARG, "gemm_ps: K must be a positive multiple of 32");
  RLKS_REQUIRE((!a.a.kmajor || a.a.rows % 8 == 0) && (!a.b.kmajor || a.b.rows % 8 == 0), RLKS_ERR_ARG,
               "gemm_ps: a K-major operand needs a multiple of 8 rows");
  PsArgs b = a;
  if (a.splits > 1) {
    RLKS_REQUIRE(a.part && a.epi == PS_STORE, RLKS_ERR_ARG, "gemm_ps: split-K needs a partial buffer and PS_STORE");
    const int kper = (cdiv(a.K, a.splits) + PK - 1) / PK * PK;
    b.splits = cdiv(a.K, kper);
  }
  int rc;
  if (!a.a.kmajor && !a.b.kmajor) rc = launch_ps_t<false, false>(b, s);
  else if (!a.a.kmajor) rc = launch_ps_t<false, true>(b, s);
  else if (!a.b.kmajor) rc = launch_ps_t<true, false>(b, s);
  else rc = launch_ps_t<true, true>(b, s);
  if (rc || a.splits <= 1) return rc;
  return launch_split_reduce(a.part, b.splits, a.M, a.N, a.C, a.ldc, 0, s);
}

int launch_split_planes(const float* x, int rows, int cols, int ld, const unsigned* maxslot, int fexp, _Float16* hi,
                        _Float16* lo, int ldp, hipStream_t s) {
  RLKS_REQUIRE(cols % 4 == 0 && ld % 4 == 0 && ldp % 4 == 0 && ((uintptr_t)x & 15) == 0, RLKS_ERR_ARG,
               "split_planes: columns / strides must be multiples of 4, x 16-byte aligned");
  const size_t n = (size_t)rows * (cols / 4);
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(8192, (n + 255) / 256));
  hipLaunchKernelGGL(k_split_planes, dim3(blocks), dim3(256), 0, s, x, rows, cols, ld, maxslot, fexp, hi, lo, ldp);
  RLKS_LAUNCHED();
  return RLKS_OK;
}

// ps_gemm tile count (split-K sizing): ~256 workgroups (one per CU) of >= 16 K chunks
int gemm_ps_splits(int M, int N, int K) {
  const int tiles = cdiv(M, PT) * cdiv(N, PT);
  int sp = std::max(1, 256 / tiles);
  sp = std::min(sp, std::max(1, K / (16 * PK)));
  return std::min(sp, 64);
}

}  // namespace rlks
