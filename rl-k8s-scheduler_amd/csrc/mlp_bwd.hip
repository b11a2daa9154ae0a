// mlp_bwd.hip — F2 and F3: the hidden-layer backward of one net (pi or vf).
//
// F2  dW2[n][k] = sum_m dZ2[m][n] H1[m][k]       (a 256 x 256 output, reduction over the rows)
//     grid = 4 output tiles of 128 x 128 x S row splits; H1 is recomputed from X (K = D = 6,
//     VALU) into LDS instead of being stored by F1 and re-read; each split writes its 128 x 128
//     fp32 partial, summed later in a fixed order (bit-reproducible).
// F3  dH1[m][k] = sum_n dZ2[m][n] W2[n][k]        (M x 256, reduction over the 256 hidden units)
//     then dZ1 = dH1 * (1 - H1^2) with H1 recomputed, and per-tile partials of
//     dW1[k][d] = sum_m dZ1[m][k] X[m][d], db1[k] = sum_m dZ1[m][k]  (dZ1 never leaves the chip).
// Both: 256-thread workgroups of 4 waves, each wave a 64 x 64 output (2 x 2 tiles of
// v_mfma_f32_32x32x2_f32), operands staged through LDS in 32-deep chunks with the next chunk's
// global loads in flight in registers during the MFMAs.
#include "mlp_common.h"

namespace rlks {

template <int DD>
__global__ __launch_bounds__(256) void k_dw2(Dw2Args g) {
  constexpr int H = HID, ds = DD + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sA = lds;                // [BK][GB]      dZ2 chunk [m][n]
  float* sB = sA + BK * GB;       // [BK][GB]      H1 chunk  [m][k]
  float* sb1 = sB + BK * GB;      // [GB]
  float* sW1 = sb1 + GB;          // [GB][DD+1]
  float* sX = sW1 + GB * ds;      // [2][BK][DD+1] double-buffered X rows

  const int tn = blockIdx.x >> 1, tk = blockIdx.x & 1, net = blockIdx.z;
  const int n0 = tn * GB, k0 = tk * GB;
  const NetPtrs P = g.P[net];
  const float* dz2 = g.dz2[net];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int h = l >> 5, li = l & 31;
  const int mbeg = blockIdx.y * g.rows_per_split, mend = mbeg + g.rows_per_split;

  for (int e = tid; e < GB * DD; e += 256) sW1[(e / DD) * ds + (e % DD)] = P.w1[(size_t)k0 * DD + e];
  for (int e = tid; e < GB; e += 256) sb1[e] = P.b1[k0 + e];

  float4 pa0, pa1, pa2, pa3;
  constexpr int XN = (BK * DD + 255) / 256;  // X values per thread per 32-row chunk
  float px[XN];
#define DW2_LOAD(mc)                                                                                \
  do {                                                                                              \
    const float* src_ = dz2 + (size_t)((mc) + (tid >> 5)) * H + n0 + 4 * (tid & 31);                   \
    pa0 = *reinterpret_cast<const float4*>(src_);                                                   \
    pa1 = *reinterpret_cast<const float4*>(src_ + 8 * H);                                           \
    pa2 = *reinterpret_cast<const float4*>(src_ + 16 * H);                                          \
    pa3 = *reinterpret_cast<const float4*>(src_ + 24 * H);                                          \
  } while (0)
#define DW2_LOAD_X(mc)                                                                              \
  _Pragma("unroll") for (int i_ = 0; i_ < XN; ++i_) {                                               \
    const int e_ = tid + 256 * i_;                                                                  \
    if (e_ < BK * DD) px[i_] = g.x[(size_t)((mc) + e_ / DD) * g.x_stride + e_ % DD];                \
  }
#define DW2_STORE_X(b)                                                                              \
  _Pragma("unroll") for (int i_ = 0; i_ < XN; ++i_) {                                               \
    const int e_ = tid + 256 * i_;                                                                  \
    if (e_ < BK * DD) sX[(b) * BK * ds + (e_ / DD) * ds + e_ % DD] = px[i_];                        \
  }
  DW2_LOAD_X(mbeg);
  DW2_STORE_X(0);
  DW2_LOAD(mbeg);
  if (mbeg + BK < mend) DW2_LOAD_X(mbeg + BK);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  __syncthreads();
  int buf = 0;
  for (int mc = mbeg; mc < mend; mc += BK) {
    {
      float* dst = sA + (tid >> 5) * GB + 4 * (tid & 31);
      *reinterpret_cast<float4*>(dst) = pa0;
      *reinterpret_cast<float4*>(dst + 8 * GB) = pa1;
      *reinterpret_cast<float4*>(dst + 16 * GB) = pa2;
      *reinterpret_cast<float4*>(dst + 24 * GB) = pa3;
    }
    if (mc + BK < mend) { DW2_STORE_X(buf ^ 1); }
    // H1 recompute: sB[m][k] = tanh(b1[k] + X[m] . W1[k]); the row is wave-uniform
    const float* xb = sX + buf * BK * ds;
    {
      const int kk = tid & (GB - 1);
      float wr[DD];
#pragma unroll
      for (int d = 0; d < DD; ++d) wr[d] = sW1[kk * ds + d];
      const float bb = sb1[kk];
#pragma unroll 4
      for (int row = tid >> 7; row < BK; row += 2) {
        float z = bb;
#pragma unroll
        for (int d = 0; d < DD; ++d) z = fmaf(xb[row * ds + d], wr[d], z);
        sB[row * GB + kk] = fast_tanh(z);
      }
    }
    __syncthreads();
    if (mc + BK < mend) DW2_LOAD(mc + BK);
    if (mc + 2 * BK < mend) DW2_LOAD_X(mc + 2 * BK);
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
    buf ^= 1;
  }
  float* out = g.part[net] + (size_t)blockIdx.y * H * H;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(size_t)(n0 + wm * 64 + i * 32 + acc_row(r, l)) * H + k0 + wn * 64 + j * 32 + li] = acc[i][j][r];
}

template <int DD>
__global__ __launch_bounds__(256) void k_dh1(Dh1Args g) {
  constexpr int H = HID, ds = DD + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sA = lds;                    // [GB][BK+1]  dZ2 chunk [m][n]
  float* sB = sA + GB * (BK + 1);     // [BK][GB]    W2 chunk  [n][k]
  float* sb1 = sB + BK * GB;          // [GB]
  float* sX = sb1 + GB;               // [GB][DD+1]
  float* sW1 = sX + GB * ds;          // [GB][DD+1]
  float* sRed = sA;                   // epilogue reuse: [2][GB][DD+1]
  static_assert(2 * GB * ds <= GB * (BK + 1) + BK * GB, "dW1 reduction must fit in the staging buffers");

  const int tile = blockIdx.x, tk = blockIdx.y, net = blockIdx.z;
  const int m0 = tile * GB, k0 = tk * GB;
  const NetPtrs P = g.P[net];
  const float* dz2 = g.dz2[net];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int h = l >> 5, li = l & 31;

  for (int e = tid; e < GB * DD; e += 256) {
    sX[(e / DD) * ds + (e % DD)] = g.x[(size_t)(m0 + e / DD) * g.x_stride + (e % DD)];
    sW1[(e / DD) * ds + (e % DD)] = P.w1[(size_t)k0 * DD + e];
  }
  for (int e = tid; e < GB; e += 256) sb1[e] = P.b1[k0 + e];

  // per thread: dZ2 rows (tid >> 3) + 32 j, columns 4 (tid & 7); W2 rows (tid >> 5) + 8 j
  float4 pa0, pa1, pa2, pa3, pb0, pb1, pb2, pb3;
#define DH1_LOAD(nc)                                                                                 \
  do {                                                                                               \
    const float* sa_ = dz2 + (size_t)(m0 + (tid >> 3)) * H + (nc) + 4 * (tid & 7);                   \
    const float* sb_ = P.w2 + (size_t)((nc) + (tid >> 5)) * H + k0 + 4 * (tid & 31);                 \
    pa0 = *reinterpret_cast<const float4*>(sa_);                                                     \
    pa1 = *reinterpret_cast<const float4*>(sa_ + 32 * H);                                            \
    pa2 = *reinterpret_cast<const float4*>(sa_ + 64 * H);                                            \
    pa3 = *reinterpret_cast<const float4*>(sa_ + 96 * H);                                            \
    pb0 = *reinterpret_cast<const float4*>(sb_);                                                     \
    pb1 = *reinterpret_cast<const float4*>(sb_ + 8 * H);                                             \
    pb2 = *reinterpret_cast<const float4*>(sb_ + 16 * H);                                            \
    pb3 = *reinterpret_cast<const float4*>(sb_ + 24 * H);                                            \
  } while (0)
  DH1_LOAD(0);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (int nc = 0; nc < H; nc += BK) {
    {
      float* da = sA + (tid >> 3) * (BK + 1) + 4 * (tid & 7);
      const float4 v[4] = {pa0, pa1, pa2, pa3};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float* d = da + j * 32 * (BK + 1);
        d[0] = v[j].x; d[1] = v[j].y; d[2] = v[j].z; d[3] = v[j].w;
      }
      float* db = sB + (tid >> 5) * GB + 4 * (tid & 31);
      *reinterpret_cast<float4*>(db) = pb0;
      *reinterpret_cast<float4*>(db + 8 * GB) = pb1;
      *reinterpret_cast<float4*>(db + 16 * GB) = pb2;
      *reinterpret_cast<float4*>(db + 24 * GB) = pb3;
    }
    __syncthreads();
    if (nc + BK < H) DH1_LOAD(nc + BK);
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

  // epilogue: dZ1 = dH1 * (1 - H1^2), H1 recomputed; per-column sums over this tile's rows
  float pw[2][DD + 1];
  float wr[2][DD], bb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kk = wn * 64 + j * 32 + li;
#pragma unroll
    for (int d = 0; d < DD; ++d) wr[j][d] = sW1[kk * ds + d];
    bb[j] = sb1[kk];
#pragma unroll
    for (int d = 0; d <= DD; ++d) pw[j][d] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll 4
    for (int r = 0; r < 16; ++r) {
      const float* xr = sX + (wm * 64 + i * 32 + acc_row(r, l)) * ds;
      float xv[DD];
#pragma unroll
      for (int d = 0; d < DD; ++d) xv[d] = xr[d];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float z = bb[j];
#pragma unroll
        for (int d = 0; d < DD; ++d) z = fmaf(xv[d], wr[j][d], z);
        const float h1 = fast_tanh(z);
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
      float* dst = sRed + (wm * GB + wn * 64 + j * 32 + l) * ds;
#pragma unroll
      for (int d = 0; d <= DD; ++d) dst[d] = pw[j][d];
    }
  }
  __syncthreads();
  for (int e = tid; e < GB * ds; e += 256) {
    const int kk = e / ds, d = e - kk * ds;
    const float s = sRed[kk * ds + d] + sRed[(GB + kk) * ds + d];
    if (d == DD)
      g.part_b1[net][(size_t)tile * H + k0 + kk] = s;
    else
      g.part_w1[net][((size_t)tile * H + k0 + kk) * DD + d] = s;
  }
}

#undef DW2_LOAD
#undef DW2_LOAD_X
#undef DW2_STORE_X
#undef DH1_LOAD

int launch_dw2(const Dw2Args& a, int D, int splits, hipStream_t s) {
  const size_t lds = ((size_t)2 * BK * GB + GB + (size_t)GB * (D + 1) + (size_t)2 * BK * (D + 1)) * sizeof(float);
  const dim3 grid((HID / GB) * (HID / GB), splits, 2);
  switch (D) {
    case 6: hipLaunchKernelGGL(k_dw2<6>, grid, dim3(256), lds, s, a); break;
    case 12: hipLaunchKernelGGL(k_dw2<12>, grid, dim3(256), lds, s, a); break;
    case 24: hipLaunchKernelGGL(k_dw2<24>, grid, dim3(256), lds, s, a); break;
    default: return fail(RLKS_ERR_UNSUPPORTED, "PPO gradient kernels are built for obs_dim 6, 12 or 24");
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}

int launch_dh1(const Dh1Args& a, int D, hipStream_t s) {
  const size_t lds = ((size_t)GB * (BK + 1) + BK * GB + GB + (size_t)2 * GB * (D + 1)) * sizeof(float);
  const dim3 grid(a.M / GB, HID / GB, 2);
  switch (D) {
    case 6: hipLaunchKernelGGL(k_dh1<6>, grid, dim3(256), lds, s, a); break;
    case 12: hipLaunchKernelGGL(k_dh1<12>, grid, dim3(256), lds, s, a); break;
    case 24: hipLaunchKernelGGL(k_dh1<24>, grid, dim3(256), lds, s, a); break;
    default: return fail(RLKS_ERR_UNSUPPORTED, "PPO gradient kernels are built for obs_dim 6, 12 or 24");
  }
  RLKS_LAUNCHED();
  return RLKS_OK;
}

}  // namespace rlks
