// sf16_layout.hip — hardware check of the operand maps the split-fp16 SGD kernels rely on
// (v_mfma_f32_32x32x16_f16 on gfx950), with exact small-integer data and asymmetric operands:
//   1. natural A/B lane maps: lane (r = l&31, h = l>>5) holds A[r][8h+j], B[8h+j][r]
//   2. an accumulator X (32x32) as the B operand of the next MFMA (Y = A . X): regs 8s..8s+7 of
//      step s carry X rows perm(s,h,j) = 16s + 8(j>>2) + 4h + (j&3)
//   3. the same accumulator as the A operand (Z = X^T . B)
//   4. split-fp16 (hi + lo, three products) dot products vs fp64 on random fp32 data
// build: hipcc --offload-arch=gfx950 -O3 sf16_layout.hip -o sf16_layout
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ int acc_row(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }
__device__ __forceinline__ int perm(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }

// X = P . Q (natural maps, K = 32 in two steps); Y = A . X; Z = X^T . B
__global__ void k_check(const float* P, const float* Q, const float* Am, const float* Bm, float* X, float* Y,
                        float* Z) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16 x = {};
  for (int s = 0; s < 2; ++s) {
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = (_Float16)P[r * 32 + 16 * s + 8 * h + j];
      b[j] = (_Float16)Q[(16 * s + 8 * h + j) * 32 + r];
    }
    x = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, x, 0, 0, 0);
  }
  for (int q = 0; q < 16; ++q) X[acc_row(q, h) * 32 + r] = x[q];
  f32x16 y = {}, z = {};
  for (int s = 0; s < 2; ++s) {
    f16x8 xa, a, b;
    for (int j = 0; j < 8; ++j) {
      xa[j] = (_Float16)x[8 * s + j];
      a[j] = (_Float16)Am[r * 32 + perm(s, h, j)];  // A[i][k] in X's permuted row order
      b[j] = (_Float16)Bm[perm(s, h, j) * 32 + r];  // B[k][j] likewise
    }
    y = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, xa, y, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa, b, z, 0, 0, 0);
  }
  for (int q = 0; q < 16; ++q) {
    Y[acc_row(q, h) * 32 + r] = y[q];
    Z[acc_row(q, h) * 32 + r] = z[q];
  }
}

__device__ __forceinline__ void split(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);
}

// D = A . B with K = 256 by three split products, operands scaled by powers of two
__global__ void k_split(const float* A, const float* B, float sa, float sb, float* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16 d = {};
  for (int s = 0; s < 16; ++s) {
    f16x8 ah, al, bh, bl;
    for (int j = 0; j < 8; ++j) {
      _Float16 t0, t1;
      split(A[r * 256 + 16 * s + 8 * h + j] * sa, t0, t1);
      ah[j] = t0; al[j] = t1;
      split(B[(16 * s + 8 * h + j) * 32 + r] * sb, t0, t1);
      bh[j] = t0; bl[j] = t1;
    }
    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, d, 0, 0, 0);
  }
  for (int q = 0; q < 16; ++q) D[acc_row(q, h) * 32 + r] = d[q] / (sa * sb);
}

int main() {
  const int n = 32 * 32;
  std::vector<float> P(n), Q(n), Am(n), Bm(n);
  srand(1);
  for (int i = 0; i < n; ++i) {
    P[i] = (float)(rand() % 7 - 3);
    Q[i] = (float)(rand() % 5 - 2) + (i % 3 == 0 ? 1.f : 0.f);
    Am[i] = (float)(rand() % 5 - 2);
    Bm[i] = (float)((i * 7) % 5 - 2);
  }
  float *dP, *dQ, *dA, *dB, *dX, *dY, *dZ;
  hipMalloc(&dP, n * 4); hipMalloc(&dQ, n * 4); hipMalloc(&dA, n * 4); hipMalloc(&dB, n * 4);
  hipMalloc(&dX, n * 4); hipMalloc(&dY, n * 4); hipMalloc(&dZ, n * 4);
  hipMemcpy(dP, P.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dQ, Q.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dA, Am.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, Bm.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, dP, dQ, dA, dB, dX, dY, dZ);
  std::vector<float> X(n), Y(n), Z(n);
  hipMemcpy(X.data(), dX, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(Y.data(), dY, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(Z.data(), dZ, n * 4, hipMemcpyDeviceToHost);
  int bad[3] = {0, 0, 0};
  std::vector<double> Xr(n);
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double s = 0;
      for (int k = 0; k < 32; ++k) s += (double)P[i * 32 + k] * Q[k * 32 + j];
      Xr[i * 32 + j] = s;
      bad[0] += s != X[i * 32 + j];
    }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double y = 0, z = 0;
      for (int k = 0; k < 32; ++k) {
        y += (double)Am[i * 32 + k] * Xr[k * 32 + j];  // Y = A . X
        z += Xr[k * 32 + i] * (double)Bm[k * 32 + j];  // Z = X^T . B
      }
      bad[1] += y != Y[i * 32 + j];
      bad[2] += z != Z[i * 32 + j];
    }
  printf("natural maps: %s (%d bad)\n", bad[0] ? "FAIL" : "PASS", bad[0]);
  printf("acc as B (A.X): %s (%d bad)\n", bad[1] ? "FAIL" : "PASS", bad[1]);
  printf("acc as A (X^T.B): %s (%d bad)\n", bad[2] ? "FAIL" : "PASS", bad[2]);

  // split precision, K = 256
  std::vector<float> SA(32 * 256), SB(256 * 32);
  for (auto& v : SA) v = (float)((rand() / (double)RAND_MAX) * 2 - 1) * 0.37f;
  for (auto& v : SB) v = (float)((rand() / (double)RAND_MAX) * 2 - 1) * 1e-6f;
  float *dSA, *dSB, *dD;
  hipMalloc(&dSA, SA.size() * 4); hipMalloc(&dSB, SB.size() * 4); hipMalloc(&dD, n * 4);
  hipMemcpy(dSA, SA.data(), SA.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dSB, SB.data(), SB.size() * 4, hipMemcpyHostToDevice);
  // scales: max|A| = 0.37 -> 2^15; max|B| = 1e-6 -> 2^34
  hipLaunchKernelGGL(k_split, dim3(1), dim3(64), 0, 0, dSA, dSB, 32768.f, 17179869184.f, dD);
  std::vector<float> D(n);
  hipMemcpy(D.data(), dD, n * 4, hipMemcpyDeviceToHost);
  double num = 0, den = 0, mx = 0, f32num = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double s = 0, sabs = 0;
      float f = 0.f;
      for (int k = 0; k < 256; ++k) {
        s += (double)SA[i * 256 + k] * SB[k * 32 + j];
        sabs += fabs((double)SA[i * 256 + k] * SB[k * 32 + j]);
        f = fmaf(SA[i * 256 + k], SB[k * 32 + j], f);
      }
      num += (D[i * 32 + j] - s) * (D[i * 32 + j] - s);
      f32num += (f - s) * (f - s);
      den += s * s;
      mx = fmax(mx, fabs(D[i * 32 + j] - s) / sabs);
    }
  printf("split-fp16 K=256: rel err (norm) %.3e, max err / sum|ab| %.3e; fp32 fmaf chain rel err %.3e\n",
         sqrt(num / den), mx, sqrt(f32num / den));
  hipError_t e = hipDeviceSynchronize();
  printf("hip: %s\n", hipGetErrorString(e));
  return (bad[0] || bad[1] || bad[2] || sqrt(num / den) > 1e-5) ? 1 : 0;
}
