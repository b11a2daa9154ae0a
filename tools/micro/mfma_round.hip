// mfma_round.hip — rounding behaviour of v_mfma_f32_16x16x32_f16 accumulation chains on gfx950:
// each output element is a K = 256 dot product of fp16 values (8 chained MFMAs, fp32 accumulator)
// with mixed signs (cancellation); compared per element against the exact sum (fp64 of exact fp16
// products) and against a sequential round-to-nearest fp32 accumulation of the same products.
// build: hipcc --offload-arch=gfx950 -O3 mfma_round.hip -o mfma_round
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using h8 = __attribute__((ext_vector_type(8))) _Float16;
using f4 = __attribute__((ext_vector_type(4))) float;

// one wave per 16 x 16 output block: A [16][256], B [256][16] (fp16), C [16][16]
__global__ void k_dot(const _Float16* A, const _Float16* B, float* C, int blocks) {
  const int blk = blockIdx.x, l = threadIdx.x, c = l & 15, g = l >> 4;
  if (blk >= blocks) return;
  const _Float16* a = A + (size_t)blk * 16 * 256;
  const _Float16* b = B + (size_t)blk * 256 * 16;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < 8; ++s) {
    h8 av, bv;
    for (int j = 0; j < 8; ++j) {
      av[j] = a[c * 256 + 32 * s + 8 * g + j];
      bv[j] = b[(32 * s + 8 * g + j) * 16 + c];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) C[(size_t)blk * 256 + (4 * g + i) * 16 + c] = acc[i];
}

int main() {
  const int blocks = 4096;
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<_Float16> A((size_t)blocks * 16 * 256), B((size_t)blocks * 256 * 16);
  for (auto& x : A) x = (_Float16)(nd(rng) * 1000.f);
  for (auto& x : B) x = (_Float16)(nd(rng) * 1000.f);
  _Float16 *dA, *dB;
  float* dC;
  hipMalloc(&dA, A.size() * 2);
  hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, (size_t)blocks * 256 * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_dot, dim3(blocks), dim3(64), 0, 0, dA, dB, dC, blocks);
  std::vector<float> C((size_t)blocks * 256);
  hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  std::vector<double> e_mf, e_seq, e_pair;
  double bias_mf = 0, bias_seq = 0;
  for (int blk = 0; blk < blocks; ++blk)
    for (int r = 0; r < 16; ++r)
      for (int c = 0; c < 16; ++c) {
        double ex = 0.0, sa = 0.0;
        float seq = 0.f;
        float part[8];
        for (int s = 0; s < 8; ++s) {
          float ps = 0.f;
          for (int k = 32 * s; k < 32 * s + 32; ++k) {
            const float p = (float)A[(size_t)blk * 4096 + r * 256 + k] * (float)B[(size_t)blk * 4096 + k * 16 + c];
            ex += (double)p;
            sa += fabs((double)p);
            seq += p;
            ps += p;
          }
          part[s] = ps;
        }
        float pair = 0.f;
        for (int s = 0; s < 8; ++s) pair += part[s];
        const double got = C[(size_t)blk * 256 + r * 16 + c];
        e_mf.push_back(fabs(got - ex) / sa);
        e_seq.push_back(fabs((double)seq - ex) / sa);
        e_pair.push_back(fabs((double)pair - ex) / sa);
        bias_mf += (got - ex) / sa;
        bias_seq += ((double)seq - ex) / sa;
      }
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q / 100.0 * (v.size() - 1))];
  };
  printf("K=256 dot products, |err| / sum|a b| (n=%zu)\n", e_mf.size());
  for (double q : {50.0, 90.0, 99.0, 100.0})
    printf("  p%-5.0f mfma %.3e   fp32 sequential %.3e   fp32 per-32 blocks %.3e\n", q, pct(e_mf, q), pct(e_seq, q),
           pct(e_pair, q));
  printf("  mean signed error / sum|ab|: mfma %.3e, fp32 sequential %.3e\n", bias_mf / e_mf.size(),
         bias_seq / e_seq.size());
  return 0;
}
