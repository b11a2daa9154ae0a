// mfma_rate.hip — cycles per MFMA on one SIMD (one wave per SIMD, every CU busy), from
// s_memtime and from wall time, for the shapes the split-fp16 kernels could use:
//   f16 32x32x16 / bf16 32x32x16 / f16 16x16x32, 8 independent accumulators, and a 1-chain case;
//   operands in VGPRs vs in AGPR-resident accumulators.
// build: hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

using h8 = __attribute__((ext_vector_type(8))) _Float16;
using b8 = __attribute__((ext_vector_type(8))) __bf16;
using f16v = __attribute__((ext_vector_type(16))) float;
using f4v = __attribute__((ext_vector_type(4))) float;

constexpr int ITERS = 2000;

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k(float* out, unsigned long long* cyc,
                                                                                   float seed) {
  h8 a, b;
  b8 ab, bb;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)(seed * (threadIdx.x + j));
    b[j] = (_Float16)(seed * (threadIdx.x - j));
    ab[j] = (__bf16)(seed * (threadIdx.x + j));
    bb[j] = (__bf16)(seed * (threadIdx.x - j));
  }
  f16v acc[8];
  f4v acc4[8];
  for (int i = 0; i < 8; ++i) {
    for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    for (int q = 0; q < 4; ++q) acc4[i][q] = 0.f;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
      if (MODE == 1) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, acc[i], 0, 0, 0);
      if (MODE == 2) acc4[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc4[i], 0, 0, 0);
      if (MODE == 3) acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[0], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) {
    for (int q = 0; q < 16; ++q) s += acc[i][q];
    for (int q = 0; q < 4; ++q) s += acc4[i][q];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, double flop_per_mfma) {
  const int blocks = 256 * 4;  // 4 rounds over the CUs would serialise; use one block per CU x4 SIMDs
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8);
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, out, cyc, 1e-3f);
  hipDeviceSynchronize();
  auto t0 = std::chrono::high_resolution_clock::now();
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, out, cyc, 1e-3f);
  hipDeviceSynchronize();
  auto t1 = std::chrono::high_resolution_clock::now();
  unsigned long long c[256];
  hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  unsigned long long mx = 0, mn = ~0ull;
  for (int i = 0; i < 256; ++i) { mx = c[i] > mx ? c[i] : mx; mn = c[i] < mn ? c[i] : mn; }
  const double n = (double)ITERS * 8;
  const double sec = std::chrono::duration<double>(t1 - t0).count();
  const double tf = flop_per_mfma * n * 256 * 4 / sec / 1e12;
  printf("%-28s memtime cyc/MFMA %.1f .. %.1f   wall %.3f ms  -> %.0f TFLOP/s (whole chip)\n", name, mn / n, mx / n,
         sec * 1e3, tf);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0>("f16 32x32x16, 8 acc", 32.0 * 32 * 16 * 2);
  run<1>("bf16 32x32x16, 8 acc", 32.0 * 32 * 16 * 2);
  run<2>("f16 16x16x32, 8 acc", 16.0 * 16 * 32 * 2);
  run<3>("f16 32x32x16, 1 chain", 32.0 * 32 * 16 * 2);
  return 0;
}
