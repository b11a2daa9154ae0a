// calib.hip — librlks_calib.so: the sustained f16 MFMA rate of this chip, measured inside the
// bench process (bench.py roofline.calibration).  Not part of the product path.
//
// One wave per SIMD (256 threads per workgroup, one workgroup per CU), eight independent
// accumulators per wave, operands loaded from a buffer of random fp16 values (the rate on random
// data is what the SGD kernels see: zero or constant operands let the chip clock higher,
// MI355X_MICROARCH.md "DVFS give-back"), back-to-back issue for `iters` x 8 MFMAs per wave.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
using h8 = __attribute__((ext_vector_type(8))) _Float16;
using f4 = __attribute__((ext_vector_type(4))) float;
using f16v = __attribute__((ext_vector_type(16))) float;

template <int SHAPE>  // 0: v_mfma_f32_16x16x32_f16 (F1a / F1b), 1: v_mfma_f32_32x32x16_f16 (F2)
__global__ __launch_bounds__(256) void k_rate(const _Float16* __restrict__ rnd, float* __restrict__ out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  h8 a[2], b[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    a[i] = *reinterpret_cast<const h8*>(rnd + ((size_t)t * 32 + 16 * i) % (1 << 20));
    b[i] = *reinterpret_cast<const h8*>(rnd + ((size_t)t * 32 + 16 * i + 8) % (1 << 20));
  }
  f4 c4[8];
  f16v c16[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c4[i] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 16; ++q) c16[i][q] = 0.f;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (SHAPE == 0) c4[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 1], b[(i >> 1) & 1], c4[i], 0, 0, 0);
      else c16[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i & 1], b[(i >> 1) & 1], c16[i], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (SHAPE == 0)
      for (int q = 0; q < 4; ++q) s += c4[i][q];
    else
      for (int q = 0; q < 16; ++q) s += c16[i][q];
  }
  out[t] = s;
}
}  // namespace

extern "C" {
// TFLOP/s of the chip running `shape` (0: 16x16x32 f16, 1: 32x32x16 f16) back to back on random
// operands, over `iters` x 8 MFMAs per wave on `cus` workgroups of four waves; rnd: 2^20 random
// fp16 values; out: cus x 256 floats; time over `reps` launches on `stream` by HIP events
int rlks_calib_mfma_f16(int shape, int cus, int iters, int reps, const void* rnd, float* out, void* stream,
                        double* tflops) {
  if (!rnd || !out || !tflops || cus <= 0 || iters <= 0 || reps <= 0) return 1;
  hipStream_t s = (hipStream_t)stream;
  auto launch = [&]() {
    if (shape == 0) hipLaunchKernelGGL(k_rate<0>, dim3(cus), dim3(256), 0, s, (const _Float16*)rnd, out, iters);
    else hipLaunchKernelGGL(k_rate<1>, dim3(cus), dim3(256), 0, s, (const _Float16*)rnd, out, iters);
  };
  launch();  // warm
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 2;
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  const double flop_per_mfma = shape == 0 ? 2.0 * 16 * 16 * 32 : 2.0 * 32 * 32 * 16;
  const double flops = flop_per_mfma * 8.0 * iters * 4.0 * cus * reps;
  *tflops = ms > 0.f ? flops / (ms * 1e-3) / 1e12 : 0.0;
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
}
