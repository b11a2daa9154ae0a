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
  h8 a[4], b[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const h8*>(rnd + ((size_t)t * 48 + 8 * i) % (1 << 20));
#pragma unroll
  for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const h8*>(rnd + ((size_t)t * 48 + 32 + 8 * i) % (1 << 20));
  float s = 0.f;
  // the eight MFMAs of an iteration as one asm block: written in C, the compiler register-renamed
  // the f32x4 accumulators with ~40 accumulator moves per 8 MFMAs (half the 16x16x32 rate); the
  // 32x32x16 form compiles clean either way.  Each accumulator is re-read 8 MFMAs after its write.
#define RATE_BODY(OP)                                                                        \
  asm volatile(OP " %0, %8, %12, %0\n\t" OP " %1, %9, %12, %1\n\t" OP " %2, %8, %13, %2\n\t"       \
               OP " %3, %9, %13, %3\n\t" OP " %4, %10, %12, %4\n\t" OP " %5, %11, %12, %5\n\t"     \
               OP " %6, %10, %13, %6\n\t" OP " %7, %11, %13, %7"                                   \
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)     \
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]))
  if constexpr (SHAPE == 0) {
    f4 c0{}, c1{}, c2{}, c3{}, c4{}, c5{}, c6{}, c7{};
    for (int it = 0; it < iters; ++it) RATE_BODY("v_mfma_f32_16x16x32_f16");
    const f4 r = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
    s = r[0] + r[1] + r[2] + r[3];
  } else {
    f16v c0{}, c1{}, c2{}, c3{}, c4{}, c5{}, c6{}, c7{};
    for (int it = 0; it < iters; ++it) RATE_BODY("v_mfma_f32_32x32x16_f16");
    const f16v r = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += r[q];
  }
#undef RATE_BODY
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
