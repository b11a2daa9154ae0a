// Microbenchmark: Philox4x32-10 throughput on gfx950 with the two multiply lowerings
// (v_mul_lo_u32 + v_mul_hi_u32 vs one v_mad_u64_u32).  Prints ns per launch and Gdraws/s; the
// outputs of both variants are compared so the faster lowering is known to be bit-identical.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox_a(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
  }
  return c;
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b) {
  uint64_t r;
  uint64_t carry;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(carry) : "v"(a), "s"(b));
  return r;
}

__device__ __forceinline__ u4 philox_b(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = mad64(c.x, 0xD2511F53u), p1 = mad64(c.z, 0xCD9E8D57u);
    c = u4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
  }
  return c;
}

template <int V>
__global__ void k(uint32_t* out, int iters, uint32_t k0, uint32_t k1) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int j = 0; j < iters; ++j) {
    u4 c{i, (uint32_t)j, 7u, 3u};
    u4 r = V == 0 ? philox_a(c, k0, k1) : philox_b(c, k0, k1);
    acc += r.x ^ r.y ^ r.z ^ r.w;
  }
  out[i] = acc;
}

int main() {
  const int n = 256 * 1024 * 4, iters = 256;
  uint32_t *a, *b;
  hipMalloc(&a, n * 4);
  hipMalloc(&b, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k<0>, dim3(n / 256), dim3(256), 0, 0, a, iters, 11u, 13u);
      else hipLaunchKernelGGL(k<1>, dim3(n / 256), dim3(256), 0, 0, b, iters, 11u, 13u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 2) printf("variant %d: %.3f ms, %.1f G philox/s\n", v, ms, (double)n * iters / (ms * 1e-3) / 1e9);
    }
  }
  uint32_t* ha = new uint32_t[n];
  uint32_t* hb = new uint32_t[n];
  hipMemcpy(ha, a, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, n * 4, hipMemcpyDeviceToHost);
  int diff = 0;
  for (int i = 0; i < n; ++i) diff += ha[i] != hb[i];
  printf("mismatches: %d\n", diff);
  return diff != 0;
}
