#include <cstring>
#include <cstdio>
#include <cmath>
#include <hip/hip_runtime.h>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(float x0, float x1, unsigned& hi, unsigned& lo) {
  const h2 h = {(_Float16)x0, (_Float16)x1};
  hi = __builtin_bit_cast(unsigned, h);
  unsigned l;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l) : "v"(x0), "v"(hi), "v"(x1));
  lo = l;
}
__global__ void k2(const float* x, unsigned* hi, unsigned* lo, unsigned* ref_hi, unsigned* ref_lo, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x0 = x[2 * i], x1 = x[2 * i + 1];
  unsigned a, b;
  split2(x0, x1, a, b);
  hi[i] = a; lo[i] = b;
  _Float16 h0 = (_Float16)x0, h1 = (_Float16)x1;
  h2 rh = {h0, h1};
  h2 rl = {(_Float16)(x0 - (float)h0), (_Float16)(x1 - (float)h1)};
  ref_hi[i] = __builtin_bit_cast(unsigned, rh); ref_lo[i] = __builtin_bit_cast(unsigned, rl);
}
int main() {
  const int n = 1 << 22;
  float* hx = (float*)malloc(8LL * n);
  unsigned s = 12345;
  for (int i = 0; i < 2 * n; ++i) {
    s = s * 1664525u + 1013904223u;
    unsigned bits = s;
    float f;
    // keep within fp16-splittable range: random exponents in [2^-10, 2^15)
    int e = (int)((s >> 8) % 25) - 10;
    f = ldexpf(1.f + (s & 0xffff) / 65536.f + ((s >> 16) & 0xff) / 16777216.f, e) * ((s >> 31) ? -1.f : 1.f);
    hx[i] = f;
  }
  float* dx; unsigned *d[4];
  hipMalloc(&dx, 8LL * n);
  for (int k = 0; k < 4; ++k) hipMalloc(&d[k], 4LL * n);
  hipMemcpy(dx, hx, 8LL * n, hipMemcpyHostToDevice);
  k2<<<n / 256, 256>>>(dx, d[0], d[1], d[2], d[3], n);
  unsigned* h[4];
  for (int k = 0; k < 4; ++k) { h[k] = (unsigned*)malloc(4LL * n); hipMemcpy(h[k], d[k], 4LL * n, hipMemcpyDeviceToHost); }
  long bad_hi = 0, bad_lo = 0;
  for (int i = 0; i < n; ++i) { bad_hi += h[0][i] != h[2][i]; bad_lo += h[1][i] != h[3][i]; }
  printf("n %d mismatches hi %ld lo %ld  sample x %g %g lo %08x ref %08x\n", n, bad_hi, bad_lo, hx[0], hx[1], h[1][0], h[3][0]);
  return (bad_hi || bad_lo) ? 1 : 0;
}
