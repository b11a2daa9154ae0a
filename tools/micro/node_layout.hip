// Microbenchmark: streaming read of the c3 node state (65,536 envs x 2,048 nodes x int2 = 1.07 GB)
// in the two candidate layouts, with the k_node_step access pattern (workgroup = 64 envs x 8
// waves, wave w sweeps nodes [w*256, (w+1)*256), 8 loads in flight per wave).
//   tiled: [envs/64][C*N][64]   row: [C*N][envs]   linear: plain grid-stride read (upper bound)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int S = 65536, CN = 2048, NPW = 256;

template <int LAYOUT>
__global__ void __launch_bounds__(512) k_read(const int2* __restrict__ a, int* __restrict__ out) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, tile = blockIdx.x;
  const int env = tile * 64 + l;
  int acc = 0;
  for (int n0 = 0; n0 < NPW; n0 += 8) {
    int2 f[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const size_t g = (size_t)w * NPW + n0 + q;
      f[q] = LAYOUT == 0 ? a[((size_t)tile * CN + g) * 64 + l] : a[g * S + env];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc += f[q].x ^ f[q].y;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {  // cheap per-node hash (~2% hit rate)
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// tiled read + write-back of ~2% of nodes (scattered 8 B stores), optional Philox-like VALU work
template <int WRITE, int WORK>
__global__ void __launch_bounds__(512) k_rw(int2* __restrict__ a, int* __restrict__ out) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, tile = blockIdx.x;
  int acc = 0;
  uint32_t h = tile * 64 + l;
  for (int n0 = 0; n0 < NPW; n0 += 8) {
    int2* p = a + ((size_t)tile * CN + (size_t)w * NPW + n0) * 64 + l;
    int2 f[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = p[q * 64];
    uint32_t r = h ^ n0;
    if (WORK) {
#pragma unroll
      for (int k = 0; k < 10; ++k) r = (uint32_t)(((uint64_t)r * 0xD2511F53u) >> 32) ^ (r * 0xCD9E8D57u) ^ k;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (WRITE && (mix(r + q * 0x9E3779B9u) & 63) == 0) {
        f[q].x += 1;
        p[q * 64] = f[q];
      }
      acc += f[q].x ^ f[q].y;
    }
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

// as k_rw<1,0> but a node row is written in aligned groups of G lanes (G*8 bytes) whenever any
// lane of the group changed it (unchanged lanes rewrite their own value)
template <int G>
__global__ void __launch_bounds__(512) k_rw_group(int2* __restrict__ a, int* __restrict__ out) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, tile = blockIdx.x;
  int acc = 0;
  uint32_t h = tile * 64 + l;
  for (int n0 = 0; n0 < NPW; n0 += 8) {
    int2* p = a + ((size_t)tile * CN + (size_t)w * NPW + n0) * 64 + l;
    int2 f[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = p[q * 64];
    uint32_t r = h ^ n0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool mine = (mix(r + q * 0x9E3779B9u) & 63) == 0;
      if (mine) f[q].x += 1;
      const unsigned long long m = __ballot(mine);
      const unsigned long long gm = ((1ull << G) - 1) << (l & ~(G - 1));
      if (G == 64 ? m != 0 : (m & gm) != 0) p[q * 64] = f[q];
      acc += f[q].x ^ f[q].y;
    }
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

__global__ void k_linear(const int4* __restrict__ a, size_t n, int* __restrict__ out) {
  int acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int4 v = a[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
  const size_t bytes = (size_t)S * CN * 8;
  int2* a;
  int* o;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  (void)hipMemset(a, 1, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[10] = {"tiled [S/64][CN][64]", "row [CN][S]", "linear grid-stride", "tiled + 1.6% writes",
                           "tiled + philox-ish work", "tiled + writes + work", "writes in 32B groups",
                           "writes in 64B groups", "writes in 128B groups", "writes in 512B rows"};
  for (int v = 0; v < 10; ++v) {
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k_read<0>, dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 1) hipLaunchKernelGGL(k_read<1>, dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 2) hipLaunchKernelGGL(k_linear, dim3(4096), dim3(256), 0, 0, (const int4*)a, bytes / 16, o);
      if (v == 3) hipLaunchKernelGGL((k_rw<1, 0>), dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 4) hipLaunchKernelGGL((k_rw<0, 1>), dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 5) hipLaunchKernelGGL((k_rw<1, 1>), dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 6) hipLaunchKernelGGL((k_rw_group<4>), dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 7) hipLaunchKernelGGL((k_rw_group<8>), dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 8) hipLaunchKernelGGL((k_rw_group<16>), dim3(S / 64), dim3(512), 0, 0, a, o);
      if (v == 9) hipLaunchKernelGGL((k_rw_group<64>), dim3(S / 64), dim3(512), 0, 0, a, o);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-24s %.3f ms  %.0f GB/s\n", names[v], best, bytes / (best * 1e-3) / 1e9);
  }
  return 0;
}
