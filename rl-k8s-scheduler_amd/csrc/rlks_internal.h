// rlks_internal.h — host + device helpers shared by the librlks.so translation units.
// gfx950 (MI355X, CDNA4) only: wave64, fp32 MFMA, 160 KiB LDS per CU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/rlks.h"

namespace rlks {

// ----------------------------------------------------------------------------- errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define RLKS_HIP(expr)                                                                   \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return ::rlks::fail(RLKS_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define RLKS_REQUIRE(cond, code, msg)                     \
  do {                                                    \
    if (!(cond)) return ::rlks::fail((code), (msg));      \
  } while (0)

// launch-error check (kernel launches are asynchronous; this catches config errors only)
#define RLKS_LAUNCHED() RLKS_HIP(hipGetLastError())

inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// ----------------------------------------------------------------------------- debug checks
// `make -C csrc debug` (librlks_debug.so, -DRLKS_DEBUG): device-side bounds checks on the indexing
// a corrupted state or a wrong shape would send out of bounds (node-state chunks and nodes, the
// minibatch gather's source rows, the SGD step's tiles).  A failed check does not fault the GPU: it
// counts the violation, records the first site and value in this translation unit's g_dcheck, and
// the caller clamps the index so that the access stays in bounds.  rlks_debug_checks() reads and
// clears the counters of every translation unit (each registers its reader at load); in the
// product build dcheck() is `true` and compiles away.
enum DcheckSite {
  DC_NODE_GROUP = 1,   // 8-chunk group of a departure scan within the cluster's chunks
  DC_NODE_CHUNK = 2,   // chunk of a departing pod
  DC_NODE_POD = 3,     // node of a departing pod within its chunk
  DC_NODE_ACTION = 4,  // chosen cluster (trusted actions)
  DC_GATHER_SRC = 5,   // minibatch gather source sample < T N
  DC_GATHER_GROUP = 6, // lane group < groups
  DC_SGD_TILE = 7,     // F1 / F2 tile < M / 16
  DC_GEMM_K = 8,       // pre-split GEMM: a DMA piece's 8 halves within the plane's row (ld)
  DC_WIDE_COL = 9,     // wide dZ2 kernel: the thread's 8 columns within H
};
#ifdef RLKS_DEBUG
// every translation unit that includes this header gets its own counters and registers their
// reader when the library loads (common.hip's registry), so no unit's checks go unread
static __device__ unsigned long long g_dcheck[3];  // violations, first site, first value
__device__ __forceinline__ bool dcheck(bool ok, int site, long long val) {
  if (!ok && atomicAdd(&g_dcheck[0], 1ull) == 0ull) {
    g_dcheck[1] = (unsigned long long)site;
    g_dcheck[2] = (unsigned long long)val;
  }
  return ok;
}
void dcheck_register(int (*reader)(unsigned long long*));
// host reader of this translation unit's counters (cleared after reading)
static int dcheck_read_tu(unsigned long long* h) {
  const unsigned long long z[3] = {0ull, 0ull, 0ull};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dcheck), sizeof(g_dcheck)) != hipSuccess) return 1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dcheck), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
static const int g_dcheck_registered = (dcheck_register(&dcheck_read_tu), 0);
#else
__device__ __forceinline__ bool dcheck(bool, int, long long) { return true; }
#endif

// ----------------------------------------------------------------------------- Philox4x32-10
// Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11). Same constants and
// round structure as oracle/rlks_oracle.c:ro_philox4x32_10.
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
  }
  return c;
}

// Same function with each 32x32->64 product as one v_mad_u64_u32 (the compiler splits it into
// v_mul_lo_u32 + v_mul_hi_u32); bit-identical, measured 14% faster (tools/micro/philox_rate.hip).
__device__ __forceinline__ uint64_t mad_u64_u32(uint32_t a, uint32_t b) {
  uint64_t r, carry;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(carry) : "v"(a), "s"(b));
  (void)carry;
  return r;
}

__device__ __forceinline__ u32x4 philox4x32_10_mad(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = mad_u64_u32(c.x, 0xD2511F53u), p1 = mad_u64_u32(c.z, 0xCD9E8D57u);
    c = u32x4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
  }
  return c;
}

// 53-bit uniform double in [0,1): CPython genrand_res53 construction (a>>5, b>>6)
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return __dmul_rn(__dadd_rn(__dmul_rn((double)(a >> 5), 67108864.0), (double)(b >> 6)),
                   1.0 / 9007199254740992.0);
}

// ----------------------------------------------------------------------------- MT19937
// CPython Modules/_randommodule.c genrand_uint32, one generator per lane, state SoA in HBM:
// word k of lane i at mt[k * stride + i] (k = 0..623), mti at mt[624 * stride + i].
constexpr int MT_N = 624;
constexpr int MT_M = 397;

__device__ __forceinline__ uint32_t mt_next(uint32_t* __restrict__ mt, int stride, int lane) {
  uint32_t mti = mt[MT_N * stride + lane];
  if (mti >= (uint32_t)MT_N) {
    int kk = 0;
    for (; kk < MT_N - MT_M; ++kk) {
      uint32_t y = (mt[kk * stride + lane] & 0x80000000u) | (mt[(kk + 1) * stride + lane] & 0x7fffffffu);
      mt[kk * stride + lane] = mt[(kk + MT_M) * stride + lane] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    for (; kk < MT_N - 1; ++kk) {
      uint32_t y = (mt[kk * stride + lane] & 0x80000000u) | (mt[(kk + 1) * stride + lane] & 0x7fffffffu);
      mt[kk * stride + lane] = mt[(kk + MT_M - MT_N) * stride + lane] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    uint32_t y = (mt[(MT_N - 1) * stride + lane] & 0x80000000u) | (mt[lane] & 0x7fffffffu);
    mt[(MT_N - 1) * stride + lane] = mt[(MT_M - 1) * stride + lane] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    mti = 0;
  }
  uint32_t y = mt[mti * stride + lane];
  mt[MT_N * stride + lane] = mti + 1;
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ double mt_random(uint32_t* __restrict__ mt, int stride, int lane) {
  uint32_t a = mt_next(mt, stride, lane);
  uint32_t b = mt_next(mt, stride, lane);
  return u53(a, b);
}

// ----------------------------------------------------------------------------- wave helpers
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace rlks
