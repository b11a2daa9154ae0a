// gemm_sf16.h — the generic split-fp16 GEMM (gemm_sf16.hip) used by the wide-MLP path (config c5).
#pragma once

#include "mlp_common.h"

namespace rlks {

enum { GEMM_STORE = RLKS_GEMM_STORE, GEMM_TANH_BIAS = RLKS_GEMM_TANH_BIAS, GEMM_BIAS = RLKS_GEMM_BIAS,
       GEMM_DTANH = RLKS_GEMM_DTANH };

struct GemmArgs {
  const float *A, *B;
  float* C;
  const float* bias;  // [N] (TANH_BIAS, BIAS)
  const float* aux;   // [M][ldaux] stored tanh output G (DTANH: C = acc (1 - G^2))
  int M, N, K, lda, ldb, ldc, ldaux;
  int ta, tb, epi, accumulate;
  const unsigned *amax, *bmax;  // operand max |x| slots (float bits)
  unsigned* cmax;               // optional: atomicMax of |C|
};

int launch_gemm_sf16(const GemmArgs& a, hipStream_t s);
int launch_absmax(const float* x, int rows, int cols, int ld, unsigned* slot, hipStream_t s);
int launch_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate, hipStream_t s);

}  // namespace rlks
