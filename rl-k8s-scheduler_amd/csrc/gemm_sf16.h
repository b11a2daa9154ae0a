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
  // split-K (weight gradients: K = minibatch rows, few output tiles): `splits` > 1 K ranges, each
  // workgroup layer z writes part[z][M][N]; a fixed-order f64 reduction then stores / adds C.
  // Epilogue GEMM_STORE only.
  int splits;
  float* part;
};

int launch_gemm_sf16(const GemmArgs& a, hipStream_t s);
// split count for an M x N x K weight-gradient GEMM (enough workgroups to fill 256 CUs)
int gemm_splits(int M, int N, int K);
int launch_absmax(const float* x, int rows, int cols, int ld, unsigned* slot, hipStream_t s);
// column sums out[c] (+)= sum_r x[r][c]; with `part` ([colsum_splits(rows)][cols] floats) the rows
// are split over workgroups and reduced in a fixed order
int colsum_splits(int rows);
int launch_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate, float* part,
                  hipStream_t s);

}  // namespace rlks
