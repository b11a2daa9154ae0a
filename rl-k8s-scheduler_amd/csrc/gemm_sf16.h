// gemm_sf16.h — the generic split-fp16 GEMM (gemm_sf16.hip) used by the wide-MLP path (config c5).
#pragma once

#include "mlp_common.h"

namespace rlks {

enum { GEMM_STORE = RLKS_GEMM_STORE, GEMM_TANH_BIAS = RLKS_GEMM_TANH_BIAS, GEMM_BIAS = RLKS_GEMM_BIAS,
       GEMM_DTANH = RLKS_GEMM_DTANH,
       GEMM_TANH_BIAS_PLANES = 4 };  // internal: tanh(acc + bias) written as fp16 hi / lo planes at 2^14

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
  _Float16 *c_hi, *c_lo;  // GEMM_TANH_BIAS_PLANES: output planes [M][ldc]
};

int launch_gemm_sf16(const GemmArgs& a, hipStream_t s);
int launch_split_reduce(const float* part, int splits, int rows, int cols, float* out, int ld, int accumulate,
                        hipStream_t s);

// ---- pre-split GEMM (gemm_ps.hip): operands as fp16 planes hi / lo of x 2^e in HBM
struct PsOperand {
  const _Float16 *hi, *lo;  // element (row, k) at row * ld + k, or k * ld + row when kmajor
  int ld, kmajor;
  int rows;                 // extent of the non-K dimension (rows past it are clamped, never stored)
  const unsigned* maxslot;  // e = exponent with max 2^e in [2^14, 2^15) (float bits); null: fexp
  int fexp;
};
enum { PS_STORE = 0, PS_TANH_BIAS = 1, PS_DTANH = 2, PS_TANH_BIAS_PLANES = 3 };
struct PsArgs {
  PsOperand a, b;           // C[m][n] = sum_k A[m][k] B[n][k]
  int M, N, K;              // K a multiple of 32
  int epi;                  // PS_STORE: C (or split-K partials); PS_TANH_BIAS: tanh(acc + bias[n]);
                            // PS_DTANH: acc (1 - G^2), G = (aux_hi + aux_lo) 2^-14;
                            // PS_TANH_BIAS_PLANES: tanh(acc + bias[n]) as fp16 planes at 2^14 in c_hi / c_lo
  float* C;
  _Float16 *c_hi, *c_lo;
  int ldc;
  const float* bias;
  const _Float16 *aux_hi, *aux_lo;
  int ldaux;
  unsigned* cmax;           // optional atomicMax of |C|
  int splits;               // split-K layers (PS_STORE): part[z][M][N], fixed-order f64 reduction into C
  float* part;
};
int launch_gemm_ps(const PsArgs& a, hipStream_t s);
int gemm_ps_splits(int M, int N, int K);
// fp32 [rows][ld] -> planes [rows][ldp] of x 2^e (e from maxslot, or fexp when null)
int launch_split_planes(const float* x, int rows, int cols, int ld, const unsigned* maxslot, int fexp, _Float16* hi,
                        _Float16* lo, int ldp, hipStream_t s);
// split count for an M x N x K weight-gradient GEMM (enough workgroups to fill 256 CUs)
int gemm_splits(int M, int N, int K);
int launch_absmax(const float* x, int rows, int cols, int ld, unsigned* slot, hipStream_t s);
// column sums out[c] (+)= sum_r x[r][c] (with wt: sum_r wt[r] x[r][c]), in f64; with `part`
// ([2][colsum_splits(rows)][cols] floats: hi, lo planes) the rows are split over workgroups and
// reduced in a fixed order
int colsum_splits(int rows);
int launch_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate, float* part,
                  hipStream_t s,
                  const float* wt = nullptr);

}  // namespace rlks
