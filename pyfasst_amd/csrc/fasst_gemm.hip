// FP64 MFMA GEMM host side: split-K planning, launch and the fixed-order
// slab reduction.  Explicit instantiations cover the operand forms the NMF
// and SIMM updates use.
#include "fasst_gemm.h"

#include <algorithm>

namespace fasst {

__global__ void k_gemm_reduce(const double *__restrict__ part, int nz, size_t slab,
                              double *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int z = 0; z < nz; ++z) s += part[z * slab + i];
    out[i] = s;
  }
}

GemmPlan gemm_plan(int M, int N, int K) {
  GemmPlan p;
  const long tiles = (long)((M + kGBM - 1) / kGBM) * ((N + kGBN - 1) / kGBN);
  int nz = 1;
  while (tiles * nz < 512 && K / (nz * 2) >= 256) nz *= 2;
  p.nz = nz;
  p.kchunk = ((K + nz - 1) / nz + kGBK - 1) / kGBK * kGBK;
  p.nz = (K + p.kchunk - 1) / p.kchunk;
  if (p.nz < 1) p.nz = 1;
  return p;
}

template <bool TA, bool TB, int NB>
int gemm(hipStream_t s, const double *A, int lda, const double *const *B, int ldb, double *const *C,
         int ldc, int M, int N, int K, double *work) {
  GemmPlan p = gemm_plan(M, N, K);
  GemmArgs g;
  g.A = A;
  g.lda = lda;
  g.ldb = ldb;
  g.M = M;
  g.N = N;
  g.K = K;
  g.kchunk = p.kchunk;
  if (p.nz == 1 || !work) {
    g.kchunk = K;
    g.ldc = ldc;
    g.slab = 0;
    for (int b = 0; b < NB; ++b) {
      g.B[b] = B[b];
      g.C[b] = C[b];
    }
    dim3 grid((N + kGBN - 1) / kGBN, (M + kGBM - 1) / kGBM, 1);
    k_gemm<TA, TB, NB><<<grid, 256, 0, s>>>(g);
    FASST_LAUNCH_CHECK();
    return FASST_OK;
  }
  // split-K into work slabs laid out [NB][nz][M][N] (ldc = N)
  const size_t slab = (size_t)M * N;
  g.ldc = N;
  g.slab = slab;
  for (int b = 0; b < NB; ++b) {
    g.B[b] = B[b];
    g.C[b] = work + (size_t)b * p.nz * slab;
  }
  dim3 grid((N + kGBN - 1) / kGBN, (M + kGBM - 1) / kGBM, p.nz);
  k_gemm<TA, TB, NB><<<grid, 256, 0, s>>>(g);
  FASST_LAUNCH_CHECK();
  for (int b = 0; b < NB; ++b) {
    if (ldc == N) {
      k_gemm_reduce<<<(int)std::min<size_t>((slab + 255) / 256, 4096), 256, 0, s>>>(
          work + (size_t)b * p.nz * slab, p.nz, slab, C[b], slab);
    } else {
      return FASST_ERR_SHAPE;  // split-K outputs must be dense
    }
    FASST_LAUNCH_CHECK();
  }
  return FASST_OK;
}

size_t gemm_workspace(int M, int N, int K, int NB) {
  GemmPlan p = gemm_plan(M, N, K);
  return p.nz > 1 ? (size_t)NB * p.nz * M * N : 0;
}

template int gemm<false, false, 1>(hipStream_t, const double *, int, const double *const *, int,
                                   double *const *, int, int, int, int, double *);
template int gemm<true, false, 1>(hipStream_t, const double *, int, const double *const *, int,
                                  double *const *, int, int, int, int, double *);
template int gemm<true, false, 2>(hipStream_t, const double *, int, const double *const *, int,
                                  double *const *, int, int, int, int, double *);
template int gemm<true, false, 4>(hipStream_t, const double *, int, const double *const *, int,
                                  double *const *, int, int, int, int, double *);
template int gemm<false, true, 1>(hipStream_t, const double *, int, const double *const *, int,
                                  double *const *, int, int, int, int, double *);
template int gemm<false, true, 2>(hipStream_t, const double *, int, const double *const *, int,
                                  double *const *, int, int, int, int, double *);

}  // namespace fasst
