// FP64 MFMA GEMM for the NMF / SIMM multiplicative updates (gfx950).
//
//   C_b[m][n] = sum_k opA[m][k] * opB_b[k][n],   b < NB (B operands share A)
//   opA[m][k] = TA ? A[k*lda + m] : A[m*lda + k]
//   opB[k][n] = TB ? B[n*ldb + k] : B[k*ldb + n]
//
// 64x64 block tile, BK = 16, 4 waves of 32x32 (2x2 v_mfma_f64_16x16x4f64
// tiles each).  A and B tiles are staged k-major in LDS (row pitch 80
// doubles: the two 16-lane row groups of a ds_read_b64 half-wave land on
// disjoint banks).  Split-K along gridDim.z writes partial C slabs
// (C + z*slab) that k_gemm_reduce sums in fixed order (deterministic).
#pragma once
#include "fasst_common.h"

namespace fasst {

constexpr int kGBM = 64, kGBN = 64, kGBK = 16, kGLD = 80;

struct GemmArgs {
  const double *A;
  const double *B[4];
  double *C[4];
  int lda, ldb, ldc;
  int M, N, K;
  int kchunk;       // K range per split (multiple of kGBK)
  size_t slab;      // element offset between split-K partial slabs of one C
};

__device__ __forceinline__ fasst::d4 gmfma(double a, double b, fasst::d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <bool TA, bool TB, int NB>
__global__ __launch_bounds__(256) void k_gemm(const GemmArgs g) {
  __shared__ __attribute__((aligned(16))) double sA[kGBK * kGLD];
  __shared__ __attribute__((aligned(16))) double sB[NB][kGBK * kGLD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fl = lane & 15, tq = lane >> 4;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.y * kGBM, n0 = blockIdx.x * kGBN;
  const int kb = blockIdx.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  fasst::d4 acc[NB][2][2];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[b][i][j] = fasst::d4{0.0, 0.0, 0.0, 0.0};

  for (int k0 = kb; k0 < ke; k0 += kGBK) {
    // stage A tile as sA[k][m]
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q;
      int k, m;
      if (TA) {
        k = idx >> 6;
        m = idx & 63;
      } else {
        m = idx >> 4;
        k = idx & 15;
      }
      const int gm = m0 + m, gk = k0 + k;
      double v = 0.0;
      if (gm < g.M && gk < ke) v = TA ? g.A[(size_t)gk * g.lda + gm] : g.A[(size_t)gm * g.lda + gk];
      sA[k * kGLD + m] = v;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = tid + 256 * q;
        int k, n;
        if (TB) {
          n = idx >> 4;
          k = idx & 15;
        } else {
          k = idx >> 6;
          n = idx & 63;
        }
        const int gn = n0 + n, gk = k0 + k;
        double v = 0.0;
        if (gn < g.N && gk < ke)
          v = TB ? g.B[b][(size_t)gn * g.ldb + gk] : g.B[b][(size_t)gk * g.ldb + gn];
        sB[b][k * kGLD + n] = v;
      }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kGBK / 4; ++kk) {
      const int kr = (4 * kk + tq) * kGLD;
      const double a0 = sA[kr + wm * 32 + fl];
      const double a1 = sA[kr + wm * 32 + 16 + fl];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const double b0 = sB[b][kr + wn * 32 + fl];
        const double b1 = sB[b][kr + wn * 32 + 16 + fl];
        acc[b][0][0] = gmfma(a0, b0, acc[b][0][0]);
        acc[b][0][1] = gmfma(a0, b1, acc[b][0][1]);
        acc[b][1][0] = gmfma(a1, b0, acc[b][1][0]);
        acc[b][1][1] = gmfma(a1, b1, acc[b][1][1]);
      }
    }
    __syncthreads();
  }
  const size_t zoff = (size_t)blockIdx.z * g.slab;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 32 + i * 16 + tq + 4 * r;
          const int col = n0 + wn * 32 + j * 16 + fl;
          if (row < g.M && col < g.N) g.C[b][zoff + (size_t)row * g.ldc + col] = acc[b][i][j][r];
        }
}

// out[i] = sum_z part[z*slab + i] (fixed order), i < n
__global__ void k_gemm_reduce(const double *__restrict__ part, int nz, size_t slab,
                              double *__restrict__ out, size_t n);

// Host helper: C_b = opA * opB_b with an automatic split-K when the output
// tile grid would leave the chip idle.  `work` must hold nz*M*ldc doubles per
// output when split (query with gemm_workspace).
struct GemmPlan {
  int nz = 1, kchunk = 0;
};
GemmPlan gemm_plan(int M, int N, int K);
template <bool TA, bool TB, int NB>
int gemm(hipStream_t s, const double *A, int lda, const double *const *B, int ldb, double *const *C,
         int ldc, int M, int N, int K, double *work);
// doubles of `work` gemm() needs for these sizes (0: no split)
size_t gemm_workspace(int M, int N, int K, int NB);

}  // namespace fasst
