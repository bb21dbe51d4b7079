// k_dgemm: FP64 GEMM for the large plain Stereo_SIMM products (gfx950).
//
//   C[m][n] = sum_k opA[m][k] * B[k][n],   opA = TA ? A[k*lda + m] : A[m*lda + k]
//
// B and C are row-major with n contiguous (the SIMM planes).  Block = 256
// threads as 2 x 2 waves, block tile 128 x 128, wave tile 64 x 64 as 4 x 4
// v_mfma_f64_16x16x4f64 accumulators; K advances in chunks of 16.
//
// What differs from k_gemm (fasst_gemm.h), each item aimed at a stall the
// rocprof / disassembly comparison with the library kernels pointed to
// (DESIGN.md §3.7):
//  * 16-byte global loads (double2 along the contiguous dimension);
//  * the A tile is stored in the layout its global rows arrive in: k-major
//    [k][m] for TA (pitch 144 = 16 mod 32 doubles), m-major [m][k] for the
//    NN form (pitch 18: a 16-lane fragment read spans the 64 banks once and
//    the b128 row writes do not serialise, where k_gemm's transposing store
//    was an 8-way bank conflict);
//  * the fragments of two k-steps are read from LDS before their 32 MFMAs,
//    the next chunk's global loads are in flight during the chunk;
//  * XCD-aware tile order: workgroup b runs on XCD b mod 8, so each XCD gets
//    a contiguous run of the m-fastest tile sequence and the tiles sharing
//    one 128-column B panel (the large streamed operand) meet in one L2.
// Requires lda, ldb and the contiguous extent of A (K for NN, M for TA) and
// N to be even (16-byte alignment); the host falls back otherwise.
#pragma once
#include "fasst_common.h"

namespace fasst {

constexpr int kDBM = 128, kDBN = 128, kDBK = 16;
constexpr int kDPK = 144;   // k-major pitch (doubles): 16 mod 32
constexpr int kDPM = 18;    // m-major pitch (doubles)

struct DgemmArgs {
  const double *A, *B;
  double *C;
  int lda, ldb, ldc, M, N, K;
  int mt, nt;   // tile counts
  int order;    // 0: XCD-aware m-fastest (default), 1: m-fastest, 2: n-fastest (A/B)
};

template <bool TA>
constexpr int dgemm_sa() { return TA ? kDBK * kDPK : kDBM * kDPM; }
constexpr int dgemm_sb() { return kDBK * kDPK; }
template <bool TA>
constexpr size_t dgemm_smem() { return 2 * (size_t)(dgemm_sa<TA>() + dgemm_sb()) * sizeof(double); }

__device__ __forceinline__ fasst::d4 dmfma(double a, double b, fasst::d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// IG > 0: __builtin_amdgcn_iglp_opt(IG - 1) scheduling hint in the chunk loop
// (A/B in tools/ubench_dgemm2.hip only)
// SM: the next chunk's LDS store after the first (1) or second (0) half of
// the chunk's MFMAs (A/B in tools/ubench_dgemm2.hip)
template <bool TA, int IG = 0, int SM = 0>
__global__ __launch_bounds__(256, 2) void k_dgemm(const DgemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int SA = dgemm_sa<TA>(), SB = dgemm_sb();
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fl = lane & 15, tq = lane >> 4, wm = wv >> 1, wn = wv & 1;
  // XCD-aware tile order (m fastest within an XCD's contiguous run)
  const int ntile = g.mt * g.nt, per = (ntile + 7) / 8;
  const int tile = g.order == 0 ? (blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
  if (tile >= ntile) return;
  const int m0 = (g.order == 2 ? tile / g.nt : tile % g.mt) * kDBM;
  const int n0 = (g.order == 2 ? tile % g.nt : tile / g.mt) * kDBN;

  fasst::d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fasst::d4{0.0, 0.0, 0.0, 0.0};

  // per chunk: A and B tiles are 128 x 16 doubles = 1024 double2, 4 per thread
  double2 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q;
      int m, k;
      if (TA) {   // A rows k, m contiguous: 16 rows x 64 double2
        k = idx >> 6;
        m = 2 * (idx & 63);
      } else {    // A rows m, k contiguous: 128 rows x 8 double2
        m = idx >> 3;
        k = 2 * (idx & 7);
      }
      const int gm = m0 + m, gk = k0 + k;
      double2 v = make_double2(0.0, 0.0);
      if (TA) {
        if (gk < g.K && gm < g.M) v = *(const double2 *)(g.A + (size_t)gk * g.lda + gm);
      } else {
        if (gm < g.M && gk < g.K) v = *(const double2 *)(g.A + (size_t)gm * g.lda + gk);
      }
      ra[q] = v;
      const int kb = idx >> 6, nb = 2 * (idx & 63);   // B: 16 rows x 64 double2
      const int gkb = k0 + kb, gn = n0 + nb;
      double2 w = make_double2(0.0, 0.0);
      if (gkb < g.K && gn < g.N) w = *(const double2 *)(g.B + (size_t)gkb * g.ldb + gn);
      rb[q] = w;
    }
  };
  auto sstore = [&](double *sA, double *sB) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q;
      if (TA) {
        *(double2 *)(sA + (idx >> 6) * kDPK + 2 * (idx & 63)) = ra[q];
      } else {
        *(double2 *)(sA + (idx >> 3) * kDPM + 2 * (idx & 7)) = ra[q];
      }
      *(double2 *)(sB + (idx >> 6) * kDPK + 2 * (idx & 63)) = rb[q];
    }
  };

  // 16-row blocks of this wave that hold rows < M (wave-uniform)
  const int nib = min(4, max(0, (g.M - m0 - wm * 64 + 15) / 16));
  const bool full = nib == 4;
  const int nch = (g.K + kDBK - 1) / kDBK;
  double *sA0 = smem, *sB0 = smem + SA, *sA1 = sB0 + SB, *sB1 = sA1 + SA;
  gload(0);
  sstore(sA0, sB0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const bool odd = c & 1;
    const double *sA = odd ? sA1 : sA0;
    const double *sB = odd ? sB1 : sB0;
    if (c + 1 < nch) gload((c + 1) * kDBK);
    if constexpr (IG > 0) __builtin_amdgcn_iglp_opt(IG - 1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // fragments of two k-steps, then their 32 MFMAs
      double a[2][4], b[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kr = 4 * (2 * h + u) + tq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = wm * 64 + i * 16 + fl;
          a[u][i] = TA ? sA[kr * kDPK + m] : sA[m * kDPM + kr];
          b[u][i] = sB[kr * kDPK + wn * 64 + i * 16 + fl];
        }
      }
      if (full) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][j] = dmfma(a[u][i], b[u][j], acc[i][j]);
      } else {   // edge tile: 16-row blocks wholly past M issue no MFMAs
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (i < nib) acc[i][j] = dmfma(a[u][i], b[u][j], acc[i][j]);
      }
      if (SM == 1 && h == 0 && c + 1 < nch) sstore(odd ? sA0 : sA1, odd ? sB0 : sB1);
    }
    if (SM == 0 && c + 1 < nch) sstore(odd ? sA0 : sA1, odd ? sB0 : sB1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + tq + 4 * r;
        const int col = n0 + wn * 64 + j * 16 + fl;
        if (row < g.M && col < g.N) g.C[(size_t)row * g.ldc + col] = acc[i][j][r];
      }
}

}  // namespace fasst
