// FP64 MFMA GEMM host side: split-K planning, launch and the fixed-order
// slab reduction.  Explicit instantiations cover the operand forms the NMF
// and SIMM updates use.
#include "fasst_gemm.h"
#include "fasst_dgemm2.h"

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

// tile shape per operand count: a WG_M x (4 / WG_M) wave grid of WT_M x WT_N
// MFMA tiles per wave per operand, at most 16 accumulators per wave.  The
// R = 40 accompaniment GEMMs (M or N <= 48) take a 48-wide single-wave strip
// so only the 40 -> 48 pad of the MFMA rows is wasted.
struct TileShape {
  int wgm, wtm, wtn;
};
static TileShape tile_shape(int M, int N, int NB) {
  if (NB == 1) {
    if (M <= 48) return {1, 3, 2};
    if (N <= 48) return {4, 2, 3};
    return {2, 4, 4};
  }
  if (NB == 2) {
    if (M <= 48) return {1, 3, 2};
    if (M <= 64) return {2, 2, 4};
    return {2, 4, 2};
  }
  if (M <= 48) return {1, 3, 1};
  return {2, 2, 2};
}

static void tile_dims(const TileShape &t, int &BM, int &BN) {
  BM = 16 * t.wgm * t.wtm;
  BN = 16 * (4 / t.wgm) * t.wtn;
}

// split K until the grid holds >= 1024 blocks (4 per CU), chunks >= 64
GemmPlan gemm_plan(int M, int N, int K, int NB) {
  GemmPlan p;
  int BM, BN;
  tile_dims(tile_shape(M, N, NB), BM, BN);
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int nz = 1;
  while (tiles * nz < 1024 && K / (nz * 2) >= 64) nz *= 2;
  p.kchunk = ((K + nz - 1) / nz + kGBK - 1) / kGBK * kGBK;
  p.nz = (K + p.kchunk - 1) / p.kchunk;
  if (p.nz < 1) p.nz = 1;
  return p;
}

template <bool TA, bool TB, int NB, int WGM, int WTM, int WTN>
static int launch_gemm(hipStream_t s, const GemmArgs &g, int nz) {
  constexpr int BM = 16 * WGM * WTM, BN = 16 * (4 / WGM) * WTN;
  const size_t smem = 2 * (size_t)kGBK * (gpitch(BM) + NB * gpitch(BN)) * sizeof(double);
  // the dynamic-LDS limit is a per-device attribute: set it before every
  // launch (a host-side call of a few us) so that a second device, or a
  // concurrent context, never launches before it holds
  if (smem > 64 * 1024)
    FASST_HIP(hipFuncSetAttribute((const void *)k_gemm<TA, TB, NB, WGM, WTM, WTN>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, nz);
  k_gemm<TA, TB, NB, WGM, WTM, WTN><<<grid, 256, smem, s>>>(g);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

// dispatch to the instantiations tile_shape can return for this NB
template <bool TA, bool TB, int NB>
static int launch_shape(hipStream_t s, const GemmArgs &g, int nz) {
  const TileShape t = tile_shape(g.M, g.N, NB);
  if constexpr (NB == 1) {
    if (t.wgm == 1) return launch_gemm<TA, TB, NB, 1, 3, 2>(s, g, nz);
    if (t.wgm == 4) return launch_gemm<TA, TB, NB, 4, 2, 3>(s, g, nz);
    return launch_gemm<TA, TB, NB, 2, 4, 4>(s, g, nz);
  } else if constexpr (NB == 2) {
    if (t.wgm == 1) return launch_gemm<TA, TB, NB, 1, 3, 2>(s, g, nz);
    if (t.wtm == 2) return launch_gemm<TA, TB, NB, 2, 2, 4>(s, g, nz);
    return launch_gemm<TA, TB, NB, 2, 4, 2>(s, g, nz);
  } else {
    if (t.wgm == 1) return launch_gemm<TA, TB, NB, 1, 3, 1>(s, g, nz);
    return launch_gemm<TA, TB, NB, 2, 2, 2>(s, g, nz);
  }
}

template <bool TA, bool TB, int NB>
int gemm(hipStream_t s, const double *A, int lda, const double *const *B, int ldb, double *const *C,
         int ldc, int M, int N, int K, double *work) {
  GemmPlan p = gemm_plan(M, N, K, NB);
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
    return launch_shape<TA, TB, NB>(s, g, 1);
  }
  // split-K into work slabs laid out [NB][nz][M][N] (ldc = N)
  const size_t slab = (size_t)M * N;
  g.ldc = N;
  g.slab = slab;
  for (int b = 0; b < NB; ++b) {
    g.B[b] = B[b];
    g.C[b] = work + (size_t)b * p.nz * slab;
  }
  int st = launch_shape<TA, TB, NB>(s, g, p.nz);
  if (st) return st;
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

// Large plain products on k_dgemm2 (fasst_dgemm2.h) in its product shapes
// (D2Prod, D2Odd).  The dynamic-LDS limit is a per-device attribute: set
// before every launch.
template <class CF, bool A4, bool B4, bool BUF = false>
static int launch_dgemm2(hipStream_t s, Dgemm2Args g) {
  g.mt = (g.M + CF::BM - 1) / CF::BM;
  g.nt = (g.N + CF::BN - 1) / CF::BN;
  FASST_HIP(hipFuncSetAttribute((const void *)k_dgemm2<CF, A4, B4, BUF>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)CF::smem));
  k_dgemm2<CF, A4, B4, BUF><<<g.mt * g.nt, CF::NT, CF::smem, s>>>(g);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int dgemm2(hipStream_t s, int M, int N, int K, const double *A, int lda, const double *B, int ldb,
           double *C, int ldc) {
  if (M <= 0 || N <= 0 || K <= 0 || lda < M || ldb < N || ldc < N) {
    set_error("dgemm2: bad shape M %d N %d K %d (lda %d ldb %d ldc %d)", M, N, K, lda, ldb, ldc);
    return FASST_ERR_SHAPE;
  }
  Dgemm2Args g{};
  g.A = A;
  g.B = B;
  g.C = C;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  const bool a16 = lda % 2 == 0 && ((uintptr_t)A & 15) == 0;
  const bool b16 = ldb % 2 == 0 && ((uintptr_t)B & 15) == 0;
  // raw-buffer LDS-DMA pieces (operands within 2 GB: 32-bit byte offsets);
  // the stereo SIMM iteration 9.19 -> 8.80 ms against the flat-address form
  const bool fits = (size_t)K * lda * sizeof(double) < (1ull << 31) &&
                    (size_t)K * ldb * sizeof(double) < (1ull << 31);
  if (a16 && b16 && fits) return launch_dgemm2<D2Prod, false, false, true>(s, g);
  if (a16 && b16) return launch_dgemm2<D2Prod, false, false>(s, g);
  if (a16) return launch_dgemm2<D2Odd, false, true>(s, g);
  if (b16) return launch_dgemm2<D2Odd, true, false>(s, g);
  return launch_dgemm2<D2Odd, true, true>(s, g);
}

size_t gemm_workspace(int M, int N, int K, int NB) {
  GemmPlan p = gemm_plan(M, N, K, NB);
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
