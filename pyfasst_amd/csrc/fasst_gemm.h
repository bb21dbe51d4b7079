// FP64 MFMA GEMM for the NMF / SIMM multiplicative updates (gfx950).
//
//   C_b[m][n] = sum_k opA[m][k] * opB_b[k][n],   b < NB (B operands share A)
//   opA[m][k] = TA ? A[k*lda + m] : A[m*lda + k]
//   opB[k][n] = TB ? B[n*ldb + k] : B[k*ldb + n]
//
// Block = 4 waves as a WG_M x WG_N grid (2 x 2, or 1 x 4 / 4 x 1 for the
// skinny R = 40 accompaniment GEMMs); a wave owns a (16 WT_M) x (16 WT_N)
// tile of every C_b as WT_M x WT_N x NB v_mfma_f64_16x16x4f64 accumulators
// (<= 16, i.e. <= 64 doubles per lane), so the block tile is
// BM = 16 WG_M WT_M by BN = 16 WG_N WT_N per operand.  K advances in chunks of BK = 16 staged k-major in LDS, double
// buffered: the next chunk's global loads are in flight in registers while
// the MFMAs consume the current chunk, then land in the other LDS buffer
// (one barrier per chunk).  LDS row pitches are 16 mod 32 doubles (gpitch).
// Split-K along gridDim.z writes partial C slabs (C + z*slab) that
// k_gemm_reduce sums in fixed order (deterministic).
#pragma once

#include "fasst_common.h"

namespace fasst {

constexpr int kGBK = 16;
// LDS row pitch (doubles) for a tile width x: == 16 (mod 32), so the two
// 16-lane row groups of a ds_read_b64 half-wave land on disjoint banks
constexpr int gpitch(int x) { return x + ((16 - x % 32) + 32) % 32; }

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

template <bool TA, bool TB, int NB, int WGM, int WTM, int WTN>
__global__ __launch_bounds__(256, 2) void k_gemm(const GemmArgs g) {
  constexpr int WGN = 4 / WGM;
  static_assert(WGM * WGN == 4 && NB * WTM * WTN <= 16, "wave grid / accumulator budget");
  constexpr int BM = 16 * WGM * WTM, BN = 16 * WGN * WTN;
  constexpr int PA = gpitch(BM), PB = gpitch(BN);        // LDS row pitches (doubles)
  constexpr int LA = kGBK * BM / 256, LB = NB * kGBK * BN / 256;  // loads per thread
  static_assert(kGBK * BM % 256 == 0 && NB * kGBK * BN % 256 == 0, "tile / thread mismatch");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *sA0 = smem, *sB0 = smem + kGBK * PA;
  double *sA1 = sB0 + NB * kGBK * PB, *sB1 = sA1 + kGBK * PA;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fl = lane & 15, tq = lane >> 4;
  const int wm = wv / WGN, wn = wv % WGN;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kb = blockIdx.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  fasst::d4 acc[NB][WTM][WTN];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < WTM; ++i)
#pragma unroll
      for (int j = 0; j < WTN; ++j) acc[b][i][j] = fasst::d4{0.0, 0.0, 0.0, 0.0};

  double ra[LA], rb[LB];
  // global -> registers for the chunk starting at k0 (coalesced along the
  // contiguous dimension of each operand, zero outside the matrices)
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int idx = tid + 256 * q;
      int k, m;
      if (TA) {
        k = idx / BM;
        m = idx % BM;
      } else {
        m = idx / kGBK;
        k = idx % kGBK;
      }
      const int gm = m0 + m, gk = k0 + k;
      ra[q] = (gm < g.M && gk < ke) ? (TA ? g.A[(size_t)gk * g.lda + gm] : g.A[(size_t)gm * g.lda + gk])
                                    : 0.0;
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int idx = tid + 256 * q;
      const int b = idx / (kGBK * BN), r = idx % (kGBK * BN);
      int k, n;
      if (TB) {
        n = r / kGBK;
        k = r % kGBK;
      } else {
        k = r / BN;
        n = r % BN;
      }
      const int gn = n0 + n, gk = k0 + k;
      const double *Bb = g.B[b];
      rb[q] = (gn < g.N && gk < ke) ? (TB ? Bb[(size_t)gn * g.ldb + gk] : Bb[(size_t)gk * g.ldb + gn])
                                    : 0.0;
    }
  };
  auto sstore = [&](double *sA, double *sB) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int idx = tid + 256 * q;
      int k, m;
      if (TA) {
        k = idx / BM;
        m = idx % BM;
      } else {
        m = idx / kGBK;
        k = idx % kGBK;
      }
      sA[k * PA + m] = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int idx = tid + 256 * q;
      const int b = idx / (kGBK * BN), r = idx % (kGBK * BN);
      int k, n;
      if (TB) {
        n = r / kGBK;
        k = r % kGBK;
      } else {
        k = r / BN;
        n = r % BN;
      }
      sB[b * kGBK * PB + k * PB + n] = rb[q];
    }
  };

  const int nch = (ke - kb + kGBK - 1) / kGBK;
  if (nch > 0) {
    gload(kb);
    sstore(sA0, sB0);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const bool odd = c & 1;
    const double *sA = odd ? sA1 : sA0;
    const double *sB = odd ? sB1 : sB0;
    if (c + 1 < nch) gload(kb + (c + 1) * kGBK);
#pragma unroll
    for (int kk = 0; kk < kGBK / 4; ++kk) {
      const int kr = 4 * kk + tq;
      double a[WTM];
#pragma unroll
      for (int i = 0; i < WTM; ++i) a[i] = sA[kr * PA + wm * 16 * WTM + i * 16 + fl];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int j = 0; j < WTN; ++j) {
          const double bv = sB[b * kGBK * PB + kr * PB + wn * 16 * WTN + j * 16 + fl];
#pragma unroll
          for (int i = 0; i < WTM; ++i) acc[b][i][j] = gmfma(a[i], bv, acc[b][i][j]);
        }
      }
    }
    if (c + 1 < nch) sstore(odd ? sA0 : sA1, odd ? sB0 : sB1);
    __syncthreads();
  }
  const size_t zoff = (size_t)blockIdx.z * g.slab;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < WTM; ++i)
#pragma unroll
      for (int j = 0; j < WTN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 16 * WTM + i * 16 + tq + 4 * r;
          const int col = n0 + wn * 16 * WTN + j * 16 + fl;
          if (row < g.M && col < g.N) g.C[b][zoff + (size_t)row * g.ldc + col] = acc[b][i][j][r];
        }
}

// ---------------------------------------------------------------------------
// k_gemm44: the same contract on v_mfma_f64_4x4x4_4b (74.7 TF measured on this
// chip vs 47.7 for 16x16x4, profiles/r1_ubench_fp64.txt).  Lane
// l = 16 X + 4 b + Y supplies A[m=Y][k=X] and B[k=X][n=Y] of block b and
// receives D[m=X][n=Y] of block b (tools/probe_mfma4.hip).  Block b of one
// instruction is rows 16 i + 4 b .. +3 of the wave tile, so the A fragment is
// a 16 x 4 slice (one double per lane) and the B fragment a 4 x 4 slice that
// all four blocks share (a broadcast LDS read):
//   C[16 i + 4 b + X][4 j + Y] += sum_k A[16 i + 4 b + .][k] B[k][4 j + .]
// A wave owns 16 RM x 4 RN outputs as RM x RN one-double accumulators and
// reads RM + RN doubles per k-step of 4 (RM x RN MFMAs).  Block = NW waves
// (WGM x WGN), tile BM = 16 RM WGM by BN = 4 RN WGN, large enough that the
// L2 feed stays ~20 flop/B.  K advances in kGBK chunks staged in LDS with the
// next chunk's loads in flight in registers.  LDS layouts are permuted so a
// lane's RM A values and RN B values of one k are contiguous (ds_read_b128):
//   A: row 16 i + q (q = 4 b + Y) of wave row wm at [k][64 wm' + q RM + i],
//      pitch PA = 18 mod 32 doubles: the 16 lanes of every ds_read_b128 group
//      cover the 64 banks once;
//   B: column 4 j + Y of wave column wn at [k][wn (4 (RN+2)) + Y (RN+2) + j],
//      pitch PB = 8 mod 32: distinct (X, Y) hit disjoint banks, equal ones
//      broadcast.
constexpr int g44pitch(int x, int r) { return x + ((r - x % 32) + 32) % 32; }

template <bool TA, bool TB, int NB, int NW, int WGM, int RM, int RN>
__global__ __launch_bounds__(64 * NW, 1) void k_gemm44(const GemmArgs g) {
  constexpr int NT = 64 * NW, WGN = NW / WGM;
  static_assert(WGM * WGN == NW && RM % 2 == 0 && RN % 2 == 0, "wave grid / b128 pairs");
  constexpr int WM = 16 * RM, WN = 4 * RN;            // wave tile
  constexpr int BM = WM * WGM, BN = WN * WGN;         // block tile
  constexpr int SBW = 4 * (RN + 2);                   // B columns per wave slab in LDS
  constexpr int PA = g44pitch(BM, 18), PB = g44pitch(SBW * WGN, 8);
  constexpr int LA = kGBK * BM / NT, LB = NB * kGBK * BN / NT;
  static_assert(kGBK * BM % NT == 0 && NB * kGBK * BN % NT == 0, "tile / thread mismatch");
  constexpr int SA = kGBK * PA, SB = NB * kGBK * PB;  // doubles per LDS buffer
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int X = lane >> 4, bq = (lane >> 2) & 3, Y = lane & 3;
  const int wm = wv / WGN, wn = wv % WGN;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kb = blockIdx.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  // block-uniform: every element of every chunk is inside the matrices
  const bool interior = m0 + BM <= g.M && n0 + BN <= g.N && (ke - kb) % kGBK == 0;
  double acc[NB][RM][RN];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[b][i][j] = 0.0;

  // element q of this thread's share of a chunk: (k, m) of A, (b, k, n) of B
  auto a_km = [&](int q, int &k, int &m) {
    const int idx = tid + NT * q;
    if (TA) {
      k = idx / BM;
      m = idx % BM;
    } else {
      m = idx / kGBK;
      k = idx % kGBK;
    }
  };
  auto b_bkn = [&](int q, int &b, int &k, int &n) {
    const int idx = tid + NT * q;
    b = idx / (kGBK * BN);
    const int r = idx % (kGBK * BN);
    if (TB) {
      n = r / kGBK;
      k = r % kGBK;
    } else {
      k = r / BN;
      n = r % BN;
    }
  };
  double ra[LA], rb[LB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      int k, m;
      a_km(q, k, m);
      const int gm = m0 + m, gk = k0 + k;
      const size_t off = TA ? (size_t)gk * g.lda + gm : (size_t)gm * g.lda + gk;
      ra[q] = (interior || (gm < g.M && gk < ke)) ? g.A[off] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      int b, k, n;
      b_bkn(q, b, k, n);
      const int gn = n0 + n, gk = k0 + k;
      const size_t off = TB ? (size_t)gn * g.ldb + gk : (size_t)gk * g.ldb + gn;
      rb[q] = (interior || (gn < g.N && gk < ke)) ? g.B[b][off] : 0.0;
    }
  };
  auto sstore = [&](double *sA, double *sB) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      int k, m;
      a_km(q, k, m);
      const int w = m / WM, r = m % WM;  // wave row, row in the wave tile
      sA[k * PA + w * WM + (r & 15) * RM + (r >> 4)] = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      int b, k, n;
      b_bkn(q, b, k, n);
      const int w = n / WN, c = n % WN;  // wave column, column in the wave tile
      sB[b * kGBK * PB + k * PB + w * SBW + (c & 3) * (RN + 2) + (c >> 2)] = rb[q];
    }
  };

  const int nch = (ke - kb + kGBK - 1) / kGBK;
  if (nch > 0) {
    gload(kb);
    sstore(smem, smem + SA);
  }
  __syncthreads();
  const int aofs = wm * WM + (4 * bq + Y) * RM;
  const int bofs = wn * SBW + Y * (RN + 2);
  for (int c = 0; c < nch; ++c) {
    const double *sA = smem + (c & 1) * (SA + SB);
    const double *sB = sA + SA;
    if (c + 1 < nch) gload(kb + (c + 1) * kGBK);
    // operands of k-step kk + 1 are read while the MFMAs of kk issue
    double a[2][RM], bv[2][NB][RN];
    auto lds_ops = [&](int kk, int slot) {
      const int kr = 4 * kk + X;
#pragma unroll
      for (int i = 0; i < RM; i += 2) {
        const double2 v = *(const double2 *)(sA + kr * PA + aofs + i);
        a[slot][i] = v.x;
        a[slot][i + 1] = v.y;
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < RN; j += 2) {
          const double2 v = *(const double2 *)(sB + b * kGBK * PB + kr * PB + bofs + j);
          bv[slot][b][j] = v.x;
          bv[slot][b][j + 1] = v.y;
        }
    };
    lds_ops(0, 0);
#pragma unroll
    for (int kk = 0; kk < kGBK / 4; ++kk) {
      const int cs = kk & 1;
      if (kk + 1 < kGBK / 4) lds_ops(kk + 1, cs ^ 1);
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[b][i][j] =
                __builtin_amdgcn_mfma_f64_4x4x4f64(a[cs][i], bv[cs][b][j], acc[b][i][j], 0, 0, 0);
    }
    if (c + 1 < nch) {
      double *dA = smem + ((c + 1) & 1) * (SA + SB);
      sstore(dA, dA + SA);
    }
    __syncthreads();
  }
  const size_t zoff = (size_t)blockIdx.z * g.slab;
  const int crow = m0 + wm * WM + 4 * bq + X;
  const int ccol = n0 + wn * WN + Y;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = crow + 16 * i, col = ccol + 4 * j;
        if (interior || (row < g.M && col < g.N))
          g.C[b][zoff + (size_t)row * g.ldc + col] = acc[b][i][j];
      }
}

template <bool TA, bool TB, int NB, int NW, int WGM, int RM, int RN>
constexpr size_t gemm44_smem() {
  constexpr int WGN = NW / WGM, BM = 16 * RM * WGM, SBW = 4 * (RN + 2);
  return 2 * (size_t)(kGBK * g44pitch(BM, 18) + NB * kGBK * g44pitch(SBW * WGN, 8)) * sizeof(double);
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
GemmPlan gemm_plan(int M, int N, int K, int NB);
template <bool TA, bool TB, int NB>
int gemm(hipStream_t s, const double *A, int lda, const double *const *B, int ldb, double *const *C,
         int ldc, int M, int N, int K, double *work);
// doubles of `work` gemm() needs for these sizes (0: no split)
size_t gemm_workspace(int M, int N, int K, int NB);

// Large plain products (the Stereo_SIMM NF0-sized ones): row-major
// C (M x N) = A^T B with A given k-major [K][lda] and B [K][ldb], on k_dgemm2
// (fasst_dgemm2.h: global_load_lds stages, 4x4x4_4b MFMA).  Rows that are not
// 16-byte aligned (odd lda / ldb) are loaded in 4-byte pieces.
int dgemm2(hipStream_t s, int M, int N, int K, const double *A, int lda, const double *B, int ldb,
           double *C, int ldc);

}  // namespace fasst
