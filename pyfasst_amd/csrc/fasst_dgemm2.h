// k_dgemm2: FP64 GEMM for the NF0-sized Stereo_SIMM products (gfx950).
//
//   C[m][n] = sum_k A[k][m] B[k][n]      (A given k-major: the "TA" form)
//
// SIMM.py:623-674 / :799 (SF0 = WF0 HF0 with WF0 kept transposed, WF0^T
// [num | den]).  Both operands arrive row by row: a 128-wide row of the
// block tile is ONE global_load_lds_dwordx4 (64 lanes x 16 B, 1 KB), written
// straight into LDS without passing through VGPRs, so NS chunk stages can be
// in flight without costing registers.  One barrier per K chunk of 16:
//   wait (counted vmcnt) for chunk c -> s_barrier -> issue the loads of chunk
//   c + NS - 1 into the buffer chunk c - 1 left -> compute chunk c.
// Block = 256 threads as 2 x 2 waves, block tile 128 x 128, wave tile 64 x 64.
// Two MFMA forms (D2Cfg::MF).  The product shape (D2Prod, two waves per SIMD)
// runs v_mfma_f64_16x16x4f64, a wave's 64 x 64 tile as 4 x 4 four-double
// accumulators fed by 8 LDS reads per k-step of 4 (16 MFMAs).  The odd-pitch
// shape (D2Odd, one wave per SIMD) runs v_mfma_f64_4x4x4_4b: lane (X, b, Y) of one instruction
// supplies A[m = Y][k = X] and B[k = X][n = Y] of block b and receives
// D[m = X][n = Y]; the four blocks are 2 (m) x 2 (n) sub-blocks of an 8 x 8
// patch, so one A register covers 8 rows, one B register 8 columns, and a
// wave's 64 x 64 tile is 8 x 8 one-double accumulators fed by 16 LDS reads
// per k-step of 4 (64 MFMAs).  Fed from LDS this shape runs at 76 TF at one
// wave per SIMD (tools/ubench_mfma_lds.hip), where 16x16x4 needs two.
// Edges: rows / columns past M / N and k rows past K load from a zero
// buffer; 8-row groups wholly past M issue no MFMAs.  16-byte row loads need
// an even leading dimension and a 16-byte aligned base; otherwise the operand
// is loaded in 4-byte pieces (A4 / B4), which only needs 4-byte alignment.
#pragma once
#include "fasst_common.h"

#include <type_traits>

namespace fasst {

// Launch shape: NS chunk stages of BK k-rows, a WGM x WGN grid of waves each
// owning a 64 x 64 tile (block tile BM x BN), OCC blocks per CU.
template <int NS_, int BK_, int WGM_, int WGN_, int OCC_, int MF_ = 0>
struct D2Cfg {
  // MF: 0 = v_mfma_f64_4x4x4_4b (8 x 8 one-double accumulators per wave),
  //     1 = v_mfma_f64_16x16x4f64 (4 x 4 four-double accumulators)
  static constexpr int NS = NS_, BK = BK_, WGM = WGM_, WGN = WGN_, OCC = OCC_, MF = MF_;
  static constexpr int NW = WGM * WGN, NT = 64 * NW;
  static constexpr int BM = 64 * WGM, BN = 64 * WGN;
  // LDS row pitches (doubles), 16 mod 32: rows X and X + 1 of one read hit
  // disjoint halves of the 64 banks
  static constexpr int PA = BM + 16, PB = BN + 16;
  static constexpr int SS = BK * (PA + PB);   // doubles per stage
  static constexpr size_t smem = (size_t)NS * SS * sizeof(double);
  // 1 KB row pieces per chunk (a row of BM doubles is BM / 128 pieces)
  static constexpr int PCA = BK * BM / 128, PCB = BK * BN / 128;
  static_assert((PCA + PCB) % NW == 0, "chunk pieces must split evenly over the waves");
  static_assert(BK % 4 == 0, "k-steps of 4");
};
// the product's shapes (tools/ubench_dgemm3.hip sweeps the others): 16-byte
// row loads; and the one for operands loaded in 4-byte pieces (odd leading
// dimension), where the two-stage shape drained its loads every chunk
// (8 vs 42-46 TF at the C5 sizes, profiles/r3_ubench_dgemm3.txt)
// (the product shape on 16x16x4 since round 5: C5 8.56 -> 8.46 ms per iteration
// with the raw-buffer pieces, profiles/r5_ab_round5b.txt; the 4x4x4_4b form was
// ahead before them, profiles/r3_ubench_dgemm3.txt)
using D2Prod = D2Cfg<2, 16, 2, 2, 2, 1>;
using D2Odd = D2Cfg<4, 8, 4, 2, 1>;

struct Dgemm2Args {
  const double *A, *B;   // A [K][lda] (k-major), B [K][ldb]
  double *C;             // [M][ldc]
  int lda, ldb, ldc, M, N, K;
  int mt, nt;            // tile counts
};

typedef __attribute__((address_space(3))) void d2_lds_t;
typedef __attribute__((address_space(1))) void d2_gbl_t;

// 16 zero bytes per lane for the loads that fall outside the operands
__device__ __attribute__((aligned(16))) double g_d2_zero[2];

__device__ __forceinline__ double d2_mfma(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// (FASST_NO_LDS_PAIRING: keep the operand reads as ds_read_b64, 2 LDS cycles
// each, not paired into ds_read2_b64 at 8)
// BUF (16-byte pieces only): the pieces as raw-buffer LDS-DMA loads
// (buffer_load_dwordx4 ... lds) off one wave-uniform resource per operand whose
// size is exactly its K rows, so rows k >= K read 0 without a test; a piece's
// per-lane byte offset is loop-invariant (columns past M / N: an offset past
// the resource, 0 as well) and the chunk's row offset rides in an SGPR.  The
// global_load_lds form selects the zero buffer per lane, which hipcc turns
// into exec-masked branches around every load.
template <class CF, bool A4 = false, bool B4 = false, bool BUF = false>
__global__ __launch_bounds__(CF::NT, CF::OCC) FASST_NO_LDS_PAIRING
void k_dgemm2(const Dgemm2Args g) {
  constexpr int NS = CF::NS, BK = CF::BK, BM = CF::BM, BN = CF::BN, NW = CF::NW;
  constexpr int PA = CF::PA, PB = CF::PB, SS = CF::SS;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int X = lane >> 4, bq = (lane >> 2) & 3, Y = lane & 3;
  const int wm = wv / CF::WGN, wn = wv % CF::WGN;
  // XCD-aware tile order: workgroups b, b + 8, ... share an XCD (and its L2);
  // give each XCD a contiguous run of the m-fastest tile sequence, so the
  // tiles reading one B column panel meet in one L2 (bijective for any count)
  const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
  const int m0 = (tile % g.mt) * BM, n0 = (tile / g.mt) * BN;

  // one 1 KB piece (128 doubles of a row): one global_load_lds_dwordx4, or,
  // for an operand whose rows are not 16-byte aligned (odd leading
  // dimension), four 4-byte loads (W4: lane l of load q carries dword l of
  // the piece's q-th 256 B)
  auto load_piece = [&](auto w4_tag, const double *base, int ld, int c0, int lim, int k, double *dst) {
    constexpr bool W4 = decltype(w4_tag)::value;
    if constexpr (!W4) {
      const double *src = (k < g.K && c0 + 2 * lane < lim) ? base + (size_t)k * ld + c0 + 2 * lane
                                                          : g_d2_zero;
      __builtin_amdgcn_global_load_lds((d2_gbl_t *)src, (d2_lds_t *)dst, 16, 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = c0 + 32 * q + (lane >> 1);
        const float *src = (k < g.K && col < lim)
                               ? (const float *)(base + (size_t)k * ld + c0 + 32 * q) + lane
                               : (const float *)g_d2_zero;
        __builtin_amdgcn_global_load_lds((d2_gbl_t *)src, (d2_lds_t *)(dst + 32 * q), 4, 0, 0);
      }
    }
  };
  // BUF: per-piece lane offsets and LDS destinations (pieces r < PCA / NW of
  // a wave are A pieces: p = wv + NW r < PCA)
  constexpr int RPB = (CF::PCA + CF::PCB) / NW;
  static_assert(!BUF || (CF::PCA % NW == 0 && !A4 && !B4), "BUF: 16-byte pieces, whole A rows per wave");
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(g.A), 0, BUF ? (int)((size_t)g.K * g.lda * sizeof(double)) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(g.B), 0, BUF ? (int)((size_t)g.K * g.ldb * sizeof(double)) : 0, 0x00020000);
  unsigned voff[BUF ? RPB : 1];
  int ldso[BUF ? RPB : 1];
  if constexpr (BUF) {
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
      const int p = wv + NW * r;
      const bool isA = r < CF::PCA / NW;
      const int q = isA ? p : p - CF::PCA;
      const int per = isA ? BM / 128 : BN / 128;
      const int kr = q / per, sg = q % per;
      const int col = (isA ? m0 : n0) + 128 * sg + 2 * lane;
      const int lim = isA ? g.M : g.N, ld = isA ? g.lda : g.ldb;
      voff[r] = col < lim ? (unsigned)((kr * ld + col) * (int)sizeof(double)) : 0x80000000u;
      ldso[r] = isA ? kr * PA + 128 * sg : BK * PA + kr * PB + 128 * sg;
    }
  }
  // chunk c: pieces wv, wv + NW, ... of the PCA A pieces then the PCB B pieces
  auto issue = [&](int c) {
    double *st = smem + (c % NS) * SS;
    if constexpr (BUF) {
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        const bool isA = r < CF::PCA / NW;
        const int so = c * BK * (isA ? g.lda : g.ldb) * (int)sizeof(double);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, (d2_lds_t *)(st + ldso[r]), 16,
                                                 (int)voff[r], so, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < (CF::PCA + CF::PCB) / NW; ++r) {
      const int p = wv + NW * r;
      if (p < CF::PCA) {
        const int kr = p / (BM / 128), sg = p % (BM / 128);
        load_piece(std::integral_constant<bool, A4>{}, g.A, g.lda, m0 + 128 * sg, g.M, c * BK + kr,
                   st + kr * PA + 128 * sg);
      } else {
        const int q = p - CF::PCA, kr = q / (BN / 128), sg = q % (BN / 128);
        load_piece(std::integral_constant<bool, B4>{}, g.B, g.ldb, n0 + 128 * sg, g.N, c * BK + kr,
                   st + BK * PA + kr * PB + 128 * sg);
      }
    }
  };
  // glds instructions a wave issues per chunk, as the vmcnt unit below: a
  // lower bound (one per piece; a 4-byte piece issues four), so that waiting
  // down to k x LPC outstanding always retires chunk c (exact without A4 / B4)
  constexpr int RPW = (CF::PCA + CF::PCB) / NW;
  constexpr int LPC = RPW;
  constexpr int W1 = LPC < 63 ? LPC : 63, W2 = 2 * LPC < 63 ? 2 * LPC : 63, W3 = 3 * LPC < 63 ? 3 * LPC : 63;

  // accumulators: 4x4x4_4b: acc1[i][j] one double, C[8 i + 4 bm + X][8 j + 4 bn + Y];
  // 16x16x4: acc4[i][j] four doubles, C[16 i + tq + 4 r][16 j + fl]
  constexpr bool M16 = CF::MF == 1;
  double acc1[M16 ? 1 : 8][M16 ? 1 : 8];
  d4 acc4[M16 ? 4 : 1][M16 ? 4 : 1];
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc4[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc1[i][j] = 0.0;
  }
  const int fl = lane & 15, tq = lane >> 4;
  // row groups (8 rows for 4x4x4_4b, 16 for 16x16x4) of this wave that hold
  // rows < M (wave-uniform)
  constexpr int RG = M16 ? 16 : 8, NRG = 64 / RG;
  const int nib = min(NRG, max(0, (g.M - m0 - wm * 64 + RG - 1) / RG));
  const int nch = (g.K + BK - 1) / BK;
#pragma unroll
  for (int c = 0; c < NS - 1; ++c)
    if (c < nch) issue(c);
  const int aoff = M16 ? wm * 64 + fl : wm * 64 + 4 * (bq >> 1) + Y;
  const int boff = M16 ? BK * PA + wn * 64 + fl : BK * PA + wn * 64 + 4 * (bq & 1) + Y;
  const int krow = M16 ? tq : X;
  // the chunk loop, once for interior waves (all row groups inside M) and
  // once for edge waves, so that no branch sits between the MFMAs
  auto mainloop = [&](auto full_tag) {
    constexpr bool FULL = decltype(full_tag)::value;
    for (int c = 0; c < nch; ++c) {
      // chunk c landed for this wave's own loads: at most LPC per younger
      // chunk still in flight (they count in issue order)
      const int ahead = min(NS - 2, nch - 1 - c);
      if (NS >= 5 && ahead >= 3)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W3) : "memory");
      else if (NS >= 4 && ahead >= 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W2) : "memory");
      else if (NS >= 3 && ahead >= 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W1) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // every wave's chunk c is in; chunk c - 1 is read
      if (c + NS - 1 < nch) issue(c + NS - 1);
      const double *st = smem + (c % NS) * SS;
      // operands of k-step kk + 1 are read while the MFMAs of kk issue
      constexpr int NA = M16 ? 4 : 8;
      double a[2][NA], b[2][NA];
      auto ldop = [&](int kk, int sl) {
        const double *ra = st + (4 * kk + krow) * PA + aoff;
        const double *rb = st + (4 * kk + krow) * PB + boff;
#pragma unroll
        for (int i = 0; i < NA; ++i) a[sl][i] = ra[(64 / NA) * i];
#pragma unroll
        for (int j = 0; j < NA; ++j) b[sl][j] = rb[(64 / NA) * j];
      };
      ldop(0, 0);
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        const int sl = kk & 1;
        if (kk + 1 < BK / 4) ldop(kk + 1, sl ^ 1);
#pragma unroll
        for (int i = 0; i < NA; ++i)
          if (FULL || i < nib)
#pragma unroll
            for (int j = 0; j < NA; ++j) {
              if constexpr (M16)
                acc4[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[sl][i], b[sl][j], acc4[i][j], 0, 0, 0);
              else
                acc1[i][j] = d2_mfma(a[sl][i], b[sl][j], acc1[i][j]);
            }
      }
    }
  };
  if (nib == NRG)
    mainloop(std::true_type{});
  else
    mainloop(std::false_type{});
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + 16 * i + tq + 4 * r;
        if (row < g.M) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int col = n0 + wn * 64 + 16 * j + fl;
            if (col < g.N) g.C[(size_t)row * g.ldc + col] = acc4[i][j][r];
          }
        }
      }
  } else {
    // lane (X, b, Y) holds C[8 i + 4 bm + X][8 j + 4 bn + Y] of the wave tile
    const int row0 = m0 + wm * 64 + 4 * (bq >> 1) + X, col0 = n0 + wn * 64 + 4 * (bq & 1) + Y;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = row0 + 8 * i;
      if (row < g.M) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = col0 + 8 * j;
          if (col < g.N) g.C[(size_t)row * g.ldc + col] = acc1[i][j];
        }
      }
    }
  }
}


}  // namespace fasst
