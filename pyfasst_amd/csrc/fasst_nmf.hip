// Itakura-Saito NMF multiplicative updates on MI355X (gfx950), FP64.
//
// Restates tools/nmf.py NMF_decomposition (:24-61) / NMF_decomp_init
// (:63-159).  One iteration:
//   hat = W H                      (MFMA GEMM, F x N x K)
//   X = SX/max(hat^2, eps), Y = 1/max(hat, eps)
//   num^T = H X^T, den^T = H Y^T   (one GEMM launch, shared H operand)
//   W *= num/max(den, eps); s = colsum(W), s[s==0] = 1; W /= s; H *= s
//   hat = W H; X, Y as above
//   num = W^T X, den = W^T Y       (one GEMM launch, shared W operand)
//   H *= num/max(den, eps)
// (the unfused GEMM path below).  The fused path (K % 16 == 0, K <= 64) runs
// an iteration in four launches: k_nmf_wnum (hat, ratios and the W
// contraction in registers), k_nmf_w_upd (W *= num / max(den, eps) and
// partial column sums), k_nmf_hnum (the H contraction on the un-renormalised
// W: the column scale cancels in the model), k_nmf_h_part (H *= s num /
// max(den, eps), W /= s).
#include "fasst_gemm.h"
#include "fasst_fft.h"

#include <algorithm>

#include "../../include/fasst_nmf.h"

namespace fasst {

constexpr double kNmfEps = 1e-10;  // tools/nmf.py:22

__global__ void k_nmf_xy(const double *__restrict__ hat, const double *__restrict__ SX,
                         double *__restrict__ X, double *__restrict__ Y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const double h = hat[i];
    X[i] = SX[i] / fmax(h * h, kNmfEps);
    Y[i] = 1.0 / fmax(h, kNmfEps);
  }
}

// one block per component k: W[:, k] update, column sum, renormalisation
__global__ __launch_bounds__(256) void k_nmf_w(double *__restrict__ W,
                                               const double *__restrict__ numT,
                                               const double *__restrict__ denT,
                                               double *__restrict__ s_out, int F, int K) {
  __shared__ double s_red[256];
  const int k = blockIdx.x;
  double part = 0.0;
  for (int f = threadIdx.x; f < F; f += 256) {
    const double w = W[(size_t)f * K + k] * (numT[(size_t)k * F + f] / fmax(denT[(size_t)k * F + f], kNmfEps));
    W[(size_t)f * K + k] = w;
    part += w;
  }
  s_red[threadIdx.x] = part;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
    __syncthreads();
  }
  double s = s_red[0];
  if (s == 0) s = 1.0;  // sumW[sumW==0] = 1. (nmf.py:46)
  for (int f = threadIdx.x; f < F; f += 256) W[(size_t)f * K + k] /= s;
  if (threadIdx.x == 0) s_out[k] = s;
}

__global__ void k_nmf_hscale(double *__restrict__ H, const double *__restrict__ s, int K,
                             int N) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)K * N;
       i += (size_t)gridDim.x * blockDim.x)
    H[i] *= s[i / N];
}

__global__ void k_nmf_h(double *__restrict__ H, const double *__restrict__ num,
                        const double *__restrict__ den, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    H[i] *= num[i] / fmax(den[i], kNmfEps);
}

// 1/x for finite normal x > 0: v_rcp_f64 + two Newton steps (<= 1 ulp), as
// the FASST E-step (fasst_em.hip rcp_nr)
__device__ __forceinline__ double nmf_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}

// raw-buffer loads for the fused contractions: wave-uniform resource in
// SGPRs + a 32-bit lane offset, so every load of a tile is issued
// unconditionally (a guarded pointer load compiles into an exec branch per
// load, and the branches made the compiler wait for ALL outstanding loads --
// the next tile's prefetch included -- before each tile's MFMAs).  An offset
// of kNmfOOB is outside every resource and reads 0.0; otherwise the accesses
// stay inside the (padded, zero-filled) allocations, see nmf_create.
typedef unsigned nmf_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t nmf_rsrc(const double *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double nmf_ld(__amdgpu_buffer_rsrc_t r, unsigned vo) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)vo, 0, 0));
}

__device__ __forceinline__ d4 nmfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Fused IS-NMF contractions (K a multiple of 16, <= 64): the model hat = W H
// is recomputed tile by tile on the MFMA pipe and never stored, the ratios
// X = SX / max(hat^2, eps), Y = 1 / max(hat, eps) stay in registers, and the
// accumulator-as-operand layout of 16x16x4 feeds them straight into the
// contraction (as the FASST FB / TW contractions, fasst_em.hip).
//
// Register layouts are chosen so that every operand a lane needs is a run of
// consecutive doubles (16-byte loads, 20 per 16 x 32 tile instead of 40
// 8-byte ones, so a tile's prefetch and the tile in flight fit the 63 loads
// the wave's vmcnt can track):
//   - the hat product's component index at step s, lane row tq is
//     k = 8 (s >> 1) + 2 tq + (s & 1): a lane's W row / frame-major H row
//     (Ht, N x K, the fused path's copy of H) values come in 16-byte pairs,
//     and the four lane rows of one load cover 64 contiguous bytes;
//   - the contraction's output column kc of lane column fl is component
//     32 (kc >> 1) + 2 fl + (kc & 1) (a 16-wide tail 16 kc + fl for odd
//     NKC): 16-byte pairs again, 16 lanes on 256 contiguous bytes;
//   - the kept dimension is split over PW = 2 interleaved 16-wide tiles
//     (element e of a 32-wide group sits in tile e & 1 at lane row e >> 1):
//     the SX values of a lane are contiguous in p.
// Each 4-wave workgroup splits its reduction range over its waves, folds the
// four partials in LDS in wave order, and writes one partial per workgroup
// row to `part`; the consumer (k_nmf_w_part / k_nmf_h_part) sums the groups
// in index order: deterministic.
constexpr int kNmfPW = 2;

typedef unsigned nmf_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nmf_ld2(__amdgpu_buffer_rsrc_t r, unsigned vo, double &a, double &b) {
  const nmf_u4 x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)vo, 0, 0);
  a = __builtin_bit_cast(double, __builtin_shufflevector(x, x, 0, 1));
  b = __builtin_bit_cast(double, __builtin_shufflevector(x, x, 2, 3));
}
// the hat operand run of a lane: pairs j at byte offset vo + 64 j
template <int NKS>
__device__ __forceinline__ void nmf_ld_hat(__amdgpu_buffer_rsrc_t r, unsigned vo, double (&d)[NKS]) {
#pragma unroll
  for (int j = 0; j < NKS / 2; ++j) nmf_ld2(r, vo + 64u * j, d[2 * j], d[2 * j + 1]);
}
__device__ __forceinline__ constexpr int nmf_hat_k(int s, int tq) { return 8 * (s >> 1) + 2 * tq + (s & 1); }
// the contraction operand of a lane: pairs m at byte offset vo + 256 m
// (vo = row + 16 fl), the odd tail at row + 8 (16 (NKC - 1) + fl)
template <int NKC>
__device__ __forceinline__ void nmf_ld_con(__amdgpu_buffer_rsrc_t r, unsigned vo, int fl, double (&d)[NKC]) {
#pragma unroll
  for (int m = 0; m < NKC / 2; ++m) nmf_ld2(r, vo + 256u * m, d[2 * m], d[2 * m + 1]);
  if constexpr (NKC & 1) d[NKC - 1] = nmf_ld(r, vo - 8u * fl + 128u * (NKC - 1));
}
template <int NKC>
__device__ __forceinline__ constexpr int nmf_con_k(int kc, int fl) {
  return kc < (NKC & ~1) ? 32 * (kc >> 1) + 2 * fl + (kc & 1) : 16 * kc + fl;
}

// interleave a tile's prefetch (NL 16-byte loads) with the first MFMAs of
// the tile in flight, one load per two MFMAs: issued all at once, the four
// waves' loads queue on the CU's address unit and hold back their MFMAs
template <int NKC>
__device__ __forceinline__ void nmf_spread_loads() {
  constexpr int NL = 4 + 2 * NKC + 4 * (NKC / 2 + (NKC & 1));
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);  // one VMEM read
    __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);   // two MFMAs
  }
}

// partial for (kept index r0 + PW (tq + 4m) + p, component nmf_con_k(kc, fl));
// TR: [r][K] rows (the H update's frame-major partials), else [K][R]
template <int NKC, bool TR>
__device__ __forceinline__ void nmf_fold_store(d4 (&num)[kNmfPW][NKC], d4 (&den)[kNmfPW][NKC],
                                               double *__restrict__ pn, double *__restrict__ pd,
                                               int r0, int R, int wv, int lane) {
  constexpr int NE = kNmfPW * NKC * 4, K = 16 * NKC;
  const int fl = lane & 15, tq = lane >> 4;
  {
    // all four partials into LDS at once (NE x 2 KB per wave), one barrier,
    // then each wave sums a quarter of the elements in wave order (the
    // sequential fold's association: bit-identical) and stores them
    __shared__ double red4[4][2][NE][64];
#pragma unroll
    for (int p = 0; p < kNmfPW; ++p)
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int e = (p * NKC + kc) * 4 + m;
          red4[wv][0][e][lane] = num[p][kc][m];
          red4[wv][1][e][lane] = den[p][kc][m];
        }
    __syncthreads();
#pragma unroll
    for (int e0 = 0; e0 < NE; e0 += 4) {
      const int e = e0 + wv, m = e & 3, kc = (e >> 2) % NKC, p = (e >> 2) / NKC;
      const double a = ((red4[0][0][e][lane] + red4[1][0][e][lane]) + red4[2][0][e][lane]) + red4[3][0][e][lane];
      const double b = ((red4[0][1][e][lane] + red4[1][1][e][lane]) + red4[2][1][e][lane]) + red4[3][1][e][lane];
      const int r = r0 + kNmfPW * (tq + 4 * m) + p, k = nmf_con_k<NKC>(kc, fl);
      if (r < R) {
        const size_t o = TR ? (size_t)r * K + k : (size_t)k * R + r;
        pn[o] = a;
        pd[o] = b;
      }
    }
  }
}

// W update (nmf.py:39-44): numT[k][f] = sum_t H[k][t] X[f][t], denT with Y.
// A workgroup owns one 32-bin group (bin g0 + 2 fl + p) and 4 frame chunks
// (one per wave); the group's W rows are loop-invariant hat operands.
template <int NKC>
__global__ __launch_bounds__(256, 1) void k_nmf_wnum(const double *__restrict__ W,
                                                     const double *__restrict__ Ht,
                                                     const double *__restrict__ SXt,
                                                     double *__restrict__ part, int F, int N, int tpc) {
  constexpr int NKS = 4 * NKC, K = 16 * NKC, PW = kNmfPW;
  const int lane = threadIdx.x & 63, fl = lane & 15, tq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g0 = blockIdx.x * 16 * PW, ntt = (N + 15) / 16;
  const __amdgpu_buffer_rsrc_t rW = nmf_rsrc(W), rH = nmf_rsrc(Ht);
  double wk[PW][NKS];  // bins past F: W's zero pad rows
#pragma unroll
  for (int p = 0; p < PW; ++p) nmf_ld_hat(rW, (unsigned)(((g0 + PW * fl + p) * K + 2 * tq) * 8), wk[p]);
  d4 num[PW][NKC], den[PW][NKC];
#pragma unroll
  for (int p = 0; p < PW; ++p)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) num[p][kc] = den[p][kc] = d4{0.0, 0.0, 0.0, 0.0};
  const int tb = (blockIdx.y * 4 + wv) * tpc, te = min(tb + tpc, ntt);
  // the next frame tile's operands are loaded while this tile's MFMAs run.
  // Frames past N read Ht's zero pad rows (hb = 0: they add nothing) and
  // SXt's pad; bins past F read the next SXt row (finite, never stored)
  double th[2][NKS], hb[2][4][NKC], sxv[2][4][PW];
  const unsigned vo_th = (unsigned)((fl * K + 2 * tq) * 8);
  const unsigned vo_hb = (unsigned)((tq * K + 2 * fl) * 8);
  const unsigned vo_sx = (unsigned)((tq * F + g0 + PW * fl) * 8);
  auto load = [&](int tt, int slot) {
    const int t0 = tt * 16;
    const unsigned ho = (unsigned)(t0 * K * 8);
    // the SX stream (HBM) first, then the L2-resident Ht tile
    const __amdgpu_buffer_rsrc_t rS = nmf_rsrc(SXt + (size_t)t0 * F);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      nmf_ld2(rS, vo_sx + (unsigned)(4 * i * F * 8), sxv[slot][i][0], sxv[slot][i][1]);
    nmf_ld_hat(rH, vo_th + ho, th[slot]);
#pragma unroll
    for (int i = 0; i < 4; ++i) nmf_ld_con(rH, vo_hb + ho + (unsigned)(4 * i * K * 8), fl, hb[slot][i]);
  };
  auto compute = [&](int cs) {
    // the hat tiles of both bin tiles first, four accumulation chains each
    // (one wave per SIMD: the MFMA latency is hidden by independent chains)
    d4 hv[PW];
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      d4 v0 = d4{0.0, 0.0, 0.0, 0.0}, v1 = v0, v2 = v0, v3 = v0;
#pragma unroll
      for (int s = 0; s < NKS; s += 4) {
        v0 = nmfma(th[cs][s], wk[p][s], v0);
        v1 = nmfma(th[cs][s + 1], wk[p][s + 1], v1);
        v2 = nmfma(th[cs][s + 2], wk[p][s + 2], v2);
        v3 = nmfma(th[cs][s + 3], wk[p][s + 3], v3);
      }
      hv[p] = (v0 + v1) + (v2 + v3);
    }
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const d4 v = hv[p];  // hat at (frame t0+tq+4i, bin g0+2fl+p)
      // no masks: frames past N meet hb = 0, bins past F are never stored,
      // and every ratio is finite (hat >= 0, floored at eps)
      double x[4], y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double h = v[i];
        x[i] = sxv[cs][i][p] * nmf_rcp(fmax(h * h, kNmfEps));
        y[i] = nmf_rcp(fmax(h, kNmfEps));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) {
          num[p][kc] = nmfma(x[i], hb[cs][i][kc], num[p][kc]);
          den[p][kc] = nmfma(y[i], hb[cs][i][kc], den[p][kc]);
        }
    }
  };
  // one tile per trip: the next tile is loaded into slot 1 while slot 0's
  // MFMAs run, then moved into slot 0 (40 register moves per 192 MFMAs).
  // The prefetch is unconditional (the last tile again past the end) and its
  // values are consumed on every path, so it can neither be sunk below the
  // MFMAs nor make the compiler's vmcnt waits cover it before they run
  if (tb < te) load(tb, 0);
  // two tiles per trip, slots alternating (no register moves); every load
  // is consumed on every path out of its trip, so none is sunk or waited
  // for early
  int tt = tb;
  for (; tt + 1 < te; tt += 2) {
    load(tt + 1, 1);
    compute(0);
    nmf_spread_loads<NKC>();
    __builtin_amdgcn_sched_barrier(0);
    load(min(tt + 2, te - 1), 0);
    compute(1);
    nmf_spread_loads<NKC>();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (tt < te) compute(0);
  const size_t slab = (size_t)K * F;
  double *pn = part + (size_t)blockIdx.y * 2 * slab;
  nmf_fold_store<NKC, false>(num, den, pn, pn + slab, g0, F, wv, lane);
}

// H update (nmf.py:53-59): num[k][t] = sum_f W[f][k] X[f][t], den with Y,
// hat from the updated W and the rescaled H (hs = W column sums from the W
// update, applied on load as k_nmf_hscale would; null when W is frozen).  A
// workgroup owns one 32-frame group (frame t0 + 2 fl + p) and 4 bin chunks
// (one per wave).
template <int NKC>
__global__ __launch_bounds__(256, 1) void k_nmf_hnum(const double *__restrict__ W,
                                                     const double *__restrict__ Ht,
                                                     const double *__restrict__ hs,
                                                     const double *__restrict__ SX,
                                                     double *__restrict__ part, int F, int N, int fpc) {
  constexpr int NKS = 4 * NKC, K = 16 * NKC, PW = kNmfPW;
  const int lane = threadIdx.x & 63, fl = lane & 15, tq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t0g = blockIdx.x * 16 * PW, nft = (F + 15) / 16;
  const __amdgpu_buffer_rsrc_t rW = nmf_rsrc(W), rH = nmf_rsrc(Ht);
  // frames past N read the next Ht rows or its zero pad: finite, and their
  // output columns are never stored
  double bt[PW][NKS], hsv[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) hsv[s] = hs ? hs[nmf_hat_k(s, tq)] : 1.0;
#pragma unroll
  for (int p = 0; p < PW; ++p) nmf_ld_hat(rH, (unsigned)(((t0g + PW * fl + p) * K + 2 * tq) * 8), bt[p]);
#pragma unroll
  for (int p = 0; p < PW; ++p)
#pragma unroll
    for (int s = 0; s < NKS; ++s) bt[p][s] *= hsv[s];
  d4 num[PW][NKC], den[PW][NKC];
#pragma unroll
  for (int p = 0; p < PW; ++p)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) num[p][kc] = den[p][kc] = d4{0.0, 0.0, 0.0, 0.0};
  const int fb = (blockIdx.y * 4 + wv) * fpc, fe = min(fb + fpc, nft);
  // the next bin tile's operands are loaded while this tile's MFMAs run;
  // bins past F read W's zero pad rows (bw = 0: they add nothing) and SX's
  // pad or the next SX row
  double ao[2][NKS], bw[2][4][NKC], sxv[2][4][PW];
  const unsigned vo_ao = (unsigned)((fl * K + 2 * tq) * 8);
  const unsigned vo_bw = (unsigned)((tq * K + 2 * fl) * 8);
  const unsigned vo_sx = (unsigned)((tq * N + t0g + PW * fl) * 8);
  auto load = [&](int ft, int slot) {
    const int f0 = ft * 16;
    const unsigned wo = (unsigned)(f0 * K * 8);
    const __amdgpu_buffer_rsrc_t rS = nmf_rsrc(SX + (size_t)f0 * N);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      nmf_ld2(rS, vo_sx + (unsigned)(4 * i * N * 8), sxv[slot][i][0], sxv[slot][i][1]);
    nmf_ld_hat(rW, vo_ao + wo, ao[slot]);
#pragma unroll
    for (int i = 0; i < 4; ++i) nmf_ld_con(rW, vo_bw + wo + (unsigned)(4 * i * K * 8), fl, bw[slot][i]);
  };
  auto compute = [&](int cs) {
    d4 hv[PW];  // as k_nmf_wnum: both hat tiles first, four chains each
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      d4 v0 = d4{0.0, 0.0, 0.0, 0.0}, v1 = v0, v2 = v0, v3 = v0;
#pragma unroll
      for (int s = 0; s < NKS; s += 4) {
        v0 = nmfma(ao[cs][s], bt[p][s], v0);
        v1 = nmfma(ao[cs][s + 1], bt[p][s + 1], v1);
        v2 = nmfma(ao[cs][s + 2], bt[p][s + 2], v2);
        v3 = nmfma(ao[cs][s + 3], bt[p][s + 3], v3);
      }
      hv[p] = (v0 + v1) + (v2 + v3);
    }
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const d4 v = hv[p];  // hat at (bin f0+tq+4i, frame t0g+2fl+p)
      double x[4], y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double h = v[i];
        x[i] = sxv[cs][i][p] * nmf_rcp(fmax(h * h, kNmfEps));
        y[i] = nmf_rcp(fmax(h, kNmfEps));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) {
          num[p][kc] = nmfma(x[i], bw[cs][i][kc], num[p][kc]);
          den[p][kc] = nmfma(y[i], bw[cs][i][kc], den[p][kc]);
        }
    }
  };
  if (fb < fe) load(fb, 0);
  // two tiles per trip, slots alternating (no register moves); every load
  // is consumed on every path out of its trip, so none is sunk or waited
  // for early
  int ft = fb;
  for (; ft + 1 < fe; ft += 2) {
    load(ft + 1, 1);
    compute(0);
    nmf_spread_loads<NKC>();
    __builtin_amdgcn_sched_barrier(0);
    load(min(ft + 2, fe - 1), 0);
    compute(1);
    nmf_spread_loads<NKC>();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (ft < fe) compute(0);
  const size_t slab = (size_t)K * N;
  double *pn = part + (size_t)blockIdx.y * 2 * slab;
  nmf_fold_store<NKC, true>(num, den, pn, pn + slab, t0g, N, wv, lane);
}

// k_nmf_w over the fused path's group partials ([g][num / den][K][F]), in
// two launches so that the update spreads over K x kNmfWS workgroups: the
// multiplicative update of a bin range with its partial column sum, then the
// renormalisation by the summed columns
constexpr int kNmfWS = 4;
__global__ __launch_bounds__(256) void k_nmf_w_upd(double *__restrict__ W,
                                                   const double *__restrict__ part, int ng,
                                                   double *__restrict__ wsum, int F, int K) {
  __shared__ double s_red[256];
  const int k = blockIdx.x, fs = blockIdx.y;
  const size_t slab = (size_t)K * F;
  double acc = 0.0;
  for (int f = fs * 256 + threadIdx.x; f < F; f += kNmfWS * 256) {
    // the ng group partials of a bin loaded 8 at a time (a per-group loop
    // was a chain of global round trips)
    const double *q = part + (size_t)k * F + f;
    double n = 0.0, d = 0.0;
    for (int g = 0; g < ng; g += 8) {
      double vn[8], vd[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        vn[u] = g + u < ng ? q[(size_t)(g + u) * 2 * slab] : 0.0;
        vd[u] = g + u < ng ? q[(size_t)(g + u) * 2 * slab + slab] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        n += vn[u];
        d += vd[u];
      }
    }
    const double w = W[(size_t)f * K + k] * (n / fmax(d, kNmfEps));
    W[(size_t)f * K + k] = w;
    acc += w;
  }
  s_red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) wsum[k * kNmfWS + fs] = s_red[0];
}

// column sum of the updated W from its kNmfWS partials (nmf.py:45-46:
// sumW[sumW==0] = 1)
__device__ __forceinline__ double nmf_colsum(const double *__restrict__ wsum, int k) {
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < kNmfWS; ++u) s += wsum[k * kNmfWS + u];
  return s == 0 ? 1.0 : s;
}

// The H update's tail over the group partials ([g][num / den][N][K]) on the
// frame-major Ht, and the W update's renormalisation (nmf.py:45-48), which
// the fused path defers to here: k_nmf_hnum forms hat = W' H from the not
// yet renormalised W' and the not yet rescaled H (the same model: the
// column scale s cancels in W' H = (W' / s)(s H)), so its numerator and
// denominator both carry the factor s and their ratio is the reference's.
// Then Ht = (Ht s) num / max(den, eps) and W = W' / s, s_out = s.  wsum is
// null when W is frozen (no rescale).
__global__ void k_nmf_h_part(double *__restrict__ Ht, const double *__restrict__ part, int ng,
                             const double *__restrict__ wsum, double *__restrict__ W,
                             double *__restrict__ s_out, int F, int K, int N) {
  const size_t slab = (size_t)K * N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < slab;
       i += (size_t)gridDim.x * blockDim.x) {
    double n = 0.0, d = 0.0;
    for (int g = 0; g < ng; g += 8) {  // 8 groups' loads in flight at once
      double vn[8], vd[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        vn[u] = g + u < ng ? part[(size_t)(g + u) * 2 * slab + i] : 0.0;
        vd[u] = g + u < ng ? part[(size_t)(g + u) * 2 * slab + slab + i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        n += vn[u];
        d += vd[u];
      }
    }
    const double h = wsum ? Ht[i] * nmf_colsum(wsum, (int)(i % K)) : Ht[i];
    Ht[i] = h * (n / fmax(d, kNmfEps));
  }
  if (wsum)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)F * K;
         i += (size_t)gridDim.x * blockDim.x) {
      const double sk = nmf_colsum(wsum, (int)(i % K));
      W[i] /= sk;
      if (i < (size_t)K) s_out[i] = sk;
    }
}

// the W update's renormalisation when H is frozen: Ht *= s, W /= s
__global__ void k_nmf_hscale_t(double *__restrict__ Ht, const double *__restrict__ wsum,
                               double *__restrict__ W, double *__restrict__ s_out, int F, int K,
                               int N) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)K * N;
       i += (size_t)gridDim.x * blockDim.x)
    Ht[i] *= nmf_colsum(wsum, (int)(i % K));
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)F * K;
       i += (size_t)gridDim.x * blockDim.x) {
    const double sk = nmf_colsum(wsum, (int)(i % K));
    W[i] /= sk;
    if (i < (size_t)K) s_out[i] = sk;
  }
}

// out[c][r] = in[r][c] for an R x C matrix (row-major), 16 x 16 LDS tiles
__global__ void k_nmf_transpose(const double *__restrict__ in, double *__restrict__ out, int R,
                                int C) {
  __shared__ double tile[16][17];
  const int c0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  if (r0 + ty < R && c0 + tx < C) tile[ty][tx] = in[(size_t)(r0 + ty) * C + c0 + tx];
  __syncthreads();
  if (c0 + ty < C && r0 + tx < R) out[(size_t)(c0 + ty) * R + r0 + tx] = tile[tx][ty];
}

// ---------------------------------------------------------------- C2 Wiener
// Per-source mono Wiener images of the IS-NMF model (BASELINE configs[1]):
// the one-channel degenerate of the FASST separation (audioModel.py:1327-1467:
// Sigma_n = V_n, Sigma_x = sum_n Sigma_n + noise PSD, its inverse with the
// inv_herm_mat_2d determinant guard of signalTools.py:177-188 reduced to
// 1 x 1, WG_n = Sigma_n Sigma_x^-1, image = WG_n X, :1205-1214).  V_n =
// W[:, comps of n] H[comps of n, :] with the components grouped by source
// on the host (koff = source boundaries in the permuted order).
//
// Block: 16 bins x 64 frames, 256 threads; the W rows and H columns of the
// tile sit in LDS; each thread owns one bin and 4 frames.  Sigma_x is summed
// over the sources in a first pass, each V_n is recomputed (K FMAs per
// point) in the second pass right before its image is written: the kernel is
// HBM-bound (X read once, J images written once), V is never stored.
constexpr int kWienerMaxK = 256;
__global__ __launch_bounds__(256) void k_nmf_wiener(const double *__restrict__ W,
                                                    const double *__restrict__ H,
                                                    const int *__restrict__ koff, int J,
                                                    const double *__restrict__ psd,
                                                    const double2 *__restrict__ X,
                                                    double2 *__restrict__ S, int F, int N, int K,
                                                    int Fp, int Np) {
  extern __shared__ __attribute__((aligned(16))) double s_wh[];
  double *s_w = s_wh;             // [16][K + 1]
  double *s_h = s_wh + 16 * (K + 1);  // [K][64]
  const int f0 = blockIdx.y * 16, t0 = blockIdx.x * 64;
  const int tid = threadIdx.x, fl = tid & 15, tq = tid >> 4;
  for (int idx = tid; idx < 16 * K; idx += 256) {
    const int r = idx / K, k = idx % K;
    s_w[r * (K + 1) + k] = f0 + r < F ? W[(size_t)(f0 + r) * K + k] : 0.0;
  }
  for (int idx = tid; idx < K * 64; idx += 256) {
    const int k = idx >> 6, tl = idx & 63;
    s_h[idx] = t0 + tl < N ? H[(size_t)k * N + t0 + tl] : 0.0;
  }
  __syncthreads();
  const int f = f0 + fl;
  const double *wr = s_w + fl * (K + 1);
  auto vsrc = [&](int n, int i) {
    double v = 0.0;
    for (int k = koff[n]; k < koff[n + 1]; ++k) v = fma(wr[k], s_h[k * 64 + tq + 16 * i], v);
    return v;
  };
  const double nz = (psd && f < F) ? psd[f] : 0.0;
  double inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double sx = 0.0;
    for (int n = 0; n < J; ++n) sx += vsrc(n, i);
    sx += nz;
    const double sg = (sx + kNmfEps) > 0.0 ? 1.0 : ((sx + kNmfEps) < 0.0 ? -1.0 : 0.0);
    inv[i] = 1.0 / (sg * fmax(fabs(sx), kNmfEps));
  }
  if (f >= Fp) return;
  double2 x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = t0 + tq + 16 * i;
    x[i] = (f < F && t < N) ? X[(size_t)t * Fp + f] : make_double2(0.0, 0.0);
  }
  for (int n = 0; n < J; ++n) {
    double2 *Sn = S + (size_t)n * Np * Fp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + tq + 16 * i;
      if (t >= Np) continue;
      const double g = vsrc(n, i) * inv[i];
      Sn[(size_t)t * Fp + f] = make_double2(g * x[i].x, g * x[i].y);
    }
  }
}

}  // namespace fasst

using namespace fasst;

namespace {

// grouped (source-contiguous) copies of W's columns / H's rows
int wiener_setup(int F, int N, int K, const double *W, const double *H, int J, const int *comp_src,
                 std::vector<double> &Wg, std::vector<double> &Hg, std::vector<int> &koff) {
  if (F < 1 || N < 1 || K < 1 || K > kWienerMaxK || J < 1 || !W || !H || !comp_src) {
    set_error("nmf wiener: bad sizes F=%d N=%d K=%d (max %d) J=%d", F, N, K, kWienerMaxK, J);
    return FASST_ERR_SHAPE;
  }
  std::vector<int> order;
  koff.assign(J + 1, 0);
  for (int n = 0; n < J; ++n) {
    for (int k = 0; k < K; ++k)
      if (comp_src[k] == n) order.push_back(k);
    koff[n + 1] = (int)order.size();
  }
  Wg.resize((size_t)F * K, 0.0);
  Hg.resize((size_t)K * N, 0.0);
  const int Ku = (int)order.size();  // components assigned to no source are dropped
  for (int f = 0; f < F; ++f)
    for (int q = 0; q < Ku; ++q) Wg[(size_t)f * K + q] = W[(size_t)f * K + order[q]];
  for (int q = 0; q < Ku; ++q)
    std::copy(H + (size_t)order[q] * N, H + (size_t)(order[q] + 1) * N, Hg.begin() + (size_t)q * N);
  return FASST_OK;
}

// device images S [J][Np][Fp] (frame-major) from host W, H, X [F][N], psd [F]
struct WienerDev {
  DBuf<double> W, H, psd;
  DBuf<int> koff;
  DBuf<double2> Xh, X, S;
  int Fp = 0, Np = 0;
};

int wiener_images_dev(hipStream_t s, int F, int N, int K, const double *W, const double *H,
                      int J, const int *comp_src, const double *psd, const double *X,
                      WienerDev &d) {
  std::vector<double> Wg, Hg;
  std::vector<int> koff;
  int st = wiener_setup(F, N, K, W, H, J, comp_src, Wg, Hg, koff);
  if (st) return st;
  if (!X) return FASST_ERR_SHAPE;
  d.Fp = round_up(F, 16);
  d.Np = round_up(N, 64);
  if ((st = d.W.alloc((size_t)F * K)) || (st = d.H.alloc((size_t)K * N)) ||
      (st = d.psd.alloc(F)) || (st = d.koff.alloc(J + 1)) || (st = d.Xh.alloc((size_t)F * N)) ||
      (st = d.X.alloc((size_t)d.Np * d.Fp)) || (st = d.S.alloc((size_t)J * d.Np * d.Fp)))
    return st;
  FASST_HIP(hipMemcpyAsync(d.W.p, Wg.data(), Wg.size() * 8, hipMemcpyHostToDevice, s));
  FASST_HIP(hipMemcpyAsync(d.H.p, Hg.data(), Hg.size() * 8, hipMemcpyHostToDevice, s));
  FASST_HIP(hipMemcpyAsync(d.koff.p, koff.data(), koff.size() * sizeof(int), hipMemcpyHostToDevice, s));
  if (psd) FASST_HIP(hipMemcpyAsync(d.psd.p, psd, (size_t)F * 8, hipMemcpyHostToDevice, s));
  FASST_HIP(hipMemcpyAsync(d.Xh.p, X, (size_t)F * N * sizeof(double2), hipMemcpyHostToDevice, s));
  if ((st = tf_launch_ft_to_tf(s, d.Xh.p, d.X.p, F, N, d.Fp, d.Np, 1))) return st;
  const size_t smem = (size_t)(16 * (K + 1) + K * 64) * sizeof(double);
  if (smem > 64 * 1024)
    FASST_HIP(hipFuncSetAttribute((const void *)k_nmf_wiener,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  k_nmf_wiener<<<dim3(d.Np / 64, d.Fp / 16), 256, smem, s>>>(d.W.p, d.H.p, d.koff.p, J,
                                                             psd ? d.psd.p : nullptr, d.X.p,
                                                             d.S.p, F, N, K, d.Fp, d.Np);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

}  // namespace

struct nmf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int F = 0, N = 0, K = 0;
  DBuf<double> SX, W, H, hat, X, Y, numT, denT, num, den, s, work;
  // fused path (K % 16 == 0, K <= 64): transposed copies and chunk partials
  // (H lives frame-major in Ht there; H is its staging copy for set / get)
  int fused = 0, ng_w = 1, tpc_w = 1, ng_h = 1, fpc_h = 1;
  DBuf<double> SXt, Ht, part, wsum;
};

namespace {

int egrid_n(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 8192); }

int model_xy(nmf_ctx *c) {
  const double *Bs[1] = {c->H.p};
  double *Cs[1] = {c->hat.p};
  int st = gemm<false, false, 1>(c->stream, c->W.p, c->K, Bs, c->N, Cs, c->N, c->F, c->N, c->K,
                                 c->work.p);
  if (st) return st;
  const size_t FN = (size_t)c->F * c->N;
  k_nmf_xy<<<egrid_n(FN), 256, 0, c->stream>>>(c->hat.p, c->SX.p, c->X.p, c->Y.p, FN);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

constexpr int kNmfCUs = 256;
template <int NKC>
static void nmf_fused(nmf_ctx *c, int update_w, int update_h) {
  const int F = c->F, N = c->N, K = c->K;
  const int gw = (F + 16 * kNmfPW - 1) / (16 * kNmfPW), gh = (N + 16 * kNmfPW - 1) / (16 * kNmfPW);
  if (update_w) {
    k_nmf_wnum<NKC><<<dim3(gw, c->ng_w), 256, 0, c->stream>>>(c->W.p, c->Ht.p, c->SXt.p, c->part.p,
                                                              F, N, c->tpc_w);
    k_nmf_w_upd<<<dim3(K, kNmfWS), 256, 0, c->stream>>>(c->W.p, c->part.p, c->ng_w, c->wsum.p, F,
                                                       K);
  }
  // the W update leaves W un-renormalised and H un-rescaled: the H update
  // (or k_nmf_hscale_t) applies both (k_nmf_h_part)
  const double *ws = update_w ? c->wsum.p : nullptr;
  const int eg = egrid_n((size_t)K * std::max(N, F));
  if (update_h) {
    k_nmf_hnum<NKC><<<dim3(gh, c->ng_h), 256, 0, c->stream>>>(c->W.p, c->Ht.p, nullptr, c->SX.p,
                                                              c->part.p, F, N, c->fpc_h);
    k_nmf_h_part<<<eg, 256, 0, c->stream>>>(c->Ht.p, c->part.p, c->ng_h, ws, c->W.p, c->s.p, F, K,
                                            N);
  } else if (update_w) {
    k_nmf_hscale_t<<<eg, 256, 0, c->stream>>>(c->Ht.p, ws, c->W.p, c->s.p, F, K, N);
  }
}

int nmf_iteration(nmf_ctx *c, int update_w, int update_h) {
  int st;
  const int F = c->F, N = c->N, K = c->K;
  if (c->fused) {
    switch (K / 16) {
      case 1: nmf_fused<1>(c, update_w, update_h); break;
      case 2: nmf_fused<2>(c, update_w, update_h); break;
      case 3: nmf_fused<3>(c, update_w, update_h); break;
      default: nmf_fused<4>(c, update_w, update_h); break;
    }
    FASST_LAUNCH_CHECK();
    return FASST_OK;
  }
  if (update_w) {
    if ((st = model_xy(c))) return st;
    const double *Bs[2] = {c->X.p, c->Y.p};
    double *Cs[2] = {c->numT.p, c->denT.p};
    if ((st = gemm<false, true, 2>(c->stream, c->H.p, N, Bs, N, Cs, F, K, F, N, c->work.p)))
      return st;
    k_nmf_w<<<K, 256, 0, c->stream>>>(c->W.p, c->numT.p, c->denT.p, c->s.p, F, K);
    k_nmf_hscale<<<egrid_n((size_t)K * N), 256, 0, c->stream>>>(c->H.p, c->s.p, K, N);
    FASST_LAUNCH_CHECK();
  }
  if (update_h) {
    if ((st = model_xy(c))) return st;
    const double *Bs[2] = {c->X.p, c->Y.p};
    double *Cs[2] = {c->num.p, c->den.p};
    if ((st = gemm<true, false, 2>(c->stream, c->W.p, K, Bs, N, Cs, N, K, N, F, c->work.p)))
      return st;
    k_nmf_h<<<egrid_n((size_t)K * N), 256, 0, c->stream>>>(c->H.p, c->num.p, c->den.p,
                                                           (size_t)K * N);
    FASST_LAUNCH_CHECK();
  }
  return FASST_OK;
}

}  // namespace

extern "C" {

int nmf_create(int device, int F, int N, int K, nmf_ctx **out) {
  if (!out || F < 1 || N < 1 || K < 1) {
    set_error("nmf_create: bad sizes F=%d N=%d K=%d", F, N, K);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  nmf_ctx *c = new nmf_ctx();
  c->device = device;
  c->F = F;
  c->N = N;
  c->K = K;
  const size_t FN = (size_t)F * N;
  int st = FASST_OK;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) st = FASST_ERR_DEVICE;
  size_t gw = std::max({gemm_workspace(F, N, K, 1), gemm_workspace(K, F, N, 2),
                        gemm_workspace(K, N, F, 2), (size_t)1});
  // zero pads read by the fused contractions' unmasked loads (tiles past
  // the last bin / frame): 32 W rows, 16 SX rows (+64 values)
  if (!st) st = c->SX.alloc((size_t)(F + 16) * N + 64);
  if (!st) st = c->W.alloc((size_t)(F + 32) * K);
  if (!st) st = c->H.alloc((size_t)K * N);
  if (!st) st = c->hat.alloc(FN);
  if (!st) st = c->X.alloc(FN);
  if (!st) st = c->Y.alloc(FN);
  if (!st) st = c->numT.alloc((size_t)K * F);
  if (!st) st = c->denT.alloc((size_t)K * F);
  if (!st) st = c->num.alloc((size_t)K * N);
  if (!st) st = c->den.alloc((size_t)K * N);
  if (!st) st = c->s.alloc(K);
  if (!st) st = c->work.alloc(gw);
  // fused path: 4-wave groups (one per CU at the kernels' occupancy of one
  // wave per SIMD), as many groups as fit in one pass over the 256 CUs
  // (their buffer offsets into W, Ht and 16-row SX / SXt slabs are 32-bit)
  c->fused = K % 16 == 0 && K <= 64 && (size_t)(N + 32) * K * 8 < 0x7fffffffu &&
             (size_t)(F + 32) * K * 8 < 0x7fffffffu && (size_t)32 * (F + N + 64) * 8 < 0x7fffffffu;
  if (c->fused) {
    const int nft = (F + 15) / 16, ntt = (N + 15) / 16;
    // launch geometry: a 32-wide group of the kept dimension per workgroup,
    // the contracted dimension split over 4 waves x ng groups so the grid
    // holds about `waves` waves (round 2 at C2, F=1025 T=2000 K=64: ~1024
    // waves best, 2048: +20%)
    const int waves = 4 * kNmfCUs;
    const int uw = (nft + kNmfPW - 1) / kNmfPW, uh = (ntt + kNmfPW - 1) / kNmfPW;
    int ng = std::max(1, std::min((ntt + 3) / 4, waves / (4 * uw)));
    c->tpc_w = (ntt + 4 * ng - 1) / (4 * ng);
    c->ng_w = ((ntt + c->tpc_w - 1) / c->tpc_w + 3) / 4;
    ng = std::max(1, std::min((nft + 3) / 4, waves / (4 * uh)));
    c->fpc_h = (nft + 4 * ng - 1) / (4 * ng);
    c->ng_h = ((nft + c->fpc_h - 1) / c->fpc_h + 3) / 4;
    const size_t np = std::max((size_t)c->ng_w * 2 * K * F, (size_t)c->ng_h * 2 * K * N);
    if (!st) st = c->SXt.alloc((size_t)(N + 16) * F + 64);
    if (!st) st = c->Ht.alloc((size_t)(N + 32) * K);
    if (!st) st = c->part.alloc(np);
    if (!st) st = c->wsum.alloc((size_t)K * kNmfWS);
  }
  if (st) {
    nmf_destroy(c);
    return st;
  }
  *out = c;
  return FASST_OK;
}

int nmf_destroy(nmf_ctx *c) {
  if (!c) return FASST_OK;
  {
    DeviceGuard g(c->device);
    if (c->stream) {
      (void)hipStreamSynchronize(c->stream);
      (void)hipStreamDestroy(c->stream);
    }
  }
  delete c;
  return FASST_OK;
}

int nmf_set_data(nmf_ctx *c, const double *SX) {
  if (!c || !SX) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  FASST_HIP(hipMemcpyAsync(c->SX.p, SX, (size_t)c->F * c->N * 8, hipMemcpyHostToDevice, c->stream));
  if (c->fused)  // frame-major copy: the W-update contraction reads 16 bins per row segment
    k_nmf_transpose<<<dim3((c->N + 15) / 16, (c->F + 15) / 16), 256, 0, c->stream>>>(
        c->SX.p, c->SXt.p, c->F, c->N);
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int nmf_set_params(nmf_ctx *c, const double *W, const double *H) {
  if (!c || !W || !H) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  FASST_HIP(hipMemcpyAsync(c->W.p, W, (size_t)c->F * c->K * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->H.p, H, (size_t)c->K * c->N * 8, hipMemcpyHostToDevice, c->stream));
  if (c->fused)
    k_nmf_transpose<<<dim3((c->N + 15) / 16, (c->K + 15) / 16), 256, 0, c->stream>>>(
        c->H.p, c->Ht.p, c->K, c->N);
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int nmf_run(nmf_ctx *c, int n_iter, int update_w, int update_h) {
  if (!c || n_iter < 0) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  for (int it = 0; it < n_iter; ++it) {
    int st = nmf_iteration(c, update_w, update_h);
    if (st) return st;
  }
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int nmf_wiener_images(int device, int F, int N, int K, const double *W, const double *H, int J,
                      const int *comp_source, const double *psd, const double *X, double *S) {
  if (!S) return FASST_ERR_SHAPE;
  DeviceGuard g(device);
  hipStream_t s = nullptr;
  FASST_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  WienerDev d;
  int st = wiener_images_dev(s, F, N, K, W, H, J, comp_source, psd, X, d);
  DBuf<double2> hS;
  if (!st) st = hS.alloc((size_t)J * F * N);
  if (!st) st = tf_launch_tf_to_ft(s, d.S.p, hS.p, F, N, d.Fp, d.Np, J);
  if (!st && hipMemcpyAsync(S, hS.p, hS.n * sizeof(double2), hipMemcpyDeviceToHost, s) != hipSuccess)
    st = FASST_ERR_DEVICE;
  if (hipStreamSynchronize(s) != hipSuccess && !st) st = FASST_ERR_DEVICE;
  (void)hipStreamDestroy(s);
  return st;
}

int nmf_wiener_waveforms(int device, int F, int N, int K, const double *W, const double *H, int J,
                         const int *comp_source, const double *psd, const double *X,
                         const double *window, const double *analysis_window, int wlen, int nfft,
                         int hop, double *y) {
  if (!y || !window || nfft / 2 + 1 != F) {
    set_error("nmf_wiener_waveforms: nfft=%d does not give F=%d bins", nfft, F);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  hipStream_t s = nullptr;
  FASST_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  WienerDev d;
  int st = wiener_images_dev(s, F, N, K, W, H, J, comp_source, psd, X, d);
  const int len_out = hop * (N - 1) + wlen - wlen / 2;  // istft (stft.py:108-129)
  DBuf<double> dw, daw, frames, dy;
  DBuf<double2> dtw;
  if (!st && ((st = dw.alloc(wlen)) || (st = daw.alloc(wlen)) || (st = dtw.alloc(nfft / 2)) ||
              (st = frames.alloc((size_t)N * wlen)) || (st = dy.alloc((size_t)J * len_out)))) {
  }
  auto tw = twiddles(nfft, +1);
  if (!st && (hipMemcpyAsync(dw.p, window, (size_t)wlen * 8, hipMemcpyHostToDevice, s) ||
              hipMemcpyAsync(daw.p, analysis_window ? analysis_window : window, (size_t)wlen * 8,
                             hipMemcpyHostToDevice, s) ||
              hipMemcpyAsync(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice, s)))
    st = FASST_ERR_DEVICE;
  for (int n = 0; n < J && !st; ++n)
    st = tf_launch_istft(s, d.S.p + (size_t)n * d.Np * d.Fp, d.Fp, N, dw.p, daw.p, dtw.p, wlen,
                         nfft, hop, frames.p, dy.p + (size_t)n * len_out, len_out);
  if (!st && hipMemcpyAsync(y, dy.p, dy.n * 8, hipMemcpyDeviceToHost, s) != hipSuccess)
    st = FASST_ERR_DEVICE;
  if (hipStreamSynchronize(s) != hipSuccess && !st) st = FASST_ERR_DEVICE;
  (void)hipStreamDestroy(s);
  return st;
}

int nmf_get_params(nmf_ctx *c, double *W, double *H) {
  if (!c) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  if (W) FASST_HIP(hipMemcpyAsync(W, c->W.p, (size_t)c->F * c->K * 8, hipMemcpyDeviceToHost, c->stream));
  if (H && c->fused)
    k_nmf_transpose<<<dim3((c->K + 15) / 16, (c->N + 15) / 16), 256, 0, c->stream>>>(
        c->Ht.p, c->H.p, c->N, c->K);
  if (H) FASST_HIP(hipMemcpyAsync(H, c->H.p, (size_t)c->K * c->N * 8, hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

}  // extern "C"
