// SIMM source/filter multiplicative updates on MI355X (gfx950), FP64.
//
// Restates SeparateLeadStereo/SIMM/SIMM.py: Stereo_SIMM (:397-943) and SIMM
// (:46-395).  The per-iteration update order is the reference's: HF0, HPHI,
// HM, HGAMMA, WM, (stereo) alpha, beta, each followed by the model refresh
//   hatSX_R = max(WM diag(bR^2) HM + aR^2 SF0*SPHI, eps)
//   hatSX_L = max(aL^2 SF0*SPHI + WM diag(bL^2) HM, eps).
// The F x NF0 x N products (WF0^T X, WF0 HF0) run on the FP64 MFMA GEMM of
// fasst_gemm.h; elementwise ratios, skinny products (K = 4 filters) and the
// renormalisations are fused VALU kernels.  One deliberate shortcut: after
// HPHI / HGAMMA renormalise the columns of HF0 (HF0 *= s), SF0 = WF0 HF0 is
// updated as SF0 *= s (the same linear map; the reference recomputes the
// GEMM) -- it saves two F x NF0 x N GEMMs per iteration.
#include "fasst_gemm.h"

#include <atomic>
#include <cmath>
#include <type_traits>

#include "../../include/fasst_simm.h"

namespace fasst {

constexpr double kSimmEps = 1e-20;  // SIMM.py:150, :506
// non-temporal access to the streamed F x N planes (see k_simm_refresh)
#define SLD(p) __builtin_nontemporal_load(&(p))
#define SST(p, v) __builtin_nontemporal_store((v), &(p))
#define CLD(p) __builtin_nontemporal_load(&(p))

// ------------------------------------------------------------------ kernels
#define GRID_STRIDE(i, n)                                                          \
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)(n); \
       i += (size_t)gridDim.x * blockDim.x)

static inline int egrid(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 8192); }

// ratio^omega with the reference's `** omega` (omega == 1 is exact)
__device__ __forceinline__ double powo(double x, double omega) {
  return omega == 1.0 ? x : pow(x, omega);
}

constexpr int kSimmKmax = 8;  // simm_create: K <= 8 filters
constexpr int kHgRowChunks = 4;  // frame chunks of k_hgamma_rows (>= 4 waves per SIMD at C5)
// bins per k_hgamma_rows block: 2 halves its accumulators and doubles the
// blocks (C5 8.92 -> 8.74 ms per iteration vs 4 bins; 1 bin the same as 2)
#ifndef FASST_HG_ROWS
#define FASST_HG_ROWS 2
#endif
constexpr int kHgRows = FASST_HG_ROWS;

// ---------------------------------------------------------------------------
// The model spectrograms are not stored between updates.  Every update of the
// reference ends with a refresh of hatSX_R / hatSX_L (SIMM.py:661-674,
// :715-728, :760-773, :812-823, :856-869, :894-906, :925-941); here each
// consumer recomputes, per point, from the resident planes SF0, SMR, SML:
//   SPHI = WPHI HPHI (K <= 8 filters: the column of HPHI in registers, the
//          row of WPHI wave-uniform), summed in k order as k_simm_refresh does
//   l = SF0 SPHI, hR = max(SMR + aR^2 l, eps), hL = max(aL^2 l + SML, eps)
//   (mono: hat = max(l + SM, eps))
// i.e. exactly the values the refresh pass would have stored.  That removes
// the four hat-refresh passes (6-7 streamed F x N planes each) and shrinks the
// three accompaniment refreshes to their two SMR / SML writes: ~45 plane
// passes per Stereo_SIMM iteration instead of ~79.  The column scale that
// HPHI / HGAMMA apply to HF0 (and so to SF0 = WF0 HF0) is left pending and
// applied (and written back) by the next kernel that streams SF0.
template <bool ST>
__device__ __forceinline__ void hat_of(double sf, double sp, double smr, double sml, double aR2,
                                       double aL2, double &hr, double &hl) {
  const double l = sf * sp;
  if constexpr (ST) {
    hr = fmax(smr + aR2 * l, kSimmEps);
    hl = fmax(l * aL2 + sml, kSimmEps);
  } else {
    hr = fmax(l + smr, kSimmEps);
    hl = 0.0;
  }
}

template <int KM>
__device__ __forceinline__ double sphi_of(const double *__restrict__ w, const double *h, int K) {
  double sp = 0.0;
#pragma unroll
  for (int k = 0; k < KM; ++k)
    if (k < K) sp += w[k] * h[k];
  return sp;
}

// the resident planes a consumer reads
struct SPl {
  const double *SF0, *SMR, *SML, *SXR, *SXL, *WPHI, *HPHI, *alpha;
  const double *pend;  // pending column scale of SF0 (null: none)
  double *SF0w;        // where the scaled SF0 is written back (null: not written)
  int F, N, K, fchunk;
};

// HF0 ratios, stereo (SIMM.py:623-630): com = aR2*SPHI/max(hR),
// d = aL2*SPHI/max(hL), num = com*SXR/max(hR) + d*SXL/max(hL), den = d + com;
// mono (:282-283): den = SPHI/max(hat), num = (den*SX)/max(hat).  Thread per
// frame n walking a chunk of bins (grid: N/256 x F chunks).
template <bool ST, int KM>
__global__ __launch_bounds__(256) void k_simm_numden(const SPl p, double *__restrict__ num,
                                                     double *__restrict__ den, size_t ldo) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= p.N) return;
  const int fb = blockIdx.y * p.fchunk, fe = min(p.F, fb + p.fchunk);
  double h[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) h[k] = k < p.K ? p.HPHI[(size_t)k * p.N + n] : 0.0;
  const double aR2 = ST ? p.alpha[0] * p.alpha[0] : 1.0;
  const double aL2 = ST ? p.alpha[1] * p.alpha[1] : 1.0;
#pragma unroll 2
  for (int f = fb; f < fe; ++f) {
    const size_t i = (size_t)f * p.N + n;
    const double sp = sphi_of<KM>(p.WPHI + (size_t)f * p.K, h, p.K);
    double hr, hl;
    hat_of<ST>(CLD(p.SF0[i]), sp, CLD(p.SMR[i]), ST ? CLD(p.SML[i]) : 0.0, aR2, aL2, hr, hl);
    if constexpr (ST) {
      const double com = aR2 * sp / hr;
      const double d = aL2 * sp / hl;
      SST(num[(size_t)f * ldo + n], com * CLD(p.SXR[i]) / hr + d * CLD(p.SXL[i]) / hl);
      SST(den[(size_t)f * ldo + n], d + com);
    } else {
      const double d = sp / hr;
      SST(den[(size_t)f * ldo + n], d);
      SST(num[(size_t)f * ldo + n], (d * CLD(p.SXR[i])) / hr);
    }
  }
}

// HF0 *= (num / max(den, eps))^omega with num / den the two halves of the
// rows of NP = WF0^T [num | den] (row stride 2N)
__global__ void k_mu_apply_nd(double *__restrict__ X, const double *__restrict__ NP, int R, int N,
                              double omega) {
  GRID_STRIDE(i, (size_t)R * N) {
    const size_t r = i / N, n = i % N;
    const double num = NP[r * 2 * N + n], den = NP[r * 2 * N + N + n];
    X[i] *= powo(num / fmax(den, kSimmEps), omega);
  }
}

// X *= (num / max(den, eps))^omega ; optional floor max(X, eps) (mono HM)
__global__ void k_mu_apply(double *__restrict__ X, const double *__restrict__ num,
                           const double *__restrict__ den, size_t n, double omega, int floor_eps) {
  GRID_STRIDE(i, n) {
    double x = X[i] * powo(num[i] / fmax(den[i], kSimmEps), omega);
    if (floor_eps) x = fmax(x, kSimmEps);
    X[i] = x;
  }
}

// HM (stereo, :747-758): HM *= ((nR + nL) / max(dR + dL, eps))^omega with
// nR = (WM bR^2)^T XR etc. given as unscaled products P_* = WM^T X_*.
__global__ void k_hm_apply(double *__restrict__ HM, const double *__restrict__ PnR,
                           const double *__restrict__ PdR, const double *__restrict__ PnL,
                           const double *__restrict__ PdL, const double *__restrict__ bR,
                           const double *__restrict__ bL, int R, int N, double omega) {
  GRID_STRIDE(i, (size_t)R * N) {
    const int r = i / N;
    const double br = bR[r] * bR[r], bl = bL[r] * bL[r];
    const double num = br * PnR[i] + bl * PnL[i];
    const double den = br * PdR[i] + bl * PdL[i];
    HM[i] *= powo(num / fmax(den, kSimmEps), omega);
  }
}

// hat refresh: optional SF0 column scale, optional SPHI = WPHI HPHI (K small).
// The F x N planes (328 MB each at C5, several per kernel: more than the
// 256 MB Infinity Cache) are streamed with non-temporal loads / stores (SLD /
// SST): -2.6% per Stereo_SIMM iteration (same-box A/B).
__global__ void k_simm_refresh(double *__restrict__ SF0, double *__restrict__ SPHI,
                               const double *__restrict__ WPHI, const double *__restrict__ HPHI,
                               const double *__restrict__ colscale, const double *__restrict__ SMR,
                               const double *__restrict__ SML, const double *__restrict__ alpha,
                               double *__restrict__ hR, double *__restrict__ hL, int F, int N,
                               int K, int stereo, int recompute_sphi) {
  const double aR2 = stereo ? alpha[0] * alpha[0] : 1.0;
  const double aL2 = stereo ? alpha[1] * alpha[1] : 1.0;
  GRID_STRIDE(i, (size_t)F * N) {
    const int f = i / N, n = i % N;
    double sf = SLD(SF0[i]);
    if (colscale) {
      sf *= colscale[n];
      SST(SF0[i], sf);
    }
    double sp;
    if (recompute_sphi) {
      sp = 0.0;
      for (int k = 0; k < K; ++k) sp += WPHI[f * K + k] * HPHI[(size_t)k * N + n];
      SST(SPHI[i], sp);
    } else {
      sp = SLD(SPHI[i]);
    }
    const double l = sf * sp;
    if (stereo) {
      SST(hR[i], fmax(SLD(SMR[i]) + aR2 * l, kSimmEps));
      SST(hL[i], fmax(l * aL2 + SLD(SML[i]), kSimmEps));
    } else {
      SST(hR[i], fmax(l + SLD(SMR[i]), kSimmEps));
    }
  }
}

// bins per k_simm_sm block: every block re-reads its frames' HM columns
// (R x 256 doubles), so 16-bin blocks read 1.25x the two planes they write
constexpr int kSmRows = 64;
// Accompaniment refresh (the step after every HM, WM and beta update,
// SIMM.py:747-773, :826-869, :909-941): stereo SMR = (WM bR^2) HM,
// SML = (WM bL^2) HM, mono SM = WM HM (R <= RMAX).  One thread per frame n
// keeps the HM column in registers for FB bins; the FB rows of WM (times
// beta^2) are wave-uniform.  Only the two planes are written: the hat is
// recomputed by its consumers (hat_of).
template <int RMAX>
__global__ __launch_bounds__(256) void k_simm_sm(const double *__restrict__ WbR,
                                                 const double *__restrict__ WbL,
                                                 const double *__restrict__ HM,
                                                 double *__restrict__ SMR, double *__restrict__ SML,
                                                 int F, int N, int R, int stereo) {
  constexpr int FB = kSmRows;
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int f0 = blockIdx.y * FB;
  if (n >= N) return;
  double hm[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) hm[r] = r < R ? HM[(size_t)r * N + n] : 0.0;
  for (int fl = 0; fl < FB; ++fl) {
    const int f = f0 + fl;
    if (f >= F) break;
    // the WM (x beta^2) rows, zero-padded to RMAX, are wave-uniform: scalar
    // loads and SGPR operands (the padded terms add exact zeros)
    const double *wr = WbR + (size_t)f * RMAX, *wl = WbL + (size_t)f * RMAX;
    double sr = 0.0, sl = 0.0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) sr += wr[r] * hm[r];
    const size_t i = (size_t)f * N + n;
    SST(SMR[i], sr);
    if (stereo) {
#pragma unroll
      for (int r = 0; r < RMAX; ++r) sl += wl[r] * hm[r];
      SST(SML[i], sl);
    }
  }
}

// stereo: X = SX/max(h^2, eps), Y = 1/max(h, eps)             (:747-753)
// mono:   Y = 1/max(h, eps), X = (Y*SX)/max(h, eps)               (:318-321)
__global__ void k_simm_xy(const double *__restrict__ h, const double *__restrict__ SX,
                          double *__restrict__ X, double *__restrict__ Y, size_t n, int stereo) {
  GRID_STRIDE(i, n) {
    const double hv = h[i];
    const double y = 1.0 / fmax(hv, kSimmEps);
    X[i] = stereo ? SX[i] / fmax(hv * hv, kSimmEps) : (y * SX[i]) / fmax(hv, kSimmEps);
    Y[i] = y;
  }
}

// k_simm_xy's operands for one element (both channels' formulas in one
// place) in the fused skinny products: reciprocals by v_rcp_f64 + two Newton
// steps (<= 1 ulp) instead of the IEEE division sequences (hv >= eps: it
// comes from hat_of)
__device__ __forceinline__ double simm_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}
template <bool ST>
__device__ __forceinline__ void xy_of(double hv, double sx, double &x, double &y) {
  y = simm_rcp(hv);
  x = ST ? sx * simm_rcp(fmax(hv * hv, kSimmEps)) : (y * sx) * y;
}

// Skinny accompaniment products with k_simm_xy fused into the operand loads
// (R <= 48 rows of WM / HM padded to three 16-row MFMA tiles).  Operand q of
// the NO = 2 (mono) or 4 (stereo) operands is {X_R, Y_R, X_L, Y_L}[q].
//
// k_simm_wmt_xy:  out_q[r][n] = sum_f WM[f][r] T_q[f][n]  (the HM and beta
//   numerators, SIMM.py:747-756, :911-919).  Wave = 16 frames x all R rows;
//   lane (fl, tq) streams T at (f = k0 + 4s + tq, n = n0 + fl): every load
//   instruction reads four 128-byte row segments.  Split-K over f along
//   gridDim.z into out + z*slab, [q][R][N] per slab.
//   The hat is formed in the loads (hat_of: SF0, SMR, SML, SPHI from this
//   lane's HPHI column and WPHI rows), and a pending SF0 column scale is
//   applied and written back here (every (f, n) is loaded by one lane once).
template <bool ST, int KM>
__global__ __launch_bounds__(256, 2) void k_simm_wmt_xy(const SPl p, const double *__restrict__ WM,
                                                        double *__restrict__ out, size_t slab,
                                                        int R, int kchunk) {
  constexpr int NC = ST ? 2 : 1, NO = 2 * NC;
  const int F = p.F, N = p.N, K = p.K;
  const int lane = threadIdx.x & 63, fl = lane & 15, tq = lane >> 4;
  const int n = blockIdx.x * 64 + (threadIdx.x >> 6) * 16 + fl;
  const int kb = blockIdx.z * kchunk, ke = min(F, kb + kchunk);
  const bool nin = n < N;
  const double *ss[2] = {p.SXR, p.SXL}, *sm[2] = {p.SMR, p.SML};
  double h[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) h[k] = (nin && k < K) ? p.HPHI[(size_t)k * N + n] : 0.0;
  const double cs = (nin && p.pend) ? p.pend[n] : 1.0;
  const double aR2 = ST ? p.alpha[0] * p.alpha[0] : 1.0;
  const double aL2 = ST ? p.alpha[1] * p.alpha[1] : 1.0;
  // the WPHI rows of this block's bin chunk, staged in LDS (lanes of one tq
  // read the same row: broadcast reads instead of K vector loads per point)
  extern __shared__ double sW[];
  for (int e = threadIdx.x; e < (ke - kb) * K; e += 256) sW[e] = p.WPHI[(size_t)kb * K + e];
  __syncthreads();
  d4 acc[NO][3];
#pragma unroll
  for (int q = 0; q < NO; ++q)
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[q][i] = d4{0.0, 0.0, 0.0, 0.0};
  // Every operand of a 16-bin step is loaded unconditionally, in one batch:
  // a bin past the chunk re-reads the chunk's last bin and a frame past N the
  // last frame (finite values: hat_of floors at eps), and the step's WM rows
  // are zeroed for them instead, so the MFMAs add exact zeros and columns
  // past N are never stored.  (Guarded loads compiled into one exec branch
  // per load with a full vmcnt wait before the MFMAs.)
  const int nc = min(n, N - 1);
  for (int k0 = kb; k0 < ke; k0 += 16) {
    double sfv[4], smv[NC][4], sv[NC][4], wa[4][3];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int f = min(k0 + 4 * s + tq, ke - 1);
      const size_t idx = (size_t)f * N + nc;
      sfv[s] = CLD(p.SF0[idx]);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        smv[c][s] = CLD(sm[c][idx]);
        sv[c][s] = CLD(ss[c][idx]);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) wa[s][i] = WM[(size_t)f * R + min(i * 16 + fl, R - 1)];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int f = k0 + 4 * s + tq;
      const bool fok = f < ke;
      if (p.SF0w) {   // pending column scale (HPHI's renormalisation of HF0)
        sfv[s] *= cs;
        if (nin && fok) SST(p.SF0w[(size_t)f * N + n], sfv[s]);
      }
      const double sp = sphi_of<KM>(sW + (size_t)(min(f, ke - 1) - kb) * K, h, K);
      double hv[2];
      hat_of<ST>(sfv[s], sp, smv[0][s], ST ? smv[NC - 1][s] : 0.0, aR2, aL2, hv[0], hv[1]);
      double a[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) a[i] = (fok && i * 16 + fl < R) ? wa[s][i] : 0.0;  // zero rows outside [kb, ke)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        double x, y;
        xy_of<ST>(hv[c], sv[c][s], x, y);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          acc[2 * c][i] = gmfma(a[i], x, acc[2 * c][i]);
          acc[2 * c + 1][i] = gmfma(a[i], y, acc[2 * c + 1][i]);
        }
      }
    }
  }
  if (!nin) return;
  double *o = out + blockIdx.z * slab;
#pragma unroll
  for (int q = 0; q < NO; ++q)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + tq + 4 * r;
        if (row < R) o[((size_t)q * R + row) * N + n] = acc[q][i][r];
      }
}

// k_simm_xy_hmt:  out_q[f][r] = sum_n T_q[f][n] HM[r][n]  (the WM numerators,
//   SIMM.py:828-845).  Wave = 16 frequency rows x all R columns.  The frame
//   sum is permuted within each 32-frame chunk: lane (fl, tq) owns frames
//   kc + tq + 4 j, j < 8, of row f = fl (every load instruction reads 32
//   contiguous bytes of 16 rows); HM's chunk [48][32] is shared by the
//   block's 4 waves through LDS (pitch 34: the half-wave's (fl, tq) pairs hit
//   32 distinct bank pairs).  Split-K over frames along gridDim.z, [q][F][R] per slab.
//   The hat is formed from SF0, SMR, SML and SPHI (this lane's WPHI row in
//   registers, HPHI's chunk columns staged in LDS next to HM's), and a pending
//   SF0 column scale (HGAMMA's renormalisation of HF0) is applied and written
//   back here.
// V16 (N even: 16-byte aligned frame pairs): lane (fl, tq) loads frames
//   kc + 8 j + 2 tq + h, h < 2, as one 16-byte load per plane and j < 4
//   (every load instruction reads 64 contiguous bytes of 16 rows); MFMA
//   2 j + h contracts them (k = tq).  The staged chunk columns are stored
//   interleaved, column c at (c & 1) 16 + (c >> 1), so the B reads of one
//   MFMA stay consecutive in tq (the pitch-34 rows keep them conflict-free).
// KC: frames per staged chunk (32; 16 halves the plane registers of a lane,
// 40 -> 20 doubles in the stereo form, which spilled at 32)
template <bool ST, int KM, bool V16 = false, int KC = 32>
__global__ __launch_bounds__(256, 2) void k_simm_xy_hmt(const SPl p, const double *__restrict__ HM,
                                                        double *__restrict__ out, size_t slab,
                                                        int R, int kchunk) {
  constexpr int NC = ST ? 2 : 1, NO = 2 * NC, PH = KC + 2, NJ = KC / 4;
  constexpr int NR = 48 + KM + 1;   // HM rows, HPHI rows, the pending scale
  __shared__ double sH[NR * PH];
  const int F = p.F, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63, fl = lane & 15, tq = lane >> 4;
  const int f = blockIdx.y * 64 + (tid >> 6) * 16 + fl;
  const int kb = blockIdx.z * kchunk, ke = min(N, kb + kchunk);
  const bool fin = f < F;
  const double *ss[2] = {p.SXR, p.SXL}, *sm[2] = {p.SMR, p.SML};
  double w[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) w[k] = (fin && k < K) ? p.WPHI[(size_t)f * K + k] : 0.0;
  const double aR2 = ST ? p.alpha[0] * p.alpha[0] : 1.0;
  const double aL2 = ST ? p.alpha[1] * p.alpha[1] : 1.0;
  d4 acc[NO][3];
#pragma unroll
  for (int q = 0; q < NO; ++q)
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[q][i] = d4{0.0, 0.0, 0.0, 0.0};
  // chunk column of MFMA j's k = tq, and its staged position
  auto kcol = [&](int j) { return V16 ? 8 * (j >> 1) + 2 * tq + (j & 1) : tq + 4 * j; };
  auto kpos = [&](int k) { return V16 ? (k & 1) * (KC / 2) + (k >> 1) : k; };
  // Every load of a chunk is issued unconditionally, in one batch: a row
  // past F re-reads row F - 1 and a frame past the chunk the chunk's last
  // frame (finite values: hat_of floors at eps); the staged B operand (HM's
  // chunk) is zero for those frames, so their products are exact zeros, and
  // rows past F are never stored.  (Guarded loads compiled into one exec
  // branch per load with a full vmcnt wait before the MFMAs.)
  const int fr = min(f, F - 1);
  for (int kc = kb; kc < ke; kc += KC) {
    double sfv[NJ], smv[NC][NJ], sv[NC][NJ];
    if constexpr (V16) {
      typedef double dv2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int j = 0; j < NJ / 2; ++j) {
        // (pairs never straddle ke: N, the chunk bounds and ke are even)
        const size_t b2 = (size_t)fr * N + min(kc + 8 * j + 2 * tq, ke - 2);
        const dv2 a0 = *(const dv2 *)(p.SF0 + b2);
        sfv[2 * j] = a0.x;
        sfv[2 * j + 1] = a0.y;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const dv2 a1 = *(const dv2 *)(sm[c] + b2);
          const dv2 a2 = *(const dv2 *)(ss[c] + b2);
          smv[c][2 * j] = a1.x;
          smv[c][2 * j + 1] = a1.y;
          sv[c][2 * j] = a2.x;
          sv[c][2 * j + 1] = a2.y;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        // plain (cached) loads: a lane group reads 32 bytes of a row per
        // instruction, the rest of the line arrives with the next j's
        const size_t i = (size_t)fr * N + min(kc + tq + 4 * j, ke - 1);
        sfv[j] = p.SF0[i];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          smv[c][j] = sm[c][i];
          sv[c][j] = ss[c][i];
        }
      }
    }
    double hm[(NR * KC + 255) / 256];  // chunk of HM (48 rows), HPHI (KM rows), pend
#pragma unroll
    for (int t = 0; t < (NR * KC + 255) / 256; ++t) {
      const int e = tid + 256 * t, r = min(e / KC, NR - 1), col = kc + e % KC, cc = min(col, ke - 1);
      // (a clamped, always valid address per row kind; the value selected after)
      const double *src = r < 48 ? HM + (size_t)min(r, R - 1) * N + cc
                          : r < 48 + KM ? p.HPHI + (size_t)min(r - 48, K - 1) * N + cc
                                        : (p.pend ? p.pend + cc : HM + cc);
      const double v = *src;
      const bool valid = r < 48 ? r < R : r < 48 + KM ? r - 48 < K : p.pend != nullptr;
      hm[t] = col >= ke ? 0.0 : valid ? v : (r == NR - 1 ? 1.0 : 0.0);
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < (NR * KC + 255) / 256; ++t) {
      const int e = tid + 256 * t;
      if (e < NR * KC) sH[(e / KC) * PH + kpos(e % KC)] = hm[t];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int kk = kcol(j), kq = kpos(kk);
      const bool ok = fin && kc + kk < ke;
      if (p.SF0w) {   // (plain store: the line's four 32-byte pieces merge in L2)
        sfv[j] *= sH[(NR - 1) * PH + kq];
        if (ok) p.SF0w[(size_t)f * N + kc + kk] = sfv[j];
      }
      double h[KM];
#pragma unroll
      for (int k = 0; k < KM; ++k) h[k] = sH[(48 + k) * PH + kq];
      const double sp = sphi_of<KM>(w, h, K);
      double hv[2];
      hat_of<ST>(sfv[j], sp, smv[0][j], ST ? smv[NC - 1][j] : 0.0, aR2, aL2, hv[0], hv[1]);
      double b[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) b[i] = sH[(i * 16 + fl) * PH + kq];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        double x, y;
        xy_of<ST>(hv[c], sv[c][j], x, y);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          acc[2 * c][i] = gmfma(x, b[i], acc[2 * c][i]);
          acc[2 * c + 1][i] = gmfma(y, b[i], acc[2 * c + 1][i]);
        }
      }
    }
  }
  double *o = out + blockIdx.z * slab;
#pragma unroll
  for (int q = 0; q < NO; ++q)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = blockIdx.y * 64 + (tid >> 6) * 16 + tq + 4 * r;
        const int col = i * 16 + fl;
        if (row < F && col < R) o[((size_t)q * F + row) * R + col] = acc[q][i][r];
      }
}

// HPHI numerator/denominator: out[m][n] = sum_f WPHI[f][m] * {num,den}(f, n),
// num/den built on the fly from Z = SF0 and the hat (hat_of) (:688-694).
// Block: 256 frames x one f-chunk; partials [chunk][2][K][N].
template <bool ST, int KM>
__global__ __launch_bounds__(256) void k_hphi_partial(const SPl p, double *__restrict__ part) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y, K = p.K, N = p.N;
  const int fb = c * p.fchunk, fe = min(p.F, fb + p.fchunk);
  if (n >= N) return;
  double sn[KM], sd[KM], h[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    sn[k] = sd[k] = 0.0;
    h[k] = k < K ? p.HPHI[(size_t)k * N + n] : 0.0;
  }
  const double aR2 = ST ? p.alpha[0] * p.alpha[0] : 1.0;
  const double aL2 = ST ? p.alpha[1] * p.alpha[1] : 1.0;
  for (int f = fb; f < fe; ++f) {
    const size_t i = (size_t)f * N + n;
    const double *w = p.WPHI + (size_t)f * K;
    const double z = CLD(p.SF0[i]);
    double mr, ml;
    hat_of<ST>(z, sphi_of<KM>(w, h, K), CLD(p.SMR[i]), ST ? CLD(p.SML[i]) : 0.0, aR2, aL2, mr, ml);
    double num, den;
    if constexpr (ST) {
      const double com = aR2 * z / mr;
      const double d = aL2 * z / ml;
      num = com * CLD(p.SXR[i]);
      num /= mr;
      num += d * CLD(p.SXL[i]) / ml;
      den = d + com;
    } else {
      den = z / mr;
      num = (den * CLD(p.SXR[i])) / mr;
    }
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < K) {
        sn[k] += w[k] * num;
        sd[k] += w[k] * den;
      }
  }
#pragma unroll
  for (int k = 0; k < KM; ++k)
    if (k < K) {
      part[(((size_t)c * 2 + 0) * K + k) * N + n] = sn[k];
      part[(((size_t)c * 2 + 1) * K + k) * N + n] = sd[k];
    }
}

// HPHI *= (num/max(den,eps))^omega; s = column sums; HPHI[:, s>0] /= s
__global__ void k_hphi_update(double *__restrict__ HPHI, const double *__restrict__ part,
                              int nchunk, double *__restrict__ s_out, int K, int N,
                              double omega) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int k = 0; k < K; ++k) {
    double num = 0.0, den = 0.0;
    for (int c = 0; c < nchunk; ++c) {
      num += part[(((size_t)c * 2 + 0) * K + k) * N + n];
      den += part[(((size_t)c * 2 + 1) * K + k) * N + n];
    }
    double h = HPHI[(size_t)k * N + n] * powo(num / fmax(den, kSimmEps), omega);
    HPHI[(size_t)k * N + n] = h;
    s += h;
  }
  if (s > 0)
    for (int k = 0; k < K; ++k) HPHI[(size_t)k * N + n] /= s;
  s_out[n] = s;
}

// X[r][n] *= s[n] over R rows (column scale)
__global__ void k_colscale(double *__restrict__ X, const double *__restrict__ s, int R, int N) {
  GRID_STRIDE(i, (size_t)R * N) X[i] *= s[i % N];
}

// HGAMMA numerator/denominator rows: out[f][k] = sum_n {num,den}(f, n) HPHI[k][n]
// (np.dot(tempNumFbyN, HPHI.T), :802), the hat formed on the fly (hat_of);
// one block per FB bins and frame chunk (gridDim.y chunks: partial rows
// [chunk][F][2K], summed in chunk order by k_hgamma_numden).
template <bool ST, int KM>
__global__ __launch_bounds__(256) void k_hgamma_rows(const SPl p, double *__restrict__ out) {
  constexpr int FB = kHgRows;  // frequency rows per block: each HPHI load serves FB rows
  __shared__ double s_red[FB * 2 * KM][4];
  const int F = p.F, N = p.N, K = p.K;
  const int f0 = blockIdx.x * FB, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double sn[FB][KM], sd[FB][KM];
#pragma unroll
  for (int r = 0; r < FB; ++r)
#pragma unroll
    for (int k = 0; k < KM; ++k) sn[r][k] = sd[r][k] = 0.0;
  const double aR2 = ST ? p.alpha[0] * p.alpha[0] : 1.0;
  const double aL2 = ST ? p.alpha[1] * p.alpha[1] : 1.0;
  const int nb = blockIdx.y * ((N + gridDim.y - 1) / gridDim.y);
  const int ne = min(N, nb + (N + gridDim.y - 1) / gridDim.y);
  for (int n = nb + threadIdx.x; n < ne; n += 256) {
    double h[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) h[k] = k < K ? p.HPHI[(size_t)k * N + n] : 0.0;
#pragma unroll
    for (int r = 0; r < FB; ++r) {
      if (f0 + r >= F) break;
      const size_t i = (size_t)(f0 + r) * N + n;
      const double z = CLD(p.SF0[i]);
      double mr, ml;
      hat_of<ST>(z, sphi_of<KM>(p.WPHI + (size_t)(f0 + r) * K, h, K), CLD(p.SMR[i]),
                 ST ? CLD(p.SML[i]) : 0.0, aR2, aL2, mr, ml);
      double num, den;
      if constexpr (ST) {
        const double com = aR2 * z / mr;
        const double d = aL2 * z / ml;
        num = com * CLD(p.SXR[i]);
        num /= mr;
        num += d * CLD(p.SXL[i]) / ml;
        den = d + com;
      } else {
        den = z / mr;
        num = (den * CLD(p.SXR[i])) / mr;
      }
#pragma unroll
      for (int k = 0; k < KM; ++k) {  // fixed trip count: sn / sd stay in registers
        sn[r][k] += num * h[k];
        sd[r][k] += den * h[k];
      }
    }
  }
  // wave butterflies, then the 4 waves' partials in fixed order
#pragma unroll
  for (int r = 0; r < FB; ++r)
#pragma unroll
    for (int q = 0; q < 2 * KM; ++q) {
      if (q % KM >= K) continue;
      double v = q < KM ? sn[r][q] : sd[r][q - KM];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) s_red[r * 2 * KM + q][wv] = v;
    }
  __syncthreads();
  for (int t = threadIdx.x; t < FB * 2 * K; t += 256) {
    const int r = t / (2 * K), q = t % (2 * K);
    const int slot = r * 2 * KM + (q < K ? q : KM + q - K);
    if (f0 + r < F)
      out[((size_t)blockIdx.y * F + f0 + r) * 2 * K + q] =
          (s_red[slot][0] + s_red[slot][1]) + (s_red[slot][2] + s_red[slot][3]);
  }
}

// HGAMMA update + renormalisations (:802-812 / :335-343) in three steps:
// k_hgamma_numden (one block per filter-basis row p) reduces
//   numH[p][k] = sum_f WGAMMA[f][p] rows[f][k], denH likewise over f;
// k_hgamma_norm: HGAMMA *= (numH / max(denH, eps))^omega, column-normalise
//   (sumHGAMMA -> sg, the HPHI row scale);
// k_wphi: WPHI = WGAMMA HGAMMA.
__global__ __launch_bounds__(256) void k_hgamma_numden(const double *__restrict__ WGAMMA,
                                                       const double *__restrict__ rows,
                                                       double *__restrict__ nd, int F, int P,
                                                       int K, int nrc) {
  __shared__ double s_red[16][8];
  const int p = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0;
  for (int f = threadIdx.x; f < F; f += 256) {
    const double w = WGAMMA[(size_t)f * P + p];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q < 2 * K) {
        double r = rows[(size_t)f * 2 * K + q];
        for (int c = 1; c < nrc; ++c) r += rows[((size_t)c * F + f) * 2 * K + q];
        acc[q] += w * r;
      }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    double v = acc[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_red[q][wv] = v;
  }
  __syncthreads();
  if (threadIdx.x < 2 * K) {
    const int q = threadIdx.x;
    nd[p * 2 * K + q] = (s_red[q][0] + s_red[q][1]) + (s_red[q][2] + s_red[q][3]);
  }
}

__global__ void k_hgamma_norm(double *__restrict__ HGAMMA, const double *__restrict__ nd,
                              double *__restrict__ sg, int P, int K, double omega) {
  const int k = threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int p = 0; p < P; ++p) {
    const double v =
        HGAMMA[p * K + k] * powo(nd[p * 2 * K + k] / fmax(nd[p * 2 * K + K + k], kSimmEps), omega);
    HGAMMA[p * K + k] = v;
    s += v;
  }
  sg[k] = s;
  if (s > 0)
    for (int p = 0; p < P; ++p) HGAMMA[p * K + k] /= s;
}

__global__ void k_wphi(const double *__restrict__ WGAMMA, const double *__restrict__ HGAMMA,
                       double *__restrict__ WPHI, int F, int P, int K) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= F * K) return;
  const int f = idx / K, k = idx % K;
  double w = 0.0;
  for (int p = 0; p < P; ++p) w += WGAMMA[(size_t)f * P + p] * HGAMMA[p * K + k];
  WPHI[idx] = w;
}

// HPHI *= outer(sg, ones); s = column sums; HPHI[:, s>0] /= s  (:808-811)
__global__ void k_hphi_rescale(double *__restrict__ HPHI, const double *__restrict__ sg,
                               double *__restrict__ s_out, int K, int N) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int k = 0; k < K; ++k) {
    const double h = HPHI[(size_t)k * N + n] * sg[k];
    HPHI[(size_t)k * N + n] = h;
    s += h;
  }
  if (s > 0)
    for (int k = 0; k < K; ++k) HPHI[(size_t)k * N + n] /= s;
  s_out[n] = s;
}

// WM update (stereo :844-853, mono :377-385) then column normalisation; one
// block per accompaniment column r.  P_* = X_* HM^T (unscaled products).
__global__ __launch_bounds__(256) void k_wm_update(double *__restrict__ WM,
                                                   const double *__restrict__ PnR,
                                                   const double *__restrict__ PdR,
                                                   const double *__restrict__ PnL,
                                                   const double *__restrict__ PdL,
                                                   const double *__restrict__ bR,
                                                   const double *__restrict__ bL,
                                                   double *__restrict__ sw, int F, int R,
                                                   double omega, int stereo) {
  __shared__ double s_red[256];
  const int r = blockIdx.x;
  double part = 0.0;
  const double br = stereo ? bR[r] * bR[r] : 1.0, bl = stereo ? bL[r] * bL[r] : 0.0;
  for (int f = threadIdx.x; f < F; f += 256) {
    const size_t i = (size_t)f * R + r;
    double ratio;
    if (stereo)
      ratio = (PnR[i] * br + PnL[i] * bl) / (PdR[i] * br + PdL[i] * bl);   // no eps floor (:844)
    else
      ratio = PnR[i] / fmax(PdR[i], kSimmEps);
    const double w = WM[i] * powo(ratio, omega);
    WM[i] = w;
    part += w;
  }
  s_red[threadIdx.x] = part;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
    __syncthreads();
  }
  const double s = s_red[0];
  if (s > 0)
    for (int f = threadIdx.x; f < F; f += 256) WM[(size_t)f * R + r] /= s;
  if (threadIdx.x == 0) sw[r] = s;
}

// HM *= vstack(sumWM) (stereo, :855) ; mono N7 quirk handled on the host
__global__ void k_rowscale(double *__restrict__ X, const double *__restrict__ s, int R, int N) {
  GRID_STRIDE(i, (size_t)R * N) X[i] *= s[i / N];
}

// WMb = WM * beta^2 (column scale), F x R
// W[f][r] (r < R) = WM[f][r] (* b[r]^2 when b), zero for R <= r < RP
__global__ void k_wm_beta_pad(const double *__restrict__ WM, const double *__restrict__ b,
                              double *__restrict__ W, int F, int R, int RP) {
  GRID_STRIDE(i, (size_t)F * RP) {
    const int f = i / RP, r = i % RP;
    double w = 0.0;
    if (r < R) {
      w = WM[(size_t)f * R + r];
      if (b) {
        const double bb = b[r];
        w = w * (bb * bb);
      }
    }
    W[i] = w;
  }
}

__global__ void k_wm_beta(const double *__restrict__ WM, const double *__restrict__ b,
                          double *__restrict__ WMb, int F, int R) {
  GRID_STRIDE(i, (size_t)F * R) {
    const double bb = b[i % R];
    WMb[i] = WM[i] * (bb * bb);
  }
}

// alpha sums (:875-885): [sum numR, sum denR, sum numL, sum denL] partials,
// one per block of the (N/256 x F chunks) walker grid, the hat on the fly
template <int KM>
__global__ __launch_bounds__(256) void k_alpha_partial(const SPl p, double *__restrict__ part) {
  __shared__ double s_red[4][256];
  const int n = blockIdx.x * 256 + threadIdx.x, N = p.N, K = p.K;
  const int fb = blockIdx.y * p.fchunk, fe = min(p.F, fb + p.fchunk);
  double a[4] = {0, 0, 0, 0};
  if (n < N) {
    double h[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) h[k] = k < K ? p.HPHI[(size_t)k * N + n] : 0.0;
    const double aR2 = p.alpha[0] * p.alpha[0], aL2 = p.alpha[1] * p.alpha[1];
    for (int f = fb; f < fe; ++f) {
      const size_t i = (size_t)f * N + n;
      const double sp = sphi_of<KM>(p.WPHI + (size_t)f * K, h, K);
      const double sf = CLD(p.SF0[i]);
      double mr, ml;
      hat_of<true>(sf, sp, CLD(p.SMR[i]), CLD(p.SML[i]), aR2, aL2, mr, ml);
      const double l = sf * sp;
      const double dR = l / mr, dL = l / ml;
      a[0] += dR * CLD(p.SXR[i]) / mr;
      a[1] += dR;
      a[2] += dL * CLD(p.SXL[i]) / ml;
      a[3] += dL;
    }
  }
  for (int q = 0; q < 4; ++q) s_red[q][threadIdx.x] = a[q];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int q = 0; q < 4; ++q) s_red[q][threadIdx.x] += s_red[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 4)
    part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + threadIdx.x] = s_red[threadIdx.x][0];
}

__global__ void k_alpha_update(const double *__restrict__ part, int nb, double *__restrict__ alpha,
                               double omega) {
  // one wave: lane-strided partial sums, then a fixed butterfly (deterministic)
  const int lane = threadIdx.x;
  double s[4] = {0, 0, 0, 0};
  for (int b = lane; b < nb; b += 64)
    for (int q = 0; q < 4; ++q) s[q] += part[(size_t)b * 4 + q];
  for (int q = 0; q < 4; ++q)
    for (int o = 32; o > 0; o >>= 1) s[q] += __shfl_xor(s[q], o, 64);
  if (lane != 0) return;
  double aR = fmax(alpha[0] * pow(s[0] / s[1], omega * .1), kSimmEps);
  double aL = fmax(alpha[1] * pow(s[2] / s[3], omega * .1), kSimmEps);
  aR = aR / fmax(aR + aL, .001);
  alpha[0] = aR;
  alpha[1] = 1 - aR;
}

// out_q[r] = sum_n T_q[r][n] HM[r][n] (diag of (WM^T X) HM^T, :910-918) for
// the four beta operands q = blockIdx.y; block per (r, q)
struct RowdotArgs {
  const double *T[4];
};
__global__ __launch_bounds__(256) void k_rowdot(const RowdotArgs ta, const double *__restrict__ HM,
                                                double *__restrict__ outq, int N) {
  __shared__ double s_red[256];
  const int r = blockIdx.x;
  const double *__restrict__ T = ta.T[blockIdx.y];
  double *__restrict__ out = outq + (size_t)blockIdx.y * gridDim.x;
  double a = 0.0;
  for (int n = threadIdx.x; n < N; n += 256) a += T[(size_t)r * N + n] * HM[(size_t)r * N + n];
  s_red[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[r] = s_red[0];
}

// beta update (:909-921): d[0..R) numR, [R..2R) denR, [2R..3R) numL, [3R..4R) denL
__global__ void k_beta_update(const double *__restrict__ d, double *__restrict__ bR,
                              double *__restrict__ bL, int R, double omega) {
  const int r = threadIdx.x;
  if (r >= R) return;
  double br = bR[r] * pow(d[r] / d[R + r], omega * .1);
  double bl = bL[r] * pow(d[2 * R + r] / d[3 * R + r], omega * .1);
  br = br / fmax(br + bl, kSimmEps);
  bR[r] = br;
  bL[r] = 1 - br;
}

// Itakura-Saito divergence partials (ISDistortion, SIMM.py:34-44) of
// SXR vs hR (+ SXL vs hL): sum(-log(r) + r - 1), r = SX/hat; the hat on the
// fly, with a pending SF0 column scale applied (not written back)
template <bool ST, int KM>
__global__ __launch_bounds__(256) void k_is_partial(const SPl p, double *__restrict__ part) {
  __shared__ double s_red[256];
  const int n = blockIdx.x * 256 + threadIdx.x, N = p.N, K = p.K;
  const int fb = blockIdx.y * p.fchunk, fe = min(p.F, fb + p.fchunk);
  double a = 0.0;
  if (n < N) {
    double h[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) h[k] = k < K ? p.HPHI[(size_t)k * N + n] : 0.0;
    const double cs = p.pend ? p.pend[n] : 1.0;
    const double aR2 = ST ? p.alpha[0] * p.alpha[0] : 1.0;
    const double aL2 = ST ? p.alpha[1] * p.alpha[1] : 1.0;
    for (int f = fb; f < fe; ++f) {
      const size_t i = (size_t)f * N + n;
      double sf = CLD(p.SF0[i]);
      if (p.pend) sf *= cs;
      double hr, hl;
      hat_of<ST>(sf, sphi_of<KM>(p.WPHI + (size_t)f * K, h, K), CLD(p.SMR[i]),
                 ST ? CLD(p.SML[i]) : 0.0, aR2, aL2, hr, hl);
      double r = CLD(p.SXR[i]) / hr;
      a += (-log(r) + r) - 1;
      if constexpr (ST) {
        r = CLD(p.SXL[i]) / hl;
        a += (-log(r) + r) - 1;
      }
    }
  }
  s_red[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)blockIdx.y * gridDim.x + blockIdx.x] = s_red[0];
}

__global__ void k_is_final(const double *__restrict__ part, int nb, double *__restrict__ out) {
  const int lane = threadIdx.x;  // one wave, as k_alpha_update
  double s = 0.0;
  for (int b = lane; b < nb; b += 64) s += part[b];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) *out = s;
}

// writeSeparatedSignals masks (SeparateLeadStereoTF.py:1785-1846), eps 1e-9:
//   hat = max(a^2 SF0 SPHI + WM b^2 HM, eps); lead = a^2 SPHI SF0 / hat X;
//   accompaniment = (WM b^2 HM) / hat X      (per channel)
__global__ void k_lead_masks(const double *__restrict__ SF0, const double *__restrict__ SPHI,
                             const double *__restrict__ SMR, const double *__restrict__ SML,
                             const double *__restrict__ alpha, const double2 *__restrict__ XR,
                             const double2 *__restrict__ XL, double2 *__restrict__ VR,
                             double2 *__restrict__ VL, double2 *__restrict__ MR,
                             double2 *__restrict__ ML, size_t n) {
  const double aR2 = alpha[0] * alpha[0], aL2 = alpha[1] * alpha[1];
  GRID_STRIDE(i, n) {
    const double sf = SF0[i], sp = SPHI[i];
    const double hr = fmax(aR2 * sf * sp + SMR[i], 1e-9);
    const double hl = fmax(aL2 * sf * sp + SML[i], 1e-9);
    const double vr = aR2 * sp * sf / hr, vl = aL2 * sp * sf / hl;
    const double mr = SMR[i] / hr, ml = SML[i] / hl;
    const double2 xr = XR[i], xl = XL[i];
    VR[i] = make_double2(vr * xr.x, vr * xr.y);
    VL[i] = make_double2(vl * xl.x, vl * xl.y);
    MR[i] = make_double2(mr * xr.x, mr * xr.y);
    ML[i] = make_double2(ml * xl.x, ml * xl.y);
  }
}

// out[c][r] = in[r][c] (R x C, row pitches ldi / ldo) through a 16 x 16 LDS tile
__global__ __launch_bounds__(256) void k_simm_transpose(const double *__restrict__ in,
                                                        double *__restrict__ out, int R, int C,
                                                        int ldi, int ldo) {
  __shared__ double t[16][17];
  const int c0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  if (r0 + ty < R && c0 + tx < C) t[ty][tx] = in[(size_t)(r0 + ty) * ldi + c0 + tx];
  __syncthreads();
  if (c0 + ty < C && r0 + tx < R) out[(size_t)(c0 + ty) * ldo + r0 + tx] = t[tx][ty];
}

}  // namespace fasst

using namespace fasst;

// ============================================================================ context
struct simm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // NF0-sized plain products (FASST_SIMM_GEMM): 0 = k_dgemm2 (default,
  // fasst_dgemm2.h), 2 = the generic k_gemm (A/B and parity reference);
  // both parity-tested against the oracle
  int gemm_kind = 0;
  int Fp = 0, NF0p = 0;   // even (16-byte) row pitches of the WF0 copies below
  int F = 0, N = 0, NF0 = 0, P = 0, K = 0, R = 0, stereo = 1;
  int nchunk_h = 1, fchunk_h = 1, nb_alpha = 1;
  int nchunk_w = 1, fchunk_w = 1;  // the frame-walker grid (N/256 x bin chunks)
  // SF0's pending column scale (s_col after HPHI / HGAMMA), applied by the
  // next kernel that streams SF0; SPHI / hR / hL hold the model only after
  // refresh_hat (rebuild_model, the R > 48 path)
  const double *pend = nullptr;
  long slots = 512;   // resident blocks of the skinny products (2 per CU)
  // WF0 [F][NF0] as given (k_gemm), WF0K [F][NF0p] and WF0T [NF0][Fp]: the
  // k-major operands of WF0^T [num | den] and of SF0 = WF0 HF0 on k_dgemm2
  DBuf<double> SXR, SXL, WF0, WF0K, WF0T, WGAMMA, HGAMMA, HPHI, HF0, HM, WM, bR, bL, alpha;
  DBuf<double> WPHI, SF0, SPHI, hR, hL, SMR, SML, T0, T1, T2, T3, TND, NPD, WMb, WMb2, s_col, sg, sw;
  DBuf<double> hpart, hrows, apart, bd, gwork, P0, P1, P2, P3, RN0, RN1, reco;
};

namespace {

// NF0-sized products dispatched per kernel since the library was loaded
// (simm_nf0_product_counts): which path a run took is observable
std::atomic<long> g_nf0_dgemm2{0}, g_nf0_kgemm{0};

int gemm_nn(simm_ctx *c, const double *A, int lda, const double *B, int ldb, double *C, int ldc,
            int M, int N, int K) {
  const double *Bs[1] = {B};
  double *Cs[1] = {C};
  return gemm<false, false, 1>(c->stream, A, lda, Bs, ldb, Cs, ldc, M, N, K, c->gwork.p);
}

// SF0 = WF0 HF0 (F x NF0)(NF0 x N)
int sf0_gemm(simm_ctx *c) {
  if (c->gemm_kind == 0) {
    ++g_nf0_dgemm2;
    return dgemm2(c->stream, c->F, c->N, c->NF0, c->WF0T.p, c->Fp, c->HF0.p, c->N, c->SF0.p, c->N);
  }
  ++g_nf0_kgemm;
  return gemm_nn(c, c->WF0.p, c->NF0, c->HF0.p, c->N, c->SF0.p, c->N, c->F, c->N, c->NF0);
}

constexpr int kWmtMaxChunk = 512;   // bins per k_simm_wmt_xy block (its LDS WPHI rows)
// split of the fused skinny products (k_simm_wmt_xy / k_simm_xy_hmt): a
// grid of >= 1024 (resp. 512) blocks, K chunks of >= 64 (256) rows
struct SkinnySplit {
  int nz, kchunk;
};
// split count for `units` blocks per split when `slots` blocks (two per CU)
// are resident: the smallest nz in [lo, hi] whose last round is >= 95% full,
// else the fullest (C5: k_simm_xy_hmt 33 x 15 blocks, one round instead of
// 33 x 16 with a 16-block tail; k_simm_wmt_xy 313 x 8: 8.70 -> 8.60 ms)
static int round_split(long units, int lo, int hi, long slots) {
  hi = std::max(lo, hi);
  int best = lo;
  double beff = 0.0;
  for (int nz = lo; nz <= hi; ++nz) {
    const long b = units * nz, rounds = (b + slots - 1) / slots;
    const double eff = (double)b / (double)(rounds * slots);
    if (eff >= 0.95) return nz;
    if (eff > beff) {
      beff = eff;
      best = nz;
    }
  }
  return best;
}
static SkinnySplit wmt_split(int F, int N, long slots) {
  const long bx = (N + 63) / 64;
  // >= 4 blocks per slot ring, chunks of >= 64 bins, WPHI rows in the LDS
  const int lo = std::max(std::max(1, (F + kWmtMaxChunk - 1) / kWmtMaxChunk),
                          (int)std::min<long>(16, (2 * slots + bx - 1) / bx));
  int nz = round_split(bx, lo, std::max(lo, std::min(16, F / 64)), slots);
  nz = std::max(nz, (F + kWmtMaxChunk - 1) / kWmtMaxChunk);
  const int kchunk = ((F + nz - 1) / nz + 15) / 16 * 16;
  return {(F + kchunk - 1) / kchunk, kchunk};
}
static SkinnySplit hmt_split(int F, int N, long slots) {
  const long by = (F + 63) / 64;
  const int hi = std::max(1, std::min(32, N / 256));
  const int nz = round_split(by, std::min(hi, (int)std::max<long>(1, slots / (2 * by))), hi, slots);
  const int kchunk = ((N + nz - 1) / nz + 31) / 32 * 32;
  return {(N + kchunk - 1) / kchunk, kchunk};
}
static size_t skinny_workspace(int F, int N, int R, int stereo, long slots) {
  if (R > 48) return 0;
  const size_t no = stereo ? 4 : 2;
  return std::max((size_t)wmt_split(F, N, slots).nz * no * R * N,
                  (size_t)hmt_split(F, N, slots).nz * no * F * R);
}

// the no outputs' split-K slabs ([z][q][n]) summed in z order, one launch
// (grid.y = q) instead of one per output
struct SlabDst {
  double *d[4];
};
__global__ void k_slab_reduce(const double *__restrict__ part, int nz, size_t zstride, SlabDst dst,
                              size_t n) {
  const double *pq = part + blockIdx.y * n;
  double *out = dst.d[blockIdx.y];
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int z = 0; z < nz; ++z) s += pq[z * zstride + i];
    out[i] = s;
  }
}
void reduce_slabs(simm_ctx *c, int no, int nz, size_t n, double *const *dst) {
  SlabDst d;
  for (int q = 0; q < 4; ++q) d.d[q] = q < no ? dst[q] : nullptr;
  k_slab_reduce<<<dim3((int)std::min<size_t>((n + 255) / 256, 4096), no), 256, 0, c->stream>>>(
      c->gwork.p, nz, (size_t)no * n, d, n);
}

// K <= 4 filters (the documented configurations) or <= 8: the per-lane
// SPHI / HPHI arrays and the HGAMMA accumulators are sized by the bound
template <class L>
void kdispatch(int K, L &&launch) {
  if (K <= 4)
    launch(std::integral_constant<int, 4>{});
  else
    launch(std::integral_constant<int, 8>{});
}

// the resident planes as the consumers read them; `apply` = the kernel
// streams every point of SF0 once and writes the pending column scale back
SPl planes(const simm_ctx *c, bool apply) {
  SPl p;
  p.SF0 = c->SF0.p;
  p.SMR = c->SMR.p;
  p.SML = c->SML.p;
  p.SXR = c->SXR.p;
  p.SXL = c->SXL.p;
  p.WPHI = c->WPHI.p;
  p.HPHI = c->HPHI.p;
  p.alpha = c->alpha.p;
  p.pend = c->pend;
  p.SF0w = (apply && c->pend) ? c->SF0.p : nullptr;
  p.F = c->F;
  p.N = c->N;
  p.K = c->K;
  p.fchunk = c->fchunk_w;
  return p;
}

dim3 walker_grid(const simm_ctx *c) { return dim3((c->N + 255) / 256, c->nchunk_w); }

int refresh_hat(simm_ctx *c, const double *colscale, int recompute_sphi);

// the model spectrograms as planes (SPHI, hR, hL) for the paths that read
// them (R > 48 products), consuming the pending SF0 scale
int materialise_hat(simm_ctx *c) {
  const int st = refresh_hat(c, c->pend, 1);
  c->pend = nullptr;
  return st;
}

// dst[q] (R x N) = WM^T {X_R, Y_R, X_L, Y_L}[q] from the current model
int wmt_xy(simm_ctx *c, double *const *dst) {
  const int F = c->F, N = c->N, R = c->R, no = c->stereo ? 4 : 2;
  if (R > 48) {  // wide accompaniment dictionaries: materialise X, Y, general GEMM
    int st = materialise_hat(c);
    if (st) return st;
    k_simm_xy<<<egrid((size_t)F * N), 256, 0, c->stream>>>(c->hR.p, c->SXR.p, c->T0.p, c->T1.p,
                                                           (size_t)F * N, c->stereo);
    if (c->stereo)
      k_simm_xy<<<egrid((size_t)F * N), 256, 0, c->stream>>>(c->hL.p, c->SXL.p, c->T2.p, c->T3.p,
                                                             (size_t)F * N, c->stereo);
    const double *Bs[4] = {c->T0.p, c->T1.p, c->T2.p, c->T3.p};
    return c->stereo ? gemm<true, false, 4>(c->stream, c->WM.p, R, Bs, N, dst, N, R, N, F, c->gwork.p)
                     : gemm<true, false, 2>(c->stream, c->WM.p, R, Bs, N, dst, N, R, N, F, c->gwork.p);
  }
  const SkinnySplit sp = wmt_split(F, N, c->slots);
  const size_t slab = (size_t)no * R * N;
  dim3 grid((N + 63) / 64, 1, sp.nz);
  const SPl p = planes(c, true);
  const size_t lds = (size_t)sp.kchunk * c->K * sizeof(double);
  kdispatch(c->K, [&](auto km) {
    constexpr int KM = decltype(km)::value;
    if (c->stereo)
      k_simm_wmt_xy<true, KM><<<grid, 256, lds, c->stream>>>(p, c->WM.p, c->gwork.p, slab, R, sp.kchunk);
    else
      k_simm_wmt_xy<false, KM><<<grid, 256, lds, c->stream>>>(p, c->WM.p, c->gwork.p, slab, R, sp.kchunk);
  });
  FASST_LAUNCH_CHECK();
  c->pend = nullptr;
  reduce_slabs(c, no, sp.nz, (size_t)R * N, dst);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

// dst[q] (F x R) = {X_R, Y_R, X_L, Y_L}[q] HM^T from the current model
int xy_hmt(simm_ctx *c, double *const *dst) {
  const int F = c->F, N = c->N, R = c->R, no = c->stereo ? 4 : 2;
  if (R > 48) {
    int st = materialise_hat(c);
    if (st) return st;
    k_simm_xy<<<egrid((size_t)F * N), 256, 0, c->stream>>>(c->hR.p, c->SXR.p, c->T0.p, c->T1.p,
                                                           (size_t)F * N, c->stereo);
    if (c->stereo)
      k_simm_xy<<<egrid((size_t)F * N), 256, 0, c->stream>>>(c->hL.p, c->SXL.p, c->T2.p, c->T3.p,
                                                             (size_t)F * N, c->stereo);
    const double *srcs[4] = {c->T0.p, c->T1.p, c->T2.p, c->T3.p};
    for (int q = 0; q < no; ++q) {  // X HM^T : (F x N)(N x R)
      const double *Bs[1] = {c->HM.p};
      double *Cs[1] = {dst[q]};
      st = gemm<false, true, 1>(c->stream, srcs[q], N, Bs, N, Cs, R, F, R, N, c->gwork.p);
      if (st) return st;
    }
    return FASST_OK;
  }
  const SkinnySplit sp = hmt_split(F, N, c->slots);
  const size_t slab = (size_t)no * F * R;
  dim3 grid(1, (F + 63) / 64, sp.nz);
  const SPl p = planes(c, true);
  // 16-byte frame pairs: even N (rows 16-byte aligned) and even chunks
  // (the stereo SIMM iteration 8.80 -> 8.61 ms against 8-byte frames)
  const bool v16 = N % 2 == 0 && sp.kchunk % 2 == 0;
  kdispatch(c->K, [&](auto km) {
    constexpr int KM = decltype(km)::value;
    if (c->stereo)
      if (v16)   // (16-frame chunks: the 32-frame form spilled, 0.672 -> 0.646 ms at C5)
        k_simm_xy_hmt<true, KM, true, 16><<<grid, 256, 0, c->stream>>>(p, c->HM.p, c->gwork.p, slab, R, sp.kchunk);
      else
        k_simm_xy_hmt<true, KM><<<grid, 256, 0, c->stream>>>(p, c->HM.p, c->gwork.p, slab, R, sp.kchunk);
    else
      if (v16)
        k_simm_xy_hmt<false, KM, true><<<grid, 256, 0, c->stream>>>(p, c->HM.p, c->gwork.p, slab, R, sp.kchunk);
      else
        k_simm_xy_hmt<false, KM><<<grid, 256, 0, c->stream>>>(p, c->HM.p, c->gwork.p, slab, R, sp.kchunk);
  });
  FASST_LAUNCH_CHECK();
  c->pend = nullptr;
  reduce_slabs(c, no, sp.nz, (size_t)F * R, dst);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

// SMR = (WM bR^2) HM, SML = (WM bL^2) HM  (stereo); SM = WM HM (mono)
int refresh_sm_gemm(simm_ctx *c) {
  if (c->stereo) {
    k_wm_beta<<<egrid((size_t)c->F * c->R), 256, 0, c->stream>>>(c->WM.p, c->bR.p, c->WMb.p, c->F, c->R);
    int st = gemm_nn(c, c->WMb.p, c->R, c->HM.p, c->N, c->SMR.p, c->N, c->F, c->N, c->R);
    if (st) return st;
    k_wm_beta<<<egrid((size_t)c->F * c->R), 256, 0, c->stream>>>(c->WM.p, c->bL.p, c->WMb.p, c->F, c->R);
    return gemm_nn(c, c->WMb.p, c->R, c->HM.p, c->N, c->SML.p, c->N, c->F, c->N, c->R);
  }
  return gemm_nn(c, c->WM.p, c->R, c->HM.p, c->N, c->SMR.p, c->N, c->F, c->N, c->R);
}

// the accompaniment planes after an HM / WM / beta update (the hat itself is
// recomputed by its consumers)
constexpr int kSmRmax = 48;
int refresh_sm(simm_ctx *c) {
  if (c->R > kSmRmax) return refresh_sm_gemm(c);
  // WM (x beta^2) rows zero-padded to RP = R rounded up to 8 (the unrolled
  // FMA count per point)
  const int RP = (c->R + 7) / 8 * 8;
  const size_t FRP = (size_t)c->F * RP;
  k_wm_beta_pad<<<egrid(FRP), 256, 0, c->stream>>>(c->WM.p, c->stereo ? c->bR.p : nullptr,
                                                   c->WMb.p, c->F, c->R, RP);
  if (c->stereo)
    k_wm_beta_pad<<<egrid(FRP), 256, 0, c->stream>>>(c->WM.p, c->bL.p, c->WMb2.p, c->F, c->R, RP);
  const dim3 grid((c->N + 255) / 256, (c->F + kSmRows - 1) / kSmRows);
#define SM_CASE(RM)                                                                           \
  case RM:                                                                                    \
    k_simm_sm<RM><<<grid, 256, 0, c->stream>>>(c->WMb.p, c->WMb2.p, c->HM.p, c->SMR.p, c->SML.p, \
                                               c->F, c->N, c->R, c->stereo);                  \
    break;
  switch (RP) {
    SM_CASE(8) SM_CASE(16) SM_CASE(24) SM_CASE(32) SM_CASE(40) SM_CASE(48)
  }
#undef SM_CASE
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int refresh_hat(simm_ctx *c, const double *colscale, int recompute_sphi) {
  k_simm_refresh<<<egrid((size_t)c->F * c->N), 256, 0, c->stream>>>(
      c->SF0.p, c->SPHI.p, c->WPHI.p, c->HPHI.p, colscale, c->SMR.p, c->SML.p, c->alpha.p,
      c->hR.p, c->hL.p, c->F, c->N, c->K, c->stereo, recompute_sphi);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

// WPHI, SF0, SPHI, SM and the model spectrograms from the parameters
// (:578-585 / :229-233)
int rebuild_model(simm_ctx *c) {
  int st;
  const int F = c->F, K = c->K;
  if ((st = gemm_nn(c, c->WGAMMA.p, c->P, c->HGAMMA.p, K, c->WPHI.p, K, F, K, c->P))) return st;
  if ((st = sf0_gemm(c))) return st;
  if ((st = refresh_sm_gemm(c))) return st;
  c->pend = nullptr;
  // the reference's initial hat is not floored by eps (:579-585); every use
  // floors it again with max(., eps), so the floored copy is equivalent
  if ((st = refresh_hat(c, nullptr, 1))) return st;
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

void reco_error(simm_ctx *c, double *slot) {
  const dim3 grid = walker_grid(c);
  const SPl p = planes(c, false);
  kdispatch(c->K, [&](auto km) {
    constexpr int KM = decltype(km)::value;
    if (c->stereo)
      k_is_partial<true, KM><<<grid, 256, 0, c->stream>>>(p, c->apart.p);
    else
      k_is_partial<false, KM><<<grid, 256, 0, c->stream>>>(p, c->apart.p);
  });
  k_is_final<<<1, 64, 0, c->stream>>>(c->apart.p, (int)(grid.x * grid.y), slot);
}

// one loop body; reco (device, may be null) receives the IS divergence
// after the HF0 and after the HPHI updates (SIMM.py:676-683, :721-728).
// Between updates the resident state is SF0 (times the pending column scale),
// SMR / SML, WPHI / HPHI and the scalars: the hat is formed by each consumer.
int simm_iteration(simm_ctx *c, double omega, int update_hgamma, double *reco) {
  const int F = c->F, N = c->N, NF0 = c->NF0, K = c->K, R = c->R;
  const bool ST = c->stereo != 0;
  const dim3 wg = walker_grid(c);
  int st;
  // ---- HF0 (:623-674 / :281-291)
  {
    const SPl p = planes(c, false);   // (no scale is pending at the iteration start)
    kdispatch(K, [&](auto km) {
      constexpr int KM = decltype(km)::value;
      // num | den side by side in the rows of TND (row stride 2N)
      if (ST)
        k_simm_numden<true, KM><<<wg, 256, 0, c->stream>>>(p, c->TND.p, c->TND.p + N, 2 * (size_t)N);
      else
        k_simm_numden<false, KM><<<wg, 256, 0, c->stream>>>(p, c->TND.p, c->TND.p + N, 2 * (size_t)N);
    });
  }
  // WF0^T [num | den]: one (NF0 x F)(F x 2N) product
  if (c->gemm_kind == 0) {
    ++g_nf0_dgemm2;
    if ((st = dgemm2(c->stream, NF0, 2 * N, F, c->WF0K.p, c->NF0p, c->TND.p, 2 * N, c->NPD.p,
                     2 * N)))
      return st;
  } else {   // FASST_SIMM_GEMM=2: k_gemm (no split-K: its outputs have ldc 2N)
    ++g_nf0_kgemm;
    const double *Bs[2] = {c->TND.p, c->TND.p + N};
    double *Cs[2] = {c->NPD.p, c->NPD.p + N};
    if ((st = gemm<true, false, 2>(c->stream, c->WF0.p, NF0, Bs, 2 * N, Cs, 2 * N, NF0, N, F,
                                   nullptr)))
      return st;
  }
  k_mu_apply_nd<<<egrid((size_t)NF0 * N), 256, 0, c->stream>>>(c->HF0.p, c->NPD.p, NF0, N, omega);
  if ((st = sf0_gemm(c))) return st;
  if (reco) reco_error(c, reco);
  // ---- HPHI (:686-729 / :296-313)
  {
    SPl p = planes(c, false);
    p.fchunk = c->fchunk_h;
    const dim3 gh((N + 255) / 256, c->nchunk_h);
    kdispatch(K, [&](auto km) {
      constexpr int KM = decltype(km)::value;
      if (ST)
        k_hphi_partial<true, KM><<<gh, 256, 0, c->stream>>>(p, c->hpart.p);
      else
        k_hphi_partial<false, KM><<<gh, 256, 0, c->stream>>>(p, c->hpart.p);
    });
  }
  k_hphi_update<<<(N + 255) / 256, 256, 0, c->stream>>>(c->HPHI.p, c->hpart.p, c->nchunk_h,
                                                         c->s_col.p, K, N, omega);
  k_colscale<<<egrid((size_t)NF0 * N), 256, 0, c->stream>>>(c->HF0.p, c->s_col.p, NF0, N);
  c->pend = c->s_col.p;   // SF0 *= s_col, applied by the HM products below
  if (reco) reco_error(c, reco + 1);
  // ---- HM (:740-773 / :318-331)
  if (ST) {
    double *Cs[4] = {c->RN0.p, c->RN1.p, c->RN0.p + (size_t)R * N, c->RN1.p + (size_t)R * N};
    if ((st = wmt_xy(c, Cs))) return st;
    k_hm_apply<<<egrid((size_t)R * N), 256, 0, c->stream>>>(c->HM.p, c->RN0.p, c->RN1.p,
                                                             c->RN0.p + (size_t)R * N,
                                                             c->RN1.p + (size_t)R * N, c->bR.p,
                                                             c->bL.p, R, N, omega);
  } else {
    double *Cs[2] = {c->RN0.p, c->RN1.p};
    if ((st = wmt_xy(c, Cs))) return st;
    k_mu_apply<<<egrid((size_t)R * N), 256, 0, c->stream>>>(c->HM.p, c->RN0.p, c->RN1.p,
                                                            (size_t)R * N, omega, 1);
  }
  if ((st = refresh_sm(c))) return st;
  // ---- HGAMMA (:776-823 / :335-350)
  if (update_hgamma) {
    const SPl p = planes(c, false);
    kdispatch(K, [&](auto km) {
      constexpr int KM = decltype(km)::value;
      if (ST)
        k_hgamma_rows<true, KM><<<dim3((F + kHgRows - 1) / kHgRows, kHgRowChunks), 256, 0, c->stream>>>(p, c->hrows.p);
      else
        k_hgamma_rows<false, KM><<<dim3((F + kHgRows - 1) / kHgRows, kHgRowChunks), 256, 0, c->stream>>>(p, c->hrows.p);
    });
    k_hgamma_numden<<<c->P, 256, 0, c->stream>>>(c->WGAMMA.p, c->hrows.p, c->apart.p, F, c->P, K,
                                                 kHgRowChunks);
    k_hgamma_norm<<<1, 64, 0, c->stream>>>(c->HGAMMA.p, c->apart.p, c->sg.p, c->P, K, omega);
    k_wphi<<<(F * K + 255) / 256, 256, 0, c->stream>>>(c->WGAMMA.p, c->HGAMMA.p, c->WPHI.p, F,
                                                       c->P, K);
    k_hphi_rescale<<<(N + 255) / 256, 256, 0, c->stream>>>(c->HPHI.p, c->sg.p, c->s_col.p, K, N);
    k_colscale<<<egrid((size_t)NF0 * N), 256, 0, c->stream>>>(c->HF0.p, c->s_col.p, NF0, N);
    c->pend = c->s_col.p;   // applied by the WM products below
  }
  // ---- WM (:826-869 / :355-387)
  if (ST) {
    double *dsts[4] = {c->P0.p, c->P1.p, c->P2.p, c->P3.p};
    if ((st = xy_hmt(c, dsts))) return st;
    k_wm_update<<<R, 256, 0, c->stream>>>(c->WM.p, c->P0.p, c->P1.p, c->P2.p, c->P3.p, c->bR.p,
                                          c->bL.p, c->sw.p, F, R, omega, 1);
    k_rowscale<<<egrid((size_t)R * N), 256, 0, c->stream>>>(c->HM.p, c->sw.p, R, N);
  } else {
    double *dsts[2] = {c->P0.p, c->P1.p};
    if ((st = xy_hmt(c, dsts))) return st;
    k_wm_update<<<R, 256, 0, c->stream>>>(c->WM.p, c->P0.p, c->P1.p, nullptr, nullptr, nullptr,
                                          nullptr, c->sw.p, F, R, omega, 0);
    // N7 (SIMM.py:388): HM *= sumWM broadcasts over the frame axis
    if (R == 1)
      k_rowscale<<<egrid((size_t)R * N), 256, 0, c->stream>>>(c->HM.p, c->sw.p, R, N);
    else
      k_colscale<<<egrid((size_t)R * N), 256, 0, c->stream>>>(c->HM.p, c->sw.p, R, N);  // R == N
  }
  if ((st = refresh_sm(c))) return st;
  if (!ST) return FASST_OK;
  // ---- alpha (:872-906)
  kdispatch(K, [&](auto km) {
    k_alpha_partial<decltype(km)::value><<<wg, 256, 0, c->stream>>>(planes(c, false), c->apart.p);
  });
  k_alpha_update<<<1, 64, 0, c->stream>>>(c->apart.p, (int)(wg.x * wg.y), c->alpha.p, omega);
  // ---- beta (:909-941)
  {
    double *Cs[4] = {c->RN0.p, c->RN1.p, c->RN0.p + (size_t)R * N, c->RN1.p + (size_t)R * N};
    if ((st = wmt_xy(c, Cs))) return st;
  }
  {
    const RowdotArgs ta = {{c->RN0.p, c->RN1.p, c->RN0.p + (size_t)R * N, c->RN1.p + (size_t)R * N}};
    k_rowdot<<<dim3(R, 4), 256, 0, c->stream>>>(ta, c->HM.p, c->bd.p, N);
  }
  k_beta_update<<<1, 64, 0, c->stream>>>(c->bd.p, c->bR.p, c->bL.p, R, omega);
  return refresh_sm(c);
}

}  // namespace

extern "C" {

int simm_create(int device, int F, int N, int NF0, int P, int K, int R, int stereo, simm_ctx **out) {
  if (!out || F < 1 || N < 1 || NF0 < 1 || P < 1 || K < 1 || K > kSimmKmax || R < 1 || P * K > 512) {
    set_error("simm_create: unsupported sizes F=%d N=%d NF0=%d P=%d K=%d R=%d", F, N, NF0, P, K, R);
    return FASST_ERR_SHAPE;
  }
  if (!stereo && R != 1 && R != N) {
    set_error("operands could not be broadcast together (SIMM.py:388 needs R == 1 or R == N)");
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  simm_ctx *c = new simm_ctx();
  c->device = device;
  c->F = F;
  c->N = N;
  c->NF0 = NF0;
  c->P = P;
  c->K = K;
  c->R = R;
  c->stereo = stereo ? 1 : 0;
  c->fchunk_h = std::max(1, (F + 15) / 16);
  c->nchunk_h = (F + c->fchunk_h - 1) / c->fchunk_h;
  // frame-walker grid: >= ~2048 blocks of 256 frames x a chunk of bins
  c->nchunk_w = std::max(1, std::min(F, (2048 + (N + 255) / 256 - 1) / ((N + 255) / 256)));
  c->fchunk_w = (F + c->nchunk_w - 1) / c->nchunk_w;
  c->nchunk_w = (F + c->fchunk_w - 1) / c->fchunk_w;
  c->nb_alpha = std::max(1024, ((N + 255) / 256) * c->nchunk_w);
  const size_t FN = (size_t)F * N;
  int st = FASST_OK;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) st = FASST_ERR_DEVICE;
  if (const char *v = getenv("FASST_SIMM_GEMM")) c->gemm_kind = atoi(v) == 2 ? 2 : 0;
  c->Fp = (F + 15) / 16 * 16;
  c->NF0p = (NF0 + 15) / 16 * 16;
  size_t gw = 0;
  gw = std::max(gw, gemm_workspace(NF0, 2 * N, F, 2));   // (num | den rows: ldc = 2N)
  gw = std::max(gw, gemm_workspace(F, N, NF0, 1));
  gw = std::max(gw, gemm_workspace(F, N, R, 1));
  gw = std::max(gw, gemm_workspace(R, N, F, stereo ? 4 : 2));
  gw = std::max(gw, gemm_workspace(F, R, N, 1));
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
    c->slots = 2L * ncu;   // resident 256-thread blocks of the skinny products
  }
  gw = std::max(gw, skinny_workspace(F, N, R, stereo, c->slots));
#define SA(buf, n) \
  if (!st) st = c->buf.alloc(n)
  SA(SXR, FN);
  SA(SXL, stereo ? FN : 1);
  SA(WF0, (size_t)F * NF0);
  SA(WF0K, (size_t)F * c->NF0p);   // zero-filled: the padding stays 0
  SA(WF0T, (size_t)NF0 * c->Fp);
  SA(WGAMMA, (size_t)F * P);
  SA(HGAMMA, (size_t)P * K);
  SA(HPHI, (size_t)K * N);
  SA(HF0, (size_t)NF0 * N);
  SA(HM, (size_t)R * N);
  SA(WM, (size_t)F * R);
  SA(bR, R);
  SA(bL, R);
  SA(alpha, 2);
  SA(WPHI, (size_t)F * K);
  SA(SF0, FN);
  SA(SPHI, FN);
  SA(hR, FN);
  SA(hL, stereo ? FN : 1);
  SA(SMR, FN);
  SA(SML, stereo ? FN : 1);
  SA(T0, FN);
  SA(T1, FN);
  SA(T2, stereo ? FN : 1);
  SA(T3, stereo ? FN : 1);
  SA(TND, 2 * FN);
  SA(NPD, 2 * (size_t)NF0 * N);
  SA(WMb, (size_t)F * std::max(R, 48));  // (48 = kSmRmax: padded rows of the fused refresh)
  SA(WMb2, (size_t)F * std::max(R, 48));
  SA(s_col, N);
  SA(sg, K);
  SA(sw, R);
  SA(hpart, (size_t)c->nchunk_h * 2 * K * N);
  SA(hrows, (size_t)kHgRowChunks * F * 2 * K);
  SA(apart, (size_t)c->nb_alpha * 4);
  SA(bd, 4 * (size_t)R);
  SA(gwork, std::max<size_t>(gw, 1));
  SA(P0, (size_t)F * R);
  SA(P1, (size_t)F * R);
  SA(P2, (size_t)F * R);
  SA(P3, (size_t)F * R);
  SA(RN0, 2 * (size_t)R * N);
  SA(RN1, 2 * (size_t)R * N);
#undef SA
  if (st) {
    simm_destroy(c);
    return st;
  }
  *out = c;
  return FASST_OK;
}

int simm_destroy(simm_ctx *c) {
  if (!c) return FASST_OK;
  {
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete c;  // DBuf destructors free device memory
  return FASST_OK;
}

int simm_set_data(simm_ctx *c, const double *SXR, const double *SXL, const double *WF0,
                  const double *WGAMMA) {
  if (!c || !WF0 || !WGAMMA) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  const size_t FN = (size_t)c->F * c->N;
  if (SXR) FASST_HIP(hipMemcpyAsync(c->SXR.p, SXR, FN * 8, hipMemcpyHostToDevice, c->stream));
  if (c->stereo && SXL)
    FASST_HIP(hipMemcpyAsync(c->SXL.p, SXL, FN * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->WF0.p, WF0, (size_t)c->F * c->NF0 * 8, hipMemcpyHostToDevice, c->stream));
  // the k-major operands of k_dgemm2: WF0 with an even row pitch, and WF0^T
  FASST_HIP(hipMemcpy2DAsync(c->WF0K.p, (size_t)c->NF0p * 8, WF0, (size_t)c->NF0 * 8,
                             (size_t)c->NF0 * 8, c->F, hipMemcpyHostToDevice, c->stream));
  k_simm_transpose<<<dim3((c->NF0 + 15) / 16, (c->F + 15) / 16), 256, 0, c->stream>>>(
      c->WF0.p, c->WF0T.p, c->F, c->NF0, c->NF0, c->Fp);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(c->WGAMMA.p, WGAMMA, (size_t)c->F * c->P * 8, hipMemcpyHostToDevice,
                           c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int simm_set_params(simm_ctx *c, const double *HGAMMA, const double *HPHI, const double *HF0,
                    const double *HM, const double *WM, const double *alpha, const double *betaR,
                    const double *betaL) {
  if (!c || !HGAMMA || !HPHI || !HF0 || !HM || !WM) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  const int F = c->F, N = c->N, K = c->K, R = c->R;
  FASST_HIP(hipMemcpyAsync(c->HGAMMA.p, HGAMMA, (size_t)c->P * K * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->HPHI.p, HPHI, (size_t)K * N * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->HF0.p, HF0, (size_t)c->NF0 * N * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->HM.p, HM, (size_t)R * N * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->WM.p, WM, (size_t)F * R * 8, hipMemcpyHostToDevice, c->stream));
  if (c->stereo) {
    std::vector<double> bl(R);
    for (int r = 0; r < R; ++r) bl[r] = betaL ? betaL[r] : 1 - betaR[r];  // (:576)
    FASST_HIP(hipMemcpyAsync(c->alpha.p, alpha, 2 * 8, hipMemcpyHostToDevice, c->stream));
    FASST_HIP(hipMemcpyAsync(c->bR.p, betaR, R * 8, hipMemcpyHostToDevice, c->stream));
    FASST_HIP(hipMemcpyAsync(c->bL.p, bl.data(), R * 8, hipMemcpyHostToDevice, c->stream));
    FASST_HIP(hipStreamSynchronize(c->stream));
  }
  return rebuild_model(c);
}

int simm_run(simm_ctx *c, int n_iter, double omega, int update_hgamma, double *reco_err) {
  if (!c || n_iter < 0) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  if (reco_err && c->reco.n < (size_t)2 * n_iter) {
    int st = c->reco.alloc(std::max(2 * n_iter, 1));
    if (st) return st;
  }
  for (int it = 0; it < n_iter; ++it) {
    int st = simm_iteration(c, omega, c->stereo ? update_hgamma : 1,
                            reco_err ? c->reco.p + 2 * it : nullptr);
    if (st) return st;
  }
  if (reco_err && n_iter > 0)
    FASST_HIP(hipMemcpyAsync(reco_err, c->reco.p, (size_t)2 * n_iter * 8, hipMemcpyDeviceToHost,
                             c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int simm_reco_error(simm_ctx *c, double *out) {
  if (!c || !out) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  if (c->reco.n < 1) {
    int st = c->reco.alloc(2);
    if (st) return st;
  }
  reco_error(c, c->reco.p);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(out, c->reco.p, 8, hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int simm_separate(simm_ctx *c, const double *XR, const double *XL, double *VR, double *VL,
                  double *MR, double *ML) {
  if (!c || !c->stereo || !XR || !XL || !VR || !VL || !MR || !ML) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  int st = rebuild_model(c);
  if (st) return st;
  const size_t FN = (size_t)c->F * c->N;
  DBuf<double2> dx[2], dout[4];
  for (auto &b : dx)
    if ((st = b.alloc(FN))) return st;
  for (auto &b : dout)
    if ((st = b.alloc(FN))) return st;
  FASST_HIP(hipMemcpyAsync(dx[0].p, XR, FN * 16, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(dx[1].p, XL, FN * 16, hipMemcpyHostToDevice, c->stream));
  k_lead_masks<<<egrid(FN), 256, 0, c->stream>>>(c->SF0.p, c->SPHI.p, c->SMR.p, c->SML.p,
                                                  c->alpha.p, dx[0].p, dx[1].p, dout[0].p,
                                                  dout[1].p, dout[2].p, dout[3].p, FN);
  FASST_LAUNCH_CHECK();
  double *outs[4] = {VR, VL, MR, ML};
  for (int q = 0; q < 4; ++q)
    FASST_HIP(hipMemcpyAsync(outs[q], dout[q].p, FN * 16, hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int simm_get_params(simm_ctx *c, double *HGAMMA, double *HPHI, double *HF0, double *HM, double *WM,
                    double *alpha, double *betaR, double *betaL) {
  if (!c) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  const int N = c->N, K = c->K, R = c->R;
  if (HGAMMA) FASST_HIP(hipMemcpyAsync(HGAMMA, c->HGAMMA.p, (size_t)c->P * K * 8, hipMemcpyDeviceToHost, c->stream));
  if (HPHI) FASST_HIP(hipMemcpyAsync(HPHI, c->HPHI.p, (size_t)K * N * 8, hipMemcpyDeviceToHost, c->stream));
  if (HF0) FASST_HIP(hipMemcpyAsync(HF0, c->HF0.p, (size_t)c->NF0 * N * 8, hipMemcpyDeviceToHost, c->stream));
  if (HM) FASST_HIP(hipMemcpyAsync(HM, c->HM.p, (size_t)R * N * 8, hipMemcpyDeviceToHost, c->stream));
  if (WM) FASST_HIP(hipMemcpyAsync(WM, c->WM.p, (size_t)c->F * R * 8, hipMemcpyDeviceToHost, c->stream));
  if (c->stereo) {
    if (alpha) FASST_HIP(hipMemcpyAsync(alpha, c->alpha.p, 2 * 8, hipMemcpyDeviceToHost, c->stream));
    if (betaR) FASST_HIP(hipMemcpyAsync(betaR, c->bR.p, R * 8, hipMemcpyDeviceToHost, c->stream));
    if (betaL) FASST_HIP(hipMemcpyAsync(betaL, c->bL.p, R * 8, hipMemcpyDeviceToHost, c->stream));
  }
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int simm_nf0_product_counts(long *dgemm2_launches, long *kgemm_launches) {
  if (dgemm2_launches) *dgemm2_launches = g_nf0_dgemm2.load();
  if (kgemm_launches) *kgemm_launches = g_nf0_kgemm.load();
  return FASST_OK;
}

}  // extern "C"
