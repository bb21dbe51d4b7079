// Time-frequency front/back end and the per-bin Wiener filter on MI355X.
//
//   k_stft_frames   Hann-windowed frames -> radix-2 FFT in LDS (FP64)
//                   (tftransforms/stft.py:3-69; numpy.fft.rfft)
//   k_istft_frames  Hermitian-extended inverse FFT per frame (stft.py:108-113)
//   k_ola           deterministic gather overlap-add + window normalisation
//                   (stft.py:110-129, same per-sample summation order)
//   k_cx_from_X     Cx packing X0 X0*, X0 X1*, X1 X1* (audioModel.py:293-302)
//   k_wiener<J>     Sigma_n = R_n V_n, Sigma_x^-1, WG_n = Sigma_n Sigma_x^-1,
//                   S_n = WG_n X  (audioModel.py:1327-1467, :1205-1214)
#include "fasst_ctx.h"
#include "fasst_fft.h"

#include <cmath>

namespace fasst {

__device__ __forceinline__ d4 mfma4b(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// One block per (frame, channel).  x: [nch][L] channel-major; output either
// [frame][bin] into a pitched device image (ld = row pitch in bins) or, for
// the stateless API, the same.
__global__ __launch_bounds__(256) void k_stft_frames(const double *__restrict__ x, int L,
                                                     const double *__restrict__ win, int wlen,
                                                     const double2 *__restrict__ tw, int N,
                                                     int logN, int hop, double2 *__restrict__ X,
                                                     int ld, size_t ch_stride) {
  extern __shared__ __attribute__((aligned(16))) double2 buf[];
  const int n = blockIdx.x, ch = blockIdx.y;
  const double *xc = x + (size_t)ch * L;
  const int half = wlen / 2;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    double v = 0.0;
    if (i < wlen) {
      const long s = (long)n * hop + i - half;
      if (s >= 0 && s < L) v = win[i] * xc[s];
    }
    buf[bitrev(i, logN)] = make_double2(v, 0.0);
  }
  __syncthreads();
  lds_fft(buf, tw, N, logN);
  double2 *out = X + ch * ch_stride + (size_t)n * ld;
  for (int k = threadIdx.x; k <= N / 2; k += blockDim.x) out[k] = buf[k];
}

// Inverse: X [frame][bin] (ld pitch) -> frames [frame][wlen] = window * irfft[:wlen]
__global__ __launch_bounds__(256) void k_istft_frames(const double2 *__restrict__ X, int ld,
                                                      const double *__restrict__ win, int wlen,
                                                      const double2 *__restrict__ tw, int N,
                                                      int logN, double *__restrict__ frames) {
  extern __shared__ __attribute__((aligned(16))) double2 buf[];
  const int n = blockIdx.x;
  const double2 *xn = X + (size_t)n * ld;
  const int h = N / 2;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    double2 z;
    if (i == 0)
      z = make_double2(xn[0].x, 0.0);
    else if (i == h)
      z = make_double2(xn[h].x, 0.0);
    else if (i < h)
      z = xn[i];
    else {
      const double2 c = xn[N - i];
      z = make_double2(c.x, -c.y);
    }
    buf[bitrev(i, logN)] = z;
  }
  __syncthreads();
  lds_fft(buf, tw, N, logN);
  const double invN = 1.0 / (double)N;
  for (int i = threadIdx.x; i < wlen; i += blockDim.x)
    frames[(size_t)n * wlen + i] = win[i] * (buf[i].x * invN);
}

// out[s] for s in [half, len): gather the frames covering s in frame order.
__global__ void k_ola(const double *__restrict__ frames, int nframes, int wlen, int hop,
                      const double *__restrict__ win, const double *__restrict__ awin,
                      double *__restrict__ y, int len_out) {
  const int half = wlen / 2;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < len_out; o += gridDim.x * blockDim.x) {
    const long s = (long)o + half;
    long nlo = (s - wlen) / hop + 1;
    if (s - wlen < 0) nlo = 0;
    long nhi = s / hop;
    if (nhi > nframes - 1) nhi = nframes - 1;
    double acc = 0.0, nrm = 0.0;
    for (long n = nlo; n <= nhi; ++n) {
      const int p = (int)(s - n * hop);
      if (p < 0 || p >= wlen) continue;
      nrm = nrm + win[p] * awin[p];
      acc = acc + frames[(size_t)n * wlen + p];
    }
    y[o] = acc / (nrm == 0.0 ? 1.0 : nrm);
  }
}

// SIMM-pipeline overlap-add (separateLeadFunctions.py:163-233): no half-window
// trim; the normalisation's first / last window are copied from the
// neighbouring window (:214-217), zeros become 1.  Needs len_out >= 2 wlen.
__device__ __forceinline__ double ola_norm(int s, int nframes, int wlen, int hop,
                                           const double *__restrict__ win,
                                           const double *__restrict__ awin) {
  long nlo = (s - wlen) / hop + 1;
  if (s - wlen < 0) nlo = 0;
  long nhi = s / hop;
  if (nhi > nframes - 1) nhi = nframes - 1;
  double nrm = 0.0;
  for (long n = nlo; n <= nhi; ++n) {
    const int p = (int)(s - n * hop);
    if (p < 0 || p >= wlen) continue;
    nrm = nrm + win[p] * awin[p];
  }
  return nrm;
}

__global__ void k_ola_simm(const double *__restrict__ frames, int nframes, int wlen, int hop,
                           const double *__restrict__ win, const double *__restrict__ awin,
                           double *__restrict__ y, int len_out) {
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < len_out; o += gridDim.x * blockDim.x) {
    long nlo = (o - wlen) / hop + 1;
    if (o - wlen < 0) nlo = 0;
    long nhi = o / hop;
    if (nhi > nframes - 1) nhi = nframes - 1;
    double acc = 0.0;
    for (long n = nlo; n <= nhi; ++n) {
      const int p = (int)(o - n * hop);
      if (p < 0 || p >= wlen) continue;
      acc = acc + frames[(size_t)n * wlen + p];
    }
    int u = o >= len_out - wlen ? o - wlen : o;  // norm[-L:] = norm[-2L:-L]
    if (u < wlen) u += wlen;                     // norm[:L] = norm[L:2L]
    double nrm = ola_norm(u, nframes, wlen, hop, win, awin);
    y[o] = acc / (nrm == 0.0 ? 1.0 : nrm);
  }
}

// Cx planes from the resident STFT images X[c][t][f].
__global__ void k_cx_from_X(const double2 *__restrict__ X, double *__restrict__ cx, size_t plane) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < plane;
       i += (size_t)gridDim.x * blockDim.x) {
    const double2 a = X[i], b = X[plane + i];
    cx[i] = a.x * a.x + a.y * a.y;
    cx[plane + i] = b.x * b.x + b.y * b.y;
    cx[2 * plane + i] = a.x * b.x + a.y * b.y;
    cx[3 * plane + i] = a.y * b.x - a.x * b.y;
  }
}

// host Cx [3][F][T] complex  <->  device planes [4][Tp][Fp]
__global__ void k_cx_unpack(const double2 *__restrict__ h, double *__restrict__ cx, int F, int T,
                            int Fp, int Tp) {
  __shared__ double2 tile[3][16][17];
  const int f0 = blockIdx.y * 16, t0 = blockIdx.x * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  for (int q = 0; q < 3; ++q) {
    const int f = f0 + ty, t = t0 + tx;
    tile[q][ty][tx] = (f < F && t < T) ? h[((size_t)q * F + f) * T + t] : make_double2(0.0, 0.0);
  }
  __syncthreads();
  const int t = t0 + ty, f = f0 + tx;
  const size_t plane = (size_t)Tp * Fp, o = (size_t)t * Fp + f;
  cx[o] = tile[0][tx][ty].x;
  cx[plane + o] = tile[2][tx][ty].x;
  cx[2 * plane + o] = tile[1][tx][ty].x;
  cx[3 * plane + o] = tile[1][tx][ty].y;
}
__global__ void k_cx_pack(const double *__restrict__ cx, double2 *__restrict__ h, int F, int T,
                          int Fp, int Tp) {
  __shared__ double tile[4][16][17];
  const int f0 = blockIdx.y * 16, t0 = blockIdx.x * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const size_t plane = (size_t)Tp * Fp;
  {
    const int t = t0 + ty, f = f0 + tx;
    const size_t o = (size_t)t * Fp + f;
    for (int q = 0; q < 4; ++q) tile[q][ty][tx] = cx[q * plane + o];
  }
  __syncthreads();
  const int f = f0 + ty, t = t0 + tx;
  if (f < F && t < T) {
    h[((size_t)0 * F + f) * T + t] = make_double2(tile[0][tx][ty], 0.0);
    h[((size_t)1 * F + f) * T + t] = make_double2(tile[2][tx][ty], tile[3][tx][ty]);
    h[((size_t)2 * F + f) * T + t] = make_double2(tile[1][tx][ty], 0.0);
  }
}

// generic complex [nm][F][T] (host order) <-> [nm][Tp][Fp] transposes
__global__ void k_ft_to_tf(const double2 *__restrict__ src, double2 *__restrict__ dst, int F, int T,
                           int Fp, int Tp) {
  __shared__ double2 tile[16][17];
  const int f0 = blockIdx.y * 16, t0 = blockIdx.x * 16, m = blockIdx.z;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  {
    const int f = f0 + ty, t = t0 + tx;
    tile[ty][tx] = (f < F && t < T) ? src[((size_t)m * F + f) * T + t] : make_double2(0.0, 0.0);
  }
  __syncthreads();
  const int t = t0 + ty, f = f0 + tx;
  if (t < Tp && f < Fp) dst[((size_t)m * Tp + t) * Fp + f] = tile[tx][ty];
}
__global__ void k_tf_to_ft(const double2 *__restrict__ src, double2 *__restrict__ dst, int F, int T,
                           int Fp, int Tp) {
  __shared__ double2 tile[16][17];
  const int f0 = blockIdx.y * 16, t0 = blockIdx.x * 16, m = blockIdx.z;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  {
    const int t = t0 + ty, f = f0 + tx;
    tile[ty][tx] = (t < Tp && f < Fp) ? src[((size_t)m * Tp + t) * Fp + f] : make_double2(0.0, 0.0);
  }
  __syncthreads();
  const int f = f0 + ty, t = t0 + tx;
  if (f < F && t < T) dst[((size_t)m * F + f) * T + t] = tile[tx][ty];
}

// mix_psd (audioModel.py:304-319): mean over t of the Cx diagonals, averaged
// over the channels.  Pass 1: block (64 bins, frame chunk), 4 frame phases
// per bin reduced in LDS -> part[chunk][f] (Cx00, Cx11 sums); pass 2 sums
// the chunks in order (deterministic; a chunked sum like NumPy's pairwise
// mean rather than one 10^4-term running sum).
constexpr int kPsdChunks = 64;
__global__ __launch_bounds__(256) void k_mix_psd_part(const double *__restrict__ cx, int F,
                                                      int T, int Fp, int Tp,
                                                      double2 *__restrict__ part) {
  __shared__ double2 s[4][64];
  const int fl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + fl;
  const int tpc = (T + kPsdChunks - 1) / kPsdChunks;
  const int tb = blockIdx.y * tpc, te = min(T, tb + tpc);
  const size_t plane = (size_t)Tp * Fp;
  double s0 = 0.0, s2 = 0.0;
  if (f < F)
    for (int t = tb + ph; t < te; t += 4) {
      s0 += cx[(size_t)t * Fp + f];
      s2 += cx[plane + (size_t)t * Fp + f];
    }
  s[ph][fl] = make_double2(s0, s2);
  __syncthreads();
  if (ph == 0 && f < F) {
    const double2 a = s[0][fl], b = s[1][fl], c = s[2][fl], d = s[3][fl];
    part[(size_t)blockIdx.y * Fp + f] = make_double2((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y));
  }
}

__global__ void k_mix_psd(const double2 *__restrict__ part, int F, int T, int Fp,
                          double *__restrict__ out) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  double s0 = 0.0, s2 = 0.0;
  for (int c = 0; c < kPsdChunks; ++c) {
    const double2 v = part[(size_t)c * Fp + f];
    s0 += v.x;
    s2 += v.y;
  }
  out[f] = ((0.0 + s0 / T) + s2 / T) / 2.0;
}

// R_n coefficients per bin: sum over the ranks of n of |a0|^2, |a1|^2, a0 conj(a1)
__global__ void k_mixcoef(const double2 *__restrict__ A, double *__restrict__ coef, int J,
                          const int *__restrict__ roff_dev, int F, int Fp) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= Fp) return;
  for (int j = 0; j < J; ++j) {
    double al = 0, be = 0, gr = 0, gi = 0;
    if (f < F)
      for (int r = roff_dev[j]; r < roff_dev[j + 1]; ++r) {
        const double2 a0 = A[(size_t)(2 * r) * Fp + f], a1 = A[(size_t)(2 * r + 1) * Fp + f];
        al += a0.x * a0.x + a0.y * a0.y;
        be += a1.x * a1.x + a1.y * a1.y;
        gr += a0.x * a1.x + a0.y * a1.y;
        gi += a0.y * a1.x - a0.x * a1.y;
      }
    coef[(size_t)(j * 4 + 0) * Fp + f] = al;
    coef[(size_t)(j * 4 + 1) * Fp + f] = be;
    coef[(size_t)(j * 4 + 2) * Fp + f] = gr;
    coef[(size_t)(j * 4 + 3) * Fp + f] = gi;
  }
}

struct WArgs {
  const double *TW, *Wkf, *coef, *psd;
  const double2 *X;  // [2][Tp][Fp]
  double2 *S;        // [J][2][Tp][Fp]
  int F, T, Fp, Tp, KP;
  int nj;            // sources (the kMaxJ instantiation's runtime bound)
};

// one wave per 16x16 (frame, bin) tile; V^T from FP64 MFMA (V = W.H, no eps,
// as comp_spat_comp_power inside compute_sigma_comp_2d)
template <int J>
__global__ __launch_bounds__(64) void k_wiener(const WArgs a) {
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const int t0 = blockIdx.x * 16, f0 = blockIdx.y * 16, f = f0 + fl;
  const int nks = a.KP >> 2;
  // (J = kMaxJ: J > 8 sources, the loops bounded by a.nj at run time)
  const int JR = J == kMaxJ ? a.nj : J;
  d4 v[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    v[j] = d4{0.0, 0.0, 0.0, 0.0};
    if (j >= JR) continue;
    const double *tw = a.TW + ((size_t)j * a.KP + tq) * a.Tp + t0 + fl;
    const double *wk = a.Wkf + ((size_t)j * a.KP + tq) * a.Fp + f;
    for (int s = 0; s < nks; ++s) v[j] = mfma4b(tw[(size_t)(4 * s) * a.Tp], wk[(size_t)(4 * s) * a.Fp], v[j]);
  }
  double cal[J], cbe[J], cgr[J], cgi[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (j >= JR) {
      cal[j] = cbe[j] = cgr[j] = cgi[j] = 0.0;
      continue;
    }
    cal[j] = a.coef[(size_t)(j * 4 + 0) * a.Fp + f];
    cbe[j] = a.coef[(size_t)(j * 4 + 1) * a.Fp + f];
    cgr[j] = a.coef[(size_t)(j * 4 + 2) * a.Fp + f];
    cgi[j] = a.coef[(size_t)(j * 4 + 3) * a.Fp + f];
  }
  const double psd = a.psd[f];
  const size_t plane = (size_t)a.Tp * a.Fp;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = t0 + tq + 4 * i;
    const size_t o = (size_t)t * a.Fp + f;
    double d0 = 0.0, d1 = 0.0, orr = 0.0, oi = 0.0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      d0 += cal[j] * v[j][i];
      d1 += cbe[j] * v[j][i];
      orr += cgr[j] * v[j][i];
      oi += cgi[j] * v[j][i];
    }
    d0 += psd;
    d1 += psd;
    double det = d0 * d1 - (orr * orr + oi * oi);
    const double dg = det + kEps;
    det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
    const double i0 = d1 / det, i1 = d0 / det;
    const double ior = -orr / det, ioi = -oi / det;
    const double2 x0 = a.X[o], x1 = a.X[plane + o];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if (j >= JR) continue;
      const double vv = v[j][i];
      const double s0 = cal[j] * vv, s1 = cbe[j] * vv, sr = cgr[j] * vv, si = cgi[j] * vv;
      // WG00 = so conj(iso) + sd0 isd0 ; WG11 = conj(so conj(iso)) + sd1 isd1
      const double pr = sr * ior + si * ioi, pi = si * ior - sr * ioi;
      const double w00r = pr + s0 * i0, w00i = pi;
      const double w11r = pr + s1 * i1, w11i = -pi;
      // WG01 = sd0 iso + so isd1 ; WG10 = conj(so) isd0 + sd1 conj(iso)
      const double w01r = s0 * ior + sr * i1, w01i = s0 * ioi + si * i1;
      const double w10r = sr * i0 + s1 * ior, w10i = -si * i0 - s1 * ioi;
      const double2 y0 = make_double2(w00r * x0.x - w00i * x0.y + (w01r * x1.x - w01i * x1.y),
                                      w00r * x0.y + w00i * x0.x + (w01r * x1.y + w01i * x1.x));
      const double2 y1 = make_double2(w10r * x0.x - w10i * x0.y + (w11r * x1.x - w11i * x1.y),
                                      w10r * x0.y + w10i * x0.x + (w11r * x1.y + w11i * x1.x));
      a.S[((size_t)j * 2 + 0) * plane + o] = y0;
      a.S[((size_t)j * 2 + 1) * plane + o] = y1;
    }
  }
}


// Sources made of spectral components (separate_comps with spec_comp_ind,
// audioModel.py:1130-1164): Sigma_n = sum over the terms of n of R_j V_{j,C}
// with V_{j,C} = W_j[:, C] H_j[C, :] (compute_sigma_comp_2d on the
// components C of n in spatial component j), Sigma_x = sum_n Sigma_n + psd
// (compute_inv_sigma_mix_2d).  Two passes per tile: Sigma_x from every term,
// then each source's Wiener gain and images (its V tiles re-formed).
struct WSArgs {
  const double *TW, *Wkf, *coef, *psd;
  const double2 *X;
  double2 *S;   // [nsrc][2][Tp][Fp]
  int F, T, Fp, Tp, KP, nsrc;
  int toff[kMaxSlot + 1], tj[kMaxSlot];
  unsigned long long tmask[kMaxSlot][2];   // 128-bit column sets (KP <= 128)
};

__device__ __forceinline__ d4 ws_term_v(const WSArgs &a, int i, int t0, int f, int tq, int fl) {
  const int j = a.tj[i];
  const unsigned long long m0 = a.tmask[i][0], m1 = a.tmask[i][1];
  const double *tw = a.TW + ((size_t)j * a.KP + tq) * a.Tp + t0 + fl;
  const double *wk = a.Wkf + ((size_t)j * a.KP + tq) * a.Fp + f;
  d4 v = d4{0.0, 0.0, 0.0, 0.0};
  for (int s = 0; s < (a.KP >> 2); ++s) {
    const int k = tq + 4 * s;
    const double w = ((k < 64 ? m0 >> k : m1 >> (k - 64)) & 1ull) ? wk[(size_t)(4 * s) * a.Fp] : 0.0;
    v = mfma4b(tw[(size_t)(4 * s) * a.Tp], w, v);
  }
  return v;
}

// Sigma_n of source n at this tile (its terms summed in order)
__device__ __forceinline__ void ws_source(const WSArgs &a, int n, int t0, int f, int tq, int fl,
                                          d4 &s0, d4 &s1, d4 &sr, d4 &si) {
  s0 = s1 = sr = si = d4{0.0, 0.0, 0.0, 0.0};
  for (int i = a.toff[n]; i < a.toff[n + 1]; ++i) {
    const d4 v = ws_term_v(a, i, t0, f, tq, fl);
    const int j = a.tj[i];
    s0 += a.coef[(size_t)(j * 4 + 0) * a.Fp + f] * v;
    s1 += a.coef[(size_t)(j * 4 + 1) * a.Fp + f] * v;
    sr += a.coef[(size_t)(j * 4 + 2) * a.Fp + f] * v;
    si += a.coef[(size_t)(j * 4 + 3) * a.Fp + f] * v;
  }
}

__global__ __launch_bounds__(64) void k_wiener_src(const WSArgs a) {
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const int t0 = blockIdx.x * 16, f0 = blockIdx.y * 16, f = f0 + fl;
  d4 d0 = d4{0.0, 0.0, 0.0, 0.0}, d1 = d0, orr = d0, oi = d0;
  for (int n = 0; n < a.nsrc; ++n) {
    d4 s0, s1, sr, si;
    ws_source(a, n, t0, f, tq, fl, s0, s1, sr, si);
    d0 += s0;
    d1 += s1;
    orr += sr;
    oi += si;
  }
  const double psd = a.psd[f];
  d4 i0, i1, ior, ioi;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double e0 = d0[q] + psd, e1 = d1[q] + psd;
    double det = e0 * e1 - (orr[q] * orr[q] + oi[q] * oi[q]);
    const double dg = det + kEps;
    det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
    i0[q] = e1 / det;
    i1[q] = e0 / det;
    ior[q] = -orr[q] / det;
    ioi[q] = -oi[q] / det;
  }
  const size_t plane = (size_t)a.Tp * a.Fp;
  for (int n = 0; n < a.nsrc; ++n) {
    d4 s0, s1, sr, si;
    ws_source(a, n, t0, f, tq, fl, s0, s1, sr, si);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const size_t o = (size_t)(t0 + tq + 4 * q) * a.Fp + f;
      // WG = Sigma_n Sigma_x^-1 (compute_Wiener_gain_2d, audioModel.py:1453-1465)
      const double pr = sr[q] * ior[q] + si[q] * ioi[q], pi = si[q] * ior[q] - sr[q] * ioi[q];
      const double w00r = pr + s0[q] * i0[q], w00i = pi;
      const double w11r = pr + s1[q] * i1[q], w11i = -pi;
      const double w01r = s0[q] * ior[q] + sr[q] * i1[q], w01i = s0[q] * ioi[q] + si[q] * i1[q];
      const double w10r = sr[q] * i0[q] + s1[q] * ior[q], w10i = -si[q] * i0[q] - s1[q] * ioi[q];
      const double2 x0 = a.X[o], x1 = a.X[plane + o];
      a.S[((size_t)n * 2 + 0) * plane + o] =
          make_double2(w00r * x0.x - w00i * x0.y + (w01r * x1.x - w01i * x1.y),
                       w00r * x0.y + w00i * x0.x + (w01r * x1.y + w01i * x1.x));
      a.S[((size_t)n * 2 + 1) * plane + o] =
          make_double2(w10r * x0.x - w10i * x0.y + (w11r * x1.x - w11i * x1.y),
                       w10r * x0.y + w10i * x0.x + (w11r * x1.y + w11i * x1.x));
    }
  }
}

__global__ void k_inv_herm(int n, const double *__restrict__ d, const double2 *__restrict__ off,
                           double *__restrict__ id, double2 *__restrict__ ioff,
                           double *__restrict__ det_out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double d0 = d[i], d1 = d[n + i];
    const double2 o = off[i];
    double det = d0 * d1 - (o.x * o.x + o.y * o.y);
    const double dg = det + kEps;
    det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
    ioff[i] = make_double2(-o.x / det, -o.y / det);
    id[i] = d1 / det;
    id[n + i] = d0 / det;
    det_out[i] = det;
  }
}


// Wiener images of the separation sources into dS [nsrc][2][Tp][Fp] (nsrc =
// J when no source table is set)
static int launch_wiener(fasst_ctx *c, const double *coef, const double *dpsd, double2 *dS) {
  const dim3 grid(c->ntt, c->nft);
  if (c->nsrc > 0) {
    WSArgs w;
    w.TW = c->TW.p;
    w.Wkf = c->Wkf.p;
    w.coef = coef;
    w.psd = dpsd;
    w.X = c->X.p;
    w.S = dS;
    w.F = c->F;
    w.T = c->T;
    w.Fp = c->Fp;
    w.Tp = c->Tp;
    w.KP = c->KP;
    w.nsrc = c->nsrc;
    for (int i = 0; i <= kMaxSlot; ++i) w.toff[i] = i <= c->nsrc ? c->toff[i] : c->toff[c->nsrc];
    for (int i = 0; i < kMaxSlot; ++i) {
      w.tj[i] = c->tj[i];
      w.tmask[i][0] = c->tmask[i][0];
      w.tmask[i][1] = c->tmask[i][1];
    }
    k_wiener_src<<<grid, 64, 0, c->stream>>>(w);
    FASST_LAUNCH_CHECK();
    return FASST_OK;
  }
  WArgs w;
  w.TW = c->TW.p;
  w.Wkf = c->Wkf.p;
  w.coef = coef;
  w.psd = dpsd;
  w.X = c->X.p;
  w.S = dS;
  w.F = c->F;
  w.T = c->T;
  w.Fp = c->Fp;
  w.Tp = c->Tp;
  w.KP = c->KP;
  w.nj = c->J;
  switch (c->J) {
    case 1: k_wiener<1><<<grid, 64, 0, c->stream>>>(w); break;
    case 2: k_wiener<2><<<grid, 64, 0, c->stream>>>(w); break;
    case 3: k_wiener<3><<<grid, 64, 0, c->stream>>>(w); break;
    case 4: k_wiener<4><<<grid, 64, 0, c->stream>>>(w); break;
    case 5: k_wiener<5><<<grid, 64, 0, c->stream>>>(w); break;
    case 6: k_wiener<6><<<grid, 64, 0, c->stream>>>(w); break;
    case 7: k_wiener<7><<<grid, 64, 0, c->stream>>>(w); break;
    case 8: k_wiener<8><<<grid, 64, 0, c->stream>>>(w); break;
    default: k_wiener<kMaxJ><<<grid, 64, 0, c->stream>>>(w); break;   // 9 .. kMaxJ
  }
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

static int check_fft(int nfft, int wlen, int hop) {
  if (ilog2(nfft) < 1 || wlen < 2 || wlen > nfft || hop < 1 || nfft > 8192) {
    set_error("FFT size %d must be a power of two >= wlen %d (hop %d)", nfft, wlen, hop);
    return FASST_ERR_SHAPE;
  }
  return FASST_OK;
}

static int fft_smem(int N) {
  const size_t bytes = (size_t)N * sizeof(double2);
  if (bytes > 64 * 1024) {
    FASST_HIP(hipFuncSetAttribute((const void *)k_stft_frames,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    FASST_HIP(hipFuncSetAttribute((const void *)k_istft_frames,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  }
  return FASST_OK;
}

int tf_launch_ft_to_tf(hipStream_t s, const double2 *src, double2 *dst, int F, int T, int Fp,
                       int Tp, int nm) {
  k_ft_to_tf<<<dim3((Tp + 15) / 16, (Fp + 15) / 16, nm), 256, 0, s>>>(src, dst, F, T, Fp, Tp);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int tf_launch_tf_to_ft(hipStream_t s, const double2 *src, double2 *dst, int F, int T, int Fp,
                       int Tp, int nm) {
  k_tf_to_ft<<<dim3((Tp + 15) / 16, (Fp + 15) / 16, nm), 256, 0, s>>>(src, dst, F, T, Fp, Tp);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int tf_launch_istft(hipStream_t s, const double2 *S, int ld, int T, const double *win,
                    const double *awin, const double2 *tw, int wlen, int nfft, int hop,
                    double *frames, double *y, int len_out) {
  int st = check_fft(nfft, wlen, hop);
  if (st) return st;
  if ((st = fft_smem(nfft))) return st;
  k_istft_frames<<<T, 256, nfft * sizeof(double2), s>>>(S, ld, win, wlen, tw, nfft, ilog2(nfft),
                                                        frames);
  FASST_LAUNCH_CHECK();
  k_ola<<<(len_out + 255) / 256, 256, 0, s>>>(frames, T, wlen, hop, win, awin, y, len_out);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

}  // namespace fasst

using namespace fasst;

extern "C" {

int fasst_stft(int device, const double *x, int L, const double *window, int wlen, int nfft,
               int hop, double *X, int *n_frames) {
  int st = check_fft(nfft, wlen, hop);
  if (st) return st;
  const int T = (L + hop - 1) / hop + 2;
  if (n_frames) *n_frames = T;
  if (!X) return FASST_OK;
  DeviceGuard g(device);
  if ((st = fft_smem(nfft))) return st;
  const int F = nfft / 2 + 1;
  DBuf<double> dx, dw;
  DBuf<double2> dtw, dX, dXt;
  if ((st = dx.alloc(std::max(L, 1))) || (st = dw.alloc(wlen)) || (st = dtw.alloc(nfft / 2)) ||
      (st = dX.alloc((size_t)T * F)) || (st = dXt.alloc((size_t)T * F)))
    return st;
  auto tw = twiddles(nfft, -1);
  FASST_HIP(hipMemcpy(dx.p, x, (size_t)L * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dw.p, window, (size_t)wlen * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice));
  k_stft_frames<<<dim3(T, 1), 256, nfft * sizeof(double2)>>>(dx.p, L, dw.p, wlen, dtw.p, nfft,
                                                             ilog2(nfft), hop, dX.p, F, 0);
  FASST_LAUNCH_CHECK();
  // [T][F] -> [F][T]
  k_tf_to_ft<<<dim3((T + 15) / 16, (F + 15) / 16, 1), 256>>>(dX.p, dXt.p, F, T, F, T);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipDeviceSynchronize());
  FASST_HIP(hipMemcpy(X, dXt.p, (size_t)T * F * sizeof(double2), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int fasst_istft(int device, const double *X, int n_frames, const double *window,
                const double *analysis_window, int wlen, int nfft, int hop, double *y) {
  int st = check_fft(nfft, wlen, hop);
  if (st) return st;
  if (n_frames < 1 || !X || !y) return FASST_ERR_SHAPE;
  DeviceGuard g(device);
  if ((st = fft_smem(nfft))) return st;
  const int F = nfft / 2 + 1, T = n_frames;
  const int len_out = hop * (T - 1) + wlen - wlen / 2;
  DBuf<double> dw, daw, dframes, dy;
  DBuf<double2> dtw, dX, dXt;
  if ((st = dw.alloc(wlen)) || (st = daw.alloc(wlen)) || (st = dtw.alloc(nfft / 2)) ||
      (st = dX.alloc((size_t)T * F)) || (st = dXt.alloc((size_t)T * F)) ||
      (st = dframes.alloc((size_t)T * wlen)) || (st = dy.alloc(len_out)))
    return st;
  auto tw = twiddles(nfft, +1);
  FASST_HIP(hipMemcpy(dw.p, window, (size_t)wlen * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(daw.p, analysis_window ? analysis_window : window,
                      (size_t)wlen * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dX.p, X, (size_t)T * F * sizeof(double2), hipMemcpyHostToDevice));
  // [F][T] -> [T][F]
  k_ft_to_tf<<<dim3((T + 15) / 16, (F + 15) / 16, 1), 256>>>(dX.p, dXt.p, F, T, F, T);
  FASST_LAUNCH_CHECK();
  k_istft_frames<<<T, 256, nfft * sizeof(double2)>>>(dXt.p, F, dw.p, wlen, dtw.p, nfft,
                                                     ilog2(nfft), dframes.p);
  FASST_LAUNCH_CHECK();
  k_ola<<<(len_out + 255) / 256, 256>>>(dframes.p, T, wlen, hop, dw.p, daw.p, dy.p, len_out);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipDeviceSynchronize());
  FASST_HIP(hipMemcpy(y, dy.p, (size_t)len_out * sizeof(double), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int fasst_istft_simm(int device, const double *X, int n_frames, const double *window,
                     const double *analysis_window, int wlen, int nfft, int hop, double *y) {
  int st = check_fft(nfft, wlen, hop);
  if (st) return st;
  if (n_frames < 1 || !X || !y) return FASST_ERR_SHAPE;
  const int F = nfft / 2 + 1, T = n_frames;
  const int len_out = hop * (T - 1) + wlen;
  if (len_out < 2 * wlen) {
    set_error("istft: %d samples < two windows (%d); the reference's edge copy fails", len_out,
              wlen);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  if ((st = fft_smem(nfft))) return st;
  DBuf<double> dw, daw, dframes, dy;
  DBuf<double2> dtw, dX, dXt;
  if ((st = dw.alloc(wlen)) || (st = daw.alloc(wlen)) || (st = dtw.alloc(nfft / 2)) ||
      (st = dX.alloc((size_t)T * F)) || (st = dXt.alloc((size_t)T * F)) ||
      (st = dframes.alloc((size_t)T * wlen)) || (st = dy.alloc(len_out)))
    return st;
  auto tw = twiddles(nfft, +1);
  FASST_HIP(hipMemcpy(dw.p, window, (size_t)wlen * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(daw.p, analysis_window ? analysis_window : window,
                      (size_t)wlen * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dX.p, X, (size_t)T * F * sizeof(double2), hipMemcpyHostToDevice));
  k_ft_to_tf<<<dim3((T + 15) / 16, (F + 15) / 16, 1), 256>>>(dX.p, dXt.p, F, T, F, T);
  FASST_LAUNCH_CHECK();
  k_istft_frames<<<T, 256, nfft * sizeof(double2)>>>(dXt.p, F, dw.p, wlen, dtw.p, nfft,
                                                     ilog2(nfft), dframes.p);
  FASST_LAUNCH_CHECK();
  k_ola_simm<<<(len_out + 255) / 256, 256>>>(dframes.p, T, wlen, hop, dw.p, daw.p, dy.p, len_out);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipDeviceSynchronize());
  FASST_HIP(hipMemcpy(y, dy.p, (size_t)len_out * sizeof(double), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int fasst_set_audio(fasst_ctx *c, const double *data, int L, const double *window, int wlen,
                    int nfft, int hop) {
  if (!c || !data || !window) return FASST_ERR_SHAPE;
  int st = check_fft(nfft, wlen, hop);
  if (st) return st;
  const int T = (L + hop - 1) / hop + 2;
  if (nfft / 2 + 1 != c->F || T != c->T) {
    set_error("fasst_set_audio: context is %dx%d, audio gives %dx%d", c->F, c->T, nfft / 2 + 1, T);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(c->device);
  if ((st = fft_smem(nfft))) return st;
  if (!c->X.p && (st = c->X.alloc((size_t)2 * c->Tp * c->Fp))) return st;
  std::vector<double> chans((size_t)2 * L);
  for (int i = 0; i < L; ++i) {
    chans[i] = data[(size_t)i * 2];
    chans[(size_t)L + i] = data[(size_t)i * 2 + 1];
  }
  DBuf<double> dx, dw;
  DBuf<double2> dtw;
  if ((st = dx.alloc((size_t)2 * L)) || (st = dw.alloc(wlen)) || (st = dtw.alloc(nfft / 2)))
    return st;
  auto tw = twiddles(nfft, -1);
  FASST_HIP(hipMemcpyAsync(dx.p, chans.data(), chans.size() * sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(dw.p, window, (size_t)wlen * sizeof(double), hipMemcpyHostToDevice,
                           c->stream));
  FASST_HIP(hipMemcpyAsync(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice,
                           c->stream));
  FASST_HIP(hipMemsetAsync(c->X.p, 0, c->X.n * sizeof(double2), c->stream));
  k_stft_frames<<<dim3(T, 2), 256, nfft * sizeof(double2), c->stream>>>(
      dx.p, L, dw.p, wlen, dtw.p, nfft, ilog2(nfft), hop, c->X.p, c->Fp, (size_t)c->Tp * c->Fp);
  FASST_LAUNCH_CHECK();
  const size_t plane = (size_t)c->Tp * c->Fp;
  k_cx_from_X<<<2048, 256, 0, c->stream>>>(c->X.p, c->cx.p, plane);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipStreamSynchronize(c->stream));
  c->have_X = true;
  c->cx_ready = true;
  return FASST_OK;
}

int fasst_mix_psd(fasst_ctx *c, double *mix_psd) {
  if (!c || !mix_psd) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  DBuf<double> d;
  DBuf<double2> part;
  int st;
  if ((st = d.alloc(c->F)) || (st = part.alloc((size_t)kPsdChunks * c->Fp))) return st;
  k_mix_psd_part<<<dim3((c->F + 63) / 64, kPsdChunks), 256, 0, c->stream>>>(c->cx.p, c->F, c->T,
                                                                           c->Fp, c->Tp, part.p);
  FASST_LAUNCH_CHECK();
  k_mix_psd<<<(c->F + 255) / 256, 256, 0, c->stream>>>(part.p, c->F, c->T, c->Fp, d.p);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(mix_psd, d.p, c->F * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_set_cx(fasst_ctx *c, const double *cx) {
  if (!c || !cx) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  DBuf<double2> h;
  int st;
  if ((st = h.alloc((size_t)3 * c->F * c->T))) return st;
  FASST_HIP(hipMemcpyAsync(h.p, cx, h.n * sizeof(double2), hipMemcpyHostToDevice, c->stream));
  k_cx_unpack<<<dim3(c->ntt, c->nft), 256, 0, c->stream>>>(h.p, c->cx.p, c->F, c->T, c->Fp, c->Tp);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipStreamSynchronize(c->stream));
  c->cx_ready = true;
  return FASST_OK;
}

int fasst_get_cx(fasst_ctx *c, double *cx) {
  if (!c || !cx) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  DBuf<double2> h;
  int st;
  if ((st = h.alloc((size_t)3 * c->F * c->T))) return st;
  k_cx_pack<<<dim3(c->ntt, c->nft), 256, 0, c->stream>>>(c->cx.p, h.p, c->F, c->T, c->Fp, c->Tp);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(cx, h.p, h.n * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

}  // extern "C"

namespace fasst {
static int upload_stft(fasst_ctx *c, const double *X) {
  int st;
  if (!c->X.p && (st = c->X.alloc((size_t)2 * c->Tp * c->Fp))) return st;
  DBuf<double2> h;
  if ((st = h.alloc((size_t)2 * c->F * c->T))) return st;
  FASST_HIP(hipMemcpyAsync(h.p, X, h.n * sizeof(double2), hipMemcpyHostToDevice, c->stream));
  k_ft_to_tf<<<dim3(c->ntt, c->nft, 2), 256, 0, c->stream>>>(h.p, c->X.p, c->F, c->T, c->Fp, c->Tp);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipStreamSynchronize(c->stream));
  c->have_X = true;
  return FASST_OK;
}
}  // namespace fasst

extern "C" {

int fasst_set_stft(fasst_ctx *c, const double *X) {
  if (!c || !X) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  int st = upload_stft(c, X);
  if (st) return st;
  k_cx_from_X<<<2048, 256, 0, c->stream>>>(c->X.p, c->cx.p, (size_t)c->Tp * c->Fp);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipStreamSynchronize(c->stream));
  c->cx_ready = true;
  return FASST_OK;
}

int fasst_set_sources(fasst_ctx *c, int nsrc, const int *term_off, const int *term_j,
                      const unsigned long long *term_mask) {
  if (!c || !c->configured) {
    set_error("fasst_set_sources: context not configured");
    return FASST_ERR_SHAPE;
  }
  if (nsrc == 0) {
    c->nsrc = 0;
    return FASST_OK;
  }
  if (nsrc < 0 || nsrc > kMaxSlot || !term_off || !term_j || !term_mask || term_off[0] != 0 ||
      term_off[nsrc] > kMaxSlot) {
    set_error("fasst_set_sources: %d sources (max %d terms in all)", nsrc, kMaxSlot);
    return nsrc > kMaxSlot ? FASST_ERR_UNSUPPORTED : FASST_ERR_SHAPE;
  }
  for (int n = 0; n < nsrc; ++n)
    if (term_off[n + 1] <= term_off[n]) {
      set_error("fasst_set_sources: source %d has no component", n);
      return FASST_ERR_SHAPE;
    }
  for (int i = 0; i < term_off[nsrc]; ++i) {
    const int j = term_j[i];
    const unsigned long long m0 = term_mask[2 * i], m1 = term_mask[2 * i + 1];
    const int K = j >= 0 && j < c->J ? c->K[j] : 0;
    // a non-empty set of the component's own columns 0 .. K - 1
    const bool past = K < 64 ? ((m0 >> K) != 0ull || m1 != 0ull)
                             : (K < 128 && (m1 >> (K - 64)) != 0ull);
    if (j < 0 || j >= c->J || !(m0 | m1) || past) {
      set_error("fasst_set_sources: bad term %d (spatial component %d)", i, j);
      return FASST_ERR_SHAPE;
    }
  }
  c->nsrc = nsrc;
  for (int n = 0; n <= nsrc; ++n) c->toff[n] = term_off[n];
  for (int i = 0; i < term_off[nsrc]; ++i) {
    c->tj[i] = term_j[i];
    c->tmask[i][0] = term_mask[2 * i];
    c->tmask[i][1] = term_mask[2 * i + 1];
  }
  return FASST_OK;
}

int fasst_wiener_images(fasst_ctx *c, const double *psd, const double *X, double *S) {
  if (!c || !c->configured || !psd || !S) {
    set_error("fasst_wiener_images: context not configured");
    return FASST_ERR_SHAPE;
  }
  int st;
  DeviceGuard g(c->device);  // before upload_stft: X and its staging live on c->device
  if (X && (st = upload_stft(c, X))) return st;
  if (!c->have_X) {
    set_error("fasst_wiener_images: no STFT available (set_audio / set_stft / X argument)");
    return FASST_ERR_SHAPE;
  }
  const int J = c->J, NS = c->nsrc > 0 ? c->nsrc : J;
  DBuf<double> dpsd, coef;
  DBuf<int> droff;
  DBuf<double2> dS, hS;
  const size_t plane = (size_t)c->Tp * c->Fp;
  if ((st = dpsd.alloc(c->Fp)) || (st = coef.alloc((size_t)J * 4 * c->Fp)) ||
      (st = droff.alloc(kMaxJ + 1)) || (st = dS.alloc((size_t)NS * 2 * plane)) ||
      (st = hS.alloc((size_t)NS * 2 * c->F * c->T)))
    return st;
  FASST_HIP(hipMemcpyAsync(dpsd.p, psd, c->F * sizeof(double), hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(droff.p, c->roff, (J + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream));
  // W = FB.FW and the per-bin mixing for 'inst'
  if ((st = build_inst_A(c))) return st;
  if ((st = launch_w_old(c))) return st;
  k_mixcoef<<<(c->Fp + 255) / 256, 256, 0, c->stream>>>(c->A.p, coef.p, J, droff.p, c->F, c->Fp);
  FASST_LAUNCH_CHECK();
  if ((st = launch_wiener(c, coef.p, dpsd.p, dS.p))) return st;
  k_tf_to_ft<<<dim3(c->ntt, c->nft, NS * 2), 256, 0, c->stream>>>(dS.p, hS.p, c->F, c->T, c->Fp, c->Tp);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(S, hS.p, hS.n * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_separate_waveforms(fasst_ctx *c, const double *psd, const double *window,
                             const double *analysis_window, int wlen, int nfft, int hop,
                             double *y) {
  if (!c || !c->configured || !psd || !window || !y) {
    set_error("fasst_separate_waveforms: context not configured");
    return FASST_ERR_SHAPE;
  }
  int st = check_fft(nfft, wlen, hop);
  if (st) return st;
  if (nfft / 2 + 1 != c->F) {
    set_error("fasst_separate_waveforms: nfft=%d gives %d bins, the model has F=%d", nfft,
              nfft / 2 + 1, c->F);
    return FASST_ERR_SHAPE;
  }
  if (!c->have_X) {
    set_error("fasst_separate_waveforms: no STFT available (set_audio / set_stft)");
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(c->device);
  if ((st = fft_smem(nfft))) return st;
  const int J = c->J, T = c->T, NS = c->nsrc > 0 ? c->nsrc : J;
  const size_t plane = (size_t)c->Tp * c->Fp;
  const int len_out = hop * (T - 1) + wlen - wlen / 2;  // istft (stft.py:108-129)
  DBuf<double> dpsd, coef, dw, daw, dframes, dy;
  DBuf<int> droff;
  DBuf<double2> dS, dtw;
  if ((st = dpsd.alloc(c->Fp)) || (st = coef.alloc((size_t)J * 4 * c->Fp)) ||
      (st = droff.alloc(kMaxJ + 1)) || (st = dS.alloc((size_t)NS * 2 * plane)) ||
      (st = dw.alloc(wlen)) || (st = daw.alloc(wlen)) || (st = dtw.alloc(nfft / 2)) ||
      (st = dframes.alloc((size_t)T * wlen)) || (st = dy.alloc((size_t)NS * 2 * len_out)))
    return st;
  auto tw = twiddles(nfft, +1);
  FASST_HIP(hipMemcpyAsync(dpsd.p, psd, c->F * sizeof(double), hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(droff.p, c->roff, (J + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(dw.p, window, (size_t)wlen * sizeof(double), hipMemcpyHostToDevice,
                           c->stream));
  FASST_HIP(hipMemcpyAsync(daw.p, analysis_window ? analysis_window : window,
                           (size_t)wlen * sizeof(double), hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice,
                           c->stream));
  if ((st = build_inst_A(c))) return st;
  if ((st = launch_w_old(c))) return st;
  k_mixcoef<<<(c->Fp + 255) / 256, 256, 0, c->stream>>>(c->A.p, coef.p, J, droff.p, c->F, c->Fp);
  FASST_LAUNCH_CHECK();
  if ((st = launch_wiener(c, coef.p, dpsd.p, dS.p))) return st;
  // each image's frames are rows of its [Tp][Fp] plane: iSTFT straight from
  // HBM (k_istft_frames takes the row stride), only waveforms leave the card
  for (int q = 0; q < 2 * NS; ++q) {
    k_istft_frames<<<T, 256, nfft * sizeof(double2), c->stream>>>(
        dS.p + (size_t)q * plane, c->Fp, dw.p, wlen, dtw.p, nfft, ilog2(nfft), dframes.p);
    FASST_LAUNCH_CHECK();
    k_ola<<<(len_out + 255) / 256, 256, 0, c->stream>>>(dframes.p, T, wlen, hop, dw.p, daw.p,
                                                        dy.p + (size_t)q * len_out, len_out);
    FASST_LAUNCH_CHECK();
  }
  FASST_HIP(hipMemcpyAsync(y, dy.p, dy.n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_inv_herm_mat_2d(int device, int n, const double *diag, const double *off,
                          double *inv_diag, double *inv_off, double *det) {
  if (n < 0 || (n > 0 && (!diag || !off || !inv_diag || !inv_off || !det))) return FASST_ERR_SHAPE;
  if (n == 0) return FASST_OK;
  DeviceGuard g(device);
  DBuf<double> dd, did, ddet;
  DBuf<double2> doff, dioff;
  int st;
  if ((st = dd.alloc((size_t)2 * n)) || (st = did.alloc((size_t)2 * n)) || (st = ddet.alloc(n)) ||
      (st = doff.alloc(n)) || (st = dioff.alloc(n)))
    return st;
  FASST_HIP(hipMemcpy(dd.p, diag, (size_t)2 * n * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(doff.p, off, (size_t)n * sizeof(double2), hipMemcpyHostToDevice));
  k_inv_herm<<<std::min((n + 255) / 256, 4096), 256>>>(n, dd.p, doff.p, did.p, dioff.p, ddet.p);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipDeviceSynchronize());
  FASST_HIP(hipMemcpy(inv_diag, did.p, (size_t)2 * n * sizeof(double), hipMemcpyDeviceToHost));
  FASST_HIP(hipMemcpy(inv_off, dioff.p, (size_t)n * sizeof(double2), hipMemcpyDeviceToHost));
  FASST_HIP(hipMemcpy(det, ddet.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
  return FASST_OK;
}

}  // extern "C"
