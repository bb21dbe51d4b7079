// Constant-Q (CQT) and minimum-Q (MinQT) transforms on MI355X (gfx950), FP64.
//
// The reference's rasterised transform (tftransforms/minqt.py:471-646, the
// perfRast=1 branch FASST always uses, audioModel.py:206-214) processes one
// octave at a time on a signal that is low-pass filtered and decimated by 2
// between octaves:
//   frames     nframes FFTs of FFTLen samples, hop fftHOP           (:569-578)
//   kernel     for each of 2^i time shifts, CQTframe = (K . phase) XX  (:579-597)
//   raster     scatter into spCQT rows, then the "drop" alignment    (:598-642)
//   filtfilt   6th-order Butterworth, forward-backward, then x[::2]  (:644-646)
// MinQT adds the linear-frequency STFT bins above the CQT range
// (computeLinearPart, :1410-1450).
//
// MI355X mapping:
//   k_cqt_frames   one block per frame: radix-2 FFT in LDS (FFTLen <= 8192,
//                  128 KB); only the kernel's non-zero band [kb, ke) of bins is
//                  kept (the thresholded one-octave kernel is zero outside a
//                  narrow band: 87 of 4096 bins for FASST's MinQT defaults).
//   k_cqt_band     per (16-frame tile, shift): the band of the 16 spectra times
//                  the shift's phase ramp staged in LDS, then the M x band
//                  complex contraction on the VALU (M = bins*winNr <= a few
//                  hundred: far too small a K for MFMA to pay), written
//                  straight to the rasterised, drop-aligned spCQT position.
//   k_iir_fwd/bwd  filtfilt as two passes of a chunked DF2T recurrence: each
//                  thread owns 128 outputs and starts `warm` samples early
//                  from a zero state (exact initial state zi*x0 on chunk 0);
//                  the filter's state transition decays below 1e-24 within
//                  `warm` samples (checked on the host from the actual
//                  coefficients), so the start-up error is far below FP64
//                  rounding.  The per-sample arithmetic is scipy's lfilter
//                  (DOUBLE_filt) operation for operation, without FMA
//                  contraction.  The backward pass fuses the decimation
//                  (forward transform) or the x2 gain (inverse).
//   k_cqt_linear   MinQT linear part: per frame, rfft in LDS of the windowed
//                  frame, bins Kmax.. written to the linear rows.
// Inverse (invertFromSpCQTRast :794-868 / invertFromCellCQT :1019-1055, then
// invertLinearPart :1469-1485): per frame, the band spectrum sparKernel . cell
// (the cell gathered from spCQT exactly as spCQT2CellCQT :949-1011 derives it,
// including the left-shifted rows of each rasterised shift), inverse FFT in
// LDS, then a deterministic gather overlap-add in the reference's (shift,
// frame) summation order; upsampling through the same filtfilt kernels.
//
// Internal spCQT layout: frame-major [W][F] (bins contiguous, the FASST
// engine's device layout); the C ABI hands out [F][W].
#include "fasst_fft.h"
#include "fasst_odgd.h"
#include "../../include/fasst_cqt.h"

#include <algorithm>
#include <cmath>

namespace fasst {

constexpr int kIirPad = 21;       // scipy filtfilt padlen = 3 * max(len(a), len(b))
constexpr int kIirOrder = 6;
constexpr int kIirChunk = 128;    // outputs per thread
constexpr int kBandFrames = 16;   // frames per k_cqt_band block
constexpr int kMaxCqtFFT = 8192;  // FFTLen in LDS (128 KB)

struct Iir {
  double b[kIirOrder + 1], a[kIirOrder + 1], zi[kIirOrder];
};

__device__ __forceinline__ double iir_src(const double *__restrict__ x, long i, int up) {
  return up ? ((i & 1) ? 0.0 : x[i >> 1]) : x[i];
}

// element j of scipy's odd extension (filtfilt padtype='odd', padlen 21) of
// the n-sample source; up = 1 reads the zero-stuffed upsampled signal
// (newy[::2] = y, minqt.py:855-856)
__device__ double iir_ext(const double *__restrict__ x, long n, long j, int up) {
#pragma clang fp contract(off)
  if (j < kIirPad) return 2.0 * iir_src(x, 0, up) - iir_src(x, kIirPad - j, up);
  if (j < n + kIirPad) return iir_src(x, j - kIirPad, up);
  return 2.0 * iir_src(x, n - 1, up) - iir_src(x, n - 2 - (j - n - kIirPad), up);
}

// one step of scipy.signal.lfilter's direct form II transposed (DOUBLE_filt)
__device__ __forceinline__ double iir_step(const Iir &f, double *z, double x) {
#pragma clang fp contract(off)
  const double y = z[0] + f.b[0] * x;
#pragma unroll
  for (int k = 0; k < kIirOrder - 1; ++k) z[k] = z[k + 1] + x * f.b[k + 1] - y * f.a[k + 1];
  z[kIirOrder - 1] = x * f.b[kIirOrder] - y * f.a[kIirOrder];
  return y;
}

// forward pass: y1 = lfilter(b, a, ext, zi * ext[0]), ne = n + 42 samples
__global__ __launch_bounds__(256) void k_iir_fwd(const double *__restrict__ x, long n, int up,
                                                 const Iir f, int warm, double *__restrict__ y1) {
  const long ne = n + 2 * kIirPad;
  const long j1 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * kIirChunk;
  if (j1 >= ne) return;
  const long j2 = min(ne, j1 + kIirChunk);
  const long j0 = max(0L, j1 - warm);
  const double x0 = j0 == 0 ? iir_ext(x, n, 0, up) : 0.0;
  double z[kIirOrder];
#pragma unroll
  for (int k = 0; k < kIirOrder; ++k) z[k] = f.zi[k] * x0;
  for (long j = j0; j < j2; ++j) {
    const double y = iir_step(f, z, iir_ext(x, n, j, up));
    if (j >= j1) y1[j] = y;
  }
}

// backward pass on the reversed y1 with zi * y1[-1]; output sample p of the
// n-sample result is reversed index ne-1-21-p.  decim: out[p/2] for even p
// (x[::2], minqt.py:646); else out[p] = scale * y.
__global__ __launch_bounds__(256) void k_iir_bwd(const double *__restrict__ y1, long n,
                                                 const Iir f, int warm, double *__restrict__ out,
                                                 int decim, double scale) {
  const long ne = n + 2 * kIirPad;
  const long j1 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * kIirChunk;
  if (j1 >= ne) return;
  const long j2 = min(ne, j1 + kIirChunk);
  const long j0 = max(0L, j1 - warm);
  const double x0 = j0 == 0 ? y1[ne - 1] : 0.0;
  double z[kIirOrder];
#pragma unroll
  for (int k = 0; k < kIirOrder; ++k) z[k] = f.zi[k] * x0;
  for (long j = j0; j < j2; ++j) {
    const double y = iir_step(f, z, y1[ne - 1 - j]);
    if (j < j1) continue;
    const long p = ne - 1 - kIirPad - j;
    if (p < 0 || p >= n) continue;
    if (decim) {
      if (!(p & 1)) out[p >> 1] = y;
    } else {
      out[p] = y * scale;
    }
  }
}

// XX[n][k - kb] = fft(x[n hop : n hop + N])[k] for k in the kernel band
__global__ __launch_bounds__(256) void k_cqt_frames(const double *__restrict__ x, long len, int hop,
                                                    const double2 *__restrict__ tw, int N, int logN,
                                                    int kb, int nb, int nbp,
                                                    double2 *__restrict__ XX) {
  extern __shared__ __attribute__((aligned(16))) double2 buf[];
  const long s0 = (long)blockIdx.x * hop;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const long s = s0 + i;
    buf[bitrev(i, logN)] = make_double2(s < len ? x[s] : 0.0, 0.0);
  }
  __syncthreads();
  lds_fft(buf, tw, N, logN);
  double2 *o = XX + (size_t)blockIdx.x * nbp;
  for (int k = threadIdx.x; k < nb; k += blockDim.x) o[k] = buf[kb + k];
}

struct BandArgs {
  const double2 *K;   // [M][nbp]: conj(sparKernel.T), band columns
  const double2 *XX;  // [nfr][nbp]
  double2 *sp;        // [W][F] frame-major spCQT
  int M, nb, nbp, kb, N, nfr, win_nr, nshifts, row0, W, F;
  long d;             // drop alignment of this octave, int(drop * nshifts)
  double inc;         // atomHOP / 2^i
};

// CQTframe_s = (K . exp(2 pi i k s inc / N)) XX for one tile of 16 frames and
// one shift s; element (nb*winNr + a, n) goes to spCQT row row0 + nb, column
// c = s + a*2^i + n*winNr*2^i (minqt.py:613-619, :633-636), then the drop
// alignment row[:W-d] = row[d:] (:639-642): c -> c - d, and the last d
// columns keep their own pre-alignment values.
__global__ __launch_bounds__(256) void k_cqt_band(const BandArgs a) {
  extern __shared__ __attribute__((aligned(16))) double2 sx[];  // [kBandFrames][nbp]
  const int n0 = blockIdx.x * kBandFrames, s = blockIdx.y;
  const double shift = (double)s * a.inc;
  for (int idx = threadIdx.x; idx < kBandFrames * a.nb; idx += blockDim.x) {
    const int fr = idx / a.nb, kk = idx - fr * a.nb;
    const int n = n0 + fr;
    double2 v = make_double2(0.0, 0.0);
    if (n < a.nfr) {
      // np.exp(1j * 2 * np.pi * np.arange(N) * shift / N)   (:590-592)
      const double ang = 2.0 * M_PI * (double)(a.kb + kk) * shift / (double)a.N;
      double sn, cs;
      sincos(ang, &sn, &cs);
      const double2 xx = a.XX[(size_t)n * a.nbp + kk];
      v = make_double2(xx.x * cs - xx.y * sn, xx.x * sn + xx.y * cs);
    }
    sx[fr * a.nbp + kk] = v;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < a.M * kBandFrames; idx += blockDim.x) {
    const int m = idx / kBandFrames, fr = idx - m * kBandFrames;
    const int n = n0 + fr;
    if (n >= a.nfr) continue;
    const double2 *kr = a.K + (size_t)m * a.nbp;
    const double2 *xr = sx + fr * a.nbp;
    double re = 0.0, im = 0.0;
    for (int kk = 0; kk < a.nb; ++kk) {
      const double2 k = kr[kk], x = xr[kk];
      re += k.x * x.x - k.y * x.y;
      im += k.x * x.y + k.y * x.x;
    }
    const int nbin = m / a.win_nr, at = m - nbin * a.win_nr;
    const long c = (long)s + (long)at * a.nshifts + (long)n * a.win_nr * a.nshifts;
    const double2 v = make_double2(re, im);
    const size_t row = (size_t)(a.row0 + nbin);
    if (c >= a.d) a.sp[(size_t)(c - a.d) * a.F + row] = v;
    if (c >= (long)a.W - a.d && c < a.W) a.sp[(size_t)c * a.F + row] = v;
  }
}

// MinQT linear part (minqt.py:1420-1435 with stft.py:3-69): frame n of the
// STFT of xpad[first_center:] (half-window zero prefix), bins kmax..N/2 to
// the linear rows of spCQT column n - drop, for n in [drop, W).
__global__ __launch_bounds__(256) void k_cqt_linear(const double *__restrict__ xp, long lp, long off,
                                                    const double *__restrict__ win,
                                                    const double2 *__restrict__ tw, int N, int logN,
                                                    int hop, int drop, int kmax, int row0, int F,
                                                    double2 *__restrict__ sp) {
  extern __shared__ __attribute__((aligned(16))) double2 buf[];
  const int n = drop + blockIdx.x;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const long s = off + (long)n * hop + i;
    const double v = (s >= 0 && s < lp) ? win[i] * xp[s] : 0.0;
    buf[bitrev(i, logN)] = make_double2(v, 0.0);
  }
  __syncthreads();
  lds_fft(buf, tw, N, logN);
  double2 *o = sp + (size_t)blockIdx.x * F + row0 - kmax;
  for (int k = kmax + threadIdx.x; k <= N / 2; k += blockDim.x) o[k] = buf[k];
}

// [W][F] <-> [F][W] complex transposes through a 16x16 LDS tile
__global__ __launch_bounds__(256) void k_cqt_transpose(const double2 *__restrict__ src,
                                                       double2 *__restrict__ dst, int rows,
                                                       int cols) {
  __shared__ double2 t[16][17];
  const int c0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  if (r0 + ty < rows && c0 + tx < cols) t[ty][tx] = src[(size_t)(r0 + ty) * cols + c0 + tx];
  __syncthreads();
  if (c0 + ty < cols && r0 + tx < rows) dst[(size_t)(c0 + ty) * rows + r0 + tx] = t[tx][ty];
}

struct ICellArgs {
  const double2 *sp;   // [W][F]
  const double2 *S;    // [nb][M]: sparKernel rows kb..ke-1
  double *frames;      // [nfr][N]
  const double2 *tw;   // inverse twiddles
  int N, logN, kb, nb, M, F, W, win_nr, row0, step, shift, nfr;
  long dropped, ncolx;
  double ns;           // divisor of the rasterised inverse (nshifts), 1 for cells
};

// cell[m][n] of spCQT2CellCQT (minqt.py:966-1011) for the octave whose rows
// start at row0 (step = 2^noct), from spCQT shifted left `shift` times
// (minqt.py:845-851: the last column repeats)
__device__ __forceinline__ double2 cell_at(const ICellArgs &a, int m, int n) {
  const int nbin = m / a.win_nr, at = m - nbin * a.win_nr;
  const long j = (long)n * a.win_nr + at;
  if (j < a.dropped) return make_double2(0.0, 0.0);
  const long q = j - a.dropped;
  if (q >= a.ncolx) return make_double2(0.0, 0.0);
  const long c = min(q * a.step + a.shift, (long)a.W - 1);
  return a.sp[(size_t)c * a.F + a.row0 + nbin];
}

// frame n: 2 Re(ifft(sparKernel . cell[:, n])) / ns   (minqt.py:829-839, :1028-1041)
__global__ __launch_bounds__(256) void k_icqt_frames(const ICellArgs a) {
  extern __shared__ __attribute__((aligned(16))) double2 buf[];  // [N] + [M] cell column
  double2 *cell = buf + a.N;
  const int n = blockIdx.x;
  for (int i = threadIdx.x; i < a.N; i += blockDim.x) buf[i] = make_double2(0.0, 0.0);
  for (int m = threadIdx.x; m < a.M; m += blockDim.x) cell[m] = cell_at(a, m, n);
  __syncthreads();
  for (int kk = threadIdx.x; kk < a.nb; kk += blockDim.x) {
    const double2 *sr = a.S + (size_t)kk * a.M;
    double re = 0.0, im = 0.0;
    for (int m = 0; m < a.M; ++m) {
      const double2 s = sr[m], c = cell[m];
      re += s.x * c.x - s.y * c.y;
      im += s.x * c.y + s.y * c.x;
    }
    buf[bitrev(a.kb + kk, a.logN)] = make_double2(re, im);
  }
  __syncthreads();
  lds_fft(buf, a.tw, a.N, a.logN);
  const double invN = 1.0 / (double)a.N;
  double *o = a.frames + (size_t)n * a.N;
  for (int t = threadIdx.x; t < a.N; t += blockDim.x) o[t] = 2.0 * ((buf[t].x * invN) / a.ns);
}

// y[p] += sum_n frame_n[p - a_n], a_n = int(n hop + off), frames in order
// (the reference's y[a:a+N] += yoct, minqt.py:840, :1042)
__global__ void k_icqt_ola(const double *__restrict__ frames, int nfr, int N, int hop, double off,
                           double *__restrict__ y, long ylen) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ylen) return;
  long nlo = (long)floor(((double)p - (double)N + 1.0 - off) / hop) - 1;
  long nhi = (long)floor(((double)p - off) / hop) + 1;
  nlo = max(nlo, 0L);
  nhi = min(nhi, (long)nfr - 1);
  double acc = y[p];
  for (long n = nlo; n <= nhi; ++n) {
    const long s = (long)((double)n * hop + off);
    if (s <= p && p < s + N) acc += frames[(size_t)n * N + (p - s)];
  }
  y[p] = acc;
}

// MinQT linear inverse frames: window * irfft(Y[:, n])[:N] with
// Y[kmax + r][n] = spCQT[row0 + r][n - dropped] (minqt.py:1476-1482, stft.py:108-113)
__global__ __launch_bounds__(256) void k_icqt_lin_frames(const double2 *__restrict__ sp, int F,
                                                         int row0, int kmax, long dropped,
                                                         const double *__restrict__ win,
                                                         const double2 *__restrict__ tw, int N,
                                                         int logN, double *__restrict__ frames) {
  extern __shared__ __attribute__((aligned(16))) double2 buf[];
  const int n = blockIdx.x, h = N / 2;
  const double2 *col = n >= dropped ? sp + (size_t)(n - dropped) * F + row0 - kmax : nullptr;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const int k = i <= h ? i : N - i;
    double2 v = make_double2(0.0, 0.0);
    if (col && k >= kmax) v = col[k];
    if (i == 0 || i == h) v.y = 0.0;
    else if (i > h) v.y = -v.y;
    buf[bitrev(i, logN)] = v;
  }
  __syncthreads();
  lds_fft(buf, tw, N, logN);
  const double invN = 1.0 / (double)N;
  for (int t = threadIdx.x; t < N; t += blockDim.x)
    frames[(size_t)n * N + t] = win[t] * (buf[t].x * invN);
}

// y[p] += istft(...)[p + off] with the window-product normalisation (stft.py:114-129)
__global__ void k_icqt_lin_ola(const double *__restrict__ frames, int nfr, int N, int hop,
                               const double *__restrict__ win, long off, double *__restrict__ y,
                               long L) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= L) return;
  const long s = p + off;
  long nlo = (s - N) / hop + 1;
  if (s - N < 0) nlo = 0;
  const long nhi = min(s / hop, (long)nfr - 1);
  double acc = 0.0, nrm = 0.0;
  for (long n = nlo; n <= nhi; ++n) {
    const long q = s - n * hop;
    if (q < 0 || q >= N) continue;
    nrm = nrm + win[q] * win[q];
    acc = acc + frames[(size_t)n * N + q];
  }
  y[p] = y[p] + acc / (nrm == 0.0 ? 1.0 : nrm);
}

// SIMM source dictionary on a CQT / MinQT (generate_WF0_TR_chirped with a
// CQT-type transform, separateLeadFunctions.py:742-886): the complex KLGLOTT88
// comb of L samples, real and imaginary parts, one thread per sample
__global__ __launch_bounds__(256) void k_odgd_synth(const double2 *__restrict__ amps, int P,
                                                    double F1, double F2, double fs, long L,
                                                    double *__restrict__ re,
                                                    double *__restrict__ im) {
  extern __shared__ __attribute__((aligned(16))) double2 amp[];
  for (int h = threadIdx.x; h < P; h += blockDim.x) amp[h] = amps[h];
  __syncthreads();
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  const double2 z = odgd_sample(amp, P, F1, F2, fs, 2.0 * (double)L / fs, t);
  re[t] = z.x;
  im[t] = z.y;
}

// column `col` of the transform ([W][F] frame-major) -> WF0[:, j]:
// pass 0 keeps T(Re odgd); pass 1 forms T(odgd) = T(Re) + i T(Im) on the CQT
// rows (the transform is linear in the signal) and T(Re) on the MinQT linear
// rows (computeLinearPart's rfft keeps the real part of its frames), then
// |.|^2 (np.abs(transfo[:, midindex]) ** 2)
__global__ __launch_bounds__(256) void k_wf0_take(const double2 *__restrict__ sp, int F, int col,
                                                  int ncq, int pass, double2 *__restrict__ keep,
                                                  double *__restrict__ wf0, int n_cols, int j) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F) return;
  const double2 v = sp[(size_t)col * F + k];
  if (pass == 0) {
    keep[k] = v;
    return;
  }
  const double2 r = keep[k];
  const double2 z = k < ncq ? make_double2(r.x - v.y, r.y + v.x) : r;
  const double m = hypot(z.x, z.y);
  wf0[(size_t)k * n_cols + j] = m * m;
}

}  // namespace fasst

using namespace fasst;

struct cqt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int bins = 0, oct = 0, win_nr = 0, N = 0, logN = 0, fft_hop = 0, atom_hop = 0, first_center = 0;
  int M = 0, kb = 0, nb = 0, nbp = 0;
  int lin_N = 0, lin_logN = 0, kmax = 0, lin_bins = 0;
  Iir iir{};
  int warm = 256;
  DBuf<double2> K, S, tw_f, tw_i, ltw_f, ltw_i;
  DBuf<double> lwin;
  // work space, sized for the last signal length
  long cap_L = -1;
  DBuf<double> xp, sa, sb, y1, frames, yb, yc;
  DBuf<double2> XX, sp, sph;
  // device time of the last forward / inverse (HIP events on the ctx stream,
  // after the host->device copy and before the device->host copy)
  hipEvent_t ev[4] = {};
  float ms_fwd = 0.f, ms_inv = 0.f;
};

namespace {

struct Geo {
  long maxBlock = 0, Lp = 0;
  int W = 0, F = 0, drop0 = 0;
  std::vector<long> len;     // signal length entering octave i
  std::vector<int> nfr;      // frames of octave i
  std::vector<long> d;       // drop alignment of octave i (columns)
};

int geometry(const cqt_ctx *c, long L, Geo &g) {
  if (L < 1) {
    set_error("empty signal");
    return FASST_ERR_SHAPE;
  }
  g.maxBlock = (long)c->N << (c->oct - 1);
  g.Lp = L + 2 * g.maxBlock;
  g.len.assign(c->oct, 0);
  g.nfr.assign(c->oct, 0);
  g.d.assign(c->oct, 0);
  long len = g.Lp;
  for (int i = 0; i < c->oct; ++i) {
    g.len[i] = len;
    const double nf = std::floor((double)(len - c->N) / (double)c->fft_hop + 1.0);
    if (nf < 1.0) {
      set_error("octave %d: signal of %ld samples shorter than FFTLen %d", i, len, c->N);
      return FASST_ERR_SHAPE;
    }
    g.nfr[i] = (int)nf;
    if (i != c->oct - 1) {
      if (len <= kIirPad) {
        set_error("filtfilt: %ld samples <= padlen %d", len, kIirPad);
        return FASST_ERR_SHAPE;
      }
      len = (len + 1) / 2;
    }
  }
  g.W = g.nfr[0] * c->win_nr;
  const double empty_hops = (double)c->first_center / (double)c->atom_hop;
  for (int i = 0; i < c->oct; ++i) {
    const long ns = 1L << i;
    if ((long)g.nfr[i] * c->win_nr * ns > g.W) {
      set_error("octave %d: %d frames do not fit the raster of width %d", i, g.nfr[i], g.W);
      return FASST_ERR_SHAPE;
    }
    const double drop = empty_hops * (double)((1L << (c->oct - i - 1)) - 1);
    g.d[i] = (long)(drop * (double)ns);
  }
  g.F = c->bins * c->oct;
  if (c->lin_N) {
    g.F += c->lin_bins;
    const long tlin = (long)std::ceil((double)(g.Lp - c->first_center) / (double)c->atom_hop) + 2;
    if (tlin < g.W) {
      set_error("linear part: %ld frames < raster width %d", tlin, g.W);
      return FASST_ERR_SHAPE;
    }
    g.drop0 = (int)(empty_hops * (double)((1L << (c->oct - 1)) - 1));
  }
  return FASST_OK;
}

int ensure_work(cqt_ctx *c, const Geo &g, long L) {
  if (c->cap_L == L) return FASST_OK;
  int st;
  const long ext = g.Lp + 2 * kIirPad;
  // inverse y: at most Lp grown by one frame extent per octave, doubled per octave
  const long ycap = 2 * (g.Lp + 2L * c->N + 4L * c->fft_hop) + 64;
  size_t fr = 0;
  for (int i = 0; i < c->oct; ++i) fr = std::max(fr, (size_t)g.nfr[i] * c->N);
  if (c->lin_N) fr = std::max(fr, (size_t)g.W * c->lin_N);
  if ((st = c->xp.alloc(g.Lp)) || (st = c->sa.alloc(g.Lp / 2 + 2)) ||
      (st = c->sb.alloc(g.Lp / 2 + 2)) || (st = c->y1.alloc(std::max(ext, 2 * ycap + 64))) ||
      (st = c->XX.alloc((size_t)g.nfr[0] * c->nbp)) || (st = c->sp.alloc((size_t)g.W * g.F)) ||
      (st = c->sph.alloc((size_t)g.W * g.F)) || (st = c->frames.alloc(fr)) ||
      (st = c->yb.alloc(ycap)) || (st = c->yc.alloc(ycap)))
    return st;
  c->cap_L = L;
  return FASST_OK;
}

int filtfilt(cqt_ctx *c, const double *src, long n, int up, double *out, int decim, double scale) {
  if (n <= kIirPad) {
    set_error("filtfilt: %ld samples <= padlen %d", n, kIirPad);
    return FASST_ERR_SHAPE;
  }
  const long ne = n + 2 * kIirPad;
  const int grid = (int)((ne + (long)kIirChunk * 256 - 1) / ((long)kIirChunk * 256));
  k_iir_fwd<<<grid, 256, 0, c->stream>>>(src, n, up, c->iir, c->warm, c->y1.p);
  FASST_LAUNCH_CHECK();
  k_iir_bwd<<<grid, 256, 0, c->stream>>>(c->y1.p, n, c->iir, c->warm, out, decim, scale);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int set_smem(const void *fn, size_t bytes) {
  if (bytes > 64 * 1024)
    FASST_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return FASST_OK;
}

// the transform of the padded signal in c->xp into c->sp ([W][F], frame-major)
int forward_dev(cqt_ctx *c, const Geo &g, hipStream_t s) {
  int st;
  FASST_HIP(hipMemsetAsync(c->sp.p, 0, (size_t)g.W * g.F * sizeof(double2), s));
  if (c->lin_N && g.W > g.drop0) {   // computeLinearPart on the padded signal
    const long off = (long)c->first_center - c->lin_N / 2;
    k_cqt_linear<<<g.W - g.drop0, 256, c->lin_N * sizeof(double2), s>>>(
        c->xp.p, g.Lp, off, c->lwin.p, c->ltw_f.p, c->lin_N, c->lin_logN, c->atom_hop, g.drop0,
        c->kmax, c->bins * c->oct, g.F, c->sp.p);
    FASST_LAUNCH_CHECK();
  }
  const double *cur = c->xp.p;
  double *next = c->sa.p;
  for (int i = 0; i < c->oct; ++i) {
    const int nfr = g.nfr[i];
    if (c->nb > 0) {
      k_cqt_frames<<<nfr, 256, c->N * sizeof(double2), s>>>(cur, g.len[i], c->fft_hop, c->tw_f.p,
                                                           c->N, c->logN, c->kb, c->nb, c->nbp,
                                                           c->XX.p);
      FASST_LAUNCH_CHECK();
      BandArgs a;
      a.K = c->K.p;
      a.XX = c->XX.p;
      a.sp = c->sp.p;
      a.M = c->M;
      a.nb = c->nb;
      a.nbp = c->nbp;
      a.kb = c->kb;
      a.N = c->N;
      a.nfr = nfr;
      a.win_nr = c->win_nr;
      a.nshifts = 1 << i;
      a.row0 = c->bins * (c->oct - i - 1);
      a.W = g.W;
      a.F = g.F;
      a.d = g.d[i];
      a.inc = (double)c->atom_hop / (double)(1L << i);
      k_cqt_band<<<dim3((nfr + kBandFrames - 1) / kBandFrames, 1 << i), 256,
                   kBandFrames * c->nbp * sizeof(double2), s>>>(a);
      FASST_LAUNCH_CHECK();
    }
    if (i != c->oct - 1) {
      if ((st = filtfilt(c, cur, g.len[i], 0, next, 1, 1.0))) return st;
      cur = next;
      next = (next == c->sa.p) ? c->sb.p : c->sa.p;
    }
  }
  return FASST_OK;
}

}  // namespace

extern "C" {

int cqt_create(int device, int bins, int octave_nr, int win_nr, int fft_len, int fft_hop,
               int atom_hop, int first_center, const double *spar_kernel, const double *iir_b,
               const double *iir_a, const double *iir_zi, int lin_ft_len, int kmax, int lin_bins,
               const double *lin_window, cqt_ctx **out) {
  if (!out || !spar_kernel || !iir_b || !iir_a || !iir_zi) return FASST_ERR_SHAPE;
  *out = nullptr;
  if (bins < 1 || octave_nr < 1 || octave_nr > 24 || win_nr < 1 || ilog2(fft_len) < 1 ||
      fft_len > kMaxCqtFFT || fft_hop < 1 || atom_hop < 1 || first_center < 0) {
    set_error("bad CQT geometry (bins %d, octaves %d, winNr %d, FFTLen %d <= %d)", bins, octave_nr,
              win_nr, fft_len, kMaxCqtFFT);
    return FASST_ERR_SHAPE;
  }
  if (lin_ft_len && (ilog2(lin_ft_len) < 1 || lin_ft_len > kMaxCqtFFT || !lin_window ||
                     kmax < 0 || lin_bins != lin_ft_len / 2 - kmax + 1)) {
    set_error("bad MinQT linear part (linFTLen %d, Kmax %d, linBins %d)", lin_ft_len, kmax,
              lin_bins);
    return FASST_ERR_SHAPE;
  }
  if (iir_a[0] != 1.0) {
    set_error("anti-aliasing filter must be normalised (a[0] = 1)");
    return FASST_ERR_SHAPE;
  }
  cqt_ctx *c = new cqt_ctx();
  c->device = device;
  c->bins = bins;
  c->oct = octave_nr;
  c->win_nr = win_nr;
  c->N = fft_len;
  c->logN = ilog2(fft_len);
  c->fft_hop = fft_hop;
  c->atom_hop = atom_hop;
  c->first_center = first_center;
  c->M = bins * win_nr;
  c->lin_N = lin_ft_len;
  c->lin_logN = lin_ft_len ? ilog2(lin_ft_len) : 0;
  c->kmax = kmax;
  c->lin_bins = lin_bins;
  for (int k = 0; k <= kIirOrder; ++k) {
    c->iir.b[k] = iir_b[k];
    c->iir.a[k] = iir_a[k];
  }
  for (int k = 0; k < kIirOrder; ++k) c->iir.zi[k] = iir_zi[k];
  // warm-up length: smallest multiple of 32 with max|A^w| < 1e-24 (A: the
  // DF2T state transition of the filter)
  {
    double A[kIirOrder][kIirOrder] = {}, P[kIirOrder][kIirOrder] = {}, T[kIirOrder][kIirOrder];
    for (int r = 0; r < kIirOrder; ++r) {
      A[r][0] = -iir_a[r + 1];
      if (r + 1 < kIirOrder) A[r][r + 1] = 1.0;
      P[r][r] = 1.0;
    }
    int w = 0;
    double mx = 1.0;
    while (mx >= 1e-24 && w < 16384) {
      for (int r = 0; r < kIirOrder; ++r)
        for (int q = 0; q < kIirOrder; ++q) {
          double s = 0.0;
          for (int u = 0; u < kIirOrder; ++u) s += A[r][u] * P[u][q];
          T[r][q] = s;
        }
      mx = 0.0;
      for (int r = 0; r < kIirOrder; ++r)
        for (int q = 0; q < kIirOrder; ++q) {
          P[r][q] = T[r][q];
          mx = std::max(mx, std::fabs(T[r][q]));
        }
      ++w;
    }
    if (mx >= 1e-24) {
      delete c;
      set_error("anti-aliasing filter is not stable enough for the chunked filtfilt");
      return FASST_ERR_SHAPE;
    }
    c->warm = (w + 31) / 32 * 32;
  }
  // kernel band: bins k where any atom of sparKernel is non-zero
  const size_t M = c->M;
  int kb = fft_len, ke = 0;
  for (int k = 0; k < fft_len; ++k)
    for (size_t m = 0; m < M; ++m) {
      const double *z = spar_kernel + 2 * ((size_t)k * M + m);
      if (z[0] != 0.0 || z[1] != 0.0) {
        kb = std::min(kb, k);
        ke = std::max(ke, k + 1);
      }
    }
  if (ke <= kb) kb = ke = 0;
  c->kb = kb;
  c->nb = ke - kb;
  c->nbp = std::max(1, c->nb | 1);  // odd pitch: LDS rows of the band tile land on distinct banks
  if ((size_t)kBandFrames * c->nbp * sizeof(double2) > 160 * 1024) {
    delete c;
    set_error("CQT kernel band of %d bins exceeds the LDS tile", c->nb);
    return FASST_ERR_SHAPE;
  }
  std::vector<double2> hK(M * c->nbp, make_double2(0.0, 0.0)), hS((size_t)std::max(c->nb, 1) * M);
  for (int kk = 0; kk < c->nb; ++kk)
    for (size_t m = 0; m < M; ++m) {
      const double *z = spar_kernel + 2 * ((size_t)(kb + kk) * M + m);
      hK[m * c->nbp + kk] = make_double2(z[0], -z[1]);   // K = conj(sparKernel.T)  (:492)
      hS[(size_t)kk * M + m] = make_double2(z[0], z[1]);
    }
  DeviceGuard g(device);
  int st;
  auto fail = [&](int s) {
    delete c;
    return s;
  };
  if ((st = c->K.alloc(hK.size())) || (st = c->S.alloc(hS.size())) ||
      (st = c->tw_f.alloc(fft_len / 2)) || (st = c->tw_i.alloc(fft_len / 2)))
    return fail(st);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(FASST_ERR_DEVICE);
  for (auto &e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(FASST_ERR_DEVICE);
  auto twf = twiddles(fft_len, -1), twi = twiddles(fft_len, +1);
  if (hipMemcpy(c->K.p, hK.data(), hK.size() * sizeof(double2), hipMemcpyHostToDevice) ||
      hipMemcpy(c->S.p, hS.data(), hS.size() * sizeof(double2), hipMemcpyHostToDevice) ||
      hipMemcpy(c->tw_f.p, twf.data(), twf.size() * sizeof(double2), hipMemcpyHostToDevice) ||
      hipMemcpy(c->tw_i.p, twi.data(), twi.size() * sizeof(double2), hipMemcpyHostToDevice))
    return fail(FASST_ERR_DEVICE);
  if (lin_ft_len) {
    if ((st = c->ltw_f.alloc(lin_ft_len / 2)) || (st = c->ltw_i.alloc(lin_ft_len / 2)) ||
        (st = c->lwin.alloc(lin_ft_len)))
      return fail(st);
    auto lf = twiddles(lin_ft_len, -1), li = twiddles(lin_ft_len, +1);
    if (hipMemcpy(c->ltw_f.p, lf.data(), lf.size() * sizeof(double2), hipMemcpyHostToDevice) ||
        hipMemcpy(c->ltw_i.p, li.data(), li.size() * sizeof(double2), hipMemcpyHostToDevice) ||
        hipMemcpy(c->lwin.p, lin_window, lin_ft_len * sizeof(double), hipMemcpyHostToDevice))
      return fail(FASST_ERR_DEVICE);
  }
  const int big = std::max(fft_len, lin_ft_len);
  if ((st = set_smem((const void *)k_cqt_frames, (size_t)fft_len * sizeof(double2))) ||
      (st = set_smem((const void *)k_icqt_frames, ((size_t)fft_len + M) * sizeof(double2))) ||
      (st = set_smem((const void *)k_cqt_band, (size_t)kBandFrames * c->nbp * sizeof(double2))) ||
      (lin_ft_len &&
       ((st = set_smem((const void *)k_cqt_linear, (size_t)lin_ft_len * sizeof(double2))) ||
        (st = set_smem((const void *)k_icqt_lin_frames, (size_t)lin_ft_len * sizeof(double2))))))
    return fail(st);
  (void)big;
  *out = c;
  return FASST_OK;
}

int cqt_destroy(cqt_ctx *c) {
  if (!c) return FASST_OK;
  {
    DeviceGuard g(c->device);
    if (c->stream) {
      (void)hipStreamSynchronize(c->stream);
      (void)hipStreamDestroy(c->stream);
    }
    for (auto &e : c->ev)
      if (e) (void)hipEventDestroy(e);
    delete c;
  }
  return FASST_OK;
}

int cqt_shape(cqt_ctx *c, long L, int *freqbins, int *width, int *nframes) {
  if (!c) return FASST_ERR_SHAPE;
  Geo g;
  int st = geometry(c, L, g);
  if (st) return st;
  if (freqbins) *freqbins = g.F;
  if (width) *width = g.W;
  if (nframes)
    for (int i = 0; i < c->oct; ++i) nframes[i] = g.nfr[i];
  return FASST_OK;
}

int cqt_forward(cqt_ctx *c, const double *x, long L, double *sp) {
  if (!c || !x || !sp) return FASST_ERR_SHAPE;
  Geo g;
  int st = geometry(c, L, g);
  if (st) return st;
  DeviceGuard dg(c->device);
  if ((st = ensure_work(c, g, L))) return st;
  hipStream_t s = c->stream;
  FASST_HIP(hipMemsetAsync(c->xp.p, 0, g.Lp * sizeof(double), s));
  FASST_HIP(hipMemcpyAsync(c->xp.p + g.maxBlock, x, L * sizeof(double), hipMemcpyHostToDevice, s));
  FASST_HIP(hipEventRecord(c->ev[0], s));
  if ((st = forward_dev(c, g, s))) return st;
  k_cqt_transpose<<<dim3((g.F + 15) / 16, (g.W + 15) / 16), 256, 0, s>>>(c->sp.p, c->sph.p, g.W,
                                                                          g.F);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipEventRecord(c->ev[1], s));
  FASST_HIP(hipMemcpyAsync(sp, c->sph.p, (size_t)g.W * g.F * sizeof(double2),
                           hipMemcpyDeviceToHost, s));
  FASST_HIP(hipStreamSynchronize(s));
  FASST_HIP(hipEventElapsedTime(&c->ms_fwd, c->ev[0], c->ev[1]));
  return FASST_OK;
}

int cqt_inverse(cqt_ctx *c, const double *sp, long L, double *y) {
  if (!c || !sp || !y) return FASST_ERR_SHAPE;
  Geo g;
  int st = geometry(c, L, g);
  if (st) return st;
  DeviceGuard dg(c->device);
  if ((st = ensure_work(c, g, L))) return st;
  hipStream_t s = c->stream;
  const bool rast = c->lin_N != 0;   // MinQT: invertFromSpCQTRast; CQT: invertFromCellCQT
  FASST_HIP(hipMemcpyAsync(c->sph.p, sp, (size_t)g.W * g.F * sizeof(double2),
                           hipMemcpyHostToDevice, s));
  FASST_HIP(hipEventRecord(c->ev[2], s));
  k_cqt_transpose<<<dim3((g.W + 15) / 16, (g.F + 15) / 16), 256, 0, s>>>(c->sph.p, c->sp.p, g.F,
                                                                          g.W);
  FASST_LAUNCH_CHECK();
  const double empty_hops = (double)c->first_center / (double)c->atom_hop;
  long ysize = (long)std::ceil((double)L / std::ldexp(1.0, c->oct - 1));
  const long ycap = (long)c->yb.n;
  double *ycur = c->yb.p, *yalt = c->yc.p;
  FASST_HIP(hipMemsetAsync(ycur, 0, ycap * sizeof(double), s));
  for (int noct = c->oct - 1; noct >= 0; --noct) {
    const long step = 1L << noct;
    const int ns = rast ? (int)step : 1;
    const double inc = (double)c->atom_hop / std::ldexp(1.0, noct);
    const long dropped = (long)(empty_hops * (std::ldexp(1.0, c->oct - noct - 1) - 1.0));
    const long ncolx = (g.W + step - 1) / step;
    const long ncell = (dropped + ncolx + c->win_nr - 1) / c->win_nr;
    int nfr = g.nfr[noct];
    if (ncell < nfr) {
      if (rast) {
        set_error("octave %d: %ld cells < %d frames", noct, ncell, nfr);
        return FASST_ERR_SHAPE;
      }
      nfr = (int)ncell;
    }
    const double ylen = (double)c->fft_hop * (nfr - 1) + c->N + (rast ? ns * inc : 0.0);
    if (ylen > (double)ysize) ysize += (long)(ylen - (double)ysize);
    if (ysize > ycap) {
      set_error("inverse CQT buffer overflow (%ld > %ld)", ysize, ycap);
      return FASST_ERR_SHAPE;
    }
    for (int sh = 0; sh < ns; ++sh) {
      ICellArgs a;
      a.sp = c->sp.p;
      a.S = c->S.p;
      a.frames = c->frames.p;
      a.tw = c->tw_i.p;
      a.N = c->N;
      a.logN = c->logN;
      a.kb = c->kb;
      a.nb = c->nb;
      a.M = c->M;
      a.F = g.F;
      a.W = g.W;
      a.win_nr = c->win_nr;
      a.row0 = c->bins * (c->oct - noct - 1);
      a.step = (int)step;
      a.shift = sh;
      a.nfr = nfr;
      a.dropped = dropped;
      a.ncolx = ncolx;
      a.ns = (double)ns;
      k_icqt_frames<<<nfr, 256, ((size_t)c->N + c->M) * sizeof(double2), s>>>(a);
      FASST_LAUNCH_CHECK();
      k_icqt_ola<<<(int)((ysize + 255) / 256), 256, 0, s>>>(c->frames.p, nfr, c->N, c->fft_hop,
                                                            rast ? sh * inc : 0.0, ycur, ysize);
      FASST_LAUNCH_CHECK();
    }
    if (noct != 0) {
      if (2 * ysize > ycap) {
        set_error("inverse CQT buffer overflow (%ld > %ld)", 2 * ysize, ycap);
        return FASST_ERR_SHAPE;
      }
      FASST_HIP(hipMemsetAsync(yalt, 0, ycap * sizeof(double), s));
      if ((st = filtfilt(c, ycur, 2 * ysize, 1, yalt, 0, 2.0))) return st;
      std::swap(ycur, yalt);
      ysize *= 2;
    }
  }
  if (ysize < g.maxBlock + L) {
    set_error("inverse CQT: %ld samples < prefix %ld + %ld", ysize, g.maxBlock, L);
    return FASST_ERR_SHAPE;
  }
  double *yout = ycur + g.maxBlock;   // y[prefixZeros:][:datalen_init]
  if (c->lin_N) {                     // + invertLinearPart (minqt.py:1469-1485)
    const long dropped0 = (long)(empty_hops * (std::ldexp(1.0, c->oct - 1) - 1.0));
    const long len_lin = (long)c->atom_hop * (g.W - 1) + c->lin_N - c->lin_N / 2;
    const long off = g.maxBlock - c->first_center;
    if (off < 0 || off + L > len_lin) {
      set_error("linear inverse: %ld samples < %ld", len_lin, off + L);
      return FASST_ERR_SHAPE;
    }
    k_icqt_lin_frames<<<g.W, 256, c->lin_N * sizeof(double2), s>>>(
        c->sp.p, g.F, c->bins * c->oct, c->kmax, dropped0, c->lwin.p, c->ltw_i.p, c->lin_N,
        c->lin_logN, c->frames.p);
    FASST_LAUNCH_CHECK();
    k_icqt_lin_ola<<<(int)((L + 255) / 256), 256, 0, s>>>(c->frames.p, g.W, c->lin_N, c->atom_hop,
                                                          c->lwin.p, off + c->lin_N / 2, yout, L);
    FASST_LAUNCH_CHECK();
  }
  FASST_HIP(hipEventRecord(c->ev[3], s));
  FASST_HIP(hipMemcpyAsync(y, yout, L * sizeof(double), hipMemcpyDeviceToHost, s));
  FASST_HIP(hipStreamSynchronize(s));
  FASST_HIP(hipEventElapsedTime(&c->ms_inv, c->ev[2], c->ev[3]));
  return FASST_OK;
}

int dict_wf0_cqt(cqt_ctx *c, int n_cols, const double *f1, const double *f2,
                 const int *n_partials, int max_partials, const double *amps, double fs,
                 long length_odgd, int col, double *wf0) {
  if (!c || n_cols < 1 || max_partials < 1 || !f1 || !f2 || !n_partials || !amps || !wf0 ||
      fs <= 0) {
    set_error("dict_wf0_cqt: bad arguments (cols %d, partials %d)", n_cols, max_partials);
    return FASST_ERR_SHAPE;
  }
  for (int j = 0; j < n_cols; ++j)
    if (n_partials[j] < 0 || n_partials[j] > max_partials) {
      set_error("dict_wf0_cqt: column %d has %d partials > %d", j, n_partials[j], max_partials);
      return FASST_ERR_SHAPE;
    }
  if ((size_t)max_partials * sizeof(double2) > 64 * 1024) {
    set_error("dict_wf0_cqt: %d partials exceed the LDS", max_partials);
    return FASST_ERR_SHAPE;
  }
  Geo g;
  int st = geometry(c, length_odgd, g);
  if (st) return st;
  if (col < 0 || col >= g.W) {
    set_error("dict_wf0_cqt: column %d outside the %d frames", col, g.W);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard dg(c->device);
  if ((st = ensure_work(c, g, length_odgd))) return st;
  const long L = length_odgd;
  DBuf<double2> damps, keep;
  DBuf<double> dim, dout;
  if ((st = damps.alloc((size_t)n_cols * max_partials)) || (st = keep.alloc(g.F)) ||
      (st = dim.alloc(L)) || (st = dout.alloc((size_t)g.F * n_cols)))
    return st;
  FASST_HIP(hipMemcpy(damps.p, amps, (size_t)n_cols * max_partials * sizeof(double2),
                      hipMemcpyHostToDevice));
  hipStream_t s = c->stream;
  FASST_HIP(hipMemsetAsync(c->xp.p, 0, g.Lp * sizeof(double), s));   // the zero padding
  FASST_HIP(hipEventRecord(c->ev[0], s));
  const int ncq = c->bins * c->oct;
  const int gF = (g.F + 255) / 256;
  for (int j = 0; j < n_cols; ++j) {
    k_odgd_synth<<<(int)((L + 255) / 256), 256, max_partials * sizeof(double2), s>>>(
        damps.p + (size_t)j * max_partials, n_partials[j], f1[j], f2[j], fs, L,
        c->xp.p + g.maxBlock, dim.p);
    FASST_LAUNCH_CHECK();
    if ((st = forward_dev(c, g, s))) return st;
    k_wf0_take<<<gF, 256, 0, s>>>(c->sp.p, g.F, col, ncq, 0, keep.p, dout.p, n_cols, j);
    FASST_LAUNCH_CHECK();
    FASST_HIP(hipMemcpyAsync(c->xp.p + g.maxBlock, dim.p, L * sizeof(double),
                             hipMemcpyDeviceToDevice, s));
    if ((st = forward_dev(c, g, s))) return st;
    k_wf0_take<<<gF, 256, 0, s>>>(c->sp.p, g.F, col, ncq, 1, keep.p, dout.p, n_cols, j);
    FASST_LAUNCH_CHECK();
  }
  FASST_HIP(hipEventRecord(c->ev[1], s));
  FASST_HIP(hipMemcpyAsync(wf0, dout.p, (size_t)g.F * n_cols * sizeof(double),
                           hipMemcpyDeviceToHost, s));
  FASST_HIP(hipStreamSynchronize(s));
  FASST_HIP(hipEventElapsedTime(&c->ms_fwd, c->ev[0], c->ev[1]));
  return FASST_OK;
}

int cqt_device_ms(cqt_ctx *c, double *forward_ms, double *inverse_ms) {
  if (!c) return FASST_ERR_SHAPE;
  if (forward_ms) *forward_ms = c->ms_fwd;
  if (inverse_ms) *inverse_ms = c->ms_inv;
  return FASST_OK;
}

}  // extern "C"
