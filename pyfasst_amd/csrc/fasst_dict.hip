// SIMM source dictionary (KLGLOTT88 harmonic combs) on MI355X (gfx950), FP64.
//
// generate_WF0_TR_chirped (separateLeadFunctions.py:696-886) synthesises, for
// each of ~1100 F0s, a complex harmonic sum of up to Fs/(2 F0) partials over
// 2 NFT samples and keeps the power spectrum of ONE frame of its STFT: the
// reference materialises the full partials x samples outer product per F0
// ("Horribly slow", :744).  Here one workgroup per column synthesises only
// the wlen samples of that frame -- each sample's partial sum in the
// reference's order, with the reference's phase expression evaluated in the
// same double operations -- windows them into LDS and runs the radix-2 FFT in
// LDS; the column of |X|^2 is written straight into WF0.
#include "fasst_fft.h"
#include "fasst_odgd.h"
#include "../../include/fasst_dict.h"

#include <algorithm>
#include <cmath>

namespace fasst {

struct DictArgs {
  const double *f1, *f2;
  const int *np_;
  const double2 *amps;   // [n_cols][max_partials]
  const double *win;
  const double2 *tw;
  double *wf0;           // [nfft/2+1][n_cols]
  double fs;
  long frame_start;
  int n_cols, max_partials, length_odgd, wlen, nfft, logn;
};

__global__ __launch_bounds__(256) void k_wf0_column(const DictArgs a) {
  extern __shared__ __attribute__((aligned(16))) double2 sm[];
  double2 *buf = sm;                 // [nfft]
  double2 *amp = sm + a.nfft;        // [max_partials]
  const int j = blockIdx.x;
  const int P = a.np_[j];
  const double F1 = a.f1[j], F2 = a.f2[j];
  for (int h = threadIdx.x; h < P; h += blockDim.x) amp[h] = a.amps[(size_t)j * a.max_partials + h];
  __syncthreads();
  const double den = 2.0 * (double)a.length_odgd / a.fs;
  for (int i = threadIdx.x; i < a.nfft; i += blockDim.x) {
    double v = 0.0;
    const long t = a.frame_start + i;
    if (i < a.wlen && t >= 0 && t < a.length_odgd)
      v = a.win[i] * odgd_sample(amp, P, F1, F2, a.fs, den, t).x;
    buf[bitrev(i, a.logn)] = make_double2(v, 0.0);
  }
  __syncthreads();
  lds_fft(buf, a.tw, a.nfft, a.logn);
  for (int k = threadIdx.x; k <= a.nfft / 2; k += blockDim.x) {
    const double m = hypot(buf[k].x, buf[k].y);      // np.abs(X) ** 2
    a.wf0[(size_t)k * a.n_cols + j] = m * m;
  }
}

static float g_dict_ms = 0.f;

}  // namespace fasst

using namespace fasst;

extern "C" {

int dict_wf0_stft(int device, int n_cols, const double *f1, const double *f2,
                  const int *n_partials, int max_partials, const double *amps, double fs,
                  int length_odgd, const double *window, int wlen, int nfft, long frame_start,
                  double *wf0) {
  if (n_cols < 1 || max_partials < 1 || !f1 || !f2 || !n_partials || !amps || !window || !wf0 ||
      ilog2(nfft) < 1 || nfft > 8192 || wlen < 1 || wlen > nfft || length_odgd < 1 || fs <= 0) {
    set_error("dict_wf0_stft: bad shape (cols %d, partials %d, nfft %d, wlen %d)", n_cols,
              max_partials, nfft, wlen);
    return FASST_ERR_SHAPE;
  }
  for (int j = 0; j < n_cols; ++j)
    if (n_partials[j] < 0 || n_partials[j] > max_partials) {
      set_error("dict_wf0_stft: column %d has %d partials > %d", j, n_partials[j], max_partials);
      return FASST_ERR_SHAPE;
    }
  const size_t smem = ((size_t)nfft + max_partials) * sizeof(double2);
  if (smem > 160 * 1024) {
    set_error("dict_wf0_stft: nfft %d + %d partials exceed the LDS", nfft, max_partials);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  int st;
  const int F = nfft / 2 + 1;
  DBuf<double> d1, d2, dw, dout;
  DBuf<int> dnp;
  DBuf<double2> damps, dtw;
  if ((st = d1.alloc(n_cols)) || (st = d2.alloc(n_cols)) || (st = dnp.alloc(n_cols)) ||
      (st = damps.alloc((size_t)n_cols * max_partials)) || (st = dw.alloc(wlen)) ||
      (st = dtw.alloc(nfft / 2)) || (st = dout.alloc((size_t)F * n_cols)))
    return st;
  auto tw = twiddles(nfft, -1);
  FASST_HIP(hipMemcpy(d1.p, f1, n_cols * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(d2.p, f2, n_cols * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dnp.p, n_partials, n_cols * sizeof(int), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(damps.p, amps, (size_t)n_cols * max_partials * sizeof(double2),
                      hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dw.p, window, wlen * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dtw.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice));
  if (smem > 64 * 1024)
    FASST_HIP(hipFuncSetAttribute((const void *)k_wf0_column,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  DictArgs a;
  a.f1 = d1.p;
  a.f2 = d2.p;
  a.np_ = dnp.p;
  a.amps = damps.p;
  a.win = dw.p;
  a.tw = dtw.p;
  a.wf0 = dout.p;
  a.fs = fs;
  a.frame_start = frame_start;
  a.n_cols = n_cols;
  a.max_partials = max_partials;
  a.length_odgd = length_odgd;
  a.wlen = wlen;
  a.nfft = nfft;
  a.logn = ilog2(nfft);
  hipEvent_t e0, e1;
  FASST_HIP(hipEventCreate(&e0));
  FASST_HIP(hipEventCreate(&e1));
  FASST_HIP(hipEventRecord(e0, 0));
  k_wf0_column<<<n_cols, 256, smem>>>(a);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipEventRecord(e1, 0));
  FASST_HIP(hipEventSynchronize(e1));
  FASST_HIP(hipEventElapsedTime(&g_dict_ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  FASST_HIP(hipMemcpy(wf0, dout.p, (size_t)F * n_cols * sizeof(double), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int dict_last_ms(double *device_ms) {
  if (device_ms) *device_ms = g_dict_ms;
  return FASST_OK;
}

}  // extern "C"
