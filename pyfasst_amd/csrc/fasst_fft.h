// Radix-2 complex FFT in LDS (FP64) shared by the STFT / iSTFT and the
// CQT / MinQT kernels, plus the host-side twiddle tables.
#pragma once
#include "fasst_common.h"

#include <cmath>

namespace fasst {

// In-LDS complex FFT of size N (power of two), data already in bit-reversed
// order.  tw[k] = exp(sign * 2 pi i k / N), k < N/2.
__device__ inline void lds_fft(double2 *x, const double2 *__restrict__ tw, int N, int logN) {
  for (int s = 0; s < logN; ++s) {
    const int m = 1 << s;
    const int stride = N >> (s + 1);
    for (int b = threadIdx.x; b < (N >> 1); b += blockDim.x) {
      const int grp = b >> s, pos = b & (m - 1);
      const int i0 = grp * 2 * m + pos, i1 = i0 + m;
      const double2 w = tw[pos * stride];
      const double2 u = x[i0], v = x[i1];
      const double2 t = make_double2(w.x * v.x - w.y * v.y, w.x * v.y + w.y * v.x);
      x[i0] = make_double2(u.x + t.x, u.y + t.y);
      x[i1] = make_double2(u.x - t.x, u.y - t.y);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ int bitrev(int i, int logN) { return (int)(__brev((unsigned)i) >> (32 - logN)); }

// twiddles exp(sign 2 pi i k / N), k < N/2, computed on the host in long double
static inline std::vector<double2> twiddles(int N, int sign) {
  std::vector<double2> tw(N / 2);
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int k = 0; k < N / 2; ++k) {
    const long double ang = 2.0L * pi * (long double)k / (long double)N;
    tw[k] = make_double2((double)cosl(ang), (double)(sign * sinl(ang)));
  }
  return tw;
}

static inline int ilog2(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return (1 << l) == n ? l : -1;
}

// Host-side launchers of the fasst_tf.hip kernels for the other translation
// units (HIP kernels do not link across TUs without -fgpu-rdc).
// [nm][F][T] (host order) <-> [nm][Tp][Fp] (frame-major, bins contiguous)
int tf_launch_ft_to_tf(hipStream_t s, const double2 *src, double2 *dst, int F, int T, int Fp,
                       int Tp, int nm);
int tf_launch_tf_to_ft(hipStream_t s, const double2 *src, double2 *dst, int F, int T, int Fp,
                       int Tp, int nm);
// iSTFT of one frame-major image (rows of `ld` bins, T frames) into y[len_out]
// (tftransforms/stft.py:71-131); frames is [T][wlen] scratch, tw the +1
// twiddles of nfft.
int tf_launch_istft(hipStream_t s, const double2 *S, int ld, int T, const double *win,
                    const double *awin, const double2 *tw, int wlen, int nfft, int hop,
                    double *frames, double *y, int len_out);

}  // namespace fasst
