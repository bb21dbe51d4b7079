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

}  // namespace fasst
