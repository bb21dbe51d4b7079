// One sample of the KLGLOTT88 harmonic comb of the SIMM source dictionary
// (generate_ODGD_spec, separateLeadFunctions.py:888-945, and
// generate_ODGD_spec_chirped, :1010-1067), shared by the STFT dictionary
// (fasst_dict.hip) and the CQT / MinQT dictionary (fasst_cqt.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace fasst {

// odgd(t) = sum_h amp[h] exp(i theta_h(t)), summed over h in the reference's
// order (np.sum over axis 0 of the partials x samples product: sequential);
//   theta_h = ((2 pi F1) h) ts                               F1 == F2
//   theta_h = 2 pi ((F1 h) ts + ((F2 - F1) h) ts^2 / den)     chirp, den = 2 L / fs
// with ts = t / fs.  amp: the partial amplitudes (LDS).
__device__ __forceinline__ double2 odgd_sample(const double2 *amp, int P, double F1, double F2,
                                               double fs, double den, long t) {
  const double two_pi = 2.0 * M_PI;
  const double w1 = two_pi * F1;
  const double dF = F2 - F1;
  const bool chirp = F1 != F2;
  const double ts = (double)t / fs;
  double re = 0.0, im = 0.0;
  for (int h = 0; h < P; ++h) {
    const double fh = (double)(h + 1);
    const double th = chirp ? two_pi * ((F1 * fh) * ts + ((dF * fh) * (ts * ts)) / den)
                            : (w1 * fh) * ts;
    double s, c;
    sincos(th, &s, &c);
    const double2 am = amp[h];
    re += c * am.x - s * am.y;   // exp(i th) * amp
    im += c * am.y + s * am.x;
  }
  return make_double2(re, im);
}

}  // namespace fasst
