/*
 * fasst_dict.h -- C ABI of the SIMM source dictionary generator (libfasst_hip.so).
 *
 * Replaces the per-F0 loop of generate_WF0_TR_chirped
 * (SeparateLeadStereo/separateLeadFunctions.py:696-886) for the STFT
 * transform SeparateLeadProcess.computeWF0 builds by default
 * (SeparateLeadStereoTF.py:646-681): for every column j,
 *   odgd_j(t)   = sum_h amps[j][h] exp(i theta_jh(t))          (KLGLOTT88 comb)
 *       theta_jh(t) = ((2 pi F1_j) h) (t / fs)                          F1 == F2
 *                     2 pi ((F1_j h) ts + ((F2_j - F1_j) h) ts^2 / (2 L / fs))  chirp
 *                     (generate_ODGD_spec :888-945 / _chirped :1010-1067)
 *   WF0[:, j]   = |rfft(window * Re odgd_j[frame_start : frame_start + wlen], nfft)|^2
 *                 (the middle frame of the transform, :838-847)
 * The partial amplitudes (a few hundred complex numbers per column) are
 * computed on the host with the reference's expression and handed over.
 * Conventions: fasst_hip.h.  amps [n_cols][max_partials] complex128;
 * wf0 [nfft/2 + 1][n_cols] row-major (the reference's WF0 layout).
 */
#ifndef FASST_DICT_H
#define FASST_DICT_H

#include "fasst_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

int dict_wf0_stft(int device, int n_cols, const double *f1, const double *f2,
                  const int *n_partials, int max_partials, const double *amps, double fs,
                  int length_odgd, const double *window, int wlen, int nfft, long frame_start,
                  double *wf0);

/* device time (HIP events) of the last dict_wf0_stft call, without copies */
int dict_last_ms(double *device_ms);

#ifdef __cplusplus
}
#endif

#endif /* FASST_DICT_H */
