/*
 * fasst_cqt.h -- C ABI of the CQT / MinQT front and back end (libfasst_hip.so).
 *
 * Replaces the constant-Q transforms the reference's FASST builds for
 * transf='cqt' / 'mqt' / 'minqt' (audioModel.py:156, :206-214, always with
 * perfRast=1):
 *
 *   cqt_forward  CQTransfo.computeCQT, rasterised branch  (tftransforms/minqt.py:471-486, 523-646)
 *                + MinQTransfo.computeLinearPart           (minqt.py:1410-1450, 1534-1549)
 *                -> the spCQT matrix `transfo` returns      (minqt.py:660-663, 722-729)
 *   cqt_inverse  MinQTransfo.invertTransform               (minqt.py:1452-1485: invertFromSpCQTRast
 *                                                          :794-868 + invertLinearPart)
 *                CQTransfo.invertTransform                 (minqt.py:1013-1055: invertFromCellCQT)
 *                both after `transfo = spCQT`              (minqt.py:648-658, spCQT2CellCQT :949-1011)
 *   dict_wf0_cqt generate_WF0_TR_chirped on this transform (separateLeadFunctions.py:742-886)
 *   cqt_shape    the frame bookkeeping of computeCQT (nframes per octave, minqt.py:553-556)
 *
 * The one-octave spectral kernel (CQTKernel / MinQTKernel, minqt.py:95-227,
 * 312-335) and the anti-aliasing Butterworth filter (scipy.signal.butter(6,
 * 0.5), minqt.py:441-447, with scipy.signal.lfilter_zi) are designed on the
 * host, exactly as the reference designs them, and handed over once.
 *
 * Conventions are those of fasst_hip.h: complex128 = interleaved doubles,
 * caller-owned host buffers, library-owned device memory, status codes
 * FASST_OK / FASST_ERR_SHAPE (-> ValueError: the shapes the reference cannot
 * broadcast either) / FASST_ERR_DEVICE / FASST_ERR_OOM.
 */
#ifndef FASST_CQT_H
#define FASST_CQT_H

#include "fasst_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cqt_ctx cqt_ctx;

/* spar_kernel: CQTKernel.sparKernel [fft_len][bins*win_nr] complex (minqt.py:194-209).
 * atom_hop, fft_hop, first_center: the kernel's integral frame geometry.
 * iir_b, iir_a [7], iir_zi [6]: anti-aliasing filter (a[0] == 1).
 * lin_ft_len == 0: CQTransfo; else MinQTransfo with lin_window [lin_ft_len]
 * (MinQTKernel.linWindow), kmax (Kmax) and lin_bins (linBins).           */
int cqt_create(int device, int bins, int octave_nr, int win_nr, int fft_len, int fft_hop,
               int atom_hop, int first_center, const double *spar_kernel, const double *iir_b,
               const double *iir_a, const double *iir_zi, int lin_ft_len, int kmax, int lin_bins,
               const double *lin_window, cqt_ctx **out);
int cqt_destroy(cqt_ctx *ctx);

/* Shape of the transform of a signal of L samples: freqbins rows, width
 * columns (nframes[0] * win_nr), nframes[octave_nr] (may be NULL).        */
int cqt_shape(cqt_ctx *ctx, long L, int *freqbins, int *width, int *nframes);

/* x [L] -> sp [freqbins][width] complex */
int cqt_forward(cqt_ctx *ctx, const double *x, long L, double *sp);

/* sp [freqbins][width] complex (the transform of a signal of L samples)
 * -> y [L]                                                                */
int cqt_inverse(cqt_ctx *ctx, const double *sp, long L, double *y);

/* SIMM source dictionary on this transform (generate_WF0_TR_chirped with a
 * CQT / MinQT transform, SeparateLeadStereo/separateLeadFunctions.py:742-886,
 * replacing its per-F0 computeTransform loop :829-879): for every column j the
 * complex KLGLOTT88 comb odgd_j of length_odgd samples (amps, f1, f2 as in
 * fasst_dict.h: generate_ODGD_spec :888-945 / _chirped :1010-1067) is
 * transformed, and wf0[k][j] = |transfo(odgd_j)[k, col]|^2, col the
 * reference's midindex (argmin |datalen_init / 2 - time_stamps|).  The
 * transform of the complex comb is T(Re) + i T(Im) on the CQT rows and T(Re)
 * on the MinQT linear rows (the linear part's rfft drops the imaginary part).
 * wf0 [freqbins][n_cols] row-major.                                        */
int dict_wf0_cqt(cqt_ctx *ctx, int n_cols, const double *f1, const double *f2,
                 const int *n_partials, int max_partials, const double *amps, double fs,
                 long length_odgd, int col, double *wf0);
/* Device time (HIP events on the context's stream) of the last cqt_forward /
 * cqt_inverse, excluding the host<->device copies of x, sp and y.         */
int cqt_device_ms(cqt_ctx *ctx, double *forward_ms, double *inverse_ms);

#ifdef __cplusplus
}
#endif

#endif /* FASST_CQT_H */
