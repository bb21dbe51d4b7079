/*
 * fasst_nmf.h -- C ABI of the IS-NMF engine (libfasst_hip.so).
 *
 * Replaces the multiplicative-update loops of the reference's tools/nmf.py:
 *   NMF_decomposition (nmf.py:24-61)  -> nmf_run(update_w=1, update_h=1)
 *   NMF_decomp_init   (nmf.py:63-159) -> nmf_run(update_w, update_h)
 * Random initialisation stays on the host (NumPy's global stream, nmf.py:30-32,
 * :119-140) and is handed over with nmf_set_params; the Python host side is
 * pyfasst_amd/tools/nmf.py.
 *
 * Conventions are those of fasst_hip.h.  SX [F][N], W [F][K], H [K][N]
 * (NMF_decomp_init's frame-major H is transposed by the host).
 */
#ifndef FASST_NMF_H
#define FASST_NMF_H

#include "fasst_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nmf_ctx nmf_ctx;

int nmf_create(int device, int F, int N, int K, nmf_ctx **out);
int nmf_destroy(nmf_ctx *ctx);
int nmf_set_data(nmf_ctx *ctx, const double *SX);
int nmf_set_params(nmf_ctx *ctx, const double *W, const double *H);

/* n_iter iterations of nmf.py:34-59 (W update, column renormalisation of W
 * with the scale moved into H, then H update); either update may be
 * switched off (NMF_decomp_init's updateW / updateH, nmf.py:142-157).      */
int nmf_run(nmf_ctx *ctx, int n_iter, int update_w, int update_h);
int nmf_get_params(nmf_ctx *ctx, double *W, double *H);

/* Per-source mono Wiener separation of the IS-NMF model (BASELINE configs[1],
 * SURVEY.md §8 N8): the one-channel degenerate of the reference's FASST
 * separation -- compute_sigma_comp_2d / compute_inv_sigma_mix_2d /
 * compute_Wiener_gain_2d (audioModel.py:1327-1467) and the image
 * sum_c2 WG X (audioModel.py:1205-1214) -- with Sigma_n = V_n =
 * W[:, k in n] H[k in n, :] (tools/nmf.py:24-61's model), Sigma_x =
 * sum_n V_n + psd (psd may be NULL = 0) and the inv_herm_mat_2d determinant
 * guard (tools/signalTools.py:177-188) on the 1 x 1 Sigma_x.
 *   W [F][K], H [K][N], comp_source[K] in [0, J) (other values: unused
 *   component), X complex [F][N] (interleaved doubles), K <= 256.
 * nmf_wiener_images   -> S complex [J][F][N]
 * nmf_wiener_waveforms -> y [J][hop (N-1) + wlen - wlen/2]: the iSTFT of each
 *   image (tftransforms/stft.py:71-131; nfft / 2 + 1 must equal F) without the
 *   images leaving the device.                                              */
int nmf_wiener_images(int device, int F, int N, int K, const double *W, const double *H, int J,
                      const int *comp_source, const double *psd, const double *X, double *S);
int nmf_wiener_waveforms(int device, int F, int N, int K, const double *W, const double *H, int J,
                         const int *comp_source, const double *psd, const double *X,
                         const double *window, const double *analysis_window, int wlen, int nfft,
                         int hop, double *y);

#ifdef __cplusplus
}
#endif

#endif /* FASST_NMF_H */
