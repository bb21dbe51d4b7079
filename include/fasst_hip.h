/*
 * fasst_hip.h -- C ABI of the MI355X FASST EM engine (libfasst_hip.so).
 *
 * The reference (s-ben/pyfasst) has no FFI layer: its seam is the Python
 * class surface of audioModel.py operating on NumPy state.
 * Each entry point below replaces one reference routine; the Python host
 * side (pyfasst_amd/audioModel.py) binds them with ctypes and keeps the
 * reference's class surface, argument meaning and exceptions.
 *
 * Conventions
 *   - all arrays are host arrays, C (row-major) order, caller-owned, copied in
 *     and out; the library owns every device allocation;
 *   - real data is float64; complex data is complex128 == interleaved
 *     (re, im) float64 pairs, exactly NumPy's memory layout;
 *   - one context = one GPU + one HIP stream; calls on a context are
 *     serialised by the caller; distinct contexts may live on distinct threads;
 *   - every function returns a status code (FASST_OK == 0); the message of
 *     the last failure of the calling thread is in fasst_last_error().
 */
#ifndef FASST_HIP_H
#define FASST_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define FASST_OK               0
#define FASST_ERR_SHAPE        1  /* -> AttributeError / ValueError          */
#define FASST_ERR_SINGULAR     2  /* -> np.linalg.LinAlgError('Singular Matrix'),
                                     audioModel.py:855-863                    */
#define FASST_ERR_DEVICE       3  /* HIP runtime / kernel failure             */
#define FASST_ERR_OOM          4  /* device allocation failed                 */
#define FASST_TW_RESTART       5  /* renormalize_parameters found sum(TW)<eps
                                     (audioModel.py:2023-2028): the host must
                                     draw the random restart and resume       */
#define FASST_ERR_UNSUPPORTED  6  /* model structure outside the HIP path     */

typedef struct fasst_ctx fasst_ctx;

/* ABI revision of this header.  A caller compares fasst_abi_version() with
 * the FASST_ABI_VERSION it was built against and refuses a mismatch (the
 * Python loader does, pyfasst_amd/_lib.py).  Revision 2: fasst_source_powers
 * and fasst_sigma_comp take 128-bit column sets (two 64-bit words per
 * spatial component; revision 1 read one word, and fasst_sigma_comp took its
 * mask by value), so a revision-1 caller would pass too short an array. */
#define FASST_ABI_VERSION 2
int fasst_abi_version(void);

const char *fasst_last_error(void);
int fasst_device_count(int *n);

/* ---- model context ------------------------------------------------------
 * Replaces the NumPy state of FASST (audioModel.py:159-248,2349-2393).
 * fasst_create allocates the observation (F freq bins x T frames, stereo:
 * the reference GEM is stereo-only, audioModel.py:394,418-420,605-607);
 * fasst_configure (re)allocates the model: J spatial components (= sources),
 * rank[J] spatial ranks, K[J] NMF components, mix_conv 0 = 'inst' (params
 * C x r), 1 = 'conv' (params r x C x F).  Reconfiguring keeps Cx / X.       */
int fasst_create(int device, int F, int T, fasst_ctx **out);
int fasst_configure(fasst_ctx *ctx, int J, const int *rank, const int *K, int mix_conv);
/* The same with the mixing type per spatial component (mix_conv[J], the
 * reference's per-component 'mix_type', retrieve_subsrc_params
 * audioModel.py:546-576).  In a model with both types, the mixing update
 * (update_mix_matrix :766-889) runs the 'inst' update over the free 'inst'
 * components with every other component held fixed; the reference's 'conv'
 * solve (:854-863) can only run when no other component exists, so its
 * free 'conv' components in a mixed model are rejected by the host layer. */
int fasst_configure_types(fasst_ctx *ctx, int J, const int *rank, const int *K,
                          const int *mix_conv);
int fasst_destroy(fasst_ctx *ctx);

/* comp_transf_Cx (audioModel.py:250-302) on the device: data[L][2] float64
 * (already scaled as AudioObject, audioObject.py:124-127), Hann or any
 * window[wlen], nfft (== fsize), hop.  Keeps the channel STFTs resident for
 * the Wiener images and builds Cx.  T must equal ceil(L/hop)+2.            */
int fasst_set_audio(fasst_ctx *ctx, const double *data, int L, const double *window,
                    int wlen, int nfft, int hop);
/* mix_psd[F] = mean_t over the channel PSDs / 2 (audioModel.py:304-319).   */
int fasst_mix_psd(fasst_ctx *ctx, double *mix_psd);

/* Cx: complex128 [3][F][T], packed upper triangle {X0 X0*, X0 X1*, X1 X1*}
 * exactly as FASST.Cx (audioModel.py:293-302).                              */
int fasst_set_cx(fasst_ctx *ctx, const double *cx);
int fasst_get_cx(fasst_ctx *ctx, double *cx);
/* X: complex128 [2][F][T] channel STFTs kept resident for the Wiener images
 * (replaces the per-source STFT recomputation of audioModel.py:1188-1192);
 * Cx is rebuilt from them on the device (audioModel.py:293-302).           */
int fasst_set_stft(fasst_ctx *ctx, const double *X);

/* Spatial component j: params in the reference layout (complex128; for
 * 'inst' the C x r matrix, for 'conv' r x C x F); free = frdm_prior=='free'.*/
int fasst_set_spatial(fasst_ctx *ctx, int j, const double *params, int free_);
int fasst_get_spatial(fasst_ctx *ctx, int j, double *params);
/* Spectral component of source j (single NMF factor, TB empty):
 * FB F x K, FW K x K, TW K x T (float64).                                    */
int fasst_set_spectral(fasst_ctx *ctx, int j, const double *FB, const double *FW,
                       const double *TW, int fb_free, int tw_free);
int fasst_get_spectral(fasst_ctx *ctx, int j, double *FB, double *FW, double *TW);
/* FW_frdm_prior of source j ('free' = 1): the FW multiplicative update of
 * update_spectral_components (audioModel.py:1578-1631) runs between the FB
 * and TW updates.  Default after fasst_configure: fixed.                     */
int fasst_set_fw_prior(fasst_ctx *ctx, int j, int fw_free);

/* Several spectral components on spatial component j (comp_spat_comp_power's
 * sum over spec_comps, audioModel.py:430-498; sequential per-component
 * update, :1479-1727): source j's FB / FW / TW (set by fasst_set_spectral)
 * hold the nblk components side by side, component b in columns / rows
 * [kb[b], kb[b + 1]) (kb[0] = 0, kb[nblk] = K_j, FW block diagonal), in the
 * reference's spec_comps key order; fb_free[b] / fw_free[b] / tw_free[b] are
 * component b's priors.  Restart flags (fasst_run / fasst_renormalize
 * restart_mask) then count one bit per component: bit (sum of nblk of the
 * sources before j) + b.                                                      */
int fasst_set_blocks(fasst_ctx *ctx, int j, int nblk, const int *kb, const int *fb_free,
                     const int *fw_free, const int *tw_free);

/* lambdaCorr (audioModel.py:1484-1507 and the corrPen terms of :1544-1719):
 * the inter-source correlation penalty of the spectral updates.  With
 * lambda > 0 the components are updated one at a time in the reference's
 * spec_comps key order: component q is block seq_b[q] of spatial component
 * seq_j[q] (fasst_set_blocks layout; nseq = every component, once).
 * lambda = 0 (the default after fasst_configure) switches it off.           */
int fasst_set_corr(fasst_ctx *ctx, double lambda, int nseq, const int *seq_j, const int *seq_b);

/* Time blobs of component b of source j (H = TW.TB, audioModel.py:486-487;
 * set through setComponentParameter(..., 'TB', ...), :2082): TW is the
 * component's factor TW (rows x L, rows = its fasst_set_blocks width), TB the
 * L x T time blobs, tb_free = TB_frdm_prior == 'free'.  The device keeps both
 * and writes H into the component's rows of the source's TW (whatever
 * fasst_set_spectral put there); TW then updates through TB (:1665-1691), TB
 * by :1931-1978, renormalisation :2029-2033.  L = 0 removes them; call after
 * fasst_set_blocks (which drops the time blobs of the source it changes).
 * A restart bit of such a component means sum(TW) < eps: the caller redraws
 * TW and performs the TB renormalisation (fasst_get_tb's TB is then not yet
 * divided by its row means).                                                 */
int fasst_set_tb(fasst_ctx *ctx, int j, int b, int L, const double *TW, const double *TB,
                 int tb_free);
int fasst_get_tb(fasst_ctx *ctx, int j, int b, double *TW, double *TB);

/* renormalize_parameters (audioModel.py:1980-2040).  restart_mask bit j (or
 * bit per spectral component, fasst_set_blocks) is set when sum(TW) < eps:
 * the caller draws the restart (host RNG order).                            */
int fasst_renormalize(fasst_ctx *ctx, int *restart_mask);

/* n_iter GEM iterations (GEM_iteration, audioModel.py:384-428), with the
 * annealed noise PSD rows psd[n_iter][F] (audioModel.py:364-373) and the NMF
 * exponent omega (nmfUpdateCoeff).  logliks[n_iter] receives the loglik of
 * each iteration.  On FASST_TW_RESTART, *iters_done iterations are complete
 * (the last one ended in the restart condition reported in restart_mask).   */
int fasst_run(fasst_ctx *ctx, int n_iter, const double *psd, double omega,
              double *logliks, int *restart_mask, int *iters_done);

/* Per-source STFT-domain Wiener images (separate_comps,
 * audioModel.py:1088-1217 up to the iSTFT; compute_sigma_comp_2d :1327,
 * compute_inv_sigma_mix_2d :1374, compute_Wiener_gain_2d :1396).  psd[F] is
 * the last annealed PSD; X complex128 [2][F][T] or NULL to use the resident
 * STFT; S out complex128 [J][2][F][T].                                       */
int fasst_wiener_images(fasst_ctx *ctx, const double *psd, const double *X, double *S);

/* Separation sources for fasst_wiener_images / fasst_separate_waveforms
 * (separate_comps' spec_comp_ind, audioModel.py:1130-1164): source n sums the
 * terms [term_off[n], term_off[n + 1]); term i is the spectral components in
 * columns term_mask[2 i .. 2 i + 1] (a 128-bit column set: bit k of word
 * k / 64 = column k, fasst_set_blocks layout; K <= 128) of spatial
 * component term_j[i] (compute_sigma_comp_2d, :1327-1372).  Sigma_x is the
 * sum over the sources plus the PSD (compute_inv_sigma_mix_2d, :1374-1394).
 * nsrc = 0 (the default): one source per spatial component, all columns.
 * The outputs then hold nsrc sources instead of J.                          */
int fasst_set_sources(fasst_ctx *ctx, int nsrc, const int *term_off, const int *term_j,
                      const unsigned long long *term_mask);

/* separate_comps up to the waveforms it writes (audioModel.py:1088-1233):
 * the Wiener images above, then the per-source, per-channel iSTFT
 * (tftransforms/stft.py:71-131, window / analysis_window as STFT's
 * synthWindow / window) of each image without leaving device memory.  Needs
 * the resident STFT (fasst_set_audio / fasst_set_stft) and nfft/2+1 == F.
 * y out float64 [J][2][len], len = hop*(T-1) + wlen - wlen/2 (istft's length
 * before the caller's [:datalen] trim).                                      */
int fasst_separate_waveforms(fasst_ctx *ctx, const double *psd, const double *window,
                             const double *analysis_window, int wlen, int nfft, int hop,
                             double *y);

/* Per-kernel timing with HIP events (used by bench.py for the roofline of
 * the dominant kernel), in the timed loop's own schedule: each pair is
 * recorded on the stream its kernel runs on (the side stream stays forked),
 * in a ring of 32 iterations between host syncs.  fasst_kernel_times
 * returns the number of kernel slots and fills the mean duration in ms of
 * each slot over the profiled iterations (a side-stream slot measures its
 * kernel while the main stream's kernels run beside it).                   */
int fasst_set_profiling(fasst_ctx *ctx, int on);
int fasst_kernel_times(fasst_ctx *ctx, double *avg_ms, long *counts, int nk);
const char *fasst_kernel_name(int i);

/* ---- stateless kernels --------------------------------------------------
 * stft (tftransforms/stft.py:3-69): x[L] float64, window[wlen], nfft a power
 * of two >= wlen, hop; X out complex128 [nfft/2+1][n_frames] with
 * n_frames = ceil(L/hop)+2 (query with X == NULL).                           */
int fasst_stft(int device, const double *x, int L, const double *window, int wlen,
               int nfft, int hop, double *X, int *n_frames);
/* istft (tftransforms/stft.py:71-131): X complex128 [nfft/2+1][n_frames];
 * y out float64 [hop*(n_frames-1)+wlen - wlen/2].                           */
int fasst_istft(int device, const double *X, int n_frames, const double *window,
                const double *analysis_window, int wlen, int nfft, int hop, double *y);
/* istft of the SIMM pipeline (SeparateLeadStereo/separateLeadFunctions.py:
 * 163-233): no half-window trim, edge normalisation copied from the
 * neighbouring window; y out float64 [hop*(n_frames-1)+wlen] (>= 2 wlen). */
int fasst_istft_simm(int device, const double *X, int n_frames, const double *window,
                     const double *analysis_window, int wlen, int nfft, int hop, double *y);
/* inv_herm_mat_2d (tools/signalTools.py:132-196) on n matrices:
 * diag[2][n], off complex128[n] -> inv_diag[2][n], inv_off complex128[n], det[n]. */
int fasst_inv_herm_mat_2d(int device, int n, const double *diag, const double *off,
                          double *inv_diag, double *inv_off, double *det);

/* ---- GEM step methods (fasst_steps.hip) ---------------------------------
 * The FASST methods GEM_iteration (audioModel.py:384-428) is made of, as
 * device calls on the reference's own arrays, for scripts that drive an
 * iteration piecewise or inspect its intermediates (fasst_run fuses them and
 * never materialises these arrays).  complex128 = interleaved (re, im).
 *
 * retrieve_subsrc_params (:514-578), the powers half: V out [nj][F][T], the
 * power of spatial components j0 .. j0+nj-1 from the context's parameters
 * (colmask[2 jj .. 2 jj + 1]: the NMF columns to include, a 128-bit set,
 * bit k of word k / 64 = column k; NULL: all).                             */
int fasst_source_powers(fasst_ctx *ctx, int j0, int nj, const unsigned long long *colmask,
                        double *V);
/* compute_suff_stat (:580-764) on the context's Cx: V [R][F][T] per-rank
 * powers, mix complex128 [R][2][F], psd [F] -> rxx complex128 [3][F]
 * (hat_Rxx: mean of Cx00, Cx01, Cx11), rxs complex128 [F][2][R],
 * rss complex128 [F][R][R], ws [R][F][T] (hat_Ws), loglik.  R <= 16.      */
int fasst_suff_stat(fasst_ctx *ctx, int R, const double *V, const double *mix, const double *psd,
                    double *rxx, double *rxs, double *rss, double *ws, double *loglik);
/* update_mix_matrix (:766-889), the solve: kind[r] = 0 fixed, 1 free
 * 'inst', 2 free 'conv' per rank; mix complex128 [R][2][F] in/out.  Free
 * 'conv' ranks next to other ranks: FASST_ERR_SHAPE (the reference's solve
 * raises); a singular system: FASST_ERR_SINGULAR, mix untouched.           */
int fasst_mix_solve(int device, int F, int R, const double *rss, const double *rxs, double *mix,
                    const int *kind);
/* update_spectral_components (:1469-1978): hat_W [J][F][T] -> the
 * context's FB / FW / TW (TB) updated in place (read back with
 * fasst_get_spectral); no renormalisation (fasst_renormalize).            */
int fasst_spectral_update(fasst_ctx *ctx, const double *hat_W, double omega);
/* compute_sigma_comp_2d (:1327-1372): spatial component j, NMF columns
 * colmask[0 .. 1] (128-bit set, bit k of word k / 64 = column k) ->
 * diag [2][F][T], off complex128 [F][T].                                   */
int fasst_sigma_comp(fasst_ctx *ctx, int j, const unsigned long long *colmask, double *diag,
                     double *off);
/* compute_inv_sigma_mix_2d (:1374-1394): n components' diag [n][2][F][T],
 * off complex128 [n][F][T], psd [F] -> inverse of their sum + PSD I:
 * idiag [2][F][T], ioff complex128 [F][T].                                 */
int fasst_inv_sigma_mix(int device, int n, int F, int T, const double *diag, const double *off,
                        const double *psd, double *idiag, double *ioff);
/* compute_Wiener_gain_2d (:1396-1467): one component's sigma (sdiag
 * [2][n], soff complex128 [n]) and the inverse mixture covariance
 * (idiag [2][n], ioff complex128 [n]) -> WG complex128 [2][2][n].         */
int fasst_wiener_gain(int device, long n, const double *sdiag, const double *soff,
                      const double *idiag, const double *ioff, double *WG);

#ifdef __cplusplus
}
#endif
#endif /* FASST_HIP_H */
