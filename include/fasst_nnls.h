/*
 * fasst_nnls.h -- C ABI of the batched non-negative least squares
 * (libfasst_hip.so).
 *
 * Replaces the per-frame scipy.optimize.nnls loop of the lead pipeline's
 * initHF00='nnls' initialisation (SeparateLeadStereo/SeparateLeadStereoTF.py
 * :982-993):  for every column q of B,
 *     X[:, q] = argmin_{x >= 0} || A x - B[:, q] ||_2  + add_eps
 * (Lawson-Hanson active set on the normal equations, one wave per column).
 * A [m][n] and B [m][nf] row-major (the reference's WF0 and SX layouts),
 * X [n][nf] row-major.  n <= 2048.  Conventions: fasst_hip.h.
 *
 * info[q] = the iteration count, every pass of Lawson & Hanson's secondary
 * loop (step E: one per outer iteration plus one per inner step that drops
 * coefficients), or -1 once the count reaches maxiter (0: 3 n, scipy's
 * default) -- the budget scipy.optimize.nnls 1.15.3 enforces (it raises
 * exactly when outer + inner passes >= maxiter; tests/test_gpu_pipeline.py).
 * The coefficient that sets the step length leaves the passive set at
 * exactly zero, as in the original algorithm.
 *
 * Tolerance (a deliberate difference): the stopping test is
 * max_free (c - G x) <= tol * max |A^T B[:, q]|, RELATIVE to the column's
 * scale, where scipy's test on its QR-based dual is absolute.  The dual here
 * comes from the normal equations, whose rounding noise scales with
 * max |A^T b| (and the dictionary's condition number), so an absolute zero
 * test could loop on that noise; on the reference's own pipeline data the
 * two give the same active sets (tests/golden/pipeline_nnls.npz), other
 * inputs are parity-unpinned at the tolerance boundary.
 */
#ifndef FASST_NNLS_H
#define FASST_NNLS_H

#include "fasst_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

int nnls_columns(int device, int m, int n, const double *A, int nf, const double *B, double tol,
                 double add_eps, int maxiter, double *X, int *info);

#ifdef __cplusplus
}
#endif

#endif /* FASST_NNLS_H */
