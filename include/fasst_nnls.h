/*
 * fasst_nnls.h -- C ABI of the batched non-negative least squares
 * (libfasst_hip.so).
 *
 * Replaces the per-frame scipy.optimize.nnls loop of the lead pipeline's
 * initHF00='nnls' initialisation (SeparateLeadStereo/SeparateLeadStereoTF.py
 * :982-993):  for every column q of B,
 *     X[:, q] = argmin_{x >= 0} || A x - B[:, q] ||_2  + add_eps
 * (Lawson-Hanson active set on the normal equations, one wave per column;
 * the dual-feasibility tolerance is tol * max |A^T B[:, q]|).  A [m][n] and
 * B [m][nf] row-major (the reference's WF0 and SX layouts), X [n][nf]
 * row-major; info[q] = outer iterations, or -1 when maxiter (0: 3 n, the
 * reference's default) was reached.  n <= 2048.  Conventions: fasst_hip.h.
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
