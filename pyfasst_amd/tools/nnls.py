"""Batched non-negative least squares on the MI355X.

`nnls_columns(A, B)` solves, for every column q of B, the problem the
reference hands to `scipy.optimize.nnls(A, B[:, q])` one frame at a time in
the lead pipeline's initHF00='nnls' initialisation
(SeparateLeadStereo/SeparateLeadStereoTF.py:982-993).  Lawson-Hanson active
set on the normal equations, one wave per column (include/fasst_nnls.h).
No CPU fallback.
"""
import numpy as np

from .. import _lib


def nnls_columns(A, B, add_eps=0.0, maxiter=None, tol=None, device=None):
    """X[:, q] = argmin_{x >= 0} ||A x - B[:, q]||_2 (+ add_eps), A (m, n),
    B (m, nf).  tol: dual-feasibility tolerance relative to max |A^T B[:, q]|
    (default 10 max(m, n) eps, scipy's scale).  Raises RuntimeError when an
    iteration limit (default 3 n, scipy's) is reached, as scipy does."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    B = np.ascontiguousarray(B, dtype=np.float64)
    if B.ndim == 1:
        return nnls_columns(A, B[:, None], add_eps, maxiter, tol, device)[:, 0]
    if A.ndim != 2 or B.ndim != 2 or A.shape[0] != B.shape[0]:
        raise ValueError("nnls_columns: A %s and B %s" % (A.shape, B.shape))
    if not (np.all(np.isfinite(A)) and np.all(np.isfinite(B))):
        raise ValueError("array must not contain infs or NaNs")   # as asarray_chkfinite
    m, n = A.shape
    nf = B.shape[1]
    if tol is None:
        tol = 10.0 * max(m, n) * np.finfo(np.float64).eps
    X = np.empty((n, nf))
    info = np.empty(nf, dtype=np.int32)
    dev = _lib.default_device() if device is None else device
    _lib.check(_lib.lib.nnls_columns(dev, m, n, _lib.dptr(A), nf, _lib.dptr(B), float(tol),
                                     float(add_eps), int(maxiter or 0), _lib.dptr(X),
                                     info.ctypes.data_as(_lib._ip)), "nnls_columns")
    if np.any(info < 0):
        raise RuntimeError("Maximum number of iterations reached.")
    return X
