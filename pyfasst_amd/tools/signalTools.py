"""Signal tools on the GPU (tools/signalTools.py of the reference)."""
import numpy as np

from .. import _lib
from .._lib import check, dptr, lib

eps = 1e-10  # signalTools.py:11


def inv_herm_mat_2d(sigma_x_diag, sigma_x_off, verbose=False, device=None):
    """Batched explicit inverse of 2x2 Hermitian matrices (signalTools.py:132-196).

    Same contract as the reference: returns (inv_diag, inv_off, det) with the
    determinant floored to sign(det+eps)*max(|det|, eps).  Runs on the GPU.
    """
    d = np.ascontiguousarray(np.asarray(sigma_x_diag, dtype=np.float64))
    o = np.asarray(sigma_x_off)
    shape = o.shape
    n = int(np.prod(shape)) if len(shape) else 1
    d = np.ascontiguousarray(d.reshape(2, n))
    o = np.ascontiguousarray(o.astype(np.complex128).reshape(n))
    inv_d = np.empty((2, n))
    inv_o = np.empty(n, dtype=np.complex128)
    det = np.empty(n)
    dev = _lib.default_device() if device is None else device
    check(lib.fasst_inv_herm_mat_2d(dev, n, dptr(d), dptr(o), dptr(inv_d), dptr(inv_o),
                                    dptr(det)), "fasst_inv_herm_mat_2d")
    return inv_d.reshape((2,) + shape), inv_o.reshape(shape), det.reshape(shape)
