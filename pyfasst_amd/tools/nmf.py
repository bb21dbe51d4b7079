"""IS-NMF on the MI355X (drop-in for the reference's tools/nmf.py).

`NMF_decomposition` (nmf.py:24-61) and `NMF_decomp_init` (nmf.py:63-159)
keep the reference's signatures, random draws (NumPy's global stream, same
order) and return values; the multiplicative-update loop runs in
libfasst_hip.so (include/fasst_nmf.h).  No CPU fallback.
"""
import ctypes

import numpy as np

from .. import _lib

eps = 1e-10     # nmf.py:22


class _NmfContext(object):
    def __init__(self, F, N, K, device):
        self.ptr = ctypes.c_void_p()
        _lib.check(_lib.lib.nmf_create(device, F, N, K, ctypes.byref(self.ptr)), "nmf_create")

    def __del__(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            _lib.lib.nmf_destroy(self.ptr)
            self.ptr = None


def _run(SX, W, H, niter, update_w, update_h, device):
    F, N = SX.shape
    K = W.shape[1]
    dev = _lib.default_device() if device is None else device
    ctx = _NmfContext(F, N, K, dev)
    SXc = np.ascontiguousarray(SX, dtype=np.float64)
    W = np.ascontiguousarray(W, dtype=np.float64)
    H = np.ascontiguousarray(H, dtype=np.float64)
    _lib.check(_lib.lib.nmf_set_data(ctx.ptr, _lib.dptr(SXc)), "nmf_set_data")
    _lib.check(_lib.lib.nmf_set_params(ctx.ptr, _lib.dptr(W), _lib.dptr(H)), "nmf_set_params")
    _lib.check(_lib.lib.nmf_run(ctx.ptr, int(niter), int(bool(update_w)), int(bool(update_h))),
               "nmf_run")
    _lib.check(_lib.lib.nmf_get_params(ctx.ptr, _lib.dptr(W), _lib.dptr(H)), "nmf_get_params")
    return W, H


def NMF_decomposition(SX, nbComps=10, niter=10, verbose=0, device=None):
    """IS-NMF multiplicative updates (nmf.py:24-61); returns (W, H)."""
    freqs, nframes = SX.shape
    W = np.random.randn(freqs, nbComps) ** 2
    H = np.random.randn(nbComps, nframes) ** 2
    W /= W.sum(axis=0)
    if verbose:
        print("    NMF: %d iterations on the GPU" % niter)
    return _run(SX, W, H, niter, True, True, device)


def NMF_decomp_init(SX, nbComps=10, niter=10, verbose=0, Winit=None, Hinit=None,
                    updateW=True, updateH=True, device=None):
    """IS-NMF with optional initial W / H and frozen factors (nmf.py:63-159).

    Returns (W, H) with H as nbComps x nframes, as the reference does.
    """
    freqs, nframes = SX.shape
    if Winit is None or (Winit.shape != (freqs, nbComps)):
        W = np.random.randn(freqs, nbComps) ** 2
    else:
        W = np.copy(Winit)
    if Hinit is not None:
        if Hinit.shape == (nbComps, nframes):
            Ht = np.copy(Hinit.T)
        elif Hinit.shape == (nframes, nbComps):
            Ht = np.copy(Hinit)
        else:
            raise AttributeError('Hinit not in the right shape.')
    else:
        Ht = np.random.randn(nframes, nbComps, ) ** 2
    if updateW:
        W /= W.sum(axis=0)
    W, H = _run(SX, W, Ht.T, niter, updateW, updateH, device)
    return W, H
