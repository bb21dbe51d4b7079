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


def _comp_source(comp_ind, K):
    """{source: [components]} (or a list of lists) -> source index per component"""
    items = comp_ind.items() if isinstance(comp_ind, dict) else enumerate(comp_ind)
    items = sorted((int(n), list(np.atleast_1d(c))) for n, c in items)
    if [n for n, _ in items] != list(range(len(items))):
        raise ValueError("sources must be numbered 0..J-1")
    src = np.full(K, -1, dtype=np.int32)
    for n, comps in items:
        for k in comps:
            if not 0 <= int(k) < K or src[int(k)] >= 0:
                raise ValueError("component %s out of range or in two sources" % k)
            src[int(k)] = n
    return len(items), src


def _wiener_args(X, W, H, comp_ind, psd):
    X = np.ascontiguousarray(X, dtype=np.complex128)
    W = np.ascontiguousarray(W, dtype=np.float64)
    H = np.ascontiguousarray(H, dtype=np.float64)
    F, N = X.shape
    K = W.shape[1]
    if W.shape != (F, K) or H.shape != (K, N):
        raise ValueError("W %s / H %s do not match X %s" % (W.shape, H.shape, X.shape))
    J, src = _comp_source(comp_ind, K)
    p = None
    if psd is not None:
        p = np.ascontiguousarray(np.asarray(psd, dtype=np.float64) * np.ones(F))
    return X, W, H, F, N, K, J, src, p


def NMF_wiener_images(X, W, H, comp_ind, psd=None, device=None):
    """Per-source mono Wiener images S[n] = V_n / (sum_m V_m + psd) * X of the
    IS-NMF model V_n = W[:, comp_ind[n]] . H[comp_ind[n]] (BASELINE configs[1]).

    The one-channel degenerate of the reference's FASST separation
    (audioModel.py:1327-1467, image :1205-1214), with the inv_herm_mat_2d
    determinant guard (signalTools.py:177-188); the reference itself has no
    mono FASST path.  X: complex STFT [F, N]; comp_ind:
    {source: [component indices]} as separate_comps' spec_comp_ind.
    Returns S complex [J, F, N].  Runs in libfasst_hip.so (nmf_wiener_images).
    """
    X, W, H, F, N, K, J, src, p = _wiener_args(X, W, H, comp_ind, psd)
    S = np.empty((J, F, N), dtype=np.complex128)
    dev = _lib.default_device() if device is None else device
    _lib.check(_lib.lib.nmf_wiener_images(dev, F, N, K, _lib.dptr(W), _lib.dptr(H), J,
                                          _lib.iptr(src), _lib.dptr(p) if p is not None else None,
                                          _lib.dptr(X), _lib.dptr(S)), "nmf_wiener_images")
    return S


def NMF_separate_waveforms(X, W, H, comp_ind, window, hopsize, nfft=None, analysis_window=None,
                           psd=None, device=None):
    """NMF_wiener_images followed by the iSTFT of each image
    (tftransforms/stft.py:71-131), the images never leaving the GPU.
    Returns [J, hopsize (N-1) + wlen - wlen // 2] float64."""
    X, W, H, F, N, K, J, src, p = _wiener_args(X, W, H, comp_ind, psd)
    w = np.ascontiguousarray(window, dtype=np.float64)
    aw = np.ascontiguousarray(w if analysis_window is None else analysis_window, dtype=np.float64)
    nfft = 2 * (F - 1) if nfft is None else int(nfft)
    hop = int(hopsize)
    y = np.empty((J, hop * (N - 1) + w.size - w.size // 2))
    dev = _lib.default_device() if device is None else device
    _lib.check(_lib.lib.nmf_wiener_waveforms(dev, F, N, K, _lib.dptr(W), _lib.dptr(H), J,
                                             _lib.iptr(src),
                                             _lib.dptr(p) if p is not None else None,
                                             _lib.dptr(X), _lib.dptr(w), _lib.dptr(aw), w.size,
                                             nfft, hop, _lib.dptr(y)), "nmf_wiener_waveforms")
    return y
