"""SIMM-pipeline STFT / iSTFT on the GPU (reference:
SeparateLeadStereo/separateLeadFunctions.py:90-233).

These differ from tftransforms/stft.py: `stft` takes a start/stop frame range
and pads half a window at both ends (:90-161); `istft` keeps the leading half
window and patches the first / last window of the normalisation from their
neighbours (:163-233).  FFTs and overlap-add run in libfasst_hip.so.
"""
import ctypes

import numpy as np

from .. import _lib
from .._lib import check, dptr, lib
from ..tools.utils import sinebell

__all__ = ["sinebell", "stft", "istft"]


def _dev(device):
    return _lib.default_device() if device is None else device


def _int_hop(hopsize):
    if float(hopsize) != int(hopsize):
        raise NotImplementedError("non-integer hopsize %r" % (hopsize,))
    return int(hopsize)


def stft(data, window=sinebell(2048), hopsize=256.0, nfft=2048.0, fs=44100.0, start=0,
         stop=None, device=None):
    """X, F, N = stft(...)  (separateLeadFunctions.py:90-161)."""
    x = np.ascontiguousarray(np.asarray(data, dtype=np.float64).ravel())
    w = np.ascontiguousarray(np.asarray(window, dtype=np.float64))
    L = w.size
    hop = _int_hop(hopsize)
    nfft_i = int(nfft)
    # frame count of :127-131 (half a window of zeros on both sides)
    n_data = x.size + 2 * int(L / 2.0)
    n_frames = int(np.ceil((n_data - L) / float(hopsize) + 1) + 1)
    T = ctypes.c_int(0)
    check(lib.fasst_stft(_dev(device), dptr(x), x.size, dptr(w), L, nfft_i, hop, None,
                         ctypes.byref(T)), "fasst_stft")
    Xall = np.empty((nfft_i // 2 + 1, T.value), dtype=np.complex128)
    check(lib.fasst_stft(_dev(device), dptr(x), x.size, dptr(w), L, nfft_i, hop, dptr(Xall),
                         ctypes.byref(T)), "fasst_stft")
    if stop is None:
        stop = n_frames
    if stop > n_frames or start < 0:
        raise ValueError("frames %d:%d outside the %d analysed frames" % (start, stop, n_frames))
    X = np.ascontiguousarray(Xall[:, start:stop])
    F = np.arange(nfft_i // 2 + 1) / nfft * fs
    N = np.arange(n_frames) * hopsize / fs
    return X, F, N


def istft(X, analysisWindow=None, window=sinebell(2048), hopsize=256.0, nfft=2048.0,
          originalDataLen=None, start=-1, stop=None, device=None):
    """data = istft(...)  (separateLeadFunctions.py:163-233)."""
    if analysisWindow is None:
        analysisWindow = window
    X = np.ascontiguousarray(X, dtype=np.complex128)
    w = np.ascontiguousarray(np.asarray(window, dtype=np.float64))
    aw = np.ascontiguousarray(np.asarray(analysisWindow, dtype=np.float64))
    nfft_i, hop = int(nfft), _int_hop(hopsize)
    if X.shape[0] != nfft_i // 2 + 1:
        raise ValueError("X has %d bins, nfft=%d needs %d" % (X.shape[0], nfft_i, nfft_i // 2 + 1))
    T = X.shape[1]
    y = np.empty(hop * (T - 1) + w.size)
    check(lib.fasst_istft_simm(_dev(device), dptr(X), T, dptr(w), dptr(aw), w.size, nfft_i, hop,
                               dptr(y)), "fasst_istft_simm")
    if originalDataLen is not None:
        y = y[:originalDataLen]
    return y
