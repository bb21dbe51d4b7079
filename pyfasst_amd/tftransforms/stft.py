"""STFT / iSTFT on the GPU (tftransforms/stft.py of the reference).

`stft` and `istft` keep the reference signatures and framing
(stft.py:3-69, :71-131): first frame centred on sample 0 (wlen/2 leading
zeros), ceil(L/hop)+2 frames, window-product normalised overlap-add.  The
FFTs are FP64 radix-2 transforms in LDS (pyfasst_amd/csrc/fasst_tf.hip).
"""
import ctypes

import numpy as np

from .. import _lib
from .._lib import check, dptr, lib
from ..tools.utils import sinebell


def _dev(device):
    return _lib.default_device() if device is None else device


def stft(data, window=sinebell(2048), hopsize=256.0, nfft=2048.0, fs=44100.0, device=None):
    """X, F, N = stft(data, window, hopsize, nfft, fs)  (stft.py:3-69)."""
    x = np.ascontiguousarray(np.asarray(data, dtype=np.float64).ravel())
    w = np.ascontiguousarray(np.asarray(window, dtype=np.float64))
    nfft_i, hop_i = int(nfft), int(hopsize)
    T = ctypes.c_int(0)
    check(lib.fasst_stft(_dev(device), dptr(x), x.size, dptr(w), w.size, nfft_i, hop_i, None,
                         ctypes.byref(T)), "fasst_stft")
    X = np.empty((nfft_i // 2 + 1, T.value), dtype=np.complex128)
    check(lib.fasst_stft(_dev(device), dptr(x), x.size, dptr(w), w.size, nfft_i, hop_i, dptr(X),
                         ctypes.byref(T)), "fasst_stft")
    F = np.arange(nfft_i // 2 + 1) / np.double(nfft) * fs
    N = np.arange(T.value) * hopsize / np.double(fs)
    return X, F, N


def istft(X, window=sinebell(2048), analysisWindow=None, hopsize=256.0, nfft=2048.0,
          device=None):
    """data = istft(X, window, analysisWindow, hopsize, nfft)  (stft.py:71-131)."""
    if analysisWindow is None:
        analysisWindow = window
    X = np.ascontiguousarray(X, dtype=np.complex128)
    w = np.ascontiguousarray(np.asarray(window, dtype=np.float64))
    aw = np.ascontiguousarray(np.asarray(analysisWindow, dtype=np.float64))
    nfft_i, hop_i = int(nfft), int(hopsize)
    if X.shape[0] != nfft_i // 2 + 1:
        raise ValueError("X has %d bins, nfft=%d needs %d" % (X.shape[0], nfft_i, nfft_i // 2 + 1))
    T = X.shape[1]
    y = np.empty(hop_i * (T - 1) + w.size - w.size // 2)
    check(lib.fasst_istft(_dev(device), dptr(X), T, dptr(w), dptr(aw), w.size, nfft_i, hop_i,
                          dptr(y)), "fasst_istft")
    return y


class STFT(object):
    """STFT transform object (stft.py:339-394): computeTransform / invertTransform."""
    transformname = 'stft'

    def __init__(self, linFTLen=2048, atomHopFactor=0.25, winFunc=np.hanning, fs=44100,
                 synthWinFunc=None, device=None, **kwargs):
        fthop = int(linFTLen * atomHopFactor)
        self.ftlen = linFTLen
        self.freqbins = self.ftlen // 2 + 1
        self.atomHopFactor = atomHopFactor
        self.fthop = fthop
        if winFunc is None:
            winFunc = np.hanning
        self.winFunc = winFunc
        self.window = self.winFunc(self.ftlen)
        self.synthWinFunc = synthWinFunc if synthWinFunc is not None else self.winFunc
        self.synthWindow = self.synthWinFunc(self.ftlen)
        self.fs = fs
        self.device = device

    def computeTransform(self, data):
        self.transfo, self.freq_stamps, self.time_stamps = stft(
            data=data, window=self.window, hopsize=self.fthop, fs=self.fs, nfft=self.ftlen,
            device=self.device)
        self.datalen_init = np.asarray(data).size
        self.time_stamps *= self.fs

    def invertTransform(self):
        return istft(X=self.transfo, window=self.synthWindow, analysisWindow=self.window,
                     hopsize=self.fthop, nfft=self.ftlen, device=self.device)[:self.datalen_init]
