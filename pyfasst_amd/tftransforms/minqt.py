"""Constant-Q / minimum-Q transforms on the GPU (tftransforms/minqt.py of the reference).

Same classes, constructor arguments and attributes as the reference:
`CQTKernel` (minqt.py:31-233), `MinQTKernel` (:309-335), `CQTransfo`
(:402-1070) and `MinQTransfo` (:1369-1550).  FASST builds them with
perfRast=1 (audioModel.py:206-214); that rasterised transform and its
inverse run on the GPU (pyfasst_amd/csrc/fasst_cqt.hip, C ABI
include/fasst_cqt.h).

Host side (setup constants only, as the reference designs them): the
one-octave spectral kernel (a few hundred FFTs of single atoms, thresholded
at `thresh` -- computed with NumPy so that the thresholding and the
normalisation weight are the reference's to the bit) and the anti-aliasing
Butterworth filter (scipy.signal.butter / lfilter_zi).  `cellCQT` is a pure
re-indexing view of spCQT (spCQT2CellCQT, :949-1011).

Not on the GPU path: perfRast=0 (its spCQT is an interpolated view of
per-octave cells, :870-947; no FASST configuration builds it) raises
NotImplementedError.  Deliberate deviation: `lowPassCoeffs=(B, A)` is used
as the anti-aliasing filter (the reference accepts the argument but then
never defines B, A and fails at the first octave).
"""
import ctypes

import numpy as np
import scipy.signal as spsig

from .. import _lib
from .._lib import check, dptr, lib
from ..tools.utils import nextpow2, sqrt_blackmanharris


def _dev(device):
    return _lib.default_device() if device is None else device


class CQTKernel(object):
    """One-octave CQT kernel (minqt.py:95-227), computed on the host."""

    def __init__(self, fmax, bins, fs, q=1, atomHopFactor=0.25, thresh=0.0005,
                 winFunc=sqrt_blackmanharris, perfRast=0):
        if fmax >= fs / 2.:
            raise ValueError("fmax (%s) is too big for fs (%s)" % (str(fmax), str(fs)))
        fmin = (fmax / 2.) * (2 ** (1. / bins))
        Q = 1. / (2 ** (1. / bins) - 1)
        Q = Q * q
        Nk_max = np.round(Q * fs / fmin)
        Nk_min = np.round(Q * fs / (fmin * (2 ** ((bins - 1.) / bins))))
        atomHOP = nextpow2(Nk_min * atomHopFactor) // 2
        first_center = np.ceil(Nk_max / 2.)
        first_center = atomHOP * np.ceil(first_center * 1. / atomHOP)
        FFTLen = nextpow2(first_center + np.ceil(Nk_max / 2.))
        winNr = np.floor((FFTLen - np.ceil(Nk_max / 2.) - first_center) / atomHOP) + 1
        if perfRast and winNr == 0:
            FFTLen = FFTLen * 2
            winNr = np.floor((FFTLen - np.ceil(Nk_max / 2.) - first_center) / atomHOP)
        last_center = first_center + (winNr - 1.) * atomHOP
        fftHOP = (last_center + atomHOP) - first_center
        fftOLP = (FFTLen - fftHOP) * (1. / FFTLen) * 100.
        sparKernel = np.zeros([int(bins * winNr), int(FFTLen)], dtype=complex)
        frequencies = []
        for k in np.arange(bins):
            Nk = np.round(Q * fs / (fmin * (2 ** ((k * 1.) / bins))))
            winFct = winFunc(int(Nk))
            fk = fmin * (2 ** ((k * 1.) / bins))
            frequencies.append(fk)
            atom = (winFct * 1. / Nk) * np.exp(2 * np.pi * 1j * fk * np.arange(Nk) / fs)
            atomOffset = first_center - np.ceil(Nk / 2.)
            for i in np.arange(winNr):
                shift = atomOffset + i * atomHOP
                tempKernel = np.zeros(int(FFTLen), dtype=complex)
                tempKernel[int(shift):int(Nk + shift)] = atom
                specKernel = np.fft.fft(tempKernel)
                specKernel[np.abs(specKernel) <= thresh] = 0
                sparKernel[int(i + k * winNr)] = specKernel
        sparKernel = (sparKernel.T) * 1. / FFTLen
        wx1 = np.argmax(sparKernel[:, 0])
        wx2 = np.argmax(sparKernel[:, -1])
        wK = sparKernel[wx1:wx2, :]
        wK = np.diag(np.dot(wK, np.conjugate(wK.T)))
        wK = wK[int(np.round(1. / q)):int(len(wK) - np.round(1. / q) - 1)]
        weight = 1. / np.mean(np.abs(wK))
        weight *= (fftHOP * 1. / FFTLen)
        weight = np.sqrt(weight)
        sparKernel *= weight
        self.sparKernel = np.ascontiguousarray(sparKernel)
        self.weight = weight
        self.atomHOP = atomHOP
        self.FFTLen = FFTLen
        self.fftOLP = fftOLP
        self.fftHOP = fftHOP
        self.bins = bins
        self.winNr = winNr
        self.Nk_max = Nk_max
        self.Q = Q
        self.fmin = fmin
        self.fmax = fmax
        self.frequencies = frequencies
        self.perfRast = perfRast
        self.first_center = first_center
        self.fs = fs
        self.winFunc = winFunc
        self.thresh = thresh
        self.q = q

    def __str__(self):
        description = "CQT Kernel structure, containing:\n"
        for k, v in self.__dict__.items():
            description += str(k) + ': ' + str(v) + '\n'
        return description


class MinQTKernel(CQTKernel):
    """MinQT kernel (minqt.py:312-335): CQT up to the frequency where the
    linear FFT bins of linFTLen are as dense as the CQT bins."""

    def __init__(self, bins, fmax, fs, linFTLen=2048, **kwargs):
        Q = 1. / (2 ** (1. / bins) - 1)
        Kmax = int(np.ceil(Q))
        fmax = 2 ** (-1. / bins) * Kmax * fs * 1. / linFTLen
        self.Q = Q
        self.Kmax = Kmax
        self.linFTLen = linFTLen
        self.fs = fs
        self.fmax = fmax
        self.bins = bins
        super(MinQTKernel, self).__init__(fmax=self.fmax, fs=self.fs, bins=self.bins, **kwargs)
        self.linBins = linFTLen // 2 - Kmax + 1
        self.linWindow = self.winFunc(linFTLen)


class CQTransfo(object):
    """Constant-Q transform (minqt.py:402-1070); perfRast=1 runs on the GPU."""
    transformname = 'cqt'

    def __init__(self, fmin, fmax, bins, fs, q=1, atomHopFactor=0.25, thresh=0.0005,
                 winFunc=sqrt_blackmanharris, perfRast=0, cqtkernel=None, lowPassCoeffs=None,
                 data=None, verbose=0, device=None, **kwargs):
        self.verbose = verbose
        self.device = device
        self.fmin = fmin
        self.fmax = fmax
        self.bins = bins
        self.bpo = bins
        self.fs = fs
        self.q = q
        self.atomHopFactor = atomHopFactor
        self.thresh = thresh
        if winFunc is None:
            winFunc = sqrt_blackmanharris
        self.winFunc = winFunc
        self.perfRast = perfRast
        self.octaveNr = np.ceil(np.log2(fmax * 1. / fmin))
        self.freqbins = bins * self.octaveNr
        self.fmin = (fmax / (2 ** self.octaveNr)) * 2 ** (1. / bins)
        if lowPassCoeffs is None:
            self.LPorder = 6
            self.cutoff = 0.5
            self.B, self.A = spsig.butter(N=self.LPorder, Wn=self.cutoff, btype='low')
        else:
            self.B, self.A = (np.asarray(c, dtype=np.float64) for c in lowPassCoeffs)
        if cqtkernel is None:
            self.cqtkernel = CQTKernel(fmax=fmax, bins=bins, fs=fs, q=q,
                                       atomHopFactor=atomHopFactor, thresh=thresh,
                                       winFunc=winFunc, perfRast=perfRast)
        else:
            self.cqtkernel = cqtkernel
        self._h = None
        if data is not None:
            self.computeTransform(data=data)

    # ---------------------------------------------------------------- device
    def _context(self):
        if self._h is not None:
            return self._h
        if not self.perfRast:
            raise NotImplementedError("perfRast=0 (interpolated cell raster) is outside the "
                                      "GPU path; FASST builds perfRast=1 transforms")
        k = self.cqtkernel
        B = np.ascontiguousarray(self.B, dtype=np.float64)
        A = np.ascontiguousarray(self.A, dtype=np.float64)
        if B.size != 7 or A.size != 7:
            raise NotImplementedError("the GPU filtfilt handles 6th-order anti-aliasing filters")
        B, A = B / A[0], A / A[0]
        zi = np.ascontiguousarray(spsig.lfilter_zi(B, A), dtype=np.float64)
        spar = np.ascontiguousarray(k.sparKernel, dtype=np.complex128)
        lin = getattr(k, 'linFTLen', 0) if isinstance(self, MinQTransfo) else 0
        lw = (np.ascontiguousarray(k.linWindow, dtype=np.float64) if lin
              else np.zeros(1))
        h = ctypes.c_void_p()
        check(lib.cqt_create(_dev(self.device), int(k.bins), int(self.octaveNr), int(k.winNr),
                             int(k.FFTLen), int(k.fftHOP), int(k.atomHOP), int(k.first_center),
                             dptr(spar), dptr(B), dptr(A), dptr(zi), int(lin),
                             int(getattr(k, 'Kmax', 0)) if lin else 0,
                             int(getattr(k, 'linBins', 0)) if lin else 0, dptr(lw),
                             ctypes.byref(h)), "cqt_create")
        self._h = h
        return h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and lib is not None:
            lib.cqt_destroy(h)
            self._h = None

    def _shape(self, L):
        F, W = ctypes.c_int(0), ctypes.c_int(0)
        nfr = np.zeros(int(self.octaveNr), dtype=np.int32)
        check(lib.cqt_shape(self._context(), L, ctypes.byref(F), ctypes.byref(W),
                            _lib.iptr(nfr)), "cqt_shape")
        return F.value, W.value, nfr

    # ---------------------------------------------------------------- forward
    def computeTransform(self, data):
        """Computes the desired transform (minqt.py:466-469)."""
        return self.computeCQT(data)

    def computeCQT(self, data):
        """Rasterised CQT of data on the GPU (minqt.py:471-646)."""
        if hasattr(self, '_spCQT'):
            del self._spCQT
        if hasattr(self, 'cellCQT'):
            del self.cellCQT
        x = np.ascontiguousarray(np.asarray(data, dtype=np.float64).ravel())
        k = self.cqtkernel
        self.datalen_init = x.shape[0]
        self.maxBlock = int(k.FFTLen * (2 ** (self.octaveNr - 1)))
        self.suffixZeros = self.maxBlock
        self.prefixZeros = self.maxBlock
        F, W, nfr = self._shape(x.size)
        self.nframes = [np.float64(n) for n in nfr]
        sp = np.empty((F, W), dtype=np.complex128)
        check(lib.cqt_forward(self._context(), dptr(x), x.size, dptr(sp)), "cqt_forward")
        self._spCQT = sp

    # ---------------------------------------------------------------- transfo
    def _set_transfo(self, X):
        if X.shape[0] == self.freqbins:
            self._spCQT = np.copy(X)
            if hasattr(self, 'cellCQT'):
                del self.cellCQT
        else:
            raise ValueError('Transfo not of the right size: ' + str(X.shape) +
                             ' instead of ' + str(self.freqbins))

    def _get_transfo(self):
        return self._get_spCQT()

    def _del_transfo(self):
        del self._spCQT
        if hasattr(self, 'cellCQT'):
            del self.cellCQT

    transfo = property(fget=_get_transfo, fdel=_del_transfo, fset=_set_transfo,
                       doc="returns the computed transform")

    def _get_spCQT(self):
        if not hasattr(self, '_spCQT'):
            raise AttributeError("Some CQT should be computed before getting it.")
        return self._spCQT

    def _set_spCQT(self, value):
        self._spCQT = value
        if hasattr(self, 'cellCQT'):
            del self.cellCQT

    spCQT = property(fget=_get_spCQT, fset=_set_spCQT,
                     doc="spCQT: the constant Q transform, in a readable format.")

    def spCQT2CellCQT(self):
        """Per-octave cells from spCQT (minqt.py:949-1011): re-indexing only."""
        k = self.cqtkernel
        bins, winNr = int(k.bins), int(k.winNr)
        emptyHops = k.first_center * 1. / k.atomHOP
        self.cellCQT = {}
        for noct in range(int(self.octaveNr)):
            dropped = emptyHops * (2. ** (self.octaveNr - noct - 1) - 1)
            X = self._spCQT[int(bins * (self.octaveNr - noct - 1)):
                            int(bins * (self.octaveNr - noct)), ::int(2 ** noct)]
            X = np.hstack([np.zeros([bins, int(dropped)]), X])
            X = np.hstack([X, np.zeros([bins, int(np.ceil(X.shape[1] / winNr) * winNr -
                                                  X.shape[1])])])
            if winNr > 1:
                cell = np.zeros([bins * winNr, int(np.ceil(X.shape[1] / winNr))], dtype=complex)
                for nbin in range(bins):
                    cell[nbin * winNr:(nbin + 1) * winNr, :] = X[nbin].reshape(
                        winNr, X.shape[1] // winNr, order='F')
            else:
                cell = np.copy(X)
            self.cellCQT[noct] = np.ascontiguousarray(cell[:, :int(self.nframes[noct])])
        return self.cellCQT

    def _get_time_stamps(self):
        nframes = self.nframes[0] * self.cqtkernel.winNr
        return (np.arange(nframes) * self.cqtkernel.atomHOP +
                self.cqtkernel.first_center * 2 ** (self.octaveNr - 1) - self.prefixZeros)

    time_stamps = property(fget=_get_time_stamps, doc="time stamps for spCQT")

    def _compute_frequencies(self):
        return (self.cqtkernel.fmin *
                2 ** (np.arange(self.cqtkernel.bins * self.octaveNr) / self.cqtkernel.bins -
                      (self.octaveNr - 1)))

    freq_stamps = property(fget=lambda self: self._compute_frequencies(),
                           doc="frequency stamps for spCQT")

    qValues = property(fget=lambda self: self.freq_stamps[:-1] / np.diff(self.freq_stamps),
                       doc="$Q$ values, approximated")

    # ---------------------------------------------------------------- inverse
    def _check_attr_inversion(self):
        for attr in ['datalen_init', 'prefixZeros', 'suffixZeros', 'octaveNr']:
            if not hasattr(self, attr):
                raise AttributeError("Missing attribute to compute the inverse "
                                     "transform: %s." % attr)
        return True

    def _invert(self):
        self._check_attr_inversion()
        sp = np.ascontiguousarray(self._spCQT, dtype=np.complex128)
        y = np.empty(int(self.datalen_init))
        check(lib.cqt_inverse(self._context(), dptr(sp), y.size, dptr(y)), "cqt_inverse")
        return y

    def invertTransform(self):
        """invertFromCellCQT (minqt.py:1013-1055), on the GPU."""
        return self._invert()


class MinQTransfo(CQTransfo):
    """Minimum-Q transform (minqt.py:1369-1550): CQT below the split
    frequency, linear STFT bins above; perfRast=1 runs on the GPU."""
    transformname = 'minqt'

    def __init__(self, fmax, bins, linFTLen, fs, fmin=70, **kwargs):
        data = kwargs.pop('data', None)
        super(MinQTransfo, self).__init__(fmax=fmax, fs=fs, bins=bins, cqtkernel=0, fmin=fmin,
                                          **kwargs)
        self.cqtkernel = MinQTKernel(linFTLen=linFTLen, fmax=fmax, bins=bins, fs=fs, q=self.q,
                                     atomHopFactor=self.atomHopFactor, thresh=self.thresh,
                                     winFunc=self.winFunc, perfRast=self.perfRast)
        self.octaveNr = np.ceil(np.log2(self.cqtkernel.fmax * 1. / fmin))
        self.fmin = (self.cqtkernel.fmax / (2. ** self.octaveNr)) * 2 ** (1. / bins)
        self.freqbins = self.octaveNr * self.cqtkernel.bins + self.cqtkernel.linBins
        if data is not None:
            self.computeTransform(data)

    def computeTransform(self, data):
        """CQT part and linear part in one GPU pass (minqt.py:1404-1450)."""
        super(MinQTransfo, self).computeTransform(data)
        self.offsetSTFT = self.cqtkernel.first_center

    def invertTransform(self):
        """invertFromSpCQTRast + invertLinearPart (minqt.py:1452-1485), on the GPU."""
        if not self.perfRast:
            raise NotImplementedError("perfRast=0 is outside the GPU path")
        return self._invert()

    def _compute_frequencies(self):
        freqs = super(MinQTransfo, self)._compute_frequencies()
        linfreqs = (np.arange(self.cqtkernel.Kmax, self.cqtkernel.Kmax + self.cqtkernel.linBins,
                              dtype=np.float64) * self.cqtkernel.fs / self.cqtkernel.linFTLen)
        return np.concatenate([freqs, linfreqs])

    def spCQT2CellCQT(self):
        """CQT cells plus the linear part (minqt.py:1500-1525): re-indexing only."""
        super(MinQTransfo, self).spCQT2CellCQT()
        k = self.cqtkernel
        emptyHops = k.first_center * 1. / k.atomHOP
        dropped = emptyHops * (2. ** (self.octaveNr - 1) - 1)
        X = self._spCQT[int(k.bins * self.octaveNr):int(k.bins * self.octaveNr + k.linBins)]
        X = np.hstack([np.zeros([int(k.linBins), int(dropped)]), X])
        self.cellCQT['linear'] = np.ascontiguousarray(X[:, :int(self.nframes[0] * k.winNr)])
        return self.cellCQT
