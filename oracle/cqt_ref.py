"""NumPy/SciPy CPU restatement of the reference CQT / MinQT front end.

TEST INFRASTRUCTURE ONLY (the checker, never the product): imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the product
package `pyfasst_amd` never imports it.

Restates /root/reference/pyfasst/tftransforms/minqt.py
for the configuration FASST uses, perfRast=1 (audioModel.py:206-214):

  cqt_kernel()        CQTKernel.__init__            minqt.py:95-227
  minqt_kernel()      MinQTKernel.__init__          minqt.py:312-335
  RefCQT.forward()    CQTransfo.computeCQT, perfRast branch   minqt.py:471-486,523-646
                      + MinQTransfo.computeLinearPart          minqt.py:1410-1450
                      + linCellCQT2LinSpCQT                    minqt.py:1534-1549
  RefCQT.sp_to_cell() CQTransfo.spCQT2CellCQT       minqt.py:949-1011
                      (+ MinQTransfo.spCQT2CellCQT  minqt.py:1500-1525)
  RefCQT.inverse()    MinQT: invertFromSpCQTRast + invertLinearPart
                      (minqt.py:794-868, 1462-1485);
                      CQT:   invertFromCellCQT      (minqt.py:1013-1055)

Pinned against golden vectors produced by running the reference itself
(scratch py3 translation, oracle/make_scratch_ref.py) in
tests/golden/make_golden.py (cases cqt_*, minqt_*).

The reference's quirks are kept: the drop alignment leaves the last
`drop*nshifts` columns of each octave's rows at their pre-shift values
(minqt.py:639-642); the rasterised inverse re-derives every octave's cells
for each shift from a left-shifted spCQT (minqt.py:824-851); 'cqt' inverts
through invertFromCellCQT even with perfRast=1 (minqt.py:1013-1017).
"""
import os
import sys

import numpy as np
import scipy.signal as spsig

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fasst_ref  # noqa: E402


def nextpow2(i):
    """tools/utils.py:30-41"""
    n = 2
    while n < i:
        n = n * 2
    return n


def sqrt_blackmanharris(M):
    """tools/utils.py:67-72"""
    return np.sqrt(spsig.windows.blackmanharris(M))


class Kernel(object):
    pass


def cqt_kernel(fmax, bins, fs, q=1, atomHopFactor=0.25, thresh=0.0005,
               winFunc=sqrt_blackmanharris, perfRast=0):
    """CQTKernel.__init__ (minqt.py:95-227)."""
    if fmax >= fs / 2.:
        raise ValueError("fmax (%s) is too big for fs (%s)" % (str(fmax), str(fs)))
    k = Kernel()
    fmin = (fmax / 2.) * (2 ** (1. / bins))
    Q = 1. / (2 ** (1. / bins) - 1) * q
    Nk_max = np.round(Q * fs / fmin)
    Nk_min = np.round(Q * fs / (fmin * (2 ** ((bins - 1.) / bins))))
    atomHOP = nextpow2(Nk_min * atomHopFactor) // 2          # py2 int / 2
    first_center = np.ceil(Nk_max / 2.)
    first_center = atomHOP * np.ceil(first_center * 1. / atomHOP)
    FFTLen = nextpow2(first_center + np.ceil(Nk_max / 2.))
    winNr = np.floor((FFTLen - np.ceil(Nk_max / 2.) - first_center) / atomHOP) + 1
    if perfRast and winNr == 0:                               # minqt.py:142-145
        FFTLen = FFTLen * 2
        winNr = np.floor((FFTLen - np.ceil(Nk_max / 2.) - first_center) / atomHOP)
    last_center = first_center + (winNr - 1.) * atomHOP
    fftHOP = (last_center + atomHOP) - first_center
    spar = np.zeros([int(bins * winNr), int(FFTLen)], dtype=complex)
    freqs = []
    for kk in np.arange(bins):                                # minqt.py:166-192
        Nk = np.round(Q * fs / (fmin * (2 ** ((kk * 1.) / bins))))
        winFct = winFunc(int(Nk))
        fk = fmin * (2 ** ((kk * 1.) / bins))
        freqs.append(fk)
        tkb = (winFct * 1. / Nk) * np.exp(2 * np.pi * 1j * fk * np.arange(Nk) / fs)
        atomOffset = first_center - np.ceil(Nk / 2.)
        for i in np.arange(winNr):
            shift = atomOffset + i * atomHOP
            temp = np.zeros(int(FFTLen), dtype=complex)
            temp[int(shift):int(Nk + shift)] = tkb
            spec = np.fft.fft(temp)
            spec[np.abs(spec) <= thresh] = 0
            spar[int(i + kk * winNr)] = spec
    spar = (spar.T) * 1. / FFTLen
    # atom magnitude normalisation (minqt.py:196-207)
    wx1 = np.argmax(spar[:, 0])
    wx2 = np.argmax(spar[:, -1])
    wK = spar[wx1:wx2, :]
    wK = np.diag(np.dot(wK, np.conjugate(wK.T)))
    wK = wK[int(np.round(1. / q)):int(len(wK) - np.round(1. / q) - 1)]
    weight = 1. / np.mean(np.abs(wK))
    weight *= (fftHOP * 1. / FFTLen)
    weight = np.sqrt(weight)
    spar *= weight
    k.sparKernel = np.ascontiguousarray(spar)       # [FFTLen, bins*winNr]
    k.weight, k.atomHOP, k.FFTLen, k.fftHOP = weight, atomHOP, FFTLen, fftHOP
    k.bins, k.winNr, k.Nk_max, k.Q, k.fmin, k.fmax = bins, winNr, Nk_max, Q, fmin, fmax
    k.frequencies, k.perfRast, k.first_center, k.fs = freqs, perfRast, first_center, fs
    k.winFunc, k.thresh, k.q = winFunc, thresh, q
    return k


def minqt_kernel(bins, fmax, fs, linFTLen=2048, **kw):
    """MinQTKernel.__init__ (minqt.py:312-335): the CQT part stops where the
    linear-frequency STFT bins are at least as dense as the CQT bins."""
    Q = 1. / (2 ** (1. / bins) - 1)
    Kmax = int(np.ceil(Q))
    fmax = 2 ** (-1. / bins) * Kmax * fs * 1. / linFTLen
    k = cqt_kernel(fmax=fmax, bins=bins, fs=fs, **kw)
    k.Qmin, k.Kmax, k.linFTLen = Q, Kmax, linFTLen
    k.linBins = linFTLen // 2 - Kmax + 1
    k.linWindow = k.winFunc(linFTLen)
    return k


def stft(data, window, hopsize, nfft):
    """tftransforms/stft.py:3-69 (fasst_ref.stft)"""
    return fasst_ref.stft(data, window, int(hopsize), int(nfft))


def istft(X, window, hopsize, nfft):
    """tftransforms/stft.py:71-131 with analysisWindow=None (fasst_ref.istft)"""
    return fasst_ref.istft(X, window, window, int(hopsize), int(nfft))


class RefCQT(object):
    """CQTransfo / MinQTransfo with perfRast=1, as FASST builds them
    (audioModel.py:206-214: fmin=tffmin, fmax=tffmax, bins=tfbpo, fs,
    perfRast=1, linFTLen=fsize, atomHopFactor=hopsize/wlen)."""

    def __init__(self, kind, fmin, fmax, bins, fs, linFTLen=2048, atomHopFactor=0.25,
                 q=1, thresh=0.0005, winFunc=None):
        if winFunc is None:
            winFunc = sqrt_blackmanharris
        self.kind = kind
        self.bins, self.fs = bins, fs
        self.B, self.A = spsig.butter(N=6, Wn=0.5, btype='low')     # minqt.py:441-447
        kw = dict(q=q, atomHopFactor=atomHopFactor, thresh=thresh, winFunc=winFunc, perfRast=1)
        if kind == 'cqt':                                             # minqt.py:436-459
            self.octaveNr = np.ceil(np.log2(fmax * 1. / fmin))
            self.k = cqt_kernel(fmax=fmax, bins=bins, fs=fs, **kw)
            self.freqbins = bins * self.octaveNr
        else:                                                         # minqt.py:1377-1399
            self.k = minqt_kernel(bins=bins, fmax=fmax, fs=fs, linFTLen=linFTLen, **kw)
            self.octaveNr = np.ceil(np.log2(self.k.fmax * 1. / fmin))
            self.freqbins = self.octaveNr * bins + self.k.linBins
        self.fmin = (self.k.fmax / (2. ** self.octaveNr)) * 2 ** (1. / bins)

    # ------------------------------------------------------------ forward
    def forward(self, data):
        """computeCQT perfRast branch (minqt.py:471-486, 523-646) and, for
        MinQT, computeLinearPart (minqt.py:1410-1450)."""
        k = self.k
        data = np.asarray(data)
        if not np.iscomplexobj(data):
            data = data.astype(np.float64)
        self.datalen_init = data.shape[0]
        oct_n = int(self.octaveNr)
        self.maxBlock = int(k.FFTLen * (2 ** (self.octaveNr - 1)))
        self.prefixZeros = self.suffixZeros = self.maxBlock
        x = np.concatenate([np.zeros(self.prefixZeros), data, np.zeros(self.suffixZeros)])
        K = np.ascontiguousarray(np.conjugate(k.sparKernel.T))      # [bins*winNr, FFTLen]
        self.nframes = []
        atomNr = int(k.winNr)
        emptyHops = k.first_center * 1. / k.atomHOP
        ahop = k.atomHOP
        N = int(k.FFTLen)
        sp = None
        for i in range(oct_n):
            inc = ahop / (2. ** i)
            binVec = np.int32(self.bins * (self.octaveNr - i - 1) + np.arange(self.bins))
            drop = emptyHops * (2 ** (self.octaveNr - i - 1) - 1)
            nframes = np.floor(((x.size - k.FFTLen) / k.fftHOP) + 1)
            self.nframes.append(nframes)
            nfr = int(nframes)
            if i == 0:
                sp = np.zeros([int(self.bins * self.octaveNr), nfr * atomNr], dtype=complex)
            XX = np.zeros([N, nfr], dtype=complex)
            for n in range(nfr):
                fs_ = int(n * k.fftHOP)
                XX[:, n] = np.fft.fft(x[fs_:fs_ + N], n=N)
            nshifts = int(2 ** i)
            for nshift in range(nshifts):
                shift = nshift * inc
                ph = np.exp(1j * 2 * np.pi * np.arange(N) * shift / N)
                CQTframe = np.dot(K * ph, XX)
                if atomNr > 1:
                    for nb, b in enumerate(binVec):
                        for a in range(atomNr):
                            sp[b, int(nshift + a * nshifts):int(nfr * atomNr * nshifts):
                               int(atomNr * nshifts)] = CQTframe[int(nb * atomNr + a)]
                else:
                    sp[binVec, int(nshift):int(nfr * nshifts):nshifts] = CQTframe
            d = int(drop * nshifts)
            for b in binVec:                                          # minqt.py:639-642
                sp[b, :(sp.shape[1] - d)] = sp[b, d:].copy()
            if i != oct_n - 1:
                x = spsig.filtfilt(self.B, self.A, x)[::2]
        if self.kind != 'cqt':
            sp = self._linear_part(data, sp)
        self.spCQT = sp
        return sp

    def _linear_part(self, data, sp):
        """computeLinearPart + linCellCQT2LinSpCQT (minqt.py:1410-1450, 1534-1549)"""
        k = self.k
        x = np.concatenate([np.zeros(self.prefixZeros), data, np.zeros(self.suffixZeros)])
        self.offsetSTFT = k.first_center
        # a complex signal (the SIMM dictionary's comb, separateLeadFunctions.py
        # :838-847): the rfft of stft.py:3-69 kept its real part (numpy < 1.13)
        X = stft(np.real(x[int(self.offsetSTFT):]), k.linWindow, k.atomHOP, k.linFTLen)
        lin = X[k.Kmax:, :int(self.nframes[0] * k.winNr)]
        W = sp.shape[1]
        out = np.vstack([sp, np.zeros([int(k.linBins), W], dtype=complex)])
        emptyHops = k.first_center * 1. / k.atomHOP
        drop = int(emptyHops * (2 ** (self.octaveNr - 1) - 1))
        out[int(self.bins * self.octaveNr):, :W - drop] = lin[:, drop:]
        return out

    # ------------------------------------------------------------ cells
    def sp_to_cell(self, sp, noct):
        """CQTransfo.spCQT2CellCQT for one octave (minqt.py:949-1011)."""
        k = self.k
        bins, winNr = self.bins, int(k.winNr)
        emptyHops = k.first_center * 1. / k.atomHOP
        dropped = emptyHops * (2. ** (self.octaveNr - noct - 1) - 1)
        X = sp[int(bins * (self.octaveNr - noct - 1)):int(bins * (self.octaveNr - noct)),
               ::int(2 ** noct)]
        X = np.hstack([np.zeros([bins, int(dropped)]), X])
        X = np.hstack([X, np.zeros([bins, int(np.ceil(X.shape[1] / winNr) * winNr - X.shape[1])])])
        if winNr > 1:
            cell = np.zeros([bins * winNr, int(np.ceil(X.shape[1] / winNr))], dtype=complex)
            for nbin in range(bins):
                cell[nbin * winNr:(nbin + 1) * winNr, :] = X[nbin].reshape(
                    winNr, X.shape[1] // winNr, order='F')
        else:
            cell = np.copy(X)
        return np.ascontiguousarray(cell[:, :int(self.nframes[noct])])

    def linear_cell(self, sp):
        """MinQTransfo.spCQT2CellCQT linear rows (minqt.py:1508-1525)."""
        k = self.k
        emptyHops = k.first_center * 1. / k.atomHOP
        dropped = emptyHops * (2. ** (self.octaveNr - 1) - 1)
        X = sp[int(self.bins * self.octaveNr):int(self.bins * self.octaveNr + k.linBins)]
        X = np.hstack([np.zeros([int(k.linBins), int(dropped)]), X])
        return np.ascontiguousarray(X[:, :int(self.nframes[0] * k.winNr)])

    # ------------------------------------------------------------ inverse
    def _upsample(self, y):
        newy = np.zeros(int(y.size * 2))
        newy[::2] = y
        return spsig.filtfilt(self.B, self.A, newy) * 2

    def inverse(self, sp):
        """invertTransform of the transform last computed by forward()."""
        if self.kind == 'cqt':
            return self._invert_from_cells(sp)
        y = self._invert_rast(sp)
        return y + self._invert_linear(sp)

    def _invert_from_cells(self, sp):
        """invertFromCellCQT (minqt.py:1019-1055)"""
        k = self.k
        K = np.ascontiguousarray(k.sparKernel)
        N = int(k.FFTLen)
        y = np.zeros(int(np.ceil(self.datalen_init / (2. ** (self.octaveNr - 1)))))
        for noct in range(int(self.octaveNr) - 1, -1, -1):
            cell = self.sp_to_cell(sp, noct)
            Y = np.dot(K, cell)
            nframes = cell.shape[1]
            ylen = int(k.fftHOP * (nframes - 1) + k.FFTLen)
            if ylen > y.size:
                y = np.concatenate([y, np.zeros(ylen - y.size)])
            for n in range(nframes):
                a = int(n * k.fftHOP)
                y[a:a + N] += 2. * np.real(np.fft.ifft(Y[:, n], n=N))
            if noct != 0:
                y = self._upsample(y)
        y = y[int(self.prefixZeros):]
        return y[:int(self.datalen_init)]

    def _invert_rast(self, sp):
        """invertFromSpCQTRast (minqt.py:794-868): for shift s of octave noct
        the cells come from the octave rows shifted left s times (the last
        column repeats)."""
        k = self.k
        K = np.ascontiguousarray(k.sparKernel)
        N = int(k.FFTLen)
        y = np.zeros(int(np.ceil(self.datalen_init / (2. ** (self.octaveNr - 1)))))
        ahop = k.atomHOP
        work = np.copy(sp)
        for noct in range(int(self.octaveNr) - 1, -1, -1):
            inc = ahop / (2. ** noct)
            nshifts = int(2 ** noct)
            nframes = int(self.nframes[noct])
            ylen = k.fftHOP * (nframes - 1) + k.FFTLen + nshifts * inc
            if ylen > y.size:
                y = np.concatenate([y, np.zeros(int(ylen - y.size))])
            r0 = int(self.bins * (self.octaveNr - noct - 1))
            r1 = int(self.bins * (self.octaveNr - noct))
            for nshift in range(nshifts):
                Y = np.dot(K, self.sp_to_cell(work, noct))
                for n in range(nframes):
                    a = int(n * k.fftHOP + nshift * inc)
                    yoct = np.fft.ifft(Y[:, n], n=N) / np.double(nshifts)
                    y[a:a + N] += 2. * np.real(yoct)
                work[r0:r1, :-1] = work[r0:r1, 1:].copy()
            if noct != 0:
                y = self._upsample(y)
        y = y[int(self.prefixZeros):]
        return y[:int(self.datalen_init)]

    def _invert_linear(self, sp):
        """invertLinearPart (minqt.py:1469-1485)"""
        k = self.k
        lin = self.linear_cell(sp)
        Y = np.zeros([k.linFTLen // 2 + 1, lin.shape[1]], dtype=complex)
        Y[k.Kmax:] = lin
        y = istft(Y, k.linWindow, k.atomHOP, k.linFTLen)
        y = y[int(self.prefixZeros - self.offsetSTFT):]
        return y[:int(self.datalen_init)]

    def freq_stamps(self):
        """_compute_frequencies (minqt.py:700-707, 1487-1498)"""
        k = self.k
        f = k.fmin * 2 ** (np.arange(k.bins * self.octaveNr) / k.bins - (self.octaveNr - 1))
        if self.kind == 'cqt':
            return f
        lin = np.arange(k.Kmax, k.Kmax + k.linBins, dtype=np.float64) * k.fs / k.linFTLen
        return np.concatenate([f, lin])
