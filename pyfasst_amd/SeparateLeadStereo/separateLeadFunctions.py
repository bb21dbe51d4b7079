"""SIMM-pipeline STFT / iSTFT and dictionaries on the GPU (reference:
SeparateLeadStereo/separateLeadFunctions.py:90-233, :696-886, :1074-1146).

These differ from tftransforms/stft.py: `stft` takes a start/stop frame range
and pads half a window at both ends (:90-161); `istft` keeps the leading half
window and patches the first / last window of the normalisation from their
neighbours (:163-233).  FFTs and overlap-add run in libfasst_hip.so.
"""
import ctypes

import numpy as np

from .. import _lib
from .._lib import check, dptr, lib
from ..tools.utils import nextpow2, sinebell

__all__ = ["nextpow2", "sinebell", "stft", "istft", "generate_WF0_TR_chirped", "generateHannBasis"]


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


# ---------------------------------------------------------------- dictionaries
def _odgd_amplitudes(F0, Ot, partialMax):
    """KLGLOTT88 partial amplitudes, the reference's expression
    (separateLeadFunctions.py:916-930); host-side parameters of the GPU synthesis."""
    frequency_numbers = np.arange(1, partialMax + 1)
    temp_array = 1j * 2.0 * np.pi * frequency_numbers * Ot
    return (F0 * 27 / 4 * (np.exp(-temp_array) + (2 * (1 + 2 * np.exp(-temp_array)) / temp_array) -
                           (6 * (1 - np.exp(-temp_array)) / (temp_array ** 2))) / temp_array)


def _comb_columns(F0Table, Fs, Ot, perF0, depthChirpInSemiTone):
    """Columns of WF0 (:829-879): the F0 comb, then perF0 - 1 chirps around
    it; per column F1, F2 and the KLGLOTT88 partial amplitudes."""
    f1, f2, amps = [], [], []
    for i in range(F0Table.size):
        F0 = F0Table[i]
        f1.append(F0)
        f2.append(F0)
        amps.append(_odgd_amplitudes(F0, np.double(Ot), np.floor((Fs / 2) / F0)))
        for c in range(perF0 - 1):
            F2 = F0 * (2 ** ((c + 1.0) * depthChirpInSemiTone / (12.0 * (perF0 - 1.0))))
            F1 = 2.0 * F0 - F2
            f1.append(np.double(F1))
            f2.append(np.double(F2))
            amps.append(_odgd_amplitudes(np.double(F1 + F2) / 2.0, np.double(Ot),
                                         np.floor((Fs / 2) / np.max([F1, F2]))))
    ncol = len(f1)
    npart = np.array([a.size for a in amps], dtype=np.int32)
    pmax = max(1, int(npart.max()))
    A = np.zeros((ncol, pmax), dtype=np.complex128)
    for j, a in enumerate(amps):
        A[j, :a.size] = a
    return (np.ascontiguousarray(f1, dtype=np.float64), np.ascontiguousarray(f2, dtype=np.float64),
            npart, pmax, A)


def generate_WF0_TR_chirped(transform, minF0, maxF0, stepNotes=4, Ot=0.5, perF0=1,
                            depthChirpInSemiTone=0.5, loadWF0=True, verbose=False,
                            device=None):
    """F0Table, WF0, transform = generate_WF0_TR_chirped(...)
    (separateLeadFunctions.py:696-886).

    WF0[:, j] = |transform(odgd_j)[:, middle frame]|^2, the KLGLOTT88 comb
    odgd_j synthesised on the GPU.  For the STFT transform
    (SeparateLeadProcess' default tfrepresentation 'stft') one workgroup per
    column synthesises and transforms only the middle frame (dict_wf0_stft,
    include/fasst_dict.h).  For a CQT / MinQT transform (tfrepresentation
    'cqt' / 'minqt' / 'mqt') the whole comb of FFTLen * 2^(octaveNr-1)
    samples goes through the GPU transform and the middle column is kept
    (dict_wf0_cqt, include/fasst_cqt.h).  The cache file holds F0Table and
    WF0 only (the reference also pickles the transform object)."""
    import os
    cqt = hasattr(transform, 'cqtkernel')
    if cqt:
        k = transform.cqtkernel
        if hasattr(transform, 'octaveNr'):                          # :742-744
            lengthWindow = int(k.FFTLen * (2 ** (transform.octaveNr - 1)))
        else:
            lengthWindow = int(k.linFTLen)
        geo = '_'.join(['atomhopfactor-%s' % str(transform.atomHopFactor),
                        'bins-%s' % str(transform.bins), 'fmax-%s' % str(transform.fmax),
                        'fmin-%s' % str(transform.fmin), 'freqbins-%s' % str(transform.freqbins),
                        'fs-%s' % str(transform.fs),
                        getattr(transform.winFunc, '__name__', 'w')])
    else:
        lengthWindow = (transform.freqbins - 1) * 2 * 2
        geo = '_'.join(['fs-%s' % str(transform.fs), 'ftlen-%d' % transform.ftlen,
                        'hop-%d' % transform.fthop,
                        'win-%s' % getattr(transform.winFunc, '__name__', 'w')])
    filename = ''.join(['wf0gpu_%s_' % transform.transformname, '_minF0-', str(minF0),
                        '_maxF0-', str(maxF0), '_stepNotes-', str(int(stepNotes)),
                        '_Ot-', str(Ot), '_perF0-', str(int(perF0)),
                        '_depthChirp-', str(depthChirpInSemiTone),
                        '_lengthWindow-%d' % lengthWindow, '_', geo, '.npz'])
    if os.path.isfile(filename) and loadWF0:
        struc = np.load(filename)
        return struc['F0Table'], struc['WF0'], transform
    minF0, maxF0 = np.double(minF0), np.double(maxF0)
    Fs, stepNotes = np.double(transform.fs), np.double(stepNotes)
    numberOfF0 = np.ceil(12.0 * stepNotes * np.log2(maxF0 / minF0)) + 1
    F0Table = minF0 * (2 ** (np.arange(numberOfF0, dtype=np.double) / (12 * stepNotes)))
    f1a, f2a, npart, pmax, A = _comb_columns(F0Table, Fs, Ot, perF0, depthChirpInSemiTone)
    ncol = f1a.size
    if cqt:
        # the transform's geometry for a signal of lengthWindow samples and
        # the reference's midindex = argmin (datalen_init / 2 - time_stamps)^2
        F, W, nfr = transform._shape(lengthWindow)
        maxBlock = int(k.FFTLen * (2 ** (transform.octaveNr - 1)))
        time_stamps = (np.arange(nfr[0] * k.winNr) * k.atomHOP +
                       k.first_center * 2 ** (transform.octaveNr - 1) - maxBlock)
        mid = int(np.argmin((lengthWindow / 2. - time_stamps) ** 2))
        WF0 = np.empty((F, ncol))
        check(lib.dict_wf0_cqt(transform._context(), ncol, dptr(f1a), dptr(f2a),
                               _lib.iptr(npart), pmax, dptr(A), float(Fs), int(lengthWindow), mid,
                               dptr(WF0)), "dict_wf0_cqt")
    else:
        # the middle frame of the transform's STFT of an lengthWindow-sample
        # signal (STFT.computeTransform, :838-847 with stft.py:3-69, :383-385)
        hop = int(transform.fthop)
        nfr = int(np.ceil(lengthWindow / np.double(hop))) + 2
        time_stamps = np.arange(nfr) * hop / np.double(transform.fs)
        time_stamps *= transform.fs
        mid = int(np.argmin((lengthWindow / 2. - time_stamps) ** 2))
        window = np.ascontiguousarray(transform.window, dtype=np.float64)
        frame_start = mid * hop - window.size // 2
        WF0 = np.empty((transform.freqbins, ncol))
        dev = _dev(device if device is not None else getattr(transform, 'device', None))
        check(lib.dict_wf0_stft(dev, ncol, dptr(f1a), dptr(f2a), _lib.iptr(npart), pmax, dptr(A),
                                float(Fs), int(lengthWindow), dptr(window), window.size,
                                int(transform.ftlen), int(frame_start), dptr(WF0)),
              "dict_wf0_stft")
    try:
        np.savez(filename, F0Table=F0Table, WF0=WF0)
    except OSError:
        pass
    return F0Table, WF0, transform


def generateHannBasis(numberFrequencyBins, sizeOfFourier, Fs, frequencyScale='linear',
                      numberOfBasis=20, overlap=.75):
    """WGAMMA: overlapping Hann bumps along the frequency axis
    (separateLeadFunctions.py:1074-1146; a few hundred host-side numbers)."""
    if frequencyScale != 'linear':
        print("The desired feature for frequencyScale is not recognized yet...")
        return 0
    numberOfWindowsForUnit = np.ceil(1.0 / (1.0 - overlap))
    overlap = 1.0 - 1.0 / np.double(numberOfWindowsForUnit)
    lengthSineWindow = np.ceil(numberFrequencyBins / ((1.0 - overlap) * (numberOfBasis - 1) + 1 -
                                                      2.0 * overlap))
    lengthSineWindow = 2.0 * np.floor(lengthSineWindow / 2.0)
    mappingFrequency = np.arange(numberFrequencyBins)
    sizeBigWindow = 2.0 * numberFrequencyBins
    firstWindowCenter = -numberOfWindowsForUnit + 1
    lastWindowCenter = numberOfBasis - numberOfWindowsForUnit + 1
    sineCenters = np.round(np.arange(firstWindowCenter, lastWindowCenter) * (1 - overlap) *
                           np.double(lengthSineWindow) + lengthSineWindow / 2.0)
    prototypeSineWindow = np.hanning(int(lengthSineWindow))
    bigWindow = np.zeros([int(sizeBigWindow * 2), 1])
    bigWindow[int(sizeBigWindow - lengthSineWindow / 2.0):
              int(sizeBigWindow + lengthSineWindow / 2.0)] = np.vstack(prototypeSineWindow)
    WGAMMA = np.zeros([numberFrequencyBins, numberOfBasis])
    for p in np.arange(numberOfBasis):
        WGAMMA[:, p] = np.hstack(bigWindow[np.int32(mappingFrequency - sineCenters[p] +
                                                    sizeBigWindow)])
    return WGAMMA
