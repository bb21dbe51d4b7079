"""Lead / accompaniment separation from SIMM parameters (reference:
SeparateLeadStereo/SeparateLeadStereoTF.py).

Provided pieces of `SeparateLeadProcess`: the Wiener-like masks of
`writeSeparatedSignals` (:1762-1871), computed on the GPU (`simm_separate`,
include/fasst_simm.h) and inverted with the SIMM-pipeline istft; and the
melody tracking `runViterbi` (:1150-1319), whose Viterbi recursion runs on
the GPU (`viterbi_tracking`, include/fasst_viterbi.h) -- the transition
matrix and log-density of the HMM are built on the host exactly as the
reference builds them.  The rest of the pipeline (file handling, F0
estimation driver, chunking) is outside the accelerated path.
"""
import ctypes

import numpy as np
import scipy.io.wavfile as wav

from .. import _lib
from . import separateLeadFunctions as slf
from .tracking._tracking import viterbiTracking as viterbiTrackingArray

eps = 10 ** -9      # SeparateLeadStereoTF.py:31


def separate_lead_stfts(SIMMParams, XR, XL, device=None):
    """(lead_R, lead_L, accomp_R, accomp_L) masked STFTs of
    writeSeparatedSignals (SeparateLeadStereoTF.py:1785-1846)."""
    P = SIMMParams
    WF0, HF0 = np.asarray(P['WF0'], float), np.asarray(P['HF0'], float)
    WGAMMA, HGAMMA = np.asarray(P['WGAMMA'], float), np.asarray(P['HGAMMA'], float)
    HPHI, HM, WM = np.asarray(P['HPHI'], float), np.asarray(P['HM'], float), np.asarray(P['WM'], float)
    F, N = XR.shape
    NF0, P_, K, R = WF0.shape[1], WGAMMA.shape[1], HPHI.shape[0], HM.shape[0]
    bR, bL = np.asarray(P['betaR'], float), np.asarray(P['betaL'], float)
    if bR.ndim == 2:        # the reference keeps the np.diag matrices (SIMM.py:943)
        bR, bL = np.diag(bR), np.diag(bL)
    from .SIMM.SIMM import _SimmContext, _c
    dev = _lib.default_device() if device is None else device
    ctx = _SimmContext(F, N, NF0, P_, K, R, True, dev)
    _lib.check(_lib.lib.simm_set_data(ctx.ptr, None, None, _lib.dptr(_c(WF0)),
                                      _lib.dptr(_c(WGAMMA))), "simm_set_data")
    alpha = np.array([float(P['alphaR']), float(P['alphaL'])])
    _lib.check(_lib.lib.simm_set_params(ctx.ptr, *[_lib.dptr(_c(a)) for a in
                                                   (HGAMMA, HPHI, HF0, HM, WM, alpha, bR, bL)]),
               "simm_set_params")
    XRc = np.ascontiguousarray(XR, dtype=np.complex128)
    XLc = np.ascontiguousarray(XL, dtype=np.complex128)
    outs = [np.empty((F, N), dtype=np.complex128) for _ in range(4)]
    _lib.check(_lib.lib.simm_separate(ctx.ptr, _lib.dptr(XRc), _lib.dptr(XLc),
                                      *[_lib.dptr(o) for o in outs]), "simm_separate")
    return tuple(outs)


class SeparateLeadProcess(object):
    """Holds the state `writeSeparatedSignals` reads (SeparateLeadStereoTF.py
    :1762-1871): SIMMParams, stftParams, XR, XL, files, fs, scaleData,
    dataType, tfrepresentation ('stft' only on this path)."""

    def __init__(self, SIMMParams=None, stftParams=None, XR=None, XL=None, files=None,
                 fs=44100, scaleData=1.0, dataType=np.int16, tfrepresentation='stft',
                 trackingParams=None, N=None, verbose=False, device=None):
        self.SIMMParams = SIMMParams
        self.stftParams = stftParams
        self.XR, self.XL = XR, XL
        self.files = files or {}
        self.fs = fs
        self.scaleData = scaleData
        self.dataType = dataType
        self.tfrepresentation = tfrepresentation
        self.trackingParams = trackingParams or {'minF0search': None, 'maxF0search': None}
        if N is not None:
            self.N = N
        self.verbose = verbose
        self.device = device

    def computeNFrames(self):
        """Number of frames; here the caller provides N (or HF0 defines it)."""
        if not hasattr(self, 'N'):
            self.N = np.asarray(self.SIMMParams['HF0']).shape[1]

    def runViterbi(self):
        """Melody line by Viterbi decoding of HF0 (SeparateLeadStereoTF.py:1150-1319)."""
        if not ('HF0' in self.SIMMParams.keys()):
            raise AttributeError("HF0 has probably not been estimated yet.")
        self.computeNFrames()
        scale = 1.0
        P = self.SIMMParams
        NF0 = P['NF0'] * P['chirpPerF0']
        nmaxF0, nminF0 = NF0, 0
        minF0, maxF0 = P['minF0'], P['maxF0']
        minF0search = self.trackingParams['minF0search']
        maxF0search = self.trackingParams['maxF0search']
        if minF0search is not None and minF0search > minF0 and minF0search < maxF0:
            nminF0 = np.where(P['F0Table'] >= minF0search)[0][0] * P['chirpPerF0']
        if (maxF0search is not None and maxF0search > minF0 and maxF0search < maxF0 and
                maxF0search > minF0search):
            nmaxF0 = (np.where(P['F0Table'] >= maxF0search)[0][0] + 1) * P['chirpPerF0']
        NF0 = nmaxF0 - nminF0
        # Toeplitz note-distance transitions + silence state, row-normalised (:1183-1208)
        transitions = np.exp(-np.floor(np.arange(0, NF0) / P['stepNotes']) * scale)
        cutoffnote = np.minimum(NF0, 2 * 5 * P['stepNotes'])
        transitions[cutoffnote:] = transitions[cutoffnote - 1]
        T = np.zeros([NF0 + 1, NF0 + 1])
        b = np.arange(NF0)
        T[0:NF0, 0:NF0] = transitions[np.array(np.abs(np.outer(np.ones(NF0), b) -
                                                      np.outer(b, np.ones(NF0))), dtype=int)]
        T[0:NF0, NF0] = transitions[cutoffnote - 1] * 10 ** (-90)
        T[NF0, 0:NF0] = transitions[cutoffnote - 1] * 10 ** (-80)
        T[NF0, NF0] = transitions[cutoffnote - 1] * 10 ** (-100)
        T = T / np.outer(np.sum(T, axis=1), np.ones(NF0 + 1))
        prior = 1 / (NF0 + 1.0) * np.ones([NF0 + 1])
        # log-density with the reference's floor for empty frames (:1210-1216)
        HF0 = np.asarray(P['HF0'])
        logHF0 = np.zeros([NF0 + 1, self.N])
        normHF0 = np.amax(HF0[nminF0:nmaxF0], axis=0)
        with np.errstate(divide='ignore'):
            logHF0[0:NF0, :] = np.log(HF0[nminF0:nmaxF0])
        logHF0[0:NF0, normHF0 == 0] = np.amin(logHF0[logHF0 > -np.inf])
        logHF0[NF0, :] = np.maximum(np.amin(logHF0[logHF0 > -np.inf]), -100)
        with np.errstate(divide='ignore'):
            logT, logprior = np.log(T), np.log(prior)
        # the pipeline tracks NF0 states of the NF0 + 1 rows (:1220-1222)
        indexBestPath = viterbiTrackingArray(NF0, self.N, logHF0, logprior, logT,
                                             verbose=False, device=self.device)
        indexBestPath += nminF0
        freqMelody = P['F0Table'][np.array(indexBestPath / P['chirpPerF0'], dtype=int)]
        freqMelody[indexBestPath == 0] = - freqMelody[indexBestPath == 0]
        if 'pitch_output_file' in self.files:
            np.savetxt(self.files['pitch_output_file'],
                       np.array([np.arange(self.N) * self.stftParams['hopsize'] /
                                 np.double(self.fs), freqMelody]).T)
        self.indexBestPath = indexBestPath
        self.freqMelody = freqMelody

    def separated_signals(self, suffix='.wav'):
        """(vest [2][L], mest [2][L]) float waveforms before int conversion."""
        if self.tfrepresentation != 'stft':
            raise NotImplementedError("tfrepresentation %r: only 'stft' runs on the GPU path"
                                      % self.tfrepresentation)
        P = dict(self.SIMMParams)
        if 'VUIMM' in suffix:
            P['WF0'], P['HF0'] = P['WUF0'], P['HUF0']
        vR, vL, mR, mL = separate_lead_stfts(P, self.XR, self.XL, device=self.device)
        w = slf.sinebell(self.stftParams['windowSizeInSamples'])
        kw = dict(hopsize=self.stftParams['hopsize'], nfft=self.stftParams['NFT'], window=w,
                  originalDataLen=None, device=self.device)
        return ([slf.istft(vR, **kw), slf.istft(vL, **kw)],
                [slf.istft(mR, **kw), slf.istft(mL, **kw)])

    def writeSeparatedSignals(self, suffix='.wav'):
        """SeparateLeadStereoTF.py:1762-1871"""
        (vR, vL), (mR, mL) = self.separated_signals(suffix)
        vR = np.array(np.round(vR * self.scaleData), dtype=self.dataType)
        vL = np.array(np.round(vL * self.scaleData), dtype=self.dataType)
        wav.write(self.files['voc_output_file'][:-4] + suffix, self.fs, np.array([vR, vL]).T)
        mR = np.array(np.round(mR * self.scaleData), dtype=self.dataType)
        mL = np.array(np.round(mL * self.scaleData), dtype=self.dataType)
        wav.write(self.files['mus_output_file'][:-4] + suffix, self.fs, np.array([mR, mL]).T)

    def writeSeparatedSignalsWithUnvoice(self):
        """SeparateLeadStereoTF.py:1873-1878"""
        self.writeSeparatedSignals(suffix='_VUIMM.wav')
