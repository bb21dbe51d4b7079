"""Lead / accompaniment separation from SIMM parameters (reference:
SeparateLeadStereo/SeparateLeadStereoTF.py).

Only the hot-path piece of `SeparateLeadProcess` is provided: the Wiener-like
masks of `writeSeparatedSignals` (:1762-1871), computed on the GPU
(`simm_separate`, include/fasst_simm.h) and inverted with the SIMM-pipeline
istft.  The rest of the pipeline (file handling, F0 estimation, Viterbi
tracking, chunking) is outside the accelerated path.
"""
import ctypes

import numpy as np
import scipy.io.wavfile as wav

from .. import _lib
from . import separateLeadFunctions as slf

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
                 device=None):
        self.SIMMParams = SIMMParams
        self.stftParams = stftParams
        self.XR, self.XL = XR, XL
        self.files = files or {}
        self.fs = fs
        self.scaleData = scaleData
        self.dataType = dataType
        self.tfrepresentation = tfrepresentation
        self.device = device

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
