"""Lead / accompaniment separation from SIMM parameters (reference:
SeparateLeadStereo/SeparateLeadStereoTF.py).

Provided pieces of `SeparateLeadProcess`: the Wiener-like masks of
`writeSeparatedSignals` (:1762-1871), computed on the GPU (`simm_separate`,
include/fasst_simm.h) and inverted with the SIMM-pipeline istft; and the
melody tracking `runViterbi` (:1150-1319), whose Viterbi recursion runs on
the GPU (`viterbi_tracking`, include/fasst_viterbi.h) -- the transition
matrix and log-density of the HMM are built on the host exactly as the
reference builds them.  `SeparateLeadProcess` (below) drives the chunked WAV
pipeline of the reference (`autoMelSepAndWrite`, `overlapAddChunks`,
`writeSeparatedSignals`) on those kernels and on the GPU
SIMM; only WAV file I/O and the chunk bookkeeping stay on the host.
"""
import ctypes

import numpy as np
import scipy.io.wavfile as wav

from .. import _lib
from . import separateLeadFunctions as slf
from .tracking._tracking import viterbiTracking as viterbiTrackingArray
from ..tools.nnls import nnls_columns

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


knownTransfos = ['stft', 'hybridcqt', 'minqt', 'cqt', 'mqt']   # SeparateLeadStereoTF.py:33


class SeparateLeadProcess(object):
    """Lead / accompaniment separation process (SeparateLeadStereoTF.py:36-1897).

    Built like the reference from a WAV file name and its keyword arguments
    (:263-540): the STFTs, the KLGLOTT88 source dictionary WF0 and the
    Hann filter basis are computed at construction; `autoMelSepAndWrite`
    (:1142-1148) runs the chunked pipeline -- mono SIMM per chunk for HF0,
    Viterbi melody, stereo SIMM per chunk with the Wiener-mask separation
    of each chunk, overlap-add of the chunk WAVs.  Every SIMM iteration,
    STFT / iSTFT, mask, the dictionary synthesis and the Viterbi recursion
    run on the GPU; chunk bookkeeping and WAV I/O are host-side, as in the
    reference.  tfrepresentation 'stft' or the CQT-type 'cqt' / 'minqt' /
    'mqt' (GPU CQT / MinQT transforms and their inverses; the source
    dictionary of a CQT-type transform transforms the complex KLGLOTT88
    comb on the GPU, dict_wf0_cqt); initHF00 'random' or 'nnls' (the per-frame
    NNLS of each chunk as one batched GPU solve, tools/nnls.py).

    Addition: with inputAudioFilename=None the state that
    writeSeparatedSignals / runViterbi read can be given directly
    (SIMMParams, stftParams, XR, XL, files, fs, scaleData, dataType,
    trackingParams, N)."""

    def __init__(self, inputAudioFilename=None, windowSize=0.0464, hopsize=None, NFT=None,
                 nbIter=10, numCompAccomp=40, minF0=39, maxF0=2000, stepNotes=16,
                 chirpPerF0=1, K_numFilters=4, P_numAtomFilters=30, imageCanvas=None,
                 wavCanvas=None, progressBar=None, verbose=True, outputDirSuffix='/',
                 minF0search=None, maxF0search=None, tfrepresentation='stft', cqtfmax=4000,
                 cqtfmin=50, cqtbins=48, cqtWinFunc=None, cqtAtomHopFactor=0.25,
                 initHF00='random', freeMemory=True, device=None, SIMMParams=None,
                 stftParams=None, XR=None, XL=None, files=None, fs=44100, scaleData=1.0,
                 dataType=np.int16, trackingParams=None, N=None):
        self.device = device
        self.verbose = verbose
        if inputAudioFilename is None:
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
            return
        import os
        from ..tools.utils import sqrt_blackmanharris
        self.files = {}
        self.SIMMParams = {}
        self.stftParams = {}
        tfrepresentation = tfrepresentation.lower()
        if tfrepresentation not in knownTransfos:
            raise AttributeError("The desired Time-Freq representation " + tfrepresentation +
                                 " is not a recognized one.\nPlease choose from " +
                                 str(knownTransfos))
        self.tfrepresentation = tfrepresentation
        self.stftParams['cqtfmin'] = cqtfmin
        self.stftParams['cqtfmax'] = cqtfmax
        self.stftParams['cqtbins'] = cqtbins
        self.stftParams['cqtWinFunc'] = cqtWinFunc if cqtWinFunc is not None else sqrt_blackmanharris
        self.stftParams['cqtAtomHopFactor'] = cqtAtomHopFactor
        self.files['inputAudioFilename'] = str(inputAudioFilename)
        self.imageCanvas = imageCanvas
        self.wavCanvas = wavCanvas
        self.displayEvolution = False
        if inputAudioFilename[-4:] != ".wav":
            raise ValueError("File not WAV file? Only WAV format support, for now...")
        # output files (:352-373)
        self._output_files(outputDirSuffix)
        # data scaling (:392-410)
        self.fs, data = wav.read(self.files['inputAudioFilename'])
        self.scaleData = 1.2 * np.abs(data).max()
        self.dataType = data.dtype
        data = np.double(data) / self.scaleData
        if data.shape[0] == data.size:
            data = np.vstack([data, data]).T
            self.numberChannels = 1
        if data.shape[1] != 2:
            data = data[:, 0:2]
            self.numberChannels = data.shape[1]
        # STFT parameters (:413-429)
        self.stftParams['windowSizeInSamples'] = slf.nextpow2(np.round(windowSize * self.fs))
        if hopsize is None:
            self.stftParams['hopsize'] = self.stftParams['windowSizeInSamples'] / 8.
        else:
            self.stftParams['hopsize'] = np.double(hopsize)
        if NFT is None:
            self.stftParams['NFT'] = self.stftParams['windowSizeInSamples']
        else:
            self.stftParams['NFT'] = NFT
        self.stftParams['offsets'] = {'stft': self.stftParams['windowSizeInSamples'] // 2,
                                      'minqt': 0, 'mqt': 0, 'hybridcqt': 0, 'cqt': 0}
        self.SIMMParams['niter'] = nbIter
        self.SIMMParams['R'] = numCompAccomp
        del data
        self.SIMMParams['minF0'] = minF0
        self.SIMMParams['maxF0'] = maxF0
        self.F = self.stftParams['NFT'] // 2 + 1
        self.SIMMParams['stepNotes'] = stepNotes
        self.SIMMParams['K'] = K_numFilters
        self.SIMMParams['P'] = P_numAtomFilters
        self.SIMMParams['chirpPerF0'] = chirpPerF0
        self.scopeAllowedHF0 = 4.0 / 1.0
        self.SIMMParams['initHF00'] = initHF00
        self.computeWF0()
        self.SIMMParams['WGAMMA'] = slf.generateHannBasis(
            numberFrequencyBins=self.F, sizeOfFourier=self.stftParams['NFT'], Fs=self.fs,
            frequencyScale='linear', numberOfBasis=self.SIMMParams['P'], overlap=.75)
        self.trackingParams = {'minF0search': self.SIMMParams['minF0'],
                               'maxF0search': self.SIMMParams['maxF0']}
        if minF0search is not None:
            self.trackingParams['minF0search'] = minF0search
        if maxF0search is not None:
            self.trackingParams['maxF0search'] = maxF0search
        self.freeMemory = freeMemory

    # ---------------------------------------------------------------- setup
    def _output_files(self, outputDirSuffix):
        """Output directory <input dir>/<suffix>/ and the lead / accompaniment
        / pitch file names (:352-373, :551-570)."""
        import os
        self.files['outputDirSuffix'] = outputDirSuffix
        self.files['outputDir'] = ('/'.join(self.files['inputAudioFilename'].split('/')[:-1]) +
                                   '/' + self.files['outputDirSuffix'] + '/')
        if not os.path.isdir(self.files['outputDir']):
            os.mkdir(self.files['outputDir'])
        self.files['pathBaseName'] = (self.files['outputDir'] +
                                      self.files['inputAudioFilename'].split('/')[-1][:-4])
        self.files['mus_output_file'] = str(self.files['pathBaseName'] + '_acc.wav')
        self.files['voc_output_file'] = str(self.files['pathBaseName'] + '_lead.wav')
        self.files['pitch_output_file'] = str(self.files['pathBaseName'] + '_pitches.txt')

    def setOutputFileNames(self, outputDirSuffix):
        """Redefine where the output files are written, e.g. between the first
        estimation and the re-estimation of the parameters (:540-585)."""
        if self.verbose:
            print("Redefining the Output Filenames !")
        self._output_files(outputDirSuffix)

    def computeWF0(self):
        """Source dictionary on the GPU and the transform object
        (SeparateLeadStereoTF.py:587-700, the transform-registry branch
        :656-700): the transform named by tfrepresentation ('stft', or the
        CQT-type 'cqt' / 'minqt' / 'mqt', tftransforms/tft.py:74-80) and
        generate_WF0_TR_chirped on it.  A CQT-type transform resets the
        frame geometry: hopsize = atomHOP, NFT = FFTLen, window =
        FFTLen * 2^(octaveNr - 1) (:689-700)."""
        from ..tftransforms import tft
        self.mqt = tft.tftransforms[self.tfrepresentation](
            fmin=self.stftParams['cqtfmin'], fmax=self.stftParams['cqtfmax'],
            bins=self.stftParams['cqtbins'], fs=self.fs, linFTLen=self.stftParams['NFT'],
            atomHopFactor=self.stftParams['cqtAtomHopFactor'],
            winFunc=self.stftParams['cqtWinFunc'], perfRast=1, verbose=0, device=self.device)
        self.SIMMParams['F0Table'], WF0, self.mqt = slf.generate_WF0_TR_chirped(
            transform=self.mqt, minF0=self.SIMMParams['minF0'], maxF0=self.SIMMParams['maxF0'],
            stepNotes=self.SIMMParams['stepNotes'], Ot=0.5,
            perF0=self.SIMMParams['chirpPerF0'], depthChirpInSemiTone=0.5, loadWF0=True,
            verbose=self.verbose, device=self.device)
        self.SIMMParams['WF0'] = WF0 / np.sum(WF0, axis=0)
        self.SIMMParams['NF0'] = self.SIMMParams['F0Table'].size
        self.F = WF0.shape[0]
        if hasattr(self.mqt, 'cqtkernel'):
            self.stftParams['hopsize'] = self.mqt.cqtkernel.atomHOP
            self.stftParams['NFT'] = self.mqt.cqtkernel.FFTLen
            self.stftParams['windowSizeInSamples'] = (self.mqt.cqtkernel.FFTLen *
                                                      (2 ** (self.mqt.octaveNr - 1)))

    def _read(self):
        _, data = wav.read(self.files['inputAudioFilename'])
        return np.double(data) / self.scaleData

    def _stft(self, x, start, stop):
        return slf.stft(x, fs=self.fs, hopsize=self.stftParams['hopsize'],
                        window=slf.sinebell(self.stftParams['windowSizeInSamples']),
                        nfft=self.stftParams['NFT'], start=start, stop=stop,
                        device=self.device)[0]

    def _cqt_span(self, data, start, stop):
        """Samples of frames start:stop for a CQT-type transform (:726-733):
        start * atomHOP to (stop - 1) * atomHOP + window (numpy < 1.12
        truncated the float bounds)."""
        start = start * self.mqt.cqtkernel.atomHOP
        if stop is not None:
            stop = (stop - 1) * self.mqt.cqtkernel.atomHOP
            stop += self.stftParams['windowSizeInSamples']
        else:
            stop = data.shape[0]
        return data[int(start):int(stop)]

    def _cqt(self, x):
        """The transform of x on the GPU (transfo), released afterwards."""
        self.mqt.computeTransform(data=x)
        X = np.copy(self.mqt.transfo)
        del self.mqt.transfo
        return X

    def computeMonoX(self, start=0, stop=None):
        """max(|X(mean of channels)|^2, 1e-8) for frames start:stop, X the
        STFT or the CQT-type transform (:702-739)."""
        data = self._read()
        if len(data.shape) > 1 and data.shape[1] > 1:
            data = data.mean(axis=1)
        if self.tfrepresentation == 'stft':
            X = self._stft(data, start, stop)
            self.F, _ = X.shape
            return np.maximum(np.abs(X) ** 2, 10 ** -8)
        return np.maximum(np.abs(self._cqt(self._cqt_span(data, start, stop))) ** 2, 10 ** -8)

    def computeStereoX(self, start=0, stop=None):
        """Complex transforms XR, XL for frames start:stop (:761-841)."""
        data = self._read()
        if self.tfrepresentation != 'stft':
            data = self._cqt_span(data, start, stop)
            self.XR = self._cqt(data[:, 0] if len(data.shape) > 1 else data)
            if len(data.shape) > 1 and data.shape[1] > 1:
                self.XL = self._cqt(data[:, 1])
            else:
                self.XL = self.XR
            self.F, _ = self.XR.shape
            return
        starttime = start * self.stftParams['hopsize']
        stoptime = stop * self.stftParams['hopsize'] if stop is not None else data.shape[0]
        self.originalDataLen = stoptime - starttime
        if len(data.shape) > 1:
            self.XR = self._stft(data[:, 0], start, stop)
        else:
            self.XR = self._stft(data, start, stop)
        if len(data.shape) > 1 and data.shape[1] > 1:
            self.XL = self._stft(data[:, 1], start, stop)
        else:
            self.XL = self.XR
        self.F, _ = self.XR.shape

    def computeStereoSX(self, start=0, stop=None):
        """max(|X|^2, 1e-8) of each channel, frames start:stop (:843-917)."""
        data = self._read()
        if self.tfrepresentation != 'stft':
            data = self._cqt_span(data, start, stop)
            SXR = np.maximum(np.abs(self._cqt(data[:, 0] if len(data.shape) > 1 else data)) ** 2,
                             10 ** -8)
            if len(data.shape) > 1 and data.shape[1] > 1:
                SXL = np.maximum(np.abs(self._cqt(data[:, 1])) ** 2, 10 ** -8)
            else:
                SXL = SXR
            self.F, _ = SXR.shape
            return SXR, SXL
        starttime = start * self.stftParams['hopsize']
        stoptime = stop * self.stftParams['hopsize'] if stop is not None else data.shape[0]
        self.originalDataLen = stoptime - starttime
        XR = self._stft(data[:, 0] if len(data.shape) > 1 else data, start, stop)
        SXR = np.maximum(np.abs(XR) ** 2, 1e-8)
        if len(data.shape) > 1 and data.shape[1] > 1:
            SXL = np.maximum(np.abs(self._stft(data[:, 1], start, stop)) ** 2, 1e-8)
        else:
            SXL = SXR
        self.F, _ = SXR.shape
        return SXR, SXL

    def checkChunkSize(self, maxFrames):
        """Chunking of the frames (:1880-1897), py2 integer divisions kept."""
        totFrames = np.int32(self.computeNFrames())
        nChunks = totFrames // maxFrames + 1
        if (totFrames - (nChunks - 1) * maxFrames <
                self.stftParams['windowSizeInSamples'] / self.stftParams['hopsize']):
            maxFrames = int(np.ceil(np.double(totFrames) / nChunks))
            nChunks = totFrames // maxFrames
        return totFrames, nChunks, maxFrames

    # ---------------------------------------------------------------- pipeline
    def autoMelSepAndWrite(self, maxFrames=1000):
        """Fully automated melody estimation and separation (:1142-1148)."""
        self.estimHF0(maxFrames=maxFrames)
        self.runViterbi()
        self.initiateHF0WithIndexBestPath()
        self.estimStereoSIMMParamsWriteSeps(maxFrames=maxFrames)

    def estimHF0(self, R=1, maxFrames=1000):
        """HF0 of the whole excerpt by mono SIMM on chunks (:959-1072)."""
        from .SIMM import SIMM
        totFrames, nChunks, maxFrames = self.checkChunkSize(maxFrames)
        P = self.SIMMParams
        P['HF0'] = np.zeros([P['NF0'] * P['chirpPerF0'], totFrames])
        for n in range(nChunks):
            start = n * maxFrames
            stop = np.minimum((n + 1) * maxFrames, totFrames)
            SX = self.computeMonoX(start=start, stop=stop)
            HF00 = None
            if P['initHF00'] == 'nnls':
                # per-frame NNLS of SX on the dictionary, + eps (:982-993), all
                # frames of the chunk at once on the GPU (tools/nnls.py); the
                # reference solves the first stop - start columns of SX
                HF00 = nnls_columns(P['WF0'], SX[:, :stop - start], add_eps=eps,
                                    device=self.device)
            HGAMMA, HPHI, HF0, HM, WM, recoError1 = SIMM.SIMM(
                SX, WF0=P['WF0'], WGAMMA=P['WGAMMA'], numberOfFilters=P['K'],
                numberOfAccompanimentSpectralShapes=R, HGAMMA0=None, HPHI0=None, HF00=HF00,
                WM0=None, HM0=None, numberOfIterations=P['niter'], updateRulePower=1.,
                stepNotes=P['stepNotes'], lambdaHF0=0.0 / (1.0 * SX.max()), alphaHF0=0.9,
                verbose=self.verbose, F0Table=P['F0Table'], chirpPerF0=P['chirpPerF0'],
                device=self.device)
            if self.tfrepresentation == 'stft':
                P['HF0'][:, start:stop] = np.copy(HF0)
            else:
                # the first frame of interest of the CQT-type raster (:1025-1032)
                startincqt = np.sort(np.where(self.mqt.time_stamps > 0)[0])[0]
                P['HF0'][:, start:stop] = np.copy(HF0[:, startincqt:startincqt + stop - start])
            del SX

    def estimSIMMParams(self, R=1):
        """Mono SIMM on the mean of the channels over the whole excerpt
        (:919-957); the parameters go to SIMMParams."""
        from .SIMM import SIMM
        P = self.SIMMParams
        SX = self.computeMonoX()
        HGAMMA, HPHI, HF0, HM, WM, recoError1 = SIMM.SIMM(
            SX, WF0=P['WF0'], WGAMMA=P['WGAMMA'], numberOfFilters=P['K'],
            numberOfAccompanimentSpectralShapes=R, HGAMMA0=None, HPHI0=None, HF00=None,
            WM0=None, HM0=None, numberOfIterations=P['niter'], updateRulePower=1.,
            stepNotes=P['stepNotes'], lambdaHF0=0.0 / (1.0 * SX.max()), alphaHF0=0.9,
            verbose=self.verbose, F0Table=P['F0Table'], chirpPerF0=P['chirpPerF0'],
            device=self.device)
        P['HGAMMA'], P['HPHI'], P['HF0'], P['HM'], P['WM'] = HGAMMA, HPHI, HF0, HM, WM
        del SX

    def _store_stereo(self, res, hf0_key='HF0'):
        """SIMMParams from a Stereo_SIMM result tuple (SIMM.py:943 order)."""
        P = self.SIMMParams
        (P['alphaR'], P['alphaL'], P['HGAMMA'], P['HPHI'], P[hf0_key], P['betaR'], P['betaL'],
         P['HM'], P['WM'], _) = res

    def estimStereoSIMMParams(self):
        """Stereo SIMM over the whole excerpt from HF00 (:1677-1713); note the
        power spectrograms here are |X|^2 without the 1e-8 floor of the
        chunked path, as in the reference."""
        from .SIMM import SIMM
        P = self.SIMMParams
        self.computeStereoX()
        SXR = np.abs(self.XR) ** 2
        SXL = np.abs(self.XL) ** 2
        self._store_stereo(SIMM.Stereo_SIMM(
            SXR, SXL, WF0=P['WF0'], WGAMMA=P['WGAMMA'], numberOfFilters=P['K'],
            numberOfAccompanimentSpectralShapes=P['R'], HGAMMA0=None, HPHI0=None,
            HF00=P['HF00'], WM0=None, HM0=None, numberOfIterations=P['niter'],
            updateRulePower=1.0, stepNotes=P['stepNotes'], lambdaHF0=0.0 / (1.0 * SXR.max()),
            alphaHF0=0.9, verbose=self.verbose, displayEvolution=False, device=self.device))
        del SXR, SXL

    @staticmethod
    def _unvoiced_basis(WF0):
        """WUF0: the source dictionary with a flat (all-ones) unvoiced atom
        appended (:1594-1596, :1720-1721)."""
        return np.hstack([WF0, np.ones([WF0.shape[0], 1])])

    def estimStereoSUIMMParams(self):
        """Stereo SIMM with the unvoiced atom (:1715-1760): WUF0 = [WF0 | 1],
        HUF0 = [HF0 ; 1], HGAMMA and HPHI from the voiced estimate, HGAMMA
        held fixed (updateHGAMMA=False).  Reads the XR / XL of the previous
        estimStereoSIMMParams, as the reference does."""
        from .SIMM import SIMM
        P = self.SIMMParams
        SXR = np.abs(self.XR) ** 2
        SXL = np.abs(self.XL) ** 2
        WUF0 = self._unvoiced_basis(P['WF0'])
        HUF0 = np.vstack([P['HF0'], np.ones([1, P['HF0'].shape[1]])])
        self._store_stereo(SIMM.Stereo_SIMM(
            SXR, SXL, WUF0, WGAMMA=P['WGAMMA'], numberOfFilters=P['K'],
            numberOfAccompanimentSpectralShapes=P['R'], HGAMMA0=P['HGAMMA'], HPHI0=P['HPHI'],
            HF00=HUF0, WM0=None, HM0=None, numberOfIterations=P['niter'], updateRulePower=1.0,
            stepNotes=P['stepNotes'], lambdaHF0=0.0 / (1.0 * SXR.max()), alphaHF0=0.9,
            verbose=self.verbose, displayEvolution=False, updateHGAMMA=False,
            device=self.device), hf0_key='HUF0')
        P['WUF0'] = WUF0

    def automaticMelodyAndSeparation(self):
        """(:1130-1140) The reference disables this un-chunked sequence: its
        `raise warnings.warn(...)` emits the warning and then raises (the
        warning call returns None), so nothing after it runs.  Kept with that
        behaviour; the steps (runViterbi, initiateHF0WithIndexBestPath,
        estimStereoSIMMParams, writeSeparatedSignals, estimStereoSUIMMParams,
        writeSeparatedSignalsWithUnvoice) are callable one by one."""
        import warnings
        warnings.warn("This function does not work well with framed estimation.")
        raise TypeError("exceptions must derive from BaseException")

    # the reference's scale patterns (:1105-1110) in the order its Python 2
    # dict iterates them (string hashes of CPython 2.7 without randomisation:
    # slots 0, 3, 5, 7 of the 8-slot table) -- the row order of
    # scoresPerTuning and the key determineTuning returns
    _tuningPatterns = (
        ('andalusPattern', (0, 1, 4, 5, 7, 8, 11)),
        ('minorHarmoPattern', (0, 2, 3, 5, 7, 8, 10)),
        ('minorMelodPattern', (0, 2, 3, 5, 7, 9, 11)),
        ('majorPattern', (0, 2, 4, 5, 7, 9, 11)),
    )

    def computeChroma(self, maxFrames=3000):
        """Chroma of the pipeline's HF0 (:1074-1094): bin n of the
        12·stepNotes-bin octave = mean over frames' HF0 rows n, n + 12·stepNotes,
        ..., then each frame normalised to sum 1.  Runs estimHF0 first when HF0
        is missing, as the reference does."""
        import warnings
        if not hasattr(self, 'SIMMParams'):
            raise AttributeError("The parameters for the SIMM are not well initialized")
        if 'HF0' not in self.SIMMParams:
            self.estimHF0(maxFrames=maxFrames)
        if not hasattr(self, 'N'):
            warnings.warn("Issues with the attributes, running again the estimation.")
            self.estimHF0(maxFrames=maxFrames)
        octave = 12 * self.SIMMParams['stepNotes']
        HF0 = np.asarray(self.SIMMParams['HF0'])
        chroma = np.zeros([octave, self.computeNFrames()])
        for n in range(octave):
            chroma[n] = HF0[n::octave].mean(axis=0)
        chroma /= chroma.sum(axis=0)
        self.chroma = chroma

    def determineTuning(self):
        """Key / tuning / scale by pattern scores on the summed chroma
        (:1096-1128): (scoresPerTuning [4, stepNotes·12], bestTuning, bestKey,
        pattern name), the indices by integer division as the reference's
        Python 2 code computes them."""
        if not hasattr(self, 'chroma'):
            self.computeChroma()
        summary = self.chroma.sum(axis=1)
        nbTunings = self.SIMMParams['stepNotes']
        nbKey = 12
        scores = np.zeros([len(self._tuningPatterns), nbTunings * nbKey])
        for ntun in range(nbTunings):
            for nk in range(nbKey):
                for npatt, (_, pattern) in enumerate(self._tuningPatterns):
                    idx = np.mod((np.array(pattern) + nk) * nbTunings + ntun, summary.size)
                    scores[npatt, ntun + nk * nbTunings] = summary[idx].sum()
        best = int(np.argmax(scores))
        bestPattern, rest = divmod(best, nbTunings * nbKey)
        bestKey, bestTuning = divmod(rest, nbTunings)
        return scores, bestTuning, bestKey, self._tuningPatterns[bestPattern][0]

    def initiateHF0WithIndexBestPath(self):
        """HF00: the melody's neighbourhood set to max HF0 (:1321-1368)."""
        NF0 = self.SIMMParams['NF0']
        chirpPerF0 = self.SIMMParams['chirpPerF0']
        stepNotes = self.SIMMParams['stepNotes']
        HF00 = np.zeros([NF0 * chirpPerF0, self.N])
        scope = self.scopeAllowedHF0
        width = int(chirpPerF0 * (2 * np.floor(stepNotes / scope) + 1))
        dim1index = np.array(np.maximum(np.minimum(
            np.outer(self.indexBestPath, np.ones(width)) +
            np.outer(np.ones(self.N), np.arange(-chirpPerF0 * np.floor(stepNotes / scope),
                                                chirpPerF0 * (np.floor(stepNotes / scope) + 1))),
            chirpPerF0 * NF0 - 1), 0), dtype=int)
        dim1index = dim1index[self.indexBestPath != 0, :]
        dim1index = dim1index.reshape(1, dim1index.size)
        dim2index = np.outer(np.arange(self.N), np.ones(width, dtype=int))
        dim2index = dim2index[self.indexBestPath != 0, :]
        dim2index = dim2index.reshape(1, dim2index.size)
        HF00[dim1index, dim2index] = self.SIMMParams['HF0'].max()
        HF00[:, self.indexBestPath == (NF0 - 1)] = 0.0
        HF00[:, self.indexBestPath == 0] = 0.0
        self.SIMMParams['HF00'] = HF00

    def estimStereoSIMMParamsWriteSeps(self, maxFrames=1000):
        """Stereo SIMM per chunk, writing each chunk's separation, then the
        overlap-add of the chunks (:1370-1467)."""
        from .SIMM import SIMM
        totFrames, nChunks, maxFrames = self.checkChunkSize(maxFrames)
        P = self.SIMMParams
        P['HGAMMA'] = None
        for n in range(nChunks):
            start = n * maxFrames
            stop = np.minimum((n + 1) * maxFrames, totFrames)
            SXR, SXL = self.computeStereoSX(start=start, stop=stop)
            HF00 = np.zeros([P['NF0'] * P['chirpPerF0'], SXR.shape[1]])
            if self.tfrepresentation == 'stft':
                startinHF00, stopinHF00 = 0, stop - start
            else:                                            # :1400-1402
                startinHF00 = np.sort(np.where(self.mqt.time_stamps > 0)[0])[0]
                stopinHF00 = startinHF00 + stop - start
            HF00[:, startinHF00:stopinHF00] = P['HF00'][:, start:stop]
            (alphaR, alphaL, HGAMMA, HPHI, HF0, betaR, betaL, HM, WM,
             recoError2) = SIMM.Stereo_SIMM(
                SXR, SXL, WF0=P['WF0'], WGAMMA=P['WGAMMA'], numberOfFilters=P['K'],
                numberOfAccompanimentSpectralShapes=P['R'], HGAMMA0=P['HGAMMA'], HPHI0=None,
                HF00=HF00, WM0=None, HM0=None, numberOfIterations=P['niter'],
                updateRulePower=1.0, stepNotes=P['stepNotes'],
                lambdaHF0=0.0 / (1.0 * SXR.max()), alphaHF0=0.9, verbose=self.verbose,
                displayEvolution=False, device=self.device)
            P['HGAMMA'], P['HPHI'], P['HF0'], P['HM'], P['WM'] = HGAMMA, HPHI, HF0, HM, WM
            P['alphaR'], P['alphaL'], P['betaR'], P['betaL'] = alphaR, alphaL, betaR, betaL
            P['HF00'][:, start:stop] = np.copy(HF0[:, startinHF00:stopinHF00])
            del SXR, SXL, HF00
            self.computeStereoX(start=start, stop=stop)
            self.writeSeparatedSignals(suffix='%05d.wav' % n)
            del self.XR, self.XL
            if self.freeMemory:
                for key in ('HM', 'HF0', 'HPHI', 'alphaR', 'alphaL', 'betaR', 'betaL'):
                    del P[key]
        self.overlapAddChunks(nChunks=nChunks, suffixIsSUIMM='.wav')

    def estimStereoSUIMMParamsWriteSeps(self, maxFrames=1000):
        """estimStereoSIMMParamsWriteSeps with the unvoiced atom (:1585-1675):
        per chunk, stereo SIMM on WUF0 = [WF0 | 1] from HUF0 = [HF00 chunk ;
        1] with the current HGAMMA held fixed, the chunk's '_VUIMM'
        separation, then the overlap-add into <lead|acc>_VUIMM.wav."""
        from .SIMM import SIMM
        totFrames, nChunks, maxFrames = self.checkChunkSize(maxFrames)
        P = self.SIMMParams
        WUF0 = self._unvoiced_basis(P['WF0'])
        P['WUF0'] = WUF0
        for n in range(nChunks):
            start = n * maxFrames
            stop = np.minimum((n + 1) * maxFrames, totFrames)
            SXR, SXL = self.computeStereoSX(start=start, stop=stop)
            HUF0 = np.zeros([P['NF0'] * P['chirpPerF0'] + 1, SXR.shape[1]])
            if self.tfrepresentation == 'stft':
                startinHF00, stopinHF00 = 0, stop - start
            else:                                            # :1610-1612
                startinHF00 = np.sort(np.where(self.mqt.time_stamps > 0)[0])[0]
                stopinHF00 = startinHF00 + stop - start
            HUF0[:-1, startinHF00:stopinHF00] = P['HF00'][:, start:stop]
            HUF0[-1] = 1
            self._store_stereo(SIMM.Stereo_SIMM(
                SXR, SXL, WUF0, WGAMMA=P['WGAMMA'], numberOfFilters=P['K'],
                numberOfAccompanimentSpectralShapes=P['R'], HGAMMA0=P['HGAMMA'], HPHI0=None,
                HF00=HUF0, WM0=None, HM0=None, numberOfIterations=P['niter'],
                updateRulePower=1.0, stepNotes=P['stepNotes'],
                lambdaHF0=0.0 / (1.0 * SXR.max()), alphaHF0=0.9, verbose=self.verbose,
                displayEvolution=False, updateHGAMMA=False, device=self.device),
                hf0_key='HUF0')
            del SXR, SXL, HUF0
            self.computeStereoX(start=start, stop=stop)
            self.writeSeparatedSignals(suffix='%05d_VUIMM.wav' % n)
            del self.XR, self.XL
            for key in ('HM', 'HUF0', 'HPHI', 'alphaR', 'alphaL', 'betaR', 'betaL'):
                del P[key]
        self.overlapAddChunks(nChunks=nChunks, suffixIsSUIMM='_VUIMM.wav')

    def overlapAddChunks(self, nChunks, suffixIsSUIMM='.wav'):
        """Concatenate the chunk WAVs with their overlaps (:1469-1583): for the
        STFT the overlap is rectangular (ones), for a CQT-type transform a
        squared sine bell over wlen - atomHOP samples; int16 arithmetic as
        the reference's."""
        import os
        wlen = self.stftParams['windowSizeInSamples']
        offsetTF = self.stftParams['offsets'][self.tfrepresentation]
        if self.tfrepresentation == 'stft':
            hopsize = self.stftParams['hopsize']
            overlapSamp = int(wlen - hopsize)
            overlapFunc = np.ones(overlapSamp)
        else:
            hopsize = self.mqt.cqtkernel.atomHOP
            overlapSamp = int(wlen - hopsize)
            overlapFunc = slf.sinebell(2 * overlapSamp)[overlapSamp:] ** 2
        nuDataLen = int(self.totFrames * hopsize + 2 * wlen)
        for key in ('voc_output_file', 'mus_output_file'):
            data = np.zeros([nuDataLen, 2], np.int16)
            cumulframe = 0
            for n in range(nChunks):
                fname = self.files[key][:-4] + '%05d%s' % (n, suffixIsSUIMM)
                _, datatmp = wav.read(fname)
                datatype = type(datatmp[0][0])
                if n == 0 and nChunks != 1:
                    datatmp[-overlapSamp:, 0] = datatype(datatmp[-overlapSamp:, 0] * overlapFunc)
                    datatmp[-overlapSamp:, 1] = datatype(datatmp[-overlapSamp:, 1] * overlapFunc)
                    lendatatmp = datatmp.shape[0] - offsetTF
                    data[:lendatatmp, :] = np.copy(datatmp[offsetTF:, :])
                    cumulframe = lendatatmp
                elif nChunks != 1:
                    if n != nChunks - 1:
                        datatmp[-overlapSamp:, 0] = datatype(datatmp[-overlapSamp:, 0] *
                                                             overlapFunc)
                        datatmp[-overlapSamp:, 1] = datatype(datatmp[-overlapSamp:, 1] *
                                                             overlapFunc)
                    datatmp[:overlapSamp, 0] = datatype(datatmp[:overlapSamp, 0] *
                                                        overlapFunc[::-1])
                    datatmp[:overlapSamp, 1] = datatype(datatmp[:overlapSamp, 1] *
                                                        overlapFunc[::-1])
                    start = int(cumulframe - wlen + hopsize)
                    lendatatmp = datatmp.shape[0]
                    stop = start + lendatatmp
                    data[start:stop, :] += datatmp
                    cumulframe = stop
                else:
                    lendatatmp = datatmp.shape[0] - offsetTF
                    data[:lendatatmp] = datatmp[offsetTF:, :]
                os.remove(fname)
            wav.write(self.files[key][:-4] + suffixIsSUIMM, self.fs, data[:self.lengthData, :])

    def computeNFrames(self):
        """Total number of frames (:741-759); in the state-injection mode the
        caller provides N (or HF0 defines it)."""
        if 'inputAudioFilename' in self.files:
            if not hasattr(self, 'totFrames'):
                _, data = wav.read(self.files['inputAudioFilename'])
                self.lengthData = data.shape[0]
                self.totFrames = np.int32(np.ceil((self.lengthData - 0) /
                                                  self.stftParams['hopsize'] + 1) + 1)
                self.N = self.totFrames
            return self.totFrames
        if not hasattr(self, 'N'):
            self.N = np.asarray(self.SIMMParams['HF0']).shape[1]
        return self.N

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
        """(vest [2][L], mest [2][L]) float waveforms before int conversion:
        the masked transforms inverted by the SIMM-pipeline istft, or by the
        CQT-type transform's invertTransform (:1795-1861)."""
        P = dict(self.SIMMParams)
        if 'VUIMM' in suffix:
            P['WF0'], P['HF0'] = P['WUF0'], P['HUF0']
        vR, vL, mR, mL = separate_lead_stfts(P, self.XR, self.XL, device=self.device)
        if self.tfrepresentation != 'stft':
            def inv(X):
                self.mqt.transfo = X
                y = self.mqt.invertTransform()
                del self.mqt.transfo
                return y
            return [inv(vR), inv(vL)], [inv(mR), inv(mL)]
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
