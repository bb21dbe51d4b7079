"""Drop-in for the reference's Cython tracker
(SeparateLeadStereo/tracking/_tracking.pyx:11-93), on the GPU through the C
ABI viterbi_tracking (include/fasst_viterbi.h, pyfasst_amd/csrc/
fasst_viterbi.hip).  Same signature and semantics: only the first
numberOfStates rows / columns are used; ties go to the first state; the path
is an int64 array, bit-identical to the reference's.
"""
import numpy as np

from ... import _lib
from ..._lib import check, dptr, lib


def viterbiTracking(numberOfStates, numberOfFrames, logDensity, logPriorDensities,
                    logTransitionMatrix, verbose=False, device=None):
    """bestStatePath = viterbiTracking(S, N, logDensity, logPriorDensities,
    logTransitionMatrix)   (_tracking.pyx:11-93)"""
    S, N = int(numberOfStates), int(numberOfFrames)
    logD = np.asarray(logDensity, dtype=np.float64)
    logT = np.asarray(logTransitionMatrix, dtype=np.float64)
    prior = np.ascontiguousarray(np.asarray(logPriorDensities, dtype=np.float64)[:S])
    if (logD.ndim != 2 or logD.shape[0] < S or logD.shape[1] < N or logT.ndim != 2 or
            logT.shape[0] < S or logT.shape[1] < S or prior.size < S):
        raise ValueError("viterbiTracking: inputs smaller than %d states x %d frames" % (S, N))
    # row-major with contiguous rows (the C ABI takes a row pitch)
    if logD.strides[1] != 8 or logD.strides[0] % 8:
        logD = np.ascontiguousarray(logD)
    if logT.strides[1] != 8 or logT.strides[0] % 8:
        logT = np.ascontiguousarray(logT)
    path = np.empty(N, dtype=np.int64)
    dev = _lib.default_device() if device is None else device
    check(lib.viterbi_tracking(dev, S, N, logD.ctypes.data_as(_lib._dp), logD.strides[0] // 8,
                               dptr(prior), logT.ctypes.data_as(_lib._dp), logT.strides[0] // 8,
                               path.ctypes.data_as(_lib._llp)), "viterbi_tracking")
    return path
