"""The reference's pure-Python tracker module (SeparateLeadStereo/tracking/
tracking.py): `viterbiTracking` (:5-85) and `viterbiTrackingArray`
(:87-151) compute the same path as the Cython tracker over all rows of
logDensity; here both run on the GPU.  (The reference returns float paths
from these two; the indices are returned as int64 here.)"""
import numpy as np

from ._tracking import viterbiTracking as _gpu_tracking


def viterbiTrackingArray(logDensity, logPriorDensities, logTransitionMatrix, verbose=False,
                         device=None):
    S, N = np.asarray(logDensity).shape
    return _gpu_tracking(S, N, logDensity, logPriorDensities, logTransitionMatrix,
                         device=device)


def viterbiTracking(logDensity, logPriorDensities, logTransitionMatrix, verbose=False,
                    device=None):
    return viterbiTrackingArray(logDensity, logPriorDensities, logTransitionMatrix,
                                device=device)
