"""CPU restatement of the reference's Viterbi melody tracker.

TEST INFRASTRUCTURE ONLY (the checker, never the product): imported by
tests/ and bench legs; the product package `pyfasst_amd` never imports it.

Restates SeparateLeadStereo/tracking/_tracking.pyx:11-93 (the Cython tracker
the pipeline calls, SeparateLeadStereoTF.py:1220-1222) and, equivalently on
NaN-free input, tracking.py:87-151 (viterbiTrackingArray):

  cum[s, 0]  = logPrior[s] + logDensity[s, 0]
  cum[s, n]  = max_{s'} (cum[s', n-1] + logTrans[s', s]) + logDensity[s, n]
  ante[s, n] = the FIRST s' reaching that max (strict '>' scan from s' = 0,
               _tracking.pyx:70-82)
  path[N-1]  = argmax_s cum[s, N-1];  path[n] = ante[path[n+1], n+1]

Only the first `numberOfStates` rows / columns are used (the pipeline passes
numberOfStates = NF0 with logHF0 of NF0 + 1 rows, SeparateLeadStereoTF.py:
1220: the silence state is never tracked).  The Cython scan's NaN rule is
kept: a NaN candidate never wins a strict comparison, so a NaN at s' = 0
sticks (cum NaN, antecedent 0) and a NaN at s' > 0 is skipped.

Pinned against tests/golden/viterbi.npz, produced by the reference's own
tracking.py (tests/golden/make_golden.py, case 'viterbi').
"""
import numpy as np


def _first_max_scan(M):
    """Column-wise (over axis 0) strict-'>' scan from row 0: value, index."""
    best = M[0].copy()
    idx = np.zeros(M.shape[1], dtype=np.int64)
    for sp in range(1, M.shape[0]):
        better = M[sp] > best          # NaN compares False either way
        best[better] = M[sp][better]
        idx[better] = sp
    return best, idx


def viterbi_tracking(numberOfStates, numberOfFrames, logDensity, logPriorDensities,
                     logTransitionMatrix):
    """_tracking.viterbiTracking (Cython signature)."""
    S, N = int(numberOfStates), int(numberOfFrames)
    logD = np.asarray(logDensity, dtype=np.float64)[:S, :N]
    logT = np.asarray(logTransitionMatrix, dtype=np.float64)[:S, :S]
    prior = np.asarray(logPriorDensities, dtype=np.float64)[:S]
    cum = np.zeros([S, N])
    ante = np.zeros([S, N], dtype=np.int64)
    ante[:, 0] = -1
    cum[:, 0] = prior + logD[:, 0]
    for n in range(1, N):
        best, idx = _first_max_scan(cum[:, n - 1][:, None] + logT)
        cum[:, n] = best + logD[:, n]
        ante[:, n] = idx
    path = np.zeros([N], dtype=np.int64)
    path[N - 1] = np.argmax(cum[:, N - 1])
    for n in range(N - 2, -1, -1):
        path[n] = ante[path[n + 1], n + 1]
    return path


def viterbi_tracking_array(logDensity, logPriorDensities, logTransitionMatrix):
    """tracking.viterbiTrackingArray (all rows of logDensity are states)."""
    S, N = np.asarray(logDensity).shape
    return viterbi_tracking(S, N, logDensity, logPriorDensities, logTransitionMatrix)


def melody_transitions(NF0, stepNotes, scale=1.0):
    """The log transition matrix and log priors runViterbi builds
    (SeparateLeadStereoTF.py:1183-1208): a Toeplitz note-distance decay with
    a silence state, row-normalised."""
    transitions = np.exp(-np.floor(np.arange(0, NF0) / stepNotes) * scale)
    cutoffnote = 2 * 5 * stepNotes
    cutoffnote = np.minimum(NF0, cutoffnote)
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
    return np.log(T), np.log(prior)


def melody_log_density(HF0):
    """logHF0 of runViterbi (SeparateLeadStereoTF.py:1210-1216), all rows."""
    NF0, N = HF0.shape
    logHF0 = np.zeros([NF0 + 1, N])
    normHF0 = np.amax(HF0, axis=0)
    with np.errstate(divide='ignore'):
        logHF0[0:NF0, :] = np.log(HF0)
    logHF0[0:NF0, normHF0 == 0] = np.amin(logHF0[logHF0 > -np.inf])
    logHF0[NF0, :] = np.maximum(np.amin(logHF0[logHF0 > -np.inf]), -100)
    return logHF0
