"""CPU restatement of the SIMM source/filter multiplicative updates.

TEST INFRASTRUCTURE ONLY (same rules as oracle/fasst_ref.py): imported by
tests/ and bench only, never by the product package.

Follows SeparateLeadStereo/SIMM/SIMM.py of the reference:
  simm()        -> SIMM        (SIMM.py:46-395), mono
  stereo_simm() -> Stereo_SIMM (SIMM.py:397-943)
Random initialisation draws from the global np.random stream in the
reference's order (HGAMMA, HPHI, HF0, HM, WM [, betaR]).  Display options are
not restated.  Stereo computeError fills recoError[0] and, per iteration, the
slots after the HF0 and HPHI updates; the reference advances its error
counter 6 (+1 with updateHGAMMA) times per iteration (SIMM.py:683-941).
"""
import numpy as np

EPS = 10 ** (-20)   # SIMM.py:150, :506


def _init(shape, given, rng):
    if given is not None and np.array(given).shape == shape:
        return np.array(given, copy=True, order='C', dtype=float)
    return np.abs(rng.randn(*shape))


def _init_params(F, N, NF0, P, K, R, HGAMMA0, HPHI0, HF00, WM0, HM0, rng):
    HGAMMA = _init((P, K), HGAMMA0, rng)
    HPHI = _init((K, N), HPHI0, rng)
    HF0 = _init((NF0, N), HF00, rng)
    HM = _init((R, N), HM0, rng)
    WM = _init((F, R), WM0, rng)
    return HGAMMA, HPHI, HF0, HM, WM


def is_distortion(X, Y):
    """ISDistortion (SIMM.py:34-44)."""
    ratio = (X / Y)
    return np.sum((-np.log(ratio) + ratio - 1))


def simm(SX, WF0, WGAMMA, numberOfFilters=4, numberOfAccompanimentSpectralShapes=10,
         HGAMMA0=None, HPHI0=None, HF00=None, WM0=None, HM0=None, numberOfIterations=1000,
         updateRulePower=1.0, rng=np.random):
    """SIMM.py:46-395 (mono)."""
    K, R, omega = numberOfFilters, numberOfAccompanimentSpectralShapes, updateRulePower
    F, N = SX.shape
    NF0 = WF0.shape[1]
    P = WGAMMA.shape[1]
    HGAMMA, HPHI, HF0, HM, WM = _init_params(F, N, NF0, P, K, R, HGAMMA0, HPHI0, HF00,
                                             WM0, HM0, rng)
    WPHI = np.dot(WGAMMA, HGAMMA)
    SF0 = np.dot(WF0, HF0)
    SPHI = np.dot(WPHI, HPHI)
    SM = np.dot(WM, HM)
    hat = SF0 * SPHI + SM
    recoError = np.zeros([numberOfIterations * 5 * 2 + NF0 * 2 + 1])
    WF0T = np.ascontiguousarray(WF0.T)
    for _ in range(numberOfIterations):
        den = SPHI / np.maximum(hat, EPS)
        num = (den * SX) / np.maximum(hat, EPS)
        HF0 *= (np.dot(WF0T, num) / np.maximum(np.dot(WF0T, den), EPS)) ** omega
        SF0 = np.dot(WF0, HF0)
        hat = np.maximum(SF0 * SPHI + SM, EPS)
        # HPHI
        den = SF0 / np.maximum(hat, EPS)
        num = (den * SX) / np.maximum(hat, EPS)
        HPHI *= (np.dot(WPHI.T, num) / np.maximum(np.dot(WPHI.T, den), EPS)) ** omega
        s = np.sum(HPHI, axis=0)
        HPHI[:, s > 0] /= s[s > 0]
        HF0 *= s
        SF0 = np.dot(WF0, HF0)
        SPHI = np.dot(WPHI, HPHI)
        hat = np.maximum(SF0 * SPHI + SM, EPS)
        # HM
        den = 1 / np.maximum(hat, EPS)
        num = den * SX
        num /= np.maximum(hat, EPS)
        HM *= (np.dot(WM.T, num) / np.maximum(np.dot(WM.T, den), EPS)) ** omega
        HM = np.maximum(HM, EPS)
        SM = np.dot(WM, HM)
        hat = np.maximum(SF0 * SPHI + SM, EPS)
        # HGAMMA
        den = SF0 / np.maximum(hat, EPS)
        num = (den * SX) / np.maximum(hat, EPS)
        HGAMMA *= (np.dot(WGAMMA.T, np.dot(num, HPHI.T)) /
                   np.maximum(np.dot(WGAMMA.T, np.dot(den, HPHI.T)), EPS)) ** omega
        sg = np.sum(HGAMMA, axis=0)
        HGAMMA[:, sg > 0] /= sg[sg > 0]
        HPHI *= np.outer(sg, np.ones(N))
        s = np.sum(HPHI, axis=0)
        HPHI[:, s > 0] /= s[s > 0]
        HF0 *= s
        WPHI = np.dot(WGAMMA, HGAMMA)
        SF0 = np.dot(WF0, HF0)
        SPHI = np.dot(WPHI, HPHI)
        hat = np.maximum(SF0 * SPHI + SM, EPS)
        # WM
        den = 1 / np.maximum(hat, EPS)
        num = den * SX
        num /= np.maximum(hat, EPS)
        WM *= (np.dot(num, HM.T) / np.maximum(np.dot(den, HM.T), EPS)) ** omega
        sw = np.sum(WM, axis=0)
        WM[:, sw > 0] /= sw[sw > 0]
        HM *= sw          # N7: broadcasts over the frame axis (R == 1 or R == N only)
        SM = np.dot(WM, HM)
        hat = np.maximum(SF0 * SPHI + SM, EPS)
    return HGAMMA, HPHI, HF0, HM, WM, recoError


def _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL):
    L = SF0 * SPHI
    Rr = np.dot(WM * (bR ** 2), HM)
    Rr += (aR ** 2) * L
    L *= (aL ** 2)
    L += np.dot(WM * (bL ** 2), HM)
    return np.maximum(Rr, EPS), np.maximum(L, EPS)


def stereo_simm(SXR, SXL, WF0, WGAMMA, numberOfFilters=4, numberOfAccompanimentSpectralShapes=10,
                HGAMMA0=None, HPHI0=None, HF00=None, WM0=None, HM0=None,
                numberOfIterations=1000, updateRulePower=1.0, updateHGAMMA=True,
                computeError=False, rng=np.random):
    """SIMM.py:397-943 (stereo)."""
    K, R, omega = numberOfFilters, numberOfAccompanimentSpectralShapes, updateRulePower
    F, N = SXR.shape
    if (F, N) != SXL.shape:
        raise ValueError("Dimension of STFT matrices must be the same.")
    NF0 = WF0.shape[1]
    P = WGAMMA.shape[1]
    HGAMMA, HPHI, HF0, HM, WM = _init_params(F, N, NF0, P, K, R, HGAMMA0, HPHI0, HF00,
                                             WM0, HM0, rng)
    aR = 0.5
    aL = 0.5
    bR = rng.rand(R)
    bL = 1 - bR
    WPHI = np.dot(WGAMMA, HGAMMA)
    SF0 = np.dot(WF0, HF0)
    SPHI = np.dot(WPHI, HPHI)
    hL = SF0 * SPHI
    hR = (aR ** 2) * hL
    hR += np.dot(WM * (bR ** 2), HM)
    hL *= (aL ** 2)
    hL += np.dot(WM * (bL ** 2), HM)
    recoError = np.zeros([numberOfIterations * 5 * 2 + NF0 * 2 + 1])
    if computeError:
        recoError[0] = is_distortion(SXR, hR) + is_distortion(SXL, hL)
    stride = 7 if updateHGAMMA else 6
    WF0T = np.ascontiguousarray(WF0.T)
    mx = np.maximum
    for it in range(numberOfIterations):
        # HF0 (:623-674)
        com = (aR ** 2) * SPHI / mx(hR, EPS)
        den = (aL ** 2) * SPHI / mx(hL, EPS)
        num = com * SXR / mx(hR, EPS) + den * SXL / mx(hL, EPS)
        den += com
        HF0 *= (np.dot(WF0T, num) / mx(np.dot(WF0T, den), EPS)) ** omega
        SF0 = np.dot(WF0, HF0)
        hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
        if computeError:
            recoError[1 + stride * it] = is_distortion(SXR, hR) + is_distortion(SXL, hL)
        # HPHI (:686-729)
        com = (aR ** 2) * SF0 / mx(hR, EPS)
        den = (aL ** 2) * SF0 / mx(hL, EPS)
        num = com * SXR
        num /= mx(hR, EPS)
        num += den * SXL / mx(hL, EPS)
        den += com
        HPHI *= (np.dot(WPHI.T, num) / mx(np.dot(WPHI.T, den), EPS)) ** omega
        s = np.sum(HPHI, axis=0)
        HPHI[:, s > 0] = HPHI[:, s > 0] / np.outer(np.ones(K), s[s > 0])
        HF0 *= np.outer(np.ones(NF0), s)
        SF0 = np.dot(WF0, HF0)
        SPHI = np.dot(WPHI, HPHI)
        hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
        if computeError:
            recoError[2 + stride * it] = is_distortion(SXR, hR) + is_distortion(SXL, hL)
        # HM (:740-773)
        HM *= ((np.dot((WM * (bR ** 2)).T, SXR / mx(hR ** 2, EPS)) +
                np.dot((WM * (bL ** 2)).T, SXL / mx(hL ** 2, EPS))) /
               mx(np.dot((WM * (bR ** 2)).T, 1 / mx(hR, EPS)) +
                  np.dot((WM * (bL ** 2)).T, 1 / mx(hL, EPS)), EPS)) ** omega
        hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
        # HGAMMA (:776-823)
        if updateHGAMMA:
            com = (aR ** 2) * SF0 / mx(hR, EPS)
            den = (aL ** 2) * SF0 / mx(hL, EPS)
            num = com * SXR
            num /= mx(hR, EPS)
            num += den * SXL / mx(hL, EPS)
            den += com
            HGAMMA *= (np.dot(WGAMMA.T, np.dot(num, HPHI.T)) /
                       mx(np.dot(WGAMMA.T, np.dot(den, HPHI.T)), EPS)) ** omega
            sg = np.sum(HGAMMA, axis=0)
            HGAMMA[:, sg > 0] /= sg[sg > 0]
            HPHI *= np.outer(sg, np.ones(N))
            s = np.sum(HPHI, axis=0)
            HPHI[:, s > 0] /= s[s > 0]
            HF0 *= s
            WPHI = np.dot(WGAMMA, HGAMMA)
            SF0 = np.dot(WF0, HF0)
            SPHI = np.dot(WPHI, HPHI)
            hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
        # WM (:826-869)
        WM = WM * ((np.dot(SXR / mx(hR ** 2, EPS), HM.T * (bR ** 2)) +
                    np.dot(SXL / mx(hL ** 2, EPS), HM.T * (bL ** 2))) /
                   (np.dot(1 / mx(hR, EPS), HM.T * (bR ** 2)) +
                    np.dot(1 / mx(hL, EPS), HM.T * (bL ** 2)))) ** omega
        sw = np.sum(WM, axis=0)
        WM[:, sw > 0] /= sw[sw > 0]
        HM *= np.vstack(sw)
        hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
        # alphaR, alphaL (:872-906)
        den = SF0 * SPHI / mx(hR, EPS)
        num = den * SXR / mx(hR, EPS)
        aR = mx(aR * (np.sum(num) / np.sum(den)) ** (omega * .1), EPS)
        den = SF0 * SPHI / mx(hL, EPS)
        num = den * SXL / mx(hL, EPS)
        aL = mx(aL * (np.sum(num) / np.sum(den)) ** (omega * .1), EPS)
        aR = aR / mx(aR + aL, .001)
        aL = np.copy(1 - aR)
        hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
        # betaR, betaL (:909-941)
        bR *= np.diag((np.dot(np.dot(WM.T, SXR / mx(hR ** 2, EPS)), HM.T)) /
                      (np.dot(np.dot(WM.T, 1 / mx(hR, EPS)), HM.T))) ** (omega * .1)
        bL *= np.diag((np.dot(np.dot(WM.T, SXL / mx(hL ** 2, EPS)), HM.T)) /
                      (np.dot(np.dot(WM.T, 1 / mx(hL, EPS)), HM.T))) ** (omega * .1)
        bR = bR / mx(bR + bL, EPS)
        bL = 1 - bR
        hR, hL = _hat(SF0, SPHI, WM, HM, aR, aL, bR, bL)
    return aR, aL, HGAMMA, HPHI, HF0, np.diag(bR), np.diag(bL), HM, WM, recoError


# ---------------------------------------------------------------- lead / accompaniment
SEP_EPS = 10 ** -9   # SeparateLeadStereoTF.py:31


def sinebell(L):
    """tools/utils.py:43-57"""
    return np.sin((np.pi * (np.arange(L))) / (1.0 * L))


def slf_stft(data, window, hopsize, nfft, fs=44100.0, start=0, stop=None):
    """SIMM-pipeline stft (separateLeadFunctions.py:90-161)."""
    L = window.size
    data = np.concatenate((np.zeros(int(L / 2.0)), data, np.zeros(int(L / 2.0))))
    n_data = data.size
    n_frames = np.ceil((n_data - L) / hopsize + 1) + 1
    new_len = (n_frames - 1) * hopsize + L
    data = np.concatenate((data, np.zeros([int(new_len - n_data)])))
    n_freqs = int(nfft / 2.0 + 1)
    if stop is None:
        stop = int(n_frames)
    X = np.zeros([n_freqs, stop - start], dtype=complex)
    for n in np.arange(start, stop):
        b = int(n * hopsize)
        X[:, n - start] = np.fft.rfft(window * data[b:b + L], int(nfft))
    return X, np.arange(n_freqs) / nfft * fs, np.arange(n_frames) * hopsize / fs


def slf_istft(X, analysisWindow=None, window=None, hopsize=256.0, nfft=2048.0,
              originalDataLen=None):
    """SIMM-pipeline istft (separateLeadFunctions.py:163-233)."""
    if analysisWindow is None:
        analysisWindow = window
    L = window.size
    n_freqs, n_frames = X.shape
    n_data = int(hopsize * (n_frames - 1) + L)
    norm = np.zeros(n_data)
    data = np.zeros(n_data)
    for n in np.arange(n_frames):
        b = int(n * hopsize)
        frame = np.fft.irfft(X[:, n], int(nfft))[:L]
        norm[b:b + L] = norm[b:b + L] + window * analysisWindow
        data[b:b + L] = data[b:b + L] + window * frame
    norm[:L] = norm[L:2 * L]
    norm[-L:] = norm[(-2 * L):(-L)]
    norm[norm == 0] = 1.
    data /= norm
    if originalDataLen is not None:
        data = data[:originalDataLen]
    return data


def lead_masks(P, XR, XL):
    """The four masked STFTs of writeSeparatedSignals
    (SeparateLeadStereoTF.py:1785-1846): lead R/L, accompaniment R/L."""
    SPHI = np.dot(np.dot(P['WGAMMA'], P['HGAMMA']), P['HPHI'])
    SF0 = np.dot(P['WF0'], P['HF0'])
    aR, aL, bR, bL, WM, HM = (P['alphaR'], P['alphaL'], P['betaR'], P['betaL'], P['WM'],
                              P['HM'])
    hR = np.maximum((aR ** 2) * SF0 * SPHI + np.dot(np.dot(WM, bR ** 2), HM), SEP_EPS)
    hL = np.maximum((aL ** 2) * SF0 * SPHI + np.dot(np.dot(WM, bL ** 2), HM), SEP_EPS)
    vR = (aR ** 2) * SPHI * SF0 / hR * XR
    vL = (aL ** 2) * SPHI * SF0 / hL * XL
    mR = (np.dot(np.dot(WM, bR ** 2), HM)) / hR * XR
    mL = (np.dot(np.dot(WM, bL ** 2), HM)) / hL * XL
    return vR, vL, mR, mL
