"""SIMM multiplicative updates on the MI355X (drop-in for SIMM/SIMM.py).

`Stereo_SIMM` (reference SIMM.py:397-943) and `SIMM` (SIMM.py:46-395) keep
the reference's signatures and return tuples.  The random initialisation
stays on the host and draws from NumPy's global stream in the reference's
order (HGAMMA, HPHI, HF0, HM, WM, then betaR for stereo; SIMM.py:525-576), so
a seeded reference run and a seeded run here start from the same point; the
update loop runs in libfasst_hip.so (include/fasst_simm.h).  There is no CPU
fallback: without the HIP library the import fails.

Display options (displayEvolution, makeMovie, imageCanvas, progressBar) are
accepted and ignored: they only draw figures in the reference.
"""
import ctypes

import numpy as np
from numpy.random import randn

from ... import _lib

__all__ = ["db", "ISDistortion", "SIMM", "Stereo_SIMM"]


def db(positiveValue):
    """SIMM.py:27-33"""
    return 10 * np.log10(np.abs(positiveValue))


def ISDistortion(X, Y):
    """Itakura-Saito divergence (SIMM.py:34-44)."""
    ratio = (X / Y)
    return np.sum((-np.log(ratio) + ratio - 1))


def _given_or_random(given, shape, name, verbose):
    # SIMM.py:525-573: a given initial matrix of the wrong shape is replaced
    # by a random one (with a message), exactly as in the reference
    if given is not None:
        arr = np.array(given, copy=True, order='C', dtype=float)
        if arr.shape == shape:
            return arr
        print("Wrong dimensions for given %s, \nrandom initialization used instead" % name)
    return np.abs(randn(*shape))


class _SimmContext(object):
    def __init__(self, F, N, NF0, P, K, R, stereo, device):
        self.ptr = ctypes.c_void_p()
        _lib.check(_lib.lib.simm_create(device, F, N, NF0, P, K, R, int(stereo),
                                        ctypes.byref(self.ptr)), "simm_create")
        self.shape = (F, N, NF0, P, K, R)

    def __del__(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            _lib.lib.simm_destroy(self.ptr)
            self.ptr = None


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _run(SXs, WF0, WGAMMA, K, R, params, alpha, betaR, n_iter, omega, update_hgamma,
         compute_error, device):
    F, N = SXs[0].shape
    NF0 = WF0.shape[1]
    P = WGAMMA.shape[1]
    stereo = len(SXs) == 2
    HGAMMA, HPHI, HF0, HM, WM = [_c(p) for p in params]
    ctx = _SimmContext(F, N, NF0, P, K, R, stereo, device)
    SXR = _c(SXs[0])
    SXL = _c(SXs[1]) if stereo else None
    WF0c, WGc = _c(WF0), _c(WGAMMA)
    _lib.check(_lib.lib.simm_set_data(ctx.ptr, _lib.dptr(SXR),
                                      _lib.dptr(SXL) if stereo else None,
                                      _lib.dptr(WF0c), _lib.dptr(WGc)), "simm_set_data")
    a = np.array(alpha if stereo else (0.5, 0.5), dtype=np.float64)
    bR = _c(betaR if stereo else np.zeros(R))
    _lib.check(_lib.lib.simm_set_params(ctx.ptr, _lib.dptr(HGAMMA), _lib.dptr(HPHI),
                                        _lib.dptr(HF0), _lib.dptr(HM), _lib.dptr(WM),
                                        _lib.dptr(a), _lib.dptr(bR), None), "simm_set_params")
    recoError = np.zeros([n_iter * 5 * 2 + NF0 * 2 + 1])
    if compute_error:
        out = np.zeros(1)
        _lib.check(_lib.lib.simm_reco_error(ctx.ptr, _lib.dptr(out)), "simm_reco_error")
        recoError[0] = out[0]
        errs = np.zeros(max(2 * n_iter, 1))
        _lib.check(_lib.lib.simm_run(ctx.ptr, int(n_iter), float(omega), int(bool(update_hgamma)),
                                     _lib.dptr(errs)), "simm_run")
        # the reference advances its error counter once per update (6, or 7
        # with updateHGAMMA, per iteration) and fills only the slots after
        # HF0 and HPHI (SIMM.py:676-729)
        stride = 7 if update_hgamma else 6
        for it in range(n_iter):
            recoError[1 + stride * it] = errs[2 * it]
            recoError[2 + stride * it] = errs[2 * it + 1]
    else:
        _lib.check(_lib.lib.simm_run(ctx.ptr, int(n_iter), float(omega),
                                     int(bool(update_hgamma)), None), "simm_run")
    bL = np.zeros(R)
    _lib.check(_lib.lib.simm_get_params(ctx.ptr, _lib.dptr(HGAMMA), _lib.dptr(HPHI),
                                        _lib.dptr(HF0), _lib.dptr(HM), _lib.dptr(WM),
                                        _lib.dptr(a), _lib.dptr(bR), _lib.dptr(bL)),
               "simm_get_params")
    return HGAMMA, HPHI, HF0, HM, WM, a, bR, bL, recoError


def SIMM(SX, WF0, WGAMMA, numberOfFilters=4, numberOfAccompanimentSpectralShapes=10,
         HGAMMA0=None, HPHI0=None, HF00=None, WM0=None, HM0=None,
         numberOfIterations=1000, updateRulePower=1.0, stepNotes=4,
         lambdaHF0=0.00, alphaHF0=0.99, displayEvolution=False, verbose=True,
         makeMovie=False, imageCanvas=None, progressBar=None, F0Table=None, chirpPerF0=1,
         device=None):
    """Mono SIMM (reference SIMM.py:46-395).

    Returns (HGAMMA, HPHI, HF0, HM, WM, recoError).  As in the reference the
    accompaniment renormalisation `HM *= sumWM` (SIMM.py:388) broadcasts over
    the frame axis, so R must be 1 or N (ValueError otherwise, like NumPy's
    broadcast error).  recoError is all zeros (the mono reference never
    fills it).
    """
    K = numberOfFilters
    R = numberOfAccompanimentSpectralShapes
    F, N = np.shape(SX)
    Fwf0, NF0 = WF0.shape
    Fwgamma, P = WGAMMA.shape
    if Fwf0 != F:
        return False    # SIMM.py:194-195
    if R != 1 and R != N:
        raise ValueError("operands could not be broadcast together: SIMM.py:388 "
                         "needs R == 1 or R == N (R=%d, N=%d)" % (R, N))
    HGAMMA = _given_or_random(HGAMMA0, (P, K), "HGAMMA0", verbose)
    HPHI = _given_or_random(HPHI0, (K, N), "HPHI0", verbose)
    HF0 = _given_or_random(HF00, (NF0, N), "HF00", verbose)
    HM = _given_or_random(HM0, (R, N), "HM0", verbose)
    WM = _given_or_random(WM0, (F, R), "WM0", verbose)
    dev = _lib.default_device() if device is None else device
    HGAMMA, HPHI, HF0, HM, WM, _, _, _, recoError = _run(
        [SX], WF0, WGAMMA, K, R, (HGAMMA, HPHI, HF0, HM, WM), None, None,
        numberOfIterations, updateRulePower, True, False, dev)
    return HGAMMA, HPHI, HF0, HM, WM, recoError


def Stereo_SIMM(SXR, SXL, WF0, WGAMMA, numberOfFilters=4,
                numberOfAccompanimentSpectralShapes=10, HGAMMA0=None, HPHI0=None,
                HF00=None, WM0=None, HM0=None, numberOfIterations=1000,
                updateRulePower=1.0, stepNotes=4, lambdaHF0=0.00, alphaHF0=0.99,
                displayEvolution=False, verbose=True, updateHGAMMA=True,
                computeError=False, device=None):
    """Stereo SIMM (reference SIMM.py:397-943).

    Returns (alphaR, alphaL, HGAMMA, HPHI, HF0, betaR, betaL, HM, WM,
    recoError) with betaR/betaL as diagonal matrices (SIMM.py:943).
    """
    K = numberOfFilters
    R = numberOfAccompanimentSpectralShapes
    F, N = SXR.shape
    if (F, N) != SXL.shape:
        print("The input STFT matrices do not have the same dimension.\n")
        print("Please check what happened...")
        raise ValueError("Dimension of STFT matrices must be the same.")
    Fwf0, NF0 = WF0.shape
    Fwgamma, P = WGAMMA.shape
    if Fwf0 != F:
        return False    # SIMM.py:520-521
    HGAMMA = _given_or_random(HGAMMA0, (P, K), "HGAMMA0", verbose)
    HPHI = _given_or_random(HPHI0, (K, N), "HPHI0", verbose)
    HF0 = _given_or_random(HF00, (NF0, N), "HF00", verbose)
    HM = _given_or_random(HM0, (R, N), "HM0", verbose)
    WM = _given_or_random(WM0, (F, R), "WM0", verbose)
    alpha = (0.5, 0.5)                  # SIMM.py:573-574
    betaR = np.random.rand(R)           # SIMM.py:575
    dev = _lib.default_device() if device is None else device
    HGAMMA, HPHI, HF0, HM, WM, a, bR, bL, recoError = _run(
        [SXR, SXL], WF0, WGAMMA, K, R, (HGAMMA, HPHI, HF0, HM, WM), alpha, betaR,
        numberOfIterations, updateRulePower, updateHGAMMA, computeError, dev)
    return (a[0], a[1], HGAMMA, HPHI, HF0, np.diag(bR), np.diag(bL), HM, WM, recoError)
