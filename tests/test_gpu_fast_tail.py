"""The fused renormalisation tail (fasst_em.hip: k_fb_update statistics,
k_renorm_scales / _rows on the side stream, TW rescale inside k_tw_update,
k_renorm_tail; renormalize_parameters, audioModel.py:1980-2040) against the
unfused kernels (FASST_FAST_TAIL=0, read when a context is created) and the
oracle, on the structures it covers: one spectral component per source,
fixed FW, no time blobs.  Both fused modes are run: FASST_FAST_TAIL=1 (the
tail alone) and 2 (the default: the tail also forms the next iteration's
(FW.TW)^T and TW row sums at KP <= 64, and the next iteration of the batch
skips its prep).  Halted batches (a TW restart raised mid-batch) are covered in every mode:
the host swaps the W buffers of iterations the device skipped, and fasst_run
rebuilds W (and the prep) from the parameters."""
import numpy as np
import pytest

import fasst_ref as R
from helpers import rel

pytestmark = pytest.mark.gpu


def _models(F, T, J, K, rank, iters, conv=True, seed=0):
    import pyfasst_amd.audioModel as am
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    X = synthetic.stereo_mixture(F, T, J=J, K_true=4, rank=rank if np.isscalar(rank) else 2,
                                 seed=seed)
    np.random.seed(1)
    cls = am.MultiChanNMFConv if conv else am.MultiChanNMFInst_FASST
    m = cls(SpectralAudio(X=X), nbComps=J, nbNMFComps=K, spatial_rank=rank, iter_num=iters,
            wlen=2 * (F - 1), hopsize=(F - 1) // 2)
    if conv:
        m.makeItConvolutive()
    o = R.RefFASST(iter_num=iters)
    o.set_transform([X[0], X[1]])
    np.random.seed(1)
    R.init_nmf_inst(o, J, K, rank)
    if conv:
        R.make_convolutive(o)
    return m, o, X


# FASST_FAST_TAIL values; UNFUSED is the reference mode
MODES = ["1", "2"]
UNFUSED = "0"


def _run(monkeypatch, mode, args, kw, prep=None, restart_seed=None):
    monkeypatch.setenv("FASST_FAST_TAIL", mode)
    m, o, X = _models(*args, **kw)
    if prep:
        prep(m)
        prep(o)
    if restart_seed is not None:
        np.random.seed(restart_seed)
    ll = m.estim_param_a_post_model()
    return m, o, X, ll


CASES = [
    # (F, T, J, K, rank, iters), conv
    ((129, 301, 4, 32, 2, 6), True),      # the C3 structure, ragged T (and ragged 64-frame blocks)
    ((129, 301, 4, 32, 2, 6), False),     # 'inst' mixing
    ((97, 203, 3, 40, [1, 2, 1], 4), True),   # mixed ranks, K padded to 64 (the LDS prep path)
    ((97, 150, 2, 100, 2, 3), True),      # K > 64 (KP = 128: FW from L2)
    ((65, 77, 6, 8, 2, 3), True),         # J > 4
    ((81, 181, 2, 16, 1, 5), True),       # J = 2, KP = 16
    ((70, 97, 4, 20, 2, 4), True),        # K = 20 padded to 32, 7 frame tiles
]


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "tail" + m)
@pytest.mark.parametrize("args,conv", CASES)
def test_fast_tail_vs_unfused_and_oracle(monkeypatch, args, conv, mode):
    mf, o, X, llf = _run(monkeypatch, mode, args, dict(conv=conv))
    ms, _, _, lls = _run(monkeypatch, UNFUSED, args, dict(conv=conv))
    llo = o.estim_param_a_post_model()
    J = args[2]
    # the fused form sums the spatial energy in another order: last bits only
    assert rel(llf, lls) < 1e-12
    assert rel(llf, llo) < 1e-10
    for j in range(J):
        for key in ('FB', 'TW', 'FW'):
            a = mf.spec_comps[j]['factor'][0][key]
            assert rel(a, ms.spec_comps[j]['factor'][0][key]) < 1e-10
            assert rel(a, o.spec_comps[j]['factor'][0][key]) < 1e-8
        assert rel(mf.spat_comps[j]['params'], ms.spat_comps[j]['params']) < 1e-10
        assert rel(mf.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    # the separation reads the device's W (the swapped buffer of the last
    # iteration's fused tail)
    Sf = mf.separated_images()
    assert rel(np.abs(Sf), np.abs(ms.separated_images())) < 1e-10
    assert rel(np.abs(Sf), np.abs(o.separated_images(X))) < 1e-8


def _dead_tw(mod):   # tiny but non-zero: the mixing solve stays regular
    mod.spec_comps[1]['factor'][0]['TW'][:] = 1e-30


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "tail" + m)
def test_fast_tail_restart_halts_the_batch(monkeypatch, mode):
    """sum(TW) < eps after the first iteration: k_renorm_tail raises the
    restart flag, the batch's later iterations return at entry, the host
    redraws TW (audioModel.py:2023-2028) and resumes; W is rebuilt after the
    halted batch (the buffers swapped for skipped iterations)."""
    args = (33, 40, 2, 4, 1, 5)
    mf, o, X, llf = _run(monkeypatch, mode, args, {}, prep=_dead_tw, restart_seed=11)
    ms, _, _, lls = _run(monkeypatch, UNFUSED, args, {}, prep=_dead_tw, restart_seed=11)
    np.random.seed(11)
    llo = o.estim_param_a_post_model()
    assert rel(llf, lls) < 1e-12
    assert rel(llf, llo) < 1e-10
    for j in range(2):
        for key in ('FB', 'TW'):
            assert rel(mf.spec_comps[j]['factor'][0][key], o.spec_comps[j]['factor'][0][key]) < 1e-8
    Sf = mf.separated_images()
    assert rel(np.abs(Sf), np.abs(o.separated_images(X))) < 1e-8


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "tail" + m)
def test_fast_tail_second_run_after_restart(monkeypatch, mode):
    """A model run again after a restarted run starts from the host
    parameters (W rebuilt at the batch start, not a stale swapped buffer)."""
    args = (33, 40, 2, 4, 1, 3)
    mf, o, X, _ = _run(monkeypatch, mode, args, {}, prep=_dead_tw, restart_seed=5)
    np.random.seed(5)
    o.estim_param_a_post_model()
    ll2 = mf.estim_param_a_post_model()
    llo2 = o.estim_param_a_post_model()
    assert rel(ll2, llo2) < 1e-10
    for j in range(2):
        assert rel(mf.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8
