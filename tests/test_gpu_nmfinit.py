"""NMF initialisation of the spectral components (audioModel.py:2091-2222)
on the GPU vs the reference's outputs (tests/golden/nmfinit_*.npz): the IS-NMF
and the renormalisation run through the C ABI, then two GEM iterations."""
import os

import numpy as np
import pytest
import scipy.io.wavfile as wf

from helpers import load, rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("same", [True, False])
def test_nmf_init_then_em_vs_reference(same, tmp_path):
    import pyfasst_amd.audioModel as am
    name = "nmfinit_same" if same else "nmfinit_indiv"
    g = load(name)
    wav = os.path.join(str(tmp_path), name + ".wav")
    wf.write(wav, int(g['fs']), g['wav'])
    np.random.seed(0)
    m = am.MultiChanNMFConv(wav, nbComps=3, nbNMFComps=4, spatial_rank=2, iter_num=2,
                            wlen=256, hopsize=64)
    m.makeItConvolutive()
    np.random.seed(5)
    m.initialize_all_spec_comps_with_NMF(sameInitAll=same, niter=4)
    for k in range(3):
        assert rel(m.spec_comps[k]['factor'][0]['FB'], g['init_FB_%d' % k]) < 1e-10
        assert rel(m.spec_comps[k]['factor'][0]['TW'], g['init_TW_%d' % k]) < 1e-10
        assert rel(m.spat_comps[k]['params'], g['init_params_%d' % k]) < 1e-12
    ll = m.estim_param_a_post_model()
    assert rel(ll, g['logliks']) < 1e-9
    for k in range(3):
        assert rel(m.spec_comps[k]['factor'][0]['FB'], g['final_FB_%d' % k]) < 1e-9
        assert rel(m.spec_comps[k]['factor'][0]['TW'], g['final_TW_%d' % k]) < 1e-9
