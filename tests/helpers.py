"""Shared test helpers (test infrastructure only)."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

# golden case -> (J, K, spatial_rank, conv, ctor kwargs); mirrors tests/golden/make_golden.py
CASES = {
    "em_inst": (2, 4, 1, False, dict(iter_num=6, wlen=256, hopsize=128)),
    "em_inst_noann": (3, 5, 2, False, dict(iter_num=4, wlen=128, hopsize=64,
                                           sim_ann_opt='no_ann', nmfUpdateCoeff=0.7)),
    "em_conv": (3, 8, 2, True, dict(iter_num=5, wlen=256, hopsize=64)),
    "em_conv_j4": (4, 16, 2, True, dict(iter_num=4, wlen=256, hopsize=64)),
    "em_conv_j1": (1, 3, [2], True, dict(iter_num=3, wlen=128, hopsize=32)),
    "em_mqt": (2, 6, 2, True, dict(iter_num=3, wlen=256, hopsize=64, transf='mqt', tffmin=200,
                                   tfbpo=12)),
    # FW_frdm_prior 'free' with a dense positive FW (audioModel.py:1578-1631)
    "em_fw_free": (3, 6, 2, True, dict(iter_num=4, wlen=256, hopsize=64, _setup='fw_free')),
    # several spectral components per spatial component (audioModel.py:430-498,
    # 1479-1727), keys interleaved over the spatial components, a fixed FB and
    # a fixed TW among them
    "em_multi": (3, 8, 2, True, dict(iter_num=4, wlen=256, hopsize=64, _setup='multi_spec')),
    "em_multi_inst": (2, 8, 1, False, dict(iter_num=5, wlen=256, hopsize=128,
                                           _setup='multi_spec')),
    # lambdaCorr > 0: the inter-source correlation penalty (audioModel.py:1484-1719)
    "em_lambda": (3, 8, 2, True, dict(iter_num=4, wlen=256, hopsize=64, lambdaCorr=0.4)),
    "em_lambda_multi": (3, 8, 2, True, dict(iter_num=3, wlen=256, hopsize=64, lambdaCorr=0.7,
                                            _setup='multi_spec')),
    # time blobs H = TW.TB (audioModel.py:1665-1691, 1931-1978, 2029-2033): TB
    # free with TW free, TB free with TW fixed, TB fixed
    "em_tb": (3, 8, 2, True, dict(iter_num=4, wlen=256, hopsize=64, _setup='tb')),
    # 'inst' and 'conv' spatial components in one model (retrieve_subsrc_params
    # :546-576, update_mix_matrix :807-841 with the others held fixed): a free
    # and a fixed 'inst' component and a fixed 'conv' one
    "em_mixed": (3, 6, 1, False, dict(iter_num=5, wlen=256, hopsize=64, _setup='mixed')),
}

# time blobs of the 'tb' setup: spectral component key -> (L, TB prior, TW prior)
TB_SETUP = {0: (4, 'free', 'free'), 1: (6, 'free', 'fixed'), 2: (3, 'fixed', 'free')}

# column blocks of the 'multi_spec' setup: spatial component j -> block widths
MULTI_SPLITS = {0: [3, 2, 3], 1: [4, 4], 2: [8]}


def apply_setup(m, name):
    """Structure changes applied after construction (and makeItConvolutive),
    identically to the reference model (make_golden.py) and to the product."""
    if name == 'fw_free':
        for k in sorted(m.spec_comps.keys()):
            fac = m.spec_comps[k]['factor'][0]
            rs = np.random.RandomState(100 + k)
            K = fac['FW'].shape[0]
            fac['FW'] = fac['FW'] + 0.3 * np.abs(rs.randn(K, K))
            fac['FW_frdm_prior'] = 'free'
    elif name == 'multi_spec':
        import copy
        pieces = {}
        for k in sorted(m.spec_comps.keys()):
            comp = m.spec_comps[k]
            j = comp['spat_comp_ind']
            fac = comp['factor'][0]
            a = 0
            pieces[j] = []
            for n in MULTI_SPLITS[j]:
                f = copy.deepcopy(fac)
                f['FB'] = np.array(fac['FB'][:, a:a + n])
                f['FW'] = np.array(fac['FW'][a:a + n, a:a + n])
                f['TW'] = np.array(fac['TW'][a:a + n])
                pieces[j].append({'spat_comp_ind': j, 'factor': {0: f}})
                a += n
        new, key = {}, 0
        for pos in range(max(len(v) for v in pieces.values())):
            for j in sorted(pieces):
                if pos < len(pieces[j]):
                    new[key] = pieces[j][pos]
                    key += 1
        new[2]['factor'][0]['FB_frdm_prior'] = 'fixed'
        new[3]['factor'][0]['TW_frdm_prior'] = 'fixed'
        m.spec_comps = new
    elif name == 'tb':
        for k, (L, tb_prior, tw_prior) in TB_SETUP.items():
            fac = m.spec_comps[k]['factor'][0]
            K, T = fac['TW'].shape
            rs = np.random.RandomState(300 + k)
            TB = np.abs(rs.randn(L, T)) + 0.2
            TW = np.abs(rs.randn(K, L)) + 0.2
            TW *= fac['TW'].mean() / np.dot(TW, TB).mean()
            fac['TW'], fac['TB'] = TW, TB
            fac['TB_frdm_prior'], fac['TW_frdm_prior'] = tb_prior, tw_prior
    elif name == 'mixed':
        # component 1 'inst' fixed; component 2 'conv' fixed, its filters the
        # 'inst' gains with a per-channel delay (a genuinely per-bin mixing)
        F = m.nbFreqsSigRepr
        m.spat_comps[1]['frdm_prior'] = 'fixed'
        sc = m.spat_comps[2]
        inst = np.asarray(sc['params'])          # C x r
        r = inst.shape[1]
        delay = np.array([0.0, 1.5])
        ph = np.exp(-1j * np.pi * np.outer(delay, np.arange(F)) / (F - 1))   # C x F
        p = np.zeros((r, 2, F), dtype=complex)
        for c in range(2):
            p[:, c, :] = np.outer(inst[c], ph[c])
        sc['params'] = p
        sc['mix_type'] = 'conv'
        sc['frdm_prior'] = 'fixed'
    else:
        raise ValueError(name)

# tests/golden/cqt.npz cases; mirrors CQT_CASES of tests/golden/make_golden.py
CQT_CASES = (
    ("mqt12", "mqt", dict(fmin=25, fmax=3000, bins=12, fs=8000, linFTLen=512,
                          atomHopFactor=0.25)),
    ("mqt48", "mqt", dict(fmin=100, fmax=18000, bins=48, fs=8000, linFTLen=256,
                          atomHopFactor=0.25)),
    ("mqt_h", "mqt", dict(fmin=300, fmax=18000, bins=24, fs=16000, linFTLen=512,
                          atomHopFactor=0.0625)),
    ("cqt12", "cqt", dict(fmin=100, fmax=3000, bins=12, fs=8000, atomHopFactor=0.25)),
    ("cqt_h", "cqt", dict(fmin=150, fmax=3500, bins=24, fs=8000, atomHopFactor=0.5)),
)


# BASELINE-size cases of tests/golden/make_fullsize.py (oracle-generated fixtures)
FULL_CASES = {
    "c3_full": dict(F=2049, T=10000, J=4, K=32, rank=2, conv=True, iters=2, K_true=8,
                    data_rank=2, data_seed=0, init_seed=1),
    "c3_t1000": dict(F=2049, T=1000, J=4, K=32, rank=2, conv=True, iters=3, K_true=8,
                     data_rank=2, data_seed=3, init_seed=1),
    # K = 128 at the full F (the production launch shapes of the K > 64
    # paths: the pipelined E-step V tiles, the LDS-staged TW contraction at
    # KP = 128, the FW-from-L2 staging kernels)
    "j8k128_t1000": dict(F=2049, T=1000, J=8, K=128, rank=1, conv=True, iters=2, K_true=8,
                         data_rank=1, data_seed=5, init_seed=1),
    "j4k128_t1000": dict(F=2049, T=1000, J=4, K=128, rank=2, conv=True, iters=2, K_true=8,
                         data_rank=2, data_seed=6, init_seed=1),
    "c1_50": dict(F=1025, T=1122, J=2, K=32, rank=1, conv=False, iters=50, K_true=8,
                  data_rank=1, data_seed=0, init_seed=0),
    "c5_full": dict(F=2049, N=20000, NF0=1092, P=30, K=4, R=40, iters=1, data_seed=0,
                    init_seed=1),
    # the pipeline's default nbIter=10 (SeparateLeadStereoTF.py:264): multiplicative-
    # update drift over the iterations the product actually runs
    "c5_10": dict(F=2049, N=20000, NF0=1092, P=30, K=4, R=40, iters=10, data_seed=0,
                  init_seed=1),
}


def sub_f(F):
    """Bins kept in the full-size fixtures (every 7th, and the last)."""
    return np.unique(np.r_[np.arange(0, F, 7), F - 1])


def sub_t(T):
    """Frames kept in the full-size fixtures (about 40, and the last)."""
    return np.unique(np.r_[np.arange(0, T, max(1, T // 40)), T - 1])


def spec_keys(g, J):
    """Spectral component keys of a golden EM case (one per spatial component
    unless the case recorded its count)."""
    return range(int(g['init_nspec'])) if 'init_nspec' in g else range(J)


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def rel(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    den = np.max(np.abs(b))
    return float(np.max(np.abs(a - b)) / (den if den > 0 else 1.0))


def rel_elem(a, b, floor=1e-6):
    """Elementwise relative error max |a - b| / max(|b|, floor * max|b|): every
    point held to its own magnitude, the floor keeping exact-zero / underflowed
    points out of the quotient."""
    a = np.asarray(a)
    b = np.asarray(b)
    den = np.maximum(np.abs(b), floor * np.max(np.abs(b)))
    den = np.where(den > 0, den, 1.0)
    return float(np.max(np.abs(a - b) / den))


def oracle_model_from_golden(g, case):
    """Oracle model on the golden wav (oracle STFT), initialised like the reference."""
    import fasst_ref as R
    J, K, rank, conv, kw = CASES[case]
    x, _ = R.read_scaled(g['wav'])
    wlen, hop = kw['wlen'], kw['hopsize']
    if kw.get('transf', 'stft') == 'stft':
        w = np.hanning(wlen)
        X = [R.stft(x[:, c], w, hop, wlen) for c in range(2)]
    else:   # FASST's MinQT / CQT front end (audioModel.py:206-214)
        import cqt_ref
        t = cqt_ref.RefCQT(kw['transf'].replace('minqt', 'mqt'), fmin=kw.get('tffmin', 25),
                           fmax=kw.get('tffmax', 18000), bins=kw.get('tfbpo', 48),
                           fs=int(g['fs']), linFTLen=wlen, atomHopFactor=hop / float(wlen))
        X = [t.forward(x[:, c]) for c in range(2)]
    okw = {k: v for k, v in kw.items() if k in ('iter_num', 'sim_ann_opt', 'nmfUpdateCoeff',
                                              'lambdaCorr')}
    m = R.RefFASST(**okw)
    m.set_transform(X)
    np.random.seed(0)
    R.init_nmf_inst(m, J, K, rank)
    if conv:
        R.make_convolutive(m)
    if kw.get('_setup'):
        apply_setup(m, kw['_setup'])
    return m, X
