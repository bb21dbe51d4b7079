"""Generate the golden fixtures in tests/golden/ by running the REFERENCE.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden.py            # all cases
    python tests/golden/make_golden.py em_inst    # one case

Each case runs in a fresh interpreter (reference quirk N2: the default
`ann_PSD_lim=[None, None]` list is shared by every model of a process,
audioModel.py:166,242,320-323).  The reference is imported from a scratch
py2->py3 translation built by oracle/make_scratch_ref.py under /tmp; only the
numeric inputs/outputs are committed (as .npz), never reference source.

Inputs are synthetic and seeded (no data derived from data/tamy.wav, which is
CC BY-NC).  Separated images are captured at the reference's own
`tft.invertTransform` call inside `separate_comps` (audioModel.py:1203), i.e.
the STFT-domain images sum_c2 WG[c1,c2] X[c2] the reference inverts.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SCRATCH = "/tmp/pyfasst_scratch"

CASES = {
    # name: (model class, kwargs, nbComps, nbNMFComps, spatial_rank, conv, wav seconds, fs)
    "em_inst": dict(cls="MultiChanNMFInst_FASST", nbComps=2, nbNMFComps=4, spatial_rank=1,
                    conv=False, n=6000, fs=8000, kw=dict(iter_num=6, wlen=256, hopsize=128)),
    "em_inst_noann": dict(cls="MultiChanNMFInst_FASST", nbComps=3, nbNMFComps=5, spatial_rank=2,
                          conv=False, n=5000, fs=8000,
                          kw=dict(iter_num=4, wlen=128, hopsize=64, sim_ann_opt='no_ann',
                                  nmfUpdateCoeff=0.7)),
    "em_conv": dict(cls="MultiChanNMFConv", nbComps=3, nbNMFComps=8, spatial_rank=2,
                    conv=True, n=6000, fs=8000, kw=dict(iter_num=5, wlen=256, hopsize=64)),
    "em_conv_j4": dict(cls="MultiChanNMFConv", nbComps=4, nbNMFComps=16, spatial_rank=2,
                       conv=True, n=6000, fs=8000, kw=dict(iter_num=4, wlen=256, hopsize=64)),
    # FASST on the MinQT front end (transf='mqt', audioModel.py:156,206-214,1187-1203)
    "em_mqt": dict(cls="MultiChanNMFConv", nbComps=2, nbNMFComps=6, spatial_rank=2,
                   conv=True, n=4000, fs=8000,
                   kw=dict(iter_num=3, wlen=256, hopsize=64, transf='mqt', tffmin=200,
                           tfbpo=12)),
    "em_conv_j1": dict(cls="MultiChanNMFConv", nbComps=1, nbNMFComps=3, spatial_rank=[2],
                       conv=True, n=3000, fs=8000, kw=dict(iter_num=3, wlen=128, hopsize=32)),
    # FW_frdm_prior 'free' with a dense FW (tests/helpers.py apply_setup)
    "em_fw_free": dict(cls="MultiChanNMFConv", nbComps=3, nbNMFComps=6, spatial_rank=2,
                       conv=True, n=5000, fs=8000, kw=dict(iter_num=4, wlen=256, hopsize=64),
                       setup='fw_free'),
    # several spectral components per spatial component (tests/helpers.py
    # apply_setup 'multi_spec': unequal column blocks, interleaved keys)
    "em_multi": dict(cls="MultiChanNMFConv", nbComps=3, nbNMFComps=8, spatial_rank=2,
                     conv=True, n=5000, fs=8000, kw=dict(iter_num=4, wlen=256, hopsize=64),
                     setup='multi_spec'),
    "em_multi_inst": dict(cls="MultiChanNMFInst_FASST", nbComps=2, nbNMFComps=8,
                          spatial_rank=1, conv=False, n=6000, fs=8000,
                          kw=dict(iter_num=5, wlen=256, hopsize=128), setup='multi_spec'),
    # lambdaCorr > 0 (audioModel.py:1484-1719), one and several components per source
    "em_lambda": dict(cls="MultiChanNMFConv", nbComps=3, nbNMFComps=8, spatial_rank=2,
                      conv=True, n=5000, fs=8000,
                      kw=dict(iter_num=4, wlen=256, hopsize=64, lambdaCorr=0.4)),
    "em_lambda_multi": dict(cls="MultiChanNMFConv", nbComps=3, nbNMFComps=8, spatial_rank=2,
                            conv=True, n=5000, fs=8000,
                            kw=dict(iter_num=3, wlen=256, hopsize=64, lambdaCorr=0.7),
                            setup='multi_spec'),
    # time blobs on the three components (tests/helpers.py apply_setup 'tb')
    "em_tb": dict(cls="MultiChanNMFConv", nbComps=3, nbNMFComps=8, spatial_rank=2,
                  conv=True, n=5000, fs=8000, kw=dict(iter_num=4, wlen=256, hopsize=64),
                  setup='tb'),
    # 'inst' (free, fixed) and 'conv' (fixed) spatial components in one model
    # (tests/helpers.py apply_setup 'mixed')
    "em_mixed": dict(cls="MultiChanNMFInst_FASST", nbComps=3, nbNMFComps=6, spatial_rank=1,
                     conv=False, n=5000, fs=8000, kw=dict(iter_num=5, wlen=256, hopsize=64),
                     setup='mixed'),
}


def synth_wav(n, fs, seed):
    """Seeded stereo int16 test signal: two panned, filtered noise bursts."""
    import numpy as np
    rs = np.random.RandomState(seed)
    t = np.arange(n) / float(fs)
    s1 = rs.randn(n) * (0.5 + 0.5 * np.sin(2 * np.pi * 1.3 * t)) + np.sin(2 * np.pi * 440 * t)
    s2 = np.convolve(rs.randn(n), np.ones(5) / 5., mode='same') * (t > 0.1)
    x = np.stack([0.8 * s1 + 0.3 * s2, 0.4 * s1 + 0.9 * np.roll(s2, 3)], axis=1)
    x = x / np.abs(x).max() * 20000
    return x.astype(np.int16)


def run_case(name):
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    import scipy.io.wavfile as wf
    import pyfasst.audioModel as am
    cfg = CASES[name]
    seed = sum(map(ord, name)) % 1000
    data = synth_wav(cfg['n'], cfg['fs'], seed)
    wav = "/tmp/golden_%s.wav" % name
    wf.write(wav, cfg['fs'], data)
    np.random.seed(0)
    cls = getattr(am, cfg['cls'])
    m = cls(wav, nbComps=cfg['nbComps'], nbNMFComps=cfg['nbNMFComps'],
            spatial_rank=cfg['spatial_rank'], verbose=0, **cfg['kw'])
    if cfg['conv']:
        m.makeItConvolutive()
    if cfg.get('setup'):
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from helpers import apply_setup
        apply_setup(m, cfg['setup'])
    out = {'wav': data, 'fs': np.array(cfg['fs']), 'Cx': m.Cx,
           'psd_lim0': np.asarray(m.noise['ann_PSD_lim'][0]),
           'psd_lim1': np.asarray(m.noise['ann_PSD_lim'][1])}

    def dump(prefix):
        out['%snspec' % prefix] = np.array(len(m.spec_comps))
        for j, sc in m.spat_comps.items():
            out['%sparams_%d' % (prefix, j)] = np.array(sc['params'])
        for k, comp in m.spec_comps.items():
            f = comp['factor'][0]
            out['%sFB_%d' % (prefix, k)] = np.array(f['FB'])
            out['%sFW_%d' % (prefix, k)] = np.array(f['FW'])
            out['%sTW_%d' % (prefix, k)] = np.array(f['TW'])
            if len(f['TB']):
                out['%sTB_%d' % (prefix, k)] = np.array(f['TB'])
    dump('init_')
    # one E-step on the initial state (pins compute_suff_stat itself)
    if m.noise['sim_ann_opt'] == 'ann':
        m.noise['PSD'] = ((np.sqrt(m.noise['ann_PSD_lim'][0]) * m.iter_num) / m.iter_num) ** 2
    else:
        m.noise['PSD'] = m.noise['ann_PSD_lim'][1]
    V, mix, parts = m.retrieve_subsrc_params()
    _, hRxs, hRss, hWs, ll = m.compute_suff_stat(V, mix)
    out.update(e_psd=np.asarray(m.noise['PSD']), e_hat_Rxs=hRxs, e_hat_Rss=hRss,
               e_hat_Ws=hWs, e_loglik=np.array(ll))
    logliks = m.estim_param_a_post_model()
    out['logliks'] = np.real(logliks)
    out['final_psd'] = np.asarray(m.noise['PSD'])
    dump('final_')
    # separation: capture STFT-domain images at invertTransform
    images = []
    orig = m.tft.invertTransform

    def capture():
        images.append(np.array(m.tft.transfo))
        return orig()
    m.tft.invertTransform = capture
    outdir = "/tmp/golden_%s_sep" % name
    os.makedirs(outdir, exist_ok=True)
    m.separate_spat_comps(dir_results=outdir)
    J = len(m.spat_comps)
    out['images'] = np.array(images).reshape(J, 2, *images[0].shape)
    for n, fn in enumerate(m.files['spat_comp']):
        out['sep_wav_%d' % n] = wf.read(fn)[1]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, {k: np.shape(v) for k, v in out.items() if k in ('Cx', 'images', 'logliks')})


def run_stft():
    sys.path.insert(0, SCRATCH)
    import numpy as np
    from pyfasst.tftransforms import stft as S
    rs = np.random.RandomState(7)
    x = rs.randn(3001)
    out = {'x': x}
    for nfft, hop in ((256, 64), (512, 128), (1024, 256)):
        tr = S.STFT(linFTLen=nfft, atomHopFactor=hop / float(nfft))
        tr.computeTransform(x)
        out['X_%d_%d' % (nfft, hop)] = tr.transfo
        out['y_%d_%d' % (nfft, hop)] = tr.invertTransform()
    np.savez_compressed(os.path.join(HERE, "stft.npz"), **out)
    print("stft")


def run_nmf():
    sys.path.insert(0, SCRATCH)
    import numpy as np
    from pyfasst.tools import nmf
    rs = np.random.RandomState(3)
    SX = rs.gamma(0.7, 1.0, size=(97, 150)) * np.outer(rs.gamma(2, 1, 97), np.ones(150))
    np.random.seed(1)
    W, H = nmf.NMF_decomposition(SX, nbComps=6, niter=7)
    res = dict(SX=SX, W=W, H=H)
    # NMF_decomp_init: random start; given W frozen; given frame-major H
    np.random.seed(2)
    res['di_W'], res['di_H'] = nmf.NMF_decomp_init(SX, nbComps=5, niter=6)
    Winit = rs.gamma(1.0, 1.0, size=(97, 4))
    Hinit = rs.gamma(1.0, 1.0, size=(150, 4))
    np.random.seed(3)
    res['Winit'], res['Hinit'] = Winit, Hinit
    res['dw_W'], res['dw_H'] = nmf.NMF_decomp_init(SX, nbComps=4, niter=5, Winit=Winit,
                                                   updateW=False)
    np.random.seed(4)
    res['dh_W'], res['dh_H'] = nmf.NMF_decomp_init(SX, nbComps=4, niter=5, Hinit=Hinit)
    np.savez_compressed(os.path.join(HERE, "nmf.npz"), **res)
    print("nmf")


def run_simm():
    """Stereo_SIMM (SIMM.py:397-943) and SIMM (SIMM.py:46-395) on seeded
    synthetic inputs (random positive bases stand in for the KLGLOTT88 WF0)."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    from pyfasst.SeparateLeadStereo.SIMM import SIMM as S
    rs = np.random.RandomState(11)
    F, N, NF0, P, K, R = 65, 40, 24, 6, 3, 5
    SXR = rs.gamma(0.8, 1.0, size=(F, N))
    SXL = rs.gamma(0.8, 1.0, size=(F, N))
    WF0 = rs.gamma(1.0, 1.0, size=(F, NF0))
    WGAMMA = rs.gamma(1.0, 1.0, size=(F, P))
    np.random.seed(1)
    out = S.Stereo_SIMM(SXR, SXL, WF0, WGAMMA, numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=R, numberOfIterations=4,
                        verbose=False)
    names = ['alphaR', 'alphaL', 'HGAMMA', 'HPHI', 'HF0', 'betaR', 'betaL', 'HM', 'WM', 'recoError']
    res = {'st_' + n: np.asarray(v) for n, v in zip(names, out)}
    # mono SIMM with R = 1 (the estimHF0 call, SeparateLeadStereoTF.py:996)
    np.random.seed(2)
    mout = S.SIMM(SXR, WF0, WGAMMA, numberOfFilters=K, numberOfAccompanimentSpectralShapes=1,
                  numberOfIterations=4, verbose=False)
    res.update({'mono_' + n: np.asarray(v) for n, v in
                zip(['HGAMMA', 'HPHI', 'HF0', 'HM', 'WM', 'recoError'], mout)})
    # stereo with computeError, frozen HGAMMA and omega != 1
    np.random.seed(3)
    out = S.Stereo_SIMM(SXR, SXL, WF0, WGAMMA, numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=R, numberOfIterations=3,
                        updateRulePower=0.7, updateHGAMMA=False, computeError=True,
                        verbose=False)
    res.update({'st2_' + n: np.asarray(v) for n, v in zip(names, out)})
    # mono with R == N (the other shape quirk N7 admits, SIMM.py:388)
    np.random.seed(4)
    mout = S.SIMM(SXR, WF0, WGAMMA, numberOfFilters=K, numberOfAccompanimentSpectralShapes=N,
                  numberOfIterations=3, verbose=False)
    res.update({'monoN_' + n: np.asarray(v) for n, v in
                zip(['HGAMMA', 'HPHI', 'HF0', 'HM', 'WM', 'recoError'], mout)})
    np.savez_compressed(os.path.join(HERE, "simm.npz"), SXR=SXR, SXL=SXL, WF0=WF0,
                        WGAMMA=WGAMMA, **res)
    print("simm")


def run_lead():
    """SIMM-pipeline stft/istft (separateLeadFunctions.py:90-233) and the
    writeSeparatedSignals masks (SeparateLeadStereoTF.py:1762-1871) applied
    with the stereo SIMM golden parameters to a seeded stereo signal."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    import scipy.io.wavfile as wf
    from pyfasst.SeparateLeadStereo import separateLeadFunctions as slf
    from pyfasst.SeparateLeadStereo import SeparateLeadStereoTF as SL
    rs = np.random.RandomState(21)
    out = {}
    x = rs.randn(1216)
    out['x'] = x
    for (wlen, hop, nfft, start, stop) in ((128, 32, 128, 0, None), (256, 64, 512, 3, 17),
                                           (100, 25, 128, 0, None)):
        tag = '%d_%d_%d' % (wlen, hop, nfft)
        X, F, N = slf.stft(x, window=slf.sinebell(wlen), hopsize=float(hop), nfft=float(nfft),
                           fs=8000., start=start, stop=stop)
        out['X_' + tag], out['F_' + tag], out['N_' + tag] = X, F, N
        out['y_' + tag] = slf.istft(X, window=slf.sinebell(wlen), hopsize=float(hop),
                                    nfft=float(nfft))
        out['yh_' + tag] = slf.istft(X, analysisWindow=np.hanning(wlen),
                                     window=slf.sinebell(wlen), hopsize=float(hop),
                                     nfft=float(nfft), originalDataLen=1000)
    g = np.load(os.path.join(HERE, "simm.npz"))
    xs = (rs.randn(1216, 2) * 3000)
    XR = slf.stft(xs[:, 0], window=slf.sinebell(128), hopsize=32., nfft=128.)[0]
    XL = slf.stft(xs[:, 1], window=slf.sinebell(128), hopsize=32., nfft=128.)[0]
    proc = object.__new__(SL.SeparateLeadProcess)
    proc.SIMMParams = {'WF0': g['WF0'], 'HF0': g['st_HF0'], 'WGAMMA': g['WGAMMA'],
                       'HGAMMA': g['st_HGAMMA'], 'HPHI': g['st_HPHI'], 'HM': g['st_HM'],
                       'WM': g['st_WM'], 'alphaR': g['st_alphaR'], 'alphaL': g['st_alphaL'],
                       'betaR': g['st_betaR'], 'betaL': g['st_betaL']}
    proc.stftParams = {'windowSizeInSamples': 128, 'hopsize': 32., 'NFT': 128}
    proc.tfrepresentation = 'stft'
    proc.XR, proc.XL = XR, XL
    proc.scaleData = 1.0
    proc.dataType = np.int16
    proc.fs = 8000
    proc.files = {'voc_output_file': '/tmp/golden_lead_voc.wav',
                  'mus_output_file': '/tmp/golden_lead_mus.wav'}
    seen = []
    orig = SL.slf.istft

    def capture(X, *a, **kw):
        y = orig(X, *a, **kw)
        seen.append((np.array(X), np.array(y)))
        return y
    SL.slf.istft = capture
    proc.writeSeparatedSignals()
    SL.slf.istft = orig
    out['XR'], out['XL'] = XR, XL
    for i, name in enumerate(('vR', 'vL', 'mR', 'mL')):
        out['mask_' + name], out['est_' + name] = seen[i]
    out['voc_wav'] = wf.read('/tmp/golden_lead_voc.wav')[1]
    out['mus_wav'] = wf.read('/tmp/golden_lead_mus.wav')[1]
    np.savez_compressed(os.path.join(HERE, "lead.npz"), **out)
    print("lead", {k: np.shape(v) for k, v in out.items() if k.startswith(('mask', 'voc'))})


CQT_CASES = (
    # name, class, kwargs (perfRast=1 as FASST builds them, audioModel.py:206-214)
    ("mqt12", "MinQTransfo", dict(fmin=25, fmax=3000, bins=12, fs=8000, linFTLen=512,
                                  atomHopFactor=0.25)),
    ("mqt48", "MinQTransfo", dict(fmin=100, fmax=18000, bins=48, fs=8000, linFTLen=256,
                                  atomHopFactor=0.25)),
    ("mqt_h", "MinQTransfo", dict(fmin=300, fmax=18000, bins=24, fs=16000, linFTLen=512,
                                  atomHopFactor=0.0625)),
    ("cqt12", "CQTransfo", dict(fmin=100, fmax=3000, bins=12, fs=8000, atomHopFactor=0.25)),
    ("cqt_h", "CQTransfo", dict(fmin=150, fmax=3500, bins=24, fs=8000, atomHopFactor=0.5)),
)


def run_cqt():
    """CQTransfo / MinQTransfo (tftransforms/minqt.py) forward + inverse with
    perfRast=1 on a seeded signal: spCQT (transfo), frame counts, frequency
    stamps and invertTransform() of the same spCQT."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    from pyfasst.tftransforms import minqt
    rs = np.random.RandomState(31)
    x = rs.randn(3000) * (1 + np.sin(np.arange(3000) / 300.))
    out = {'x': x}
    for name, cls, kw in CQT_CASES:
        t = getattr(minqt, cls)(perfRast=1, **kw)
        t.computeTransform(x)
        X = np.array(t.transfo)
        out['X_' + name] = X
        out['nframes_' + name] = np.array(t.nframes)
        out['freqs_' + name] = np.array(t.freq_stamps)
        t.transfo = X
        out['y_' + name] = np.array(t.invertTransform())
    np.savez_compressed(os.path.join(HERE, "cqt.npz"), **out)
    print("cqt", {k: np.shape(v) for k, v in out.items() if k.startswith('X_')})


def run_viterbi():
    """Viterbi tracker (SeparateLeadStereo/tracking/tracking.py, the reference's
    own pure-Python tracker; same algorithm as _tracking.pyx) on seeded
    inputs, and runViterbi's transition / log-density construction
    (SeparateLeadStereoTF.py:1150-1319) captured at its tracker call."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    from pyfasst.SeparateLeadStereo.tracking import tracking as TR
    from pyfasst.SeparateLeadStereo import SeparateLeadStereoTF as SL
    rs = np.random.RandomState(41)
    out = {}
    # random dense HMM
    S, N = 37, 53
    T = rs.gamma(0.5, 1.0, size=(S, S))
    T /= T.sum(axis=1)[:, None]
    out['r_logD'] = np.log(rs.gamma(1.0, 1.0, size=(S, N)))
    out['r_logT'] = np.log(T)
    out['r_prior'] = np.log(np.ones(S) / S)
    out['r_path'] = TR.viterbiTrackingArray(out['r_logD'], out['r_prior'], out['r_logT'])
    out['r_path_naive'] = TR.viterbiTracking(out['r_logD'], out['r_prior'], out['r_logT'])
    # ties everywhere (small integers) and impossible transitions (-inf)
    S, N = 19, 40
    out['t_logD'] = rs.randint(-3, 1, size=(S, N)).astype(float)
    lt = rs.randint(-2, 1, size=(S, S)).astype(float)
    lt[rs.rand(S, S) < 0.2] = -np.inf
    lt[np.arange(S), np.arange(S)] = 0.0
    out['t_logT'] = lt
    out['t_prior'] = rs.randint(-1, 1, size=S).astype(float)
    out['t_path'] = TR.viterbiTrackingArray(out['t_logD'], out['t_prior'], out['t_logT'])
    out['t_path_naive'] = TR.viterbiTracking(out['t_logD'], out['t_prior'], out['t_logT'])
    # runViterbi on a stub process: NF0 = 64 states + silence, stepNotes = 4
    NF0, N = 64, 75
    HF0 = rs.gamma(0.3, 1.0, size=(NF0, N))
    HF0[:, 5] = 0.0
    HF0[rs.rand(NF0, N) < 0.05] = 0.0
    proc = object.__new__(SL.SeparateLeadProcess)
    proc.SIMMParams = {'HF0': HF0, 'NF0': NF0, 'chirpPerF0': 1, 'minF0': 100., 'maxF0': 800.,
                       'F0Table': 100. * 2 ** (np.arange(NF0) / 12.), 'stepNotes': 4}
    proc.trackingParams = {'minF0search': 100., 'maxF0search': 800.}
    proc.N = N
    proc.computeNFrames = lambda: None
    proc.files = {'pitch_output_file': '/tmp/golden_pitch.txt'}
    proc.stftParams = {'hopsize': 256.}
    proc.fs = 8000.
    proc.verbose = False
    seen = {}

    def tracker(S_, N_, logD, prior, logT, verbose=False):
        seen.update(S=S_, N=N_, logD=np.array(logD), prior=np.array(prior), logT=np.array(logT))
        # Cython semantics: the first S_ states only
        return TR.viterbiTrackingArray(logD[:S_, :N_], prior[:S_], logT[:S_, :S_])
    SL.viterbiTrackingArray = tracker
    proc.runViterbi()
    out['m_HF0'] = HF0
    out['m_S'] = np.array(seen['S'])
    out['m_logD'], out['m_prior'], out['m_logT'] = seen['logD'], seen['prior'], seen['logT']
    out['m_path'] = np.array(proc.indexBestPath)
    out['m_freq'] = np.array(proc.freqMelody)
    np.savez_compressed(os.path.join(HERE, "viterbi.npz"), **out)
    print("viterbi", {k: np.shape(v) for k, v in out.items() if 'path' in k})


def run_wf0():
    """SIMM dictionaries: generate_WF0_TR_chirped with the STFT transform
    SeparateLeadProcess.computeWF0 builds for tfrepresentation='stft'
    (SeparateLeadStereoTF.py:646-681), with and without chirps, and
    generateHannBasis (separateLeadFunctions.py:1074-1146)."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    os.chdir("/tmp")        # the reference writes its .npz cache to the cwd
    import numpy as np
    from pyfasst.SeparateLeadStereo import separateLeadFunctions as slf
    from pyfasst.tftransforms import tft
    from pyfasst.tools.utils import sqrt_blackmanharris
    out = {}
    for tag, (fs, nft, minF0, maxF0, stepNotes, perF0) in {
            'a': (8000, 256, 100, 800, 4, 1), 'b': (8000, 512, 150, 600, 2, 3),
            'c': (16000, 256, 60, 1000, 1, 1)}.items():
        t = tft.tftransforms['stft'](fmin=25, fmax=18000, bins=48, fs=fs, linFTLen=nft,
                                     atomHopFactor=0.25, winFunc=sqrt_blackmanharris, perfRast=1)
        F0Table, WF0, _ = slf.generate_WF0_TR_chirped(
            transform=t, minF0=minF0, maxF0=maxF0, stepNotes=stepNotes, Ot=0.5, perF0=perF0,
            depthChirpInSemiTone=0.5, loadWF0=False)
        out['F0Table_' + tag], out['WF0_' + tag] = F0Table, WF0
    for tag, (F, nft, fs, P, ov) in {'h1': (129, 256, 8000, 10, 0.75),
                                     'h2': (257, 512, 16000, 30, 0.5),
                                     'h3': (2049, 4096, 44100, 30, 0.75)}.items():
        out['WGAMMA_' + tag] = slf.generateHannBasis(F, nft, fs, numberOfBasis=P, overlap=ov)
    np.savez_compressed(os.path.join(HERE, "wf0.npz"), **out)
    print("wf0", {k: np.shape(v) for k, v in out.items()})


def run_wf0_cqt():
    """generate_WF0_TR_chirped on CQT-type transforms (separateLeadFunctions.py
    :742-886 with the tft.py registry's MinQTransfo / CQTransfo, as
    SeparateLeadProcess.computeWF0 builds them for tfrepresentation 'mqt' /
    'cqt', SeparateLeadStereoTF.py:656-681): the complex comb goes through
    the transform; with and without chirps."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import shutil
    work = "/tmp/golden_wf0_cqt"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    os.chdir(work)          # the reference writes its .npz cache to the cwd
    import numpy as np
    from pyfasst.SeparateLeadStereo import separateLeadFunctions as slf
    from pyfasst.tftransforms import tft
    from pyfasst.tools.utils import sqrt_blackmanharris
    out = {}
    for tag, (kind, fs, nft, fmin, fmax, bins, minF0, maxF0, stepNotes, perF0) in {
            'm1': ('mqt', 8000, 512, 50, 4000, 12, 100, 800, 4, 1),
            'm2': ('mqt', 8000, 1024, 60, 4000, 24, 150, 600, 2, 3),
            'c1': ('cqt', 8000, 512, 100, 1600, 12, 100, 400, 2, 1)}.items():
        t = tft.tftransforms[kind](fmin=fmin, fmax=fmax, bins=bins, fs=fs, linFTLen=nft,
                                   atomHopFactor=0.25, winFunc=sqrt_blackmanharris, perfRast=1)
        F0Table, WF0, _ = slf.generate_WF0_TR_chirped(
            transform=t, minF0=minF0, maxF0=maxF0, stepNotes=stepNotes, Ot=0.5, perF0=perF0,
            depthChirpInSemiTone=0.5, loadWF0=False)
        out['F0Table_' + tag], out['WF0_' + tag] = F0Table, WF0
        out['cfg_' + tag] = np.array([fs, nft, fmin, fmax, bins, minF0, maxF0, stepNotes, perF0],
                                     dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "wf0_cqt.npz"), **out)
    print("wf0_cqt", {k: np.shape(v) for k, v in out.items()})


def run_nmfinit(same):
    """initialize_all_spec_comps_with_NMF (audioModel.py:2091-2222) on a
    seeded model, then 2 GEM iterations from that initial state."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    import scipy.io.wavfile as wf
    import pyfasst.audioModel as am
    name = "nmfinit_same" if same else "nmfinit_indiv"
    data = synth_wav(4000, 8000, 77 if same else 78)
    wav = "/tmp/golden_%s.wav" % name
    wf.write(wav, 8000, data)
    np.random.seed(0)
    m = am.MultiChanNMFConv(wav, nbComps=3, nbNMFComps=4, spatial_rank=2, verbose=0,
                            iter_num=2, wlen=256, hopsize=64)
    m.makeItConvolutive()
    out = {'wav': data, 'fs': np.array(8000)}
    np.random.seed(5)
    if same:
        m.initialize_all_spec_comps_with_NMF(sameInitAll=True, niter=4)
    else:
        m.initialize_all_spec_comps_with_NMF(sameInitAll=False, niter=4,
                                             updateFreqBasis=True, updateTimeWeight=True)
    for k, comp in m.spec_comps.items():
        out['init_FB_%d' % k] = np.array(comp['factor'][0]['FB'])
        out['init_TW_%d' % k] = np.array(comp['factor'][0]['TW'])
    for j, sc in m.spat_comps.items():
        out['init_params_%d' % j] = np.array(sc['params'])
    out['logliks'] = np.real(m.estim_param_a_post_model())
    for k, comp in m.spec_comps.items():
        out['final_FB_%d' % k] = np.array(comp['factor'][0]['FB'])
        out['final_TW_%d' % k] = np.array(comp['factor'][0]['TW'])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, out['logliks'])


def run_convinit():
    """initializeConvParams(initMethod='rand') (audioModel.py:2224-2294) on a
    seeded model: the random steering vectors' RNG order, the 'conv'
    parameters they fill, then 3 GEM iterations from that state."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import numpy as np
    import scipy.io.wavfile as wf
    import pyfasst.audioModel as am
    name = "convinit_rand"
    data = synth_wav(4000, 8000, 79)
    wav = "/tmp/golden_%s.wav" % name
    wf.write(wav, 8000, data)
    np.random.seed(0)
    m = am.MultiChanNMFConv(wav, nbComps=3, nbNMFComps=4, spatial_rank=[1, 2, 1], verbose=0,
                            iter_num=3, wlen=256, hopsize=64)
    out = {'wav': data, 'fs': np.array(8000)}
    np.random.seed(9)
    m.initializeConvParams(initMethod='rand')
    for j, sc in m.spat_comps.items():
        out['init_params_%d' % j] = np.array(sc['params'])
        out['mix_type_%d' % j] = np.array(sc['mix_type'])
    out['logliks'] = np.real(m.estim_param_a_post_model())
    for j, sc in m.spat_comps.items():
        out['final_params_%d' % j] = np.array(sc['params'])
    for k, comp in m.spec_comps.items():
        out['final_FB_%d' % k] = np.array(comp['factor'][0]['FB'])
        out['final_TW_%d' % k] = np.array(comp['factor'][0]['TW'])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, out['logliks'])


def run_pipeline():
    """The full lead/accompaniment pipeline SeparateLeadProcess(...)
    .autoMelSepAndWrite(maxFrames) (SeparateLeadStereoTF.py:263-540,
    1142-1148: chunked mono SIMM -> Viterbi melody -> chunked stereo SIMM with
    per-chunk Wiener masks -> overlap-add of the chunk WAVs) on a short
    seeded stereo signal, 3 chunks.  The Cython tracker is called with its
    5-argument signature, so it is served by the reference's pure-Python
    twin (tracking.py) on the first NF0 states, as _tracking.pyx does."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import shutil
    import numpy as np
    import scipy.io.wavfile as wf
    from pyfasst.SeparateLeadStereo import SeparateLeadStereoTF as SL
    from pyfasst.SeparateLeadStereo.tracking import tracking as TR

    def tracker(S_, N_, logD, prior, logT, verbose=False):
        return TR.viterbiTrackingArray(logD[:S_, :N_], prior[:S_], logT[:S_, :S_])
    SL.viterbiTrackingArray = tracker
    work = "/tmp/golden_pipeline"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    os.chdir(work)
    rs = np.random.RandomState(61)
    fs, n = 8000, 9000
    t = np.arange(n) / float(fs)
    f0 = 220 * 2 ** (np.floor(t * 2) / 12.)                 # a stepped melody
    lead = sum(np.sin(2 * np.pi * h * np.cumsum(f0) / fs) / h for h in range(1, 8))
    acc = np.convolve(rs.randn(n), np.ones(9) / 9., mode='same') * 0.7
    x = np.stack([0.7 * lead + 0.4 * acc, 0.5 * lead + 0.6 * np.roll(acc, 5)], axis=1)
    x = (x / np.abs(x).max() * 12000).astype(np.int16)
    wav = os.path.join(work, "mix.wav")
    wf.write(wav, fs, x)
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out')
    proc.autoMelSepAndWrite(maxFrames=60)
    out = {'wav': x, 'fs': np.array(fs), 'WF0': proc.SIMMParams['WF0'],
           'WGAMMA': proc.SIMMParams['WGAMMA'], 'F0Table': proc.SIMMParams['F0Table'],
           'indexBestPath': np.array(proc.indexBestPath), 'freqMelody': np.array(proc.freqMelody),
           'HF00': proc.SIMMParams['HF00'], 'totFrames': np.array(proc.totFrames),
           'lead': wf.read(proc.files['voc_output_file'])[1],
           'acc': wf.read(proc.files['mus_output_file'])[1],
           'pitches': np.loadtxt(proc.files['pitch_output_file'])}
    np.savez_compressed(os.path.join(HERE, "pipeline.npz"), **out)
    print("pipeline", {k: np.shape(v) for k, v in out.items()})


def pipeline_signal(fs, n, seed=61):
    """The stepped-melody stereo test signal of the pipeline fixtures."""
    import numpy as np
    rs = np.random.RandomState(seed)
    t = np.arange(n) / float(fs)
    f0 = 220 * 2 ** (np.floor(t * 2) / 12.)                 # a stepped melody
    lead = sum(np.sin(2 * np.pi * h * np.cumsum(f0) / fs) / h for h in range(1, 8))
    acc = np.convolve(rs.randn(n), np.ones(9) / 9., mode='same') * 0.7
    x = np.stack([0.7 * lead + 0.4 * acc, 0.5 * lead + 0.6 * np.roll(acc, 5)], axis=1)
    return (x / np.abs(x).max() * 12000).astype(np.int16)


def run_pipeline_nnls():
    """The STFT lead pipeline of run_pipeline with initHF00='nnls'
    (SeparateLeadStereoTF.py:982-993: per-frame scipy.optimize.nnls of each
    chunk's SX on WF0, + eps, as the mono SIMM's HF00).  Records each chunk's
    SX and the HF00 handed to SIMM, and the pipeline's outputs."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import shutil
    import numpy as np
    import scipy
    import scipy.io.wavfile as wf
    from pyfasst.SeparateLeadStereo import SeparateLeadStereoTF as SL
    from pyfasst.SeparateLeadStereo.tracking import tracking as TR

    def tracker(S_, N_, logD, prior, logT, verbose=False):
        return TR.viterbiTrackingArray(logD[:S_, :N_], prior[:S_], logT[:S_, :S_])
    SL.viterbiTrackingArray = tracker
    caps = []
    orig = SL.SIMM.SIMM

    def rec(SX, *a, **kw):
        if kw.get('HF00') is not None:
            caps.append((np.array(SX), np.array(kw['HF00'])))
        return orig(SX, *a, **kw)
    SL.SIMM.SIMM = rec
    work = "/tmp/golden_pipeline_nnls"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    os.chdir(work)
    fs = 8000
    g = np.load(os.path.join(HERE, "pipeline.npz"))
    x = g['wav']
    wav = os.path.join(work, "mix.wav")
    wf.write(wav, fs, x)
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out', initHF00='nnls')
    proc.autoMelSepAndWrite(maxFrames=60)
    SL.SIMM.SIMM = orig
    out = {'wav': x, 'fs': np.array(fs), 'WF0': proc.SIMMParams['WF0'],
           'indexBestPath': np.array(proc.indexBestPath),
           'HF00': proc.SIMMParams['HF00'],
           'lead': wf.read(proc.files['voc_output_file'])[1],
           'acc': wf.read(proc.files['mus_output_file'])[1],
           'scipy_version': np.array(scipy.__version__), 'nchunks': np.array(len(caps))}
    for i, (SX, H) in enumerate(caps):
        out['SX_%d' % i] = SX
        out['nnls_HF00_%d' % i] = H
    np.savez_compressed(os.path.join(HERE, "pipeline_nnls.npz"), **out)
    print("pipeline_nnls", {k: np.shape(v) for k, v in out.items()})


def run_pipeline_mqt():
    """The lead/accompaniment pipeline on the MinQT, tfrepresentation='mqt'
    (the reference's own MinQTSLStest, pyfasst_tests/.../
    test_SeparateLeadStereoTF.py:40-47): WF0 on the MinQT
    (SeparateLeadStereoTF.py:656-700), chunked mono SIMM with the
    startincqt realignment (:1023-1032), Viterbi, chunked stereo SIMM, the
    MinQT inverse of each masked chunk (:1802-1861) and the sine-bell^2
    overlap-add (:1481-1491); 5 s at 8 kHz, 3 chunks of 140, 140 and 35
    frames (maxFrames=100 would leave the last 78 frames unestimated: the
    reference's chunk count 315 // 79 = 3, :1880-1897, whose all-zero HF0
    makes the Viterbi tail a tie)."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import shutil
    import numpy as np
    import scipy.io.wavfile as wf
    from pyfasst.SeparateLeadStereo import SeparateLeadStereoTF as SL
    from pyfasst.SeparateLeadStereo.tracking import tracking as TR

    def tracker(S_, N_, logD, prior, logT, verbose=False):
        return TR.viterbiTrackingArray(logD[:S_, :N_], prior[:S_], logT[:S_, :S_])
    SL.viterbiTrackingArray = tracker
    work = "/tmp/golden_pipeline_mqt"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    os.chdir(work)
    fs = 8000
    x = pipeline_signal(fs, 40000)
    wav = os.path.join(work, "mix.wav")
    wf.write(wav, fs, x)
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out', tfrepresentation='mqt',
                                  cqtbins=12, cqtfmin=50)
    proc.autoMelSepAndWrite(maxFrames=140)
    out = {'wav': x, 'fs': np.array(fs), 'WF0': proc.SIMMParams['WF0'],
           'WGAMMA': proc.SIMMParams['WGAMMA'], 'F0Table': proc.SIMMParams['F0Table'],
           'indexBestPath': np.array(proc.indexBestPath), 'freqMelody': np.array(proc.freqMelody),
           'HF00': proc.SIMMParams['HF00'], 'totFrames': np.array(proc.totFrames),
           'hopsize': np.array(proc.stftParams['hopsize']),
           'window': np.array(proc.stftParams['windowSizeInSamples']),
           'lead': wf.read(proc.files['voc_output_file'])[1],
           'acc': wf.read(proc.files['mus_output_file'])[1],
           'pitches': np.loadtxt(proc.files['pitch_output_file'])}
    np.savez_compressed(os.path.join(HERE, "pipeline_mqt.npz"), **out)
    print("pipeline_mqt", {k: np.shape(v) for k, v in out.items()})


def run_pipeline_suimm():
    """The unvoiced-lead (SUIMM) stages of SeparateLeadProcess on the signal
    and settings of run_pipeline: after autoMelSepAndWrite(maxFrames=60),
    estimStereoSUIMMParamsWriteSeps(maxFrames=60) (SeparateLeadStereoTF.py:
    1585-1675: per chunk Stereo_SIMM on WUF0 = [WF0 | 1] with HGAMMA fixed,
    the '_VUIMM' masks, the overlap-add); then, into a second output
    directory (setOutputFileNames, :540-585), the un-chunked
    estimStereoSIMMParams (:1677-1713) + writeSeparatedSignals and
    estimStereoSUIMMParams (:1715-1760) + writeSeparatedSignalsWithUnvoice."""
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import shutil
    import numpy as np
    import scipy.io.wavfile as wf
    from pyfasst.SeparateLeadStereo import SeparateLeadStereoTF as SL
    from pyfasst.SeparateLeadStereo.tracking import tracking as TR

    def tracker(S_, N_, logD, prior, logT, verbose=False):
        return TR.viterbiTrackingArray(logD[:S_, :N_], prior[:S_], logT[:S_, :S_])
    SL.viterbiTrackingArray = tracker
    work = "/tmp/golden_pipeline_suimm"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    os.chdir(work)
    fs = 8000
    x = pipeline_signal(fs, 9000)
    wav = os.path.join(work, "mix.wav")
    wf.write(wav, fs, x)
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out')
    proc.autoMelSepAndWrite(maxFrames=60)
    hg0 = np.array(proc.SIMMParams['HGAMMA'])
    proc.estimStereoSUIMMParamsWriteSeps(maxFrames=60)
    out = {'wav': x, 'fs': np.array(fs), 'HGAMMA_in': hg0,
           'HGAMMA_suimm': np.array(proc.SIMMParams['HGAMMA']),
           'WM_suimm': np.array(proc.SIMMParams['WM']),
           'lead': wf.read(proc.files['voc_output_file'])[1],
           'lead_vuimm': wf.read(proc.files['voc_output_file'][:-4] + '_VUIMM.wav')[1],
           'acc_vuimm': wf.read(proc.files['mus_output_file'][:-4] + '_VUIMM.wav')[1]}
    proc.setOutputFileNames('out2')
    proc.estimStereoSIMMParams()
    proc.writeSeparatedSignals()
    P = proc.SIMMParams
    out.update({'whole_HF0': np.array(P['HF0']), 'whole_HGAMMA': np.array(P['HGAMMA']),
                'whole_alphaR': np.array(P['alphaR']), 'whole_alphaL': np.array(P['alphaL']),
                'whole_lead': wf.read(proc.files['voc_output_file'])[1],
                'whole_acc': wf.read(proc.files['mus_output_file'])[1]})
    proc.estimStereoSUIMMParams()
    proc.writeSeparatedSignalsWithUnvoice()
    out.update({'whole_HUF0': np.array(P['HUF0']), 'whole_HGAMMA_u': np.array(P['HGAMMA']),
                'whole_alphaR_u': np.array(P['alphaR']), 'whole_betaR_u': np.array(P['betaR']),
                'whole_lead_vuimm': wf.read(proc.files['voc_output_file'][:-4] + '_VUIMM.wav')[1],
                'whole_acc_vuimm': wf.read(proc.files['mus_output_file'][:-4] + '_VUIMM.wav')[1]})
    np.savez_compressed(os.path.join(HERE, "pipeline_suimm.npz"), **out)
    print("pipeline_suimm", {k: np.shape(v) for k, v in out.items()})


def run_inv_herm():
    """Known-answer data of pyfasst_tests/pyfasst/tools/test_signalTools.py:27-64."""
    import numpy as np
    sys.path.insert(0, SCRATCH)
    src = open("/root/reference/pyfasst_tests/pyfasst/tools/test_signalTools.py").read()
    ns = {'np': np}
    start = src.index("sigma_x_diag = np.array(")
    stop = src.index("def test_inv_herm_mat_2d")
    exec(compile(src[start:stop], "fixture", "exec"), ns)
    from pyfasst.tools import signalTools as st
    d, o, det = st.inv_herm_mat_2d(ns['sigma_x_diag'], ns['sigma_x_off'])
    np.savez_compressed(os.path.join(HERE, "inv_herm.npz"),
                        sigma_x_diag=ns['sigma_x_diag'], sigma_x_off=ns['sigma_x_off'],
                        inv_diag_ref=ns['inv_sigma_x_diag_ref'], inv_off_ref=ns['inv_sigma_x_off_ref'],
                        inv_diag_run=d, inv_off_run=o, det_run=det)
    print("inv_herm")


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    if len(sys.argv) > 2 and sys.argv[1] == "--case":
        name = sys.argv[2]
        {"stft": run_stft, "nmf": run_nmf, "inv_herm": run_inv_herm, "simm": run_simm,
         "lead": run_lead, "cqt": run_cqt, "viterbi": run_viterbi, "wf0": run_wf0, "nmfinit_same": lambda: run_nmfinit(True),
         "nmfinit_indiv": lambda: run_nmfinit(False), "convinit_rand": run_convinit,
         "pipeline": run_pipeline,
         "wf0_cqt": run_wf0_cqt, "pipeline_mqt": run_pipeline_mqt,
         "pipeline_nnls": run_pipeline_nnls, "pipeline_suimm": run_pipeline_suimm}.get(
            name, lambda: run_case(name))()
        sys.exit(0)
    import make_scratch_ref
    if not os.path.isdir(os.path.join(SCRATCH, "pyfasst")):
        make_scratch_ref.build(SCRATCH)
    names = sys.argv[1:] or (["inv_herm", "stft", "nmf", "simm", "lead", "cqt", "viterbi", "wf0", "nmfinit_same",
                              "nmfinit_indiv", "convinit_rand", "pipeline", "wf0_cqt", "pipeline_mqt",
                              "pipeline_nnls", "pipeline_suimm"] + list(CASES))
    for name in names:
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--case", name])
