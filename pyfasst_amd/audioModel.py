"""FASST model classes with the reference's surface, running on MI355X.

Drop-in for pyfasst.audioModel (audioModel.py:66-2508): same class names,
constructor keyword arguments, `spat_comps` / `spec_comps` / `noise` dicts
and public methods.  Between calls the NumPy dicts are the source of truth;
`estim_param_a_post_model()` uploads them once, runs every GEM iteration on
the GPU (pyfasst_amd/csrc/fasst_em.hip) and downloads the result;
`separate_spat_comps()` computes the Wiener images and iSTFTs on the GPU.

There is no CPU fallback: structures outside the HIP path raise
NotImplementedError, a missing library raises ImportError.

Deliberate deviation: the reference stores the shared
mutable default `ann_PSD_lim=[None, None]` by reference, so a second model
in the same process inherits the first model's annealing limits
(audioModel.py:166,242,320-323); here each model copies the list.
"""
import os
import warnings

import numpy as np

from . import audioObject as ao
from .engine import Engine
from .tftransforms import minqt as minqt_mod
from .tftransforms import stft as stft_mod

eps = 1e-10              # audioModel.py:61
log_prior_small_cst = 1e-70
soundCelerity = 340.


class FASST(object):
    """FASST base class (audioModel.py:66-248)."""
    implemented_transf = ['stft', 'mqt', 'minqt', 'cqt']
    implemented_annealing = ['ann', 'no_ann']

    def __init__(self, audio, transf='stft', wlen=2048, hopsize=512, iter_num=50,
                 sim_ann_opt='ann', ann_PSD_lim=[None, None], verbose=0, nmfUpdateCoeff=1.,
                 tffmin=25, tffmax=18000, tfWinFunc=None, tfbpo=48, lambdaCorr=0.,
                 device=None):
        self.verbose = verbose
        self.nmfUpdateCoeff = nmfUpdateCoeff
        if isinstance(audio, ao.AudioObject):
            self.audioObject = audio
        elif isinstance(audio, str):
            self.audioObject = ao.AudioObject(filename=audio)
        else:
            raise AttributeError("The provided audio parameter is" + "not a supported format.")
        self.device = device
        self.sig_repr_params = {}
        self.sig_repr_params['transf'] = transf.lower()
        self.sig_repr_params['wlen'] = ao.nextpow2(wlen)
        self.sig_repr_params['fsize'] = ao.nextpow2(wlen)
        self.sig_repr_params['hopsize'] = hopsize
        self.sig_repr_params['tffmin'] = tffmin
        self.sig_repr_params['tffmax'] = tffmax
        self.sig_repr_params['tfbpo'] = tfbpo
        self.sig_repr_params['tfWinFunc'] = tfWinFunc
        self.sig_repr_params['hopfactor'] = 1. * hopsize / self.sig_repr_params['wlen']
        if self.sig_repr_params['transf'] not in self.implemented_transf:
            raise NotImplementedError(self.sig_repr_params['transf'] + " not yet implemented.")
        # the transform object (audioModel.py:205-214): STFT, or the rasterised
        # MinQT / CQT (perfRast=1) on the GPU
        tf_cls = {'stft': stft_mod.STFT, 'mqt': minqt_mod.MinQTransfo,
                  'minqt': minqt_mod.MinQTransfo, 'cqt': minqt_mod.CQTransfo}[
                      self.sig_repr_params['transf']]
        self.tft = tf_cls(fmin=tffmin, fmax=tffmax, bins=tfbpo, fs=self._samplerate_or_default(),
                          perfRast=1, linFTLen=self.sig_repr_params['fsize'],
                          atomHopFactor=self.sig_repr_params['hopfactor'], device=device)
        self.demixParams = {
            'tffmin': tffmin, 'tffmax': tffmax, 'tfbpo': tfbpo,
            'tfrepresentation': transf.lower(), 'wlen': self.sig_repr_params['wlen'],
            'hopsize': self.sig_repr_params['wlen'] // 2, 'neighbors': 20, 'winFunc': tfWinFunc}
        self.noise = {}
        self.noise['PSD'] = np.zeros(self.sig_repr_params['fsize'] // 2 + 1)
        self.noise['sim_ann_opt'] = sim_ann_opt
        self.noise['ann_PSD_lim'] = list(ann_PSD_lim)
        self.spat_comps = {}
        self.spec_comps = {}
        self.iter_num = iter_num
        self.lambdaCorr = lambdaCorr
        self._engine = None
        self._Cx = None

    def _samplerate_or_default(self):
        try:
            return self.audioObject.samplerate
        except Exception:
            return 44100

    # ---------------------------------------------------------------- Cx
    @property
    def Cx(self):
        """Packed covariance [3, F, T] (audioModel.py:293-302), fetched lazily."""
        if self._Cx is None and self._engine is not None:
            self._Cx = self._engine.get_cx()
        return self._Cx

    @Cx.setter
    def Cx(self, value):
        value = np.asarray(value, dtype=np.complex128)
        self._Cx = value
        if value.ndim == 3:
            self.nbFreqsSigRepr, self.nbFramesSigRepr = value.shape[1:]
            if (self._engine is None or self._engine.F != value.shape[1]
                    or self._engine.T != value.shape[2]):
                self._engine = Engine(value.shape[1], value.shape[2], self.device)
            self._engine.set_cx(value)

    def comp_transf_Cx(self):
        """Signal representation on the GPU (audioModel.py:250-328)."""
        if self.sig_repr_params['transf'] not in self.implemented_transf:
            raise ValueError(self.sig_repr_params['transf'] + " not implemented - yet?")
        aud = self.audioObject
        if isinstance(aud, ao.SpectralAudio):
            F, T = aud.nbFreqs, aud.nbFrames
            self._engine = Engine(F, T, self.device)
            self.nbFreqsSigRepr, self.nbFramesSigRepr = F, T
            if aud.X is not None:
                self._engine.set_stft(aud.X)   # Cx packed on the device
                self._Cx = None
            else:
                self.Cx = aud.Cx
        else:
            if not hasattr(aud, '_data'):
                aud._read()
            nc = aud.channels
            if nc != 2:
                raise NotImplementedError("the HIP path handles stereo signals (got %d)" % nc)
            data = np.asarray(aud.data, dtype=np.float64)
            L = data.shape[0]
            if self.sig_repr_params['transf'] != 'stft':
                # MinQT / CQT of each channel on the GPU (audioModel.py:266-280), then
                # the channel transforms become the engine's resident observation
                X = []
                for n in range(nc):
                    self.tft.computeTransform(data[:, n])
                    X.append(self.tft.transfo)
                F, T = X[0].shape
                self._engine = Engine(F, T, self.device)
                self._engine.set_stft(np.array(X))
                self.nbFreqsSigRepr, self.nbFramesSigRepr = F, T
                self._Cx = None
                self._finish_noise_limits()
                return
            hop = self.tft.fthop
            T = int(np.ceil(L / np.double(hop))) + 2
            F = self.tft.freqbins
            self._engine = Engine(F, T, self.device)
            self._engine.set_audio(data, self.tft.window, self.tft.ftlen, hop)
            self.tft.datalen_init = L
            self.nbFreqsSigRepr, self.nbFramesSigRepr = F, T
            self._Cx = None
        self._finish_noise_limits()

    def _finish_noise_limits(self):
        """Annealing limits from the mean diagonal PSD (audioModel.py:304-325)."""
        lim = self.noise['ann_PSD_lim']
        if lim[0] is None or lim[1] is None:
            mix_psd = self._engine.mix_psd()
            if lim[0] is None:
                lim[0] = np.real(mix_psd) / 100.
            if lim[1] is None:
                lim[1] = np.real(mix_psd) / 10000.
        if self.noise['sim_ann_opt'] in ('ann'):   # substring test, as the reference (:324)
            self.noise['PSD'] = lim[0]

    # ---------------------------------------------------------------- structure
    def _structure(self):
        """Check the model is on the HIP path; return (order, ranks, Ks, conv),
        order[j] = the keys of spatial component j's spectral components in
        the reference's key order (update_spectral_components iterates
        spec_comps.items(), audioModel.py:1479).

        HIP path: stereo; single-factor NMF spectral components (TW_constr
        'NMF'; FB, FW, TW each free or fixed; time blobs TB, free or fixed, or
        none), one or several per spatial component (comp_spat_comp_power sums
        them, :469-498); 'inst' and 'conv' spatial components in any
        combination the reference's mixing update can run (free 'conv' ones
        only when every component is free 'conv'); any lambdaCorr >= 0 (the
        inter-source correlation penalty, :1484-1719).
        """
        if self.audioObject.channels != 2:
            raise AttributeError("Nb channels " + str(self.audioObject.channels) +
                                 " not implemented yet")
        J = len(self.spat_comps)
        if sorted(self.spat_comps.keys()) != list(range(J)):
            raise NotImplementedError("spatial components must be numbered 0..J-1")
        owner = {}
        for k in sorted(self.spec_comps.keys()):
            comp = self.spec_comps[k]
            owner.setdefault(comp['spat_comp_ind'], []).append(k)
            facs = comp['factor']
            if list(facs.keys()) != [0]:
                raise NotImplementedError("multi-factor spectral components are outside the HIP path")
            fac = facs[0]
            if len(fac['TB']):
                TB = np.asarray(fac['TB'])
                if TB.ndim != 2 or TB.shape[1] != self.nbFramesSigRepr or \
                        np.shape(fac['TW']) != (fac['FB'].shape[1], TB.shape[0]):
                    raise ValueError("time blobs of spectral component %d: TW %s, TB %s"
                                     % (k, np.shape(fac['TW']), TB.shape))
            if fac.get('TW_constr', 'NMF') != 'NMF':
                raise NotImplementedError("TW_constr=%s is outside the HIP path" % fac['TW_constr'])
        if sorted(owner.keys()) != list(range(J)):
            raise NotImplementedError("every spatial component needs a spectral component")
        conv = [self.spat_comps[j]['mix_type'] == 'conv' for j in range(J)]
        free = [self.spat_comps[j]['frdm_prior'] == 'free' for j in range(J)]
        # update_mix_matrix (:843-863) solves the free 'conv' components with
        # the FULL hat_Rss[f] against the right-hand side of those components
        # only, which the reference can evaluate only when no other (fixed or
        # 'inst') component exists: any other component makes np.linalg.solve
        # raise at the first M-step.  Raise the same exception type up front.
        if any(c and f for c, f in zip(conv, free)) and not all(c and f for c, f in zip(conv, free)):
            raise ValueError("update_mix_matrix: free 'conv' spatial components next to fixed or "
                             "'inst' ones (audioModel.py:856-857 solves hat_Rss[f].T of all %d "
                             "components against the free components' right-hand side only)"
                             % J)
        ranks, Ks = [], []
        for j in range(J):
            p = self.spat_comps[j]['params']
            ranks.append(p.shape[0] if conv[j] else p.shape[1])
            Ks.append(int(sum(self.spec_comps[k]['factor'][0]['FB'].shape[1] for k in owner[j])))
        return [owner[j] for j in range(J)], ranks, Ks, (all(conv) if len(set(conv)) == 1 else conv)

    def _upload(self):
        order, ranks, Ks, conv = self._structure()
        eng = self._engine
        eng.configure(ranks, Ks, conv)
        for j in range(len(order)):
            sc = self.spat_comps[j]
            eng.set_spatial(j, sc['params'], sc['frdm_prior'] == 'free')
            facs = [self.spec_comps[k]['factor'][0] for k in order[j]]
            fb_free = [f.get('FB_frdm_prior', 'free') == 'free' for f in facs]
            fw_free = [f.get('FW_frdm_prior', 'fixed') == 'free' for f in facs]
            tw_free = [f.get('TW_frdm_prior', 'free') == 'free' for f in facs]
            # a component with time blobs: the device forms H = TW.TB (fasst_set_tb)
            TWs = [np.zeros((f['FB'].shape[1], self.nbFramesSigRepr)) if len(f['TB'])
                   else f['TW'] for f in facs]
            if len(facs) == 1:
                FB, FW, TW = facs[0]['FB'], facs[0]['FW'], TWs[0]
            else:   # the components side by side, FW block diagonal
                FB = np.hstack([f['FB'] for f in facs])
                TW = np.vstack(TWs)
                FW = np.zeros((Ks[j], Ks[j]))
                a = 0
                for f in facs:
                    n = f['FB'].shape[1]
                    FW[a:a + n, a:a + n] = f['FW']
                    a += n
            eng.set_spectral(j, FB, FW, TW, any(fb_free), any(tw_free), any(fw_free))
            eng.set_blocks(j, np.cumsum([0] + [f['FB'].shape[1] for f in facs]), fb_free, fw_free,
                           tw_free)
            for b, f in enumerate(facs):
                if len(f['TB']):
                    eng.set_tb(j, b, f['TW'], f['TB'], f.get('TB_frdm_prior') == 'free')
        if self.lambdaCorr > 0:   # components one at a time in key order (:1479)
            pos = {k: (j, b) for j, keys in enumerate(order) for b, k in enumerate(keys)}
            seq = [pos[k] for k in sorted(self.spec_comps.keys())]
            eng.set_corr(self.lambdaCorr, [j for j, _ in seq], [b for _, b in seq])
        else:
            eng.set_corr(0.0)
        return order, Ks, conv

    def _download(self, order, Ks, conv, updated_spatial=True):
        eng = self._engine
        for j in range(len(order)):
            sc = self.spat_comps[j]
            p = eng.get_spatial(j, sc['params'].shape)
            if not np.iscomplexobj(sc['params']) and not (updated_spatial and
                                                          sc['frdm_prior'] == 'free'):
                p = p.real.copy()
            sc['params'] = p
            FB, FW, TW = eng.get_spectral(j, Ks[j])
            a = 0
            for b, k in enumerate(order[j]):
                fac = self.spec_comps[k]['factor'][0]
                n = fac['FB'].shape[1]
                parts = (('FB', FB[:, a:a + n]), ('FW', FW[a:a + n, a:a + n]),
                         ('TW', TW[a:a + n]))
                if len(fac['TB']):   # the factor TW and TB, not H
                    TWs, TB = eng.get_tb(j, b, n, np.shape(fac['TB'])[0])
                    parts = parts[:2] + (('TW', TWs), ('TB', TB))
                if len(order[j]) > 1:
                    parts = tuple((key, np.ascontiguousarray(val)) for key, val in parts)
                for key, val in parts:
                    if isinstance(fac[key], np.ndarray) and fac[key].shape == val.shape \
                            and fac[key].dtype == val.dtype:
                        fac[key][...] = val
                    else:
                        fac[key] = val
                a += n

    def _restart_tw(self, mask, order):
        """Random TW restart of renormalize_parameters (audioModel.py:2023-2028),
        drawn on the host RNG in spectral-component key order; mask has one bit
        per spectral component, spatial component by spatial component."""
        dead = set()
        bit = 0
        for keys in order:
            for k in keys:
                if mask & (1 << bit):
                    dead.add(k)
                bit += 1
        for k in sorted(self.spec_comps.keys()):
            if k in dead:
                fac = self.spec_comps[k]['factor'][0]
                fac['TW'] = np.random.randn(*fac['TW'].shape) ** 2
                fac['TW'] *= 1e3 * eps
                if self.verbose:
                    print("    renorm: reinitialized TW for spec", k, "factor", 0)
                if len(fac['TB']):   # the rest of the renormalisation (:2029-2033)
                    w = fac['TB'].mean(axis=1)
                    w[w == 0] = 1.
                    fac['TB'] /= np.vstack(w)
                    fac['TW'] *= w

    # ---------------------------------------------------------------- EM
    def _annealed_psd(self, i):
        lim = self.noise['ann_PSD_lim']
        return ((np.sqrt(lim[0]) * (self.iter_num - i) + np.sqrt(lim[1]) * i)
                / self.iter_num) ** 2

    def estim_param_a_post_model(self,):
        """Run iter_num GEM iterations on the GPU (audioModel.py:330-382)."""
        logliks = np.ones(self.iter_num)
        opt = self.noise['sim_ann_opt']
        if opt in ['ann', ]:
            self.noise['PSD'] = self.noise['ann_PSD_lim'][0]
        elif opt == 'no_ann':
            self.noise['PSD'] = self.noise['ann_PSD_lim'][1]
        else:
            warnings.warn("To add noise to the signal, provide the " +
                          "sim_ann_opt from any of 'ann', " + "'no_ann' or 'ann_ns_inj' ")
        rows = []
        for i in range(self.iter_num):
            if opt in ['ann', 'ann_ns_inj']:
                rows.append(self._annealed_psd(i))
            else:
                rows.append(np.asarray(self.noise['PSD'], dtype=np.float64) *
                            np.ones(self.nbFreqsSigRepr))
        if not rows:
            return logliks
        rows = np.array(rows, dtype=np.float64)
        order, Ks, conv = self._upload()
        i0 = 0
        while i0 < self.iter_num:
            ll, done, mask = self._engine.run(rows[i0:], self.nmfUpdateCoeff)
            logliks[i0:i0 + done] = ll
            i0 += done
            if mask:
                self._download(order, Ks, conv)
                self._restart_tw(mask, order)
                order, Ks, conv = self._upload()
        self._download(order, Ks, conv)
        self.noise['PSD'] = rows[-1]
        if self.verbose:
            for i in range(self.iter_num):
                print("Iteration", i + 1, "on", self.iter_num, "    log-likelihood:", logliks[i])
        return logliks

    def GEM_iteration(self,):
        """One GEM iteration with the current noise PSD (audioModel.py:384-428)."""
        order, Ks, conv = self._upload()
        psd = np.asarray(self.noise['PSD'], dtype=np.float64) * np.ones(self.nbFreqsSigRepr)
        ll, done, mask = self._engine.run(psd[None, :], self.nmfUpdateCoeff)
        self._download(order, Ks, conv)
        if mask:
            self._restart_tw(mask, order)
        return ll[0]

    def renormalize_parameters(self):
        """renormalize_parameters on the GPU (audioModel.py:1980-2040)."""
        order, Ks, conv = self._upload()
        mask = self._engine.renormalize()
        self._download(order, Ks, conv, updated_spatial=False)
        if mask:
            self._restart_tw(mask, order)

    # ---------------------------------------------------------------- GEM steps
    # The methods GEM_iteration is made of (audioModel.py:384-428), each a
    # device call on the reference's own arrays (fasst_steps.hip).  GEM_iteration
    # itself runs the fused iteration (fasst_run) and never materialises them.
    def _psd_row(self):
        return np.asarray(self.noise['PSD'], dtype=np.float64) * np.ones(self.nbFreqsSigRepr)

    def retrieve_subsrc_params(self,):
        """(spat_comp_powers [R, F, T], mix_matrix [R, 2, F], rank_part_ind)
        (audioModel.py:514-578); the powers come from the device."""
        order, Ks, conv = self._upload()
        J = len(order)
        rank_part_ind, total = {}, 0
        for j in range(J):
            sc = self.spat_comps[j]
            rank = sc['params'].shape[1] if sc['mix_type'] == 'inst' else sc['params'].shape[0]
            rank_part_ind[j] = total + np.arange(rank)
            total += rank
        V = self._engine.source_powers(0, J)
        spat_comp_powers = np.empty((total, self.nbFreqsSigRepr, self.nbFramesSigRepr))
        mix_matrix = np.zeros((total, self.audioObject.channels, self.nbFreqsSigRepr),
                              dtype=complex)
        for j in range(J):
            sc = self.spat_comps[j]
            spat_comp_powers[rank_part_ind[j]] = V[j]
            if sc['mix_type'] == 'inst':
                mix_matrix[rank_part_ind[j]] = np.asarray(sc['params']).T[:, :, None]
            else:
                mix_matrix[rank_part_ind[j]] = sc['params']
        return spat_comp_powers, mix_matrix, rank_part_ind

    def compute_suff_stat(self, spat_comp_powers, mix_matrix):
        """(hat_Rxx, hat_Rxs, hat_Rss, hat_Ws, loglik) on the device
        (audioModel.py:580-764), with the current noise PSD."""
        if self.audioObject.channels != 2:
            raise ValueError("Nb channels not supported:" + str(self.audioObject.channels))
        if self._engine is None:
            raise AttributeError("no observation: call comp_transf_Cx() first")
        return self._engine.suff_stat(spat_comp_powers, mix_matrix, self._psd_row())

    def update_mix_matrix(self, hat_Rxs, hat_Rss, mix_matrix, rank_part_ind):
        """Mixing update (audioModel.py:766-889): mix_matrix updated in place,
        the free spatial components' params replaced."""
        kind = np.zeros(mix_matrix.shape[0], dtype=np.int32)
        for j, sc in self.spat_comps.items():
            if sc['frdm_prior'] == 'free':
                kind[rank_part_ind[j]] = 1 if sc['mix_type'] == 'inst' else 2
        m = np.ascontiguousarray(mix_matrix, dtype=np.complex128)
        self._engine.mix_solve(hat_Rss, hat_Rxs, m, kind)
        if m is not mix_matrix:
            mix_matrix[...] = m
        for j, sc in self.spat_comps.items():
            if sc['frdm_prior'] == 'free':
                if sc['mix_type'] == 'inst':
                    sc['params'] = np.mean(mix_matrix[rank_part_ind[j]], axis=2).T
                else:
                    sc['params'] = mix_matrix[rank_part_ind[j]]

    def update_spectral_components(self, hat_W):
        """FB / FW / TW (TB) updates from hat_W [J, F, T] on the device
        (audioModel.py:1469-1978); no renormalisation."""
        order, Ks, conv = self._upload()
        self._engine.spectral_update(hat_W, self.nmfUpdateCoeff)
        self._download(order, Ks, conv, updated_spatial=False)

    def _colmask(self, spat_ind, spec_comp_ind, order):
        keys = spec_comp_ind if len(spec_comp_ind) else order[spat_ind]
        mask, a = 0, 0
        for k in order[spat_ind]:
            n = self.spec_comps[k]['factor'][0]['FB'].shape[1]
            if k in keys:
                mask |= ((1 << n) - 1) << a
            a += n
        return mask

    def compute_sigma_comp_2d(self, spat_ind, spec_comp_ind):
        """(sigma_comp_diag [2, F, T], sigma_comp_off [F, T]) of one spatial
        component's spectral components (audioModel.py:1327-1372)."""
        order, Ks, conv = self._upload()
        return self._engine.sigma_comp(spat_ind, self._colmask(spat_ind, spec_comp_ind, order))

    def compute_inv_sigma_mix_2d(self, sigma_comps_diag, sigma_comps_off):
        """Inverse of sum_n Sigma_n + PSD I (audioModel.py:1374-1394)."""
        return self._engine.inv_sigma_mix(sigma_comps_diag, sigma_comps_off, self._psd_row())

    def compute_Wiener_gain_2d(self, sigma_comp_diag, sigma_comp_off, inv_sigma_mix_diag,
                               inv_sigma_mix_off, timeInvariant=False):
        """WG [2, 2, F(, T)] (audioModel.py:1396-1467)."""
        from .engine import wiener_gain
        dev = self._engine.device if self._engine is not None else \
            (0 if self.device is None else self.device)
        return wiener_gain(dev, sigma_comp_diag, sigma_comp_off, inv_sigma_mix_diag,
                           inv_sigma_mix_off)

    # ---------------------------------------------------------------- NMF init
    def _mono_power(self):
        """Channel-averaged power sum_c Re Cx[c, c] / nc (audioModel.py:2150-2158)."""
        nc = self.audioObject.channels
        Cx = np.copy(np.real(self.Cx[0]))
        Cx += np.real(self.Cx[2])
        Cx /= np.double(nc)
        return Cx

    def initialize_all_spec_comps_with_NMF(self, sameInitAll=False, **kwargs):
        """IS-NMF of the mono power initialises FB / TW (audioModel.py:2091-2116);
        the NMF iterations and the renormalisation run on the GPU."""
        if sameInitAll:
            return self.initialize_all_spec_comps_with_NMF_same(**kwargs)
        return self.initialize_all_spec_comps_with_NMF_indiv(**kwargs)

    def initialize_all_spec_comps_with_NMF_indiv(self, niter=10, updateFreqBasis=True,
                                                 updateTimeWeight=True, **kwargs):
        """One NMF over all components, started from the current FB / TW
        (audioModel.py:2118-2177)."""
        from .tools.nmf import NMF_decomp_init
        nbSpecComps = [sc['factor'][0]['FB'].shape[1] for sc in self.spec_comps.values()]
        total = int(np.sum(nbSpecComps))
        FBinit = np.zeros([self.nbFreqsSigRepr, total])
        TWinit = np.zeros([total, self.nbFramesSigRepr])
        for k, sc in self.spec_comps.items():
            a = int(np.sum(nbSpecComps[:k]))
            FBinit[:, a:a + nbSpecComps[k]] = sc['factor'][0]['FB']
            TWinit[a:a + nbSpecComps[k]] = sc['factor'][0]['TW']
        W, H = NMF_decomp_init(SX=self._mono_power(), nbComps=total, niter=niter,
                               verbose=self.verbose, Winit=FBinit, Hinit=TWinit,
                               updateW=updateFreqBasis, updateH=updateTimeWeight,
                               device=self.device)
        for k, sc in self.spec_comps.items():
            a = int(np.sum(nbSpecComps[:k]))
            if updateFreqBasis:
                sc['factor'][0]['FB'] = np.maximum(W[:, a:a + nbSpecComps[k]], eps)
            if updateTimeWeight:
                sc['factor'][0]['TW'] = np.maximum(H[a:a + nbSpecComps[k]], eps)
        self.renormalize_parameters()

    def initialize_all_spec_comps_with_NMF_same(self, niter=10, **kwargs):
        """One NMF, the same W / H (most energetic first) for every component
        (audioModel.py:2179-2222)."""
        from .tools.nmf import NMF_decomposition
        if not np.all([len(sc['factor']) == 1 for sc in self.spec_comps.values()]):
            raise NotImplementedError("NMF init not implemented for multi factor models.")
        nbSpecComps = [sc['factor'][0]['FB'].shape[1] for sc in self.spec_comps.values()]
        W, H = NMF_decomposition(SX=self._mono_power(), verbose=self.verbose,
                                 nbComps=int(np.max(nbSpecComps)), niter=niter,
                                 device=self.device)
        indexSort = np.argsort(H.sum(axis=1))[::-1]
        W = W[:, indexSort]
        H = H[indexSort]
        for sc in self.spec_comps.values():
            n = sc['factor'][0]['FB'].shape[1]
            sc['factor'][0]['FB'][:] = W[:, :n]
            sc['factor'][0]['TW'][:] = H[:n]
        self.renormalize_parameters()

    # ---------------------------------------------------------------- separation
    def separate_spat_comps(self, dir_results=None, suffix=None):
        """One source per spatial component (audioModel.py:1063-1086)."""
        spec_comp_ind = {}
        for spat_ind in range(len(self.spat_comps)):
            spec_comp_ind[spat_ind] = []
        for spec_ind, spec_comp in self.spec_comps.items():
            spec_comp_ind[spec_comp['spat_comp_ind']].append(spec_ind)
        self.separate_comps(dir_results=dir_results, spec_comp_ind=spec_comp_ind, suffix=suffix)

    def separated_images(self, spec_comp_ind=None):
        """STFT-domain Wiener images S[n, c] = sum_c2 WG_n[c, c2] X[c2], as the
        reference computes before its iSTFT (audioModel.py:1136-1214)."""
        src_spat, psd = self._separation_plan(spec_comp_ind)
        S = self._engine.wiener_images(psd)
        return S[src_spat]

    def separated_waveforms(self, spec_comp_ind=None):
        """The per-source, per-channel iSTFT of separated_images() without the
        images leaving the GPU (STFT transform only): [n, channel, sample],
        trimmed to the input length as tft.invertTransform() does
        (audioModel.py:1187-1217, tftransforms/stft.py:71-131)."""
        t = self.tft
        if getattr(t, 'transformname', None) != 'stft':
            raise NotImplementedError("device-resident separation needs the STFT transform "
                                      "(use separated_images() + tft.invertTransform())")
        src_spat, psd = self._separation_plan(spec_comp_ind)
        Y = self._engine.separate_waveforms(psd, t.synthWindow, t.window, t.ftlen, t.fthop)
        return Y[src_spat][:, :, :t.datalen_init]

    def _separation_plan(self, spec_comp_ind):
        """Set the engine's separation sources; return (output order, last
        annealed PSD).  Source n holds the spectral components spec_comp_ind[n]
        (default: one source per spectral component, audioModel.py:1130-1133):
        Sigma_n sums, per spatial component, R_j times the power of those of
        its components (compute_sigma_comp_2d, :1327-1372) and Sigma_x sums
        the sources (compute_inv_sigma_mix_2d, :1374-1394).  Sources that are
        whole spatial components, all of them, take the per-spatial-component
        kernel (outputs reordered); others the source-table kernel."""
        if spec_comp_ind is None:
            spec_comp_ind = {}
            for spec_ind in range(len(self.spec_comps)):
                spec_comp_ind[spec_ind] = [spec_ind, ]
        order, Ks, conv = self._upload()
        col = {}
        for j, keys in enumerate(order):
            a = 0
            for k in keys:
                n = self.spec_comps[k]['factor'][0]['FB'].shape[1]
                col[k] = (j, a, n)
                a += n
        sources = []
        for n in range(len(spec_comp_ind)):
            terms = {}
            for k in spec_comp_ind[n]:
                j, a, w = col[k]
                terms[j] = terms.get(j, 0) | (((1 << w) - 1) << a)
            sources.append(sorted(terms.items()))
        full = [(j, (1 << Ks[j]) - 1) for j in range(len(order))]
        whole = all(len(t) == 1 and t[0] == full[t[0][0]] for t in sources)
        psd = np.asarray(self.noise['PSD'], dtype=np.float64) * np.ones(self.nbFreqsSigRepr)
        if whole and sorted(t[0][0] for t in sources) == list(range(len(order))):
            self._engine.set_sources(None)
            return [t[0][0] for t in sources], psd
        self._engine.set_sources(sources)
        return list(range(len(sources))), psd

    def separate_comps(self, dir_results=None, spec_comp_ind=None, suffix=None):
        """Wiener-filter and write one WAV per source (audioModel.py:1088-1236)."""
        if dir_results is None:
            dir_results = '/'.join(self.audioObject.filename.split('/')[:-1])
        nc = self.audioObject.channels
        if nc != 2:
            raise NotImplementedError()
        if getattr(self.tft, 'transformname', None) == 'stft':
            Y = self.separated_waveforms(spec_comp_ind)   # iSTFT on the device
            S = None
            nbSources = Y.shape[0]
        else:
            S = self.separated_images(spec_comp_ind)
            nbSources = S.shape[0]
        if not hasattr(self, "files"):
            self.files = {}
        self.files['spat_comp'] = []
        fileroot = self.audioObject.filename.split('/')[-1][:-4]
        for n in range(nbSources):
            if S is None:
                ndata = Y[n].T
            else:
                ndata = []
                for chan1 in range(nc):
                    self.tft.transfo = S[n, chan1]
                    ndata.append(self.tft.invertTransform())
                    del self.tft.transfo
                ndata = np.array(ndata).T
            _suffix = ''
            if suffix is not None and n in suffix:
                _suffix = '_' + suffix[n]
            outAudioName = (dir_results + '/' + fileroot + '_' + str(n) + '-' +
                            str(nbSources) + _suffix + '.wav')
            self.files['spat_comp'].append(outAudioName)
            out = ao.AudioObject(filename=outAudioName, mode='w')
            out._data = np.int16(ndata[:self.audioObject.nframes, :] * self.audioObject._maxdata)
            out._maxdata = 1
            out._encoding = 'pcm16'
            out.samplerate = self.audioObject.samplerate
            out._write()

    # ---------------------------------------------------------------- helpers
    def comp_spat_comp_power(self, spat_comp_ind, spec_comp_ind=[], factor_ind=[]):
        """Host-side V = prod_factors (FB.FW).(TW[.TB]) (audioModel.py:430-498);
        a parameter inspection helper, not used by the GPU iteration."""
        V = np.zeros([self.nbFreqsSigRepr, self.nbFramesSigRepr])
        keys = spec_comp_ind if len(spec_comp_ind) else list(self.spec_comps.keys())
        for k in keys:
            if spat_comp_ind != self.spec_comps[k]['spat_comp_ind']:
                continue
            Vc = np.ones([self.nbFreqsSigRepr, self.nbFramesSigRepr])
            facs = factor_ind if len(factor_ind) else list(self.spec_comps[k]['factor'].keys())
            for fi in facs:
                fac = self.spec_comps[k]['factor'][fi]
                H = np.dot(fac['TW'], fac['TB']) if len(fac['TB']) else fac['TW']
                Vc *= np.dot(np.dot(fac['FB'], fac['FW']), H)
            V += Vc
        return V

    def comp_spat_cmps_powers(self, spat_comp_ind, spec_comp_ind=[], factor_ind=[]):
        """Sum of the spectral powers of the spatial components listed in
        spat_comp_ind (audioModel.py:500-512; spec_comp_ind / factor_ind are
        accepted and unused, as there).  Each component's power comes from
        the device (fasst_source_powers on the uploaded parameters) and the
        sum runs on the host in the list's order."""
        self._upload()
        V = 0
        for i in spat_comp_ind:
            V += self._engine.source_powers(int(i), 1)[0]
        return V

    def setComponentParameter(self, newValue, spec_ind, fact_ind=0, partLabel='FB',
                              prior='free', keepDimensions=True):
        """The reference's unfinished helper (audioModel.py:2042-2089): it
        prints its notice, then its first statement reads the misspelt name
        `keepDimenstions` and raises NameError before touching anything.
        Kept as that behaviour so the class surface is the same; set the
        components directly (spec_comps[k]['factor'][f][...]), as its notice
        says."""
        print("NOT IMPLEMENTED YET, PLEASE SET THE COMPONENTS DIRECTLY")
        raise NameError("name 'keepDimenstions' is not defined")

    def initializeConvParams(self, initMethod='demix'):
        """Convolutive spatial parameters (audioModel.py:2224-2294): every
        spatial component becomes 'conv'; 'rand' draws the steering vectors
        A = randn(J, F, nc) + 1j randn(J, F, nc) from the global np.random
        stream (the reference's draw order) and gives every rank of
        component j the parameters A[j].T.  'demix' needs the DEMIX
        estimator (pyfasst.demixTF), which is outside this engine's scope
        (DESIGN.md §7): NotImplementedError.  The method is checked before
        any component changes type (the reference sets every 'mix_type' to
        'conv' first, so a caught error left 'conv' components holding 'inst'
        parameters): a refused call leaves the model as it was."""
        nc = self.audioObject.channels
        for spat_ind, spat_comp in self.spat_comps.items():
            if spat_comp['mix_type'] != 'inst':
                warnings.warn("Spatial component %d " % spat_ind +
                              "already not instantaneous, overwriting...")
        if initMethod == 'demix':
            raise NotImplementedError("initializeConvParams('demix'): the DEMIX estimator "
                                      "(demixTF) is outside the HIP engine's scope; use 'rand'")
        elif 'rand' not in initMethod:
            raise ValueError("Init method not implemented.")
        J = len(self.spat_comps)
        A = (np.random.randn(J, self.nbFreqsSigRepr, nc) +
             1j * np.random.randn(J, self.nbFreqsSigRepr, nc))
        for spat_comp in self.spat_comps.values():
            spat_comp['mix_type'] = 'conv'
        for nspat, (spat_ind, spat_comp) in enumerate(self.spat_comps.items()):
            spat_comp['params'] = np.zeros([self.rank[nspat], nc, self.nbFreqsSigRepr],
                                           dtype=complex)
            for r in range(self.rank[nspat]):
                spat_comp['params'][r] = A[spat_ind].T


class MultiChanNMFInst_FASST(FASST):
    """Multichannel NMF, instantaneous mixing (audioModel.py:2296-2420)."""

    def __init__(self, audio, nbComps=3, nbNMFComps=4, spatial_rank=2, **kwargs):
        super(MultiChanNMFInst_FASST, self).__init__(audio=audio, **kwargs)
        self.comp_transf_Cx()
        self.nbComps = nbComps
        self.nbNMFComps = nbNMFComps
        self.rank = np.atleast_1d(spatial_rank)
        if self.rank.size < self.nbComps:
            self.rank = [self.rank[0], ] * self.nbComps
        self._initialize_structures()

    def _initialize_structures(self):
        """Initial parameters; consumes the global np.random stream in the
        reference's order (audioModel.py:2349-2393)."""
        nc = self.audioObject.channels
        self.spat_comps = {}
        self.spec_comps = {}
        for j in range(self.nbComps):
            self.spat_comps[j] = {}
            self.spat_comps[j]['time_dep'] = 'indep'
            self.spat_comps[j]['mix_type'] = 'inst'
            self.spat_comps[j]['frdm_prior'] = 'free'
            self.spat_comps[j]['params'] = np.random.randn(nc, self.rank[j])
            if nc == 2:
                self.spat_comps[j]['params'] = (
                    np.array([np.sin((j + 1) * np.pi / (2. * (self.nbComps + 1))) +
                              np.random.randn(self.rank[j]) * np.sqrt(0.01),
                              np.cos((j + 1) * np.pi / (2. * (self.nbComps + 1))) +
                              np.random.randn(self.rank[j]) * np.sqrt(0.01)]))
            self.spec_comps[j] = {}
            self.spec_comps[j]['spat_comp_ind'] = j
            self.spec_comps[j]['factor'] = {}
            fac = {}
            fac['FB'] = 0.75 * np.abs(np.random.randn(self.nbFreqsSigRepr, self.nbNMFComps)) + 0.25
            fac['FW'] = np.eye(self.nbNMFComps)
            fac['TW'] = 0.75 * np.abs(np.random.randn(self.nbNMFComps, self.nbFramesSigRepr)) + 0.25
            fac['TB'] = []
            fac['FB_frdm_prior'] = 'free'
            fac['FW_frdm_prior'] = 'fixed'
            fac['TW_frdm_prior'] = 'free'
            fac['TB_frdm_prior'] = []
            fac['TW_constr'] = 'NMF'
            self.spec_comps[j]['factor'][0] = fac
        self.renormalize_parameters()

    def setSpecCompFB(self, compNb, FB, FB_frdm_prior='fixed'):
        """audioModel.py:2395-2420"""
        speccomp = self.spec_comps[compNb]['factor'][0]
        if self.nbFreqsSigRepr != FB.shape[0]:
            raise AttributeError("Size of provided FB is not consistent" + " with inner attributes")
        speccomp['FB'] = np.copy(FB)
        ncomp = FB.shape[1]
        speccomp['FW'] = np.eye(ncomp)
        speccomp['TW'] = 0.75 * np.abs(np.random.randn(ncomp, self.nbFramesSigRepr)) + 0.25
        speccomp['FB_frdm_prior'] = FB_frdm_prior


class MultiChanNMFConv(MultiChanNMFInst_FASST):
    """Convolutive multichannel NMF (audioModel.py:2422-2508)."""

    def __init__(self, audio, nbComps=3, nbNMFComps=4, spatial_rank=2, **kwargs):
        super(MultiChanNMFConv, self).__init__(audio=audio, nbComps=nbComps,
                                               nbNMFComps=nbNMFComps,
                                               spatial_rank=spatial_rank, **kwargs)

    def makeItConvolutive(self):
        """Replicate the instantaneous params over bins (audioModel.py:2488-2508)."""
        nc = self.audioObject.channels
        for nspat, (spat_ind, spat_comp) in enumerate(self.spat_comps.items()):
            if spat_comp['mix_type'] != 'inst':
                warnings.warn("Spatial component %d " % spat_ind +
                              "already not instantaneous, skipping...")
            else:
                spat_comp['mix_type'] = 'conv'
                inst = spat_comp['params']
                p = np.zeros([self.rank[nspat], nc, self.nbFreqsSigRepr], dtype=complex)
                p[:] = inst.T[:, :, None]
                spat_comp['params'] = p
