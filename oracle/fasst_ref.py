"""CPU restatement of pyfasst's FASST EM hot path (NumPy, float64/complex128).

TEST INFRASTRUCTURE ONLY -- the checker, never the product.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module.  The product package `pyfasst_amd` never imports it and has no CPU
fallback.

Every function restates the reference algorithm step by step, keeping the
reference's operation structure (same R x R pair loop, same per-frequency
Python loops) so that its CPU timing is representative of the reference.
Citations are `file:line` in /root/reference/pyfasst.

Parity pinning: this restatement is pinned against golden vectors produced by
running the reference itself (a mechanical py2->py3 scratch translation, see
oracle/make_scratch_ref.py and tests/golden/make_golden.py) and against the
reference's own known-answer test for inv_herm_mat_2d
(pyfasst_tests/pyfasst/tools/test_signalTools.py:27-64).
"""
import numpy as np

EPS = 1e-10  # audioModel.py:61 ; tools/signalTools.py:11 ; tools/nmf.py:22


# ----------------------------------------------------------------------------
# tools/signalTools.py:132-196
def inv_herm_mat_2d(sigma_diag, sigma_off):
    """Explicit 2x2 Hermitian inverse with the determinant guard."""
    det = sigma_diag[0] * sigma_diag[1] - np.abs(sigma_off) ** 2
    det = np.sign(det + EPS) * np.maximum(np.abs(det), EPS)
    inv_off = -sigma_off / det
    inv_diag = np.zeros_like(sigma_diag)
    inv_diag[0] = sigma_diag[1] / det
    inv_diag[1] = sigma_diag[0] / det
    return inv_diag, inv_off, det


# ----------------------------------------------------------------------------
# tftransforms/stft.py:3-69 (stft) and :71-131 (istft)
def stft(x, window, hop, nfft):
    lw = window.size
    n_frames = int(np.ceil(x.size / float(hop))) + 2
    total = (n_frames - 1) * hop + lw
    buf = np.concatenate((np.zeros(lw // 2), x))
    buf = np.concatenate((buf, np.zeros(total - buf.size)))
    n_freq = nfft // 2 + 1
    X = np.zeros([n_freq, n_frames], dtype=complex)
    for n in range(n_frames):
        b = n * hop
        X[:, n] = np.fft.rfft(window * buf[b:b + lw], nfft)
    return X


def istft(X, window, analysis_window, hop, nfft):
    lw = window.size
    n_frames = X.shape[1]
    length = hop * (n_frames - 1) + lw
    norm = np.zeros(length)
    out = np.zeros(length)
    for n in range(n_frames):
        b = n * hop
        frame = np.fft.irfft(X[:, n], nfft)[:lw]
        norm[b:b + lw] = norm[b:b + lw] + window * analysis_window
        out[b:b + lw] = out[b:b + lw] + window * frame
    out = out[lw // 2:]
    norm = norm[lw // 2:]
    norm[norm == 0] = 1.
    return out / norm


def read_scaled(data_int):
    """audioObject.py:112-127: divide by max(1.1*max|x|, 1e-10)."""
    maxdata = np.maximum(1.1 * np.abs(data_int).max(), 1e-10)
    return data_int / maxdata, maxdata


# ----------------------------------------------------------------------------
class RefFASST(object):
    """Model state + EM/GEM iteration, following audioModel.py:66-2040.

    State keeps the reference's layout: `Cx` complex [3,F,T] (packed upper
    triangle), `spat_comps`/`spec_comps` dicts, `noise` dict.
    """

    def __init__(self, iter_num=50, sim_ann_opt='ann', nmfUpdateCoeff=1.,
                 lambdaCorr=0., channels=2):
        self.iter_num = iter_num
        self.nmfUpdateCoeff = nmfUpdateCoeff
        self.lambdaCorr = lambdaCorr
        self.channels = channels
        self.noise = {'sim_ann_opt': sim_ann_opt, 'ann_PSD_lim': [None, None]}
        self.spat_comps = {}
        self.spec_comps = {}

    # audioModel.py:285-325
    def set_transform(self, Xchan):
        nc = len(Xchan)
        self.nbFreqsSigRepr, self.nbFramesSigRepr = Xchan[0].shape
        if nc == 1:
            self.Cx = np.abs(Xchan[0]) ** 2
        else:
            self.Cx = np.zeros([nc * (nc + 1) // 2, self.nbFreqsSigRepr,
                                self.nbFramesSigRepr], dtype=complex)
            for a in range(nc):
                for b in range(a, nc):
                    self.Cx[b - a + int(np.sum(np.arange(nc, nc - a, -1)))] = (
                        Xchan[a] * np.conj(Xchan[b]))
        self.set_annealing_limits()

    def set_annealing_limits(self):
        nc = self.channels
        lim = self.noise['ann_PSD_lim']
        if lim[0] is None or lim[1] is None:
            mix_psd = 0
            if nc == 1:
                mix_psd += np.mean(self.Cx, axis=1)
            else:
                for a in range(nc):
                    mix_psd += np.mean(self.Cx[int(np.sum(np.arange(nc, nc - a, -1)))], axis=1)
            mix_psd /= nc
            if lim[0] is None:
                lim[0] = np.real(mix_psd) / 100.
            if lim[1] is None:
                lim[1] = np.real(mix_psd) / 10000.
        self.noise['PSD'] = lim[0]

    # audioModel.py:364-373
    def annealed_psd(self, i):
        lim = self.noise['ann_PSD_lim']
        N = self.iter_num
        return ((np.sqrt(lim[0]) * (N - i) + np.sqrt(lim[1]) * i) / N) ** 2

    # audioModel.py:330-382
    def estim_param_a_post_model(self, callback=None):
        logliks = np.ones(self.iter_num)
        opt = self.noise['sim_ann_opt']
        if opt == 'ann':
            self.noise['PSD'] = self.noise['ann_PSD_lim'][0]
        elif opt == 'no_ann':
            self.noise['PSD'] = self.noise['ann_PSD_lim'][1]
        for i in range(self.iter_num):
            if opt in ('ann', 'ann_ns_inj'):
                self.noise['PSD'] = self.annealed_psd(i)
            logliks[i] = np.real(self.GEM_iteration())
            if callback is not None:
                callback(i, self)
        return logliks

    # audioModel.py:384-428
    def GEM_iteration(self):
        if self.channels != 2:
            raise AttributeError("Nb channels %d not implemented yet" % self.channels)
        V, mix, parts = self.retrieve_subsrc_params()
        hat_Rxx, hat_Rxs, hat_Rss, hat_Ws, loglik = self.compute_suff_stat(V, mix)
        self.update_mix_matrix(hat_Rxs, hat_Rss, mix, parts)
        hat_W = np.zeros([len(parts), self.nbFreqsSigRepr, self.nbFramesSigRepr])
        for j in range(len(parts)):
            hat_W[j] = np.mean(hat_Ws[parts[j]], axis=0)
        self.last_hat_W = hat_W
        self.update_spectral_components(hat_W)
        self.renormalize_parameters()
        return loglik

    # audioModel.py:430-498 (note N1: an empty factor list means ALL factors)
    def comp_spat_comp_power(self, spat_comp_ind, spec_comp_ind=(), factor_ind=()):
        V = np.zeros([self.nbFreqsSigRepr, self.nbFramesSigRepr])
        keys = list(spec_comp_ind) if len(spec_comp_ind) else list(self.spec_comps.keys())
        for k in keys:
            comp = self.spec_comps[k]
            if comp['spat_comp_ind'] != spat_comp_ind:
                continue
            Vk = np.ones([self.nbFreqsSigRepr, self.nbFramesSigRepr])
            facs = list(factor_ind) if len(factor_ind) else list(comp['factor'].keys())
            for fi in facs:
                fac = comp['factor'][fi]
                W = np.dot(fac['FB'], fac['FW'])
                H = np.dot(fac['TW'], fac['TB']) if len(fac['TB']) else fac['TW']
                Vk *= np.dot(W, H)
            V += Vk
        return V

    # audioModel.py:514-578
    def retrieve_subsrc_params(self):
        parts = {}
        total = 0
        for j in range(len(self.spat_comps)):
            p = self.spat_comps[j]['params']
            rank = p.shape[1] if self.spat_comps[j]['mix_type'] == 'inst' else p.shape[0]
            parts[j] = total + np.arange(rank)
            total += rank
        V = np.zeros([total, self.nbFreqsSigRepr, self.nbFramesSigRepr])
        mix = np.zeros([total, self.channels, self.nbFreqsSigRepr], dtype=complex)
        for j, sc in self.spat_comps.items():
            Vj = self.comp_spat_comp_power(spat_comp_ind=j)
            for r in parts[j]:
                V[r] = Vj
            if sc['mix_type'] == 'inst':
                for f in range(self.nbFreqsSigRepr):
                    mix[parts[j], :, f] = sc['params'].T
            else:
                mix[parts[j]] = sc['params']
        return V, mix, parts

    # audioModel.py:580-764 (E-step; the R x R pair loop is kept as is)
    def compute_suff_stat(self, V, mix):
        if self.channels != 2:
            raise ValueError("Nb channels not supported:%d" % self.channels)
        R = V.shape[0]
        col = lambda a: a[:, None]
        sd = np.empty([2, self.nbFreqsSigRepr, self.nbFramesSigRepr])
        sd[0] = col(np.abs(mix[0][0]) ** 2) * V[0]
        sd[1] = col(np.abs(mix[0][1]) ** 2) * V[0]
        so = col(mix[0][0] * np.conj(mix[0][1])) * V[0]
        for c in range(2):
            sd[c] += col(self.noise['PSD'])
        for r in range(1, R):
            sd[0] += col(np.abs(mix[r][0]) ** 2) * V[r]
            sd[1] += col(np.abs(mix[r][1]) ** 2) * V[r]
            so += col(mix[r][0] * np.conj(mix[r][1])) * V[r]
        isd, iso, det = inv_herm_mat_2d(sd, so)
        del sd, so
        Cx = self.Cx
        loglik = -np.mean(np.log(det * np.pi) + isd[0] * Cx[0] + isd[1] * Cx[2]
                          + 2. * np.real(iso * np.conj(Cx[1])))
        G = np.empty((2, R, self.nbFreqsSigRepr, self.nbFramesSigRepr), dtype=complex)
        for r in range(R):
            G[0, r] = (col(np.conj(mix[r][0])) * isd[0]
                       + col(np.conj(mix[r][1])) * np.conj(iso)) * V[r]
            G[1, r] = (col(np.conj(mix[r][0])) * iso
                       + col(np.conj(mix[r][1])) * isd[1]) * V[r]
        hat_Rss = np.empty([self.nbFreqsSigRepr, R, R], dtype=complex)
        hat_Ws = np.empty([R, self.nbFreqsSigRepr, self.nbFramesSigRepr])
        t1 = np.empty_like(Cx[0])
        t2 = np.empty_like(Cx[0])
        t3 = np.empty_like(Cx[0])
        for r1 in range(R):
            for r2 in range(R):
                t1[:] = Cx[0]
                t1 *= np.conj(G[0, r2])
                t1 += np.conj(G[1, r2]) * Cx[1]
                t1 *= G[0, r1]
                t2[:] = Cx[2]
                t2 *= np.conj(G[1, r2])
                t2 += np.conj(G[0, r2] * Cx[1])
                t2 *= G[1, r1]
                t3[:] = G[0, r1]
                t3 *= col(mix[r2, 0])
                t3 += G[1, r1] * col(mix[r2, 1])
                t3 *= V[r2]
                t1 += t2
                t1 -= t3
                if r1 == r2:
                    t1 += V[r1]
                    hat_Ws[r1] = np.abs(np.real(t1))
                hat_Rss[:, r1, r2] = np.mean(t1, axis=1)
        for f in range(self.nbFreqsSigRepr):
            hat_Rss[f] = (hat_Rss[f] + np.conj(hat_Rss[f]).T) / 2.
        hat_Rxs = np.empty([self.nbFreqsSigRepr, 2, R], dtype=complex)
        for r in range(R):
            hat_Rxs[:, 0, r] = np.mean(np.conj(G[0][r]) * Cx[0] + np.conj(G[1][r]) * Cx[1], axis=1)
            hat_Rxs[:, 1, r] = np.mean(np.conj(G[0][r]) * np.conj(Cx[1]) + np.conj(G[1][r]) * Cx[2], axis=1)
        del G
        hat_Rxx = np.mean(Cx, axis=-1)
        return hat_Rxx, hat_Rxs, hat_Rss, hat_Ws, loglik

    # audioModel.py:766-889 (M-step, mixing parameters)
    def update_mix_matrix(self, hat_Rxs, hat_Rss, mix, parts):
        inst, inst_other, conv, conv_other = [], [], [], []
        for j, sc in self.spat_comps.items():
            free = sc['frdm_prior'] == 'free'
            (inst if free and sc['mix_type'] == 'inst' else inst_other).extend(parts[j])
            (conv if free and sc['mix_type'] == 'conv' else conv_other).extend(parts[j])
        F = self.nbFreqsSigRepr
        if len(inst):
            bis = hat_Rxs[:, :, inst]
            if len(inst_other):
                for f in range(F):
                    bis[f] -= np.dot(mix[inst_other, :, f].T,
                                     hat_Rss[f][np.vstack(inst_other), inst])
            bis = np.real(np.mean(bis, axis=0))
            rss = np.real(np.mean(hat_Rss[:, np.vstack(inst), inst], axis=0))
            sol = np.linalg.solve(rss.T, bis.T)
            for f in range(F):
                mix[inst, :, f] = sol
        if len(conv):
            bis = hat_Rxs[:, :, conv]
            if len(conv_other):
                for f in range(F):
                    bis[f] -= np.dot(mix[conv_other, :, f].T,
                                     hat_Rss[f][np.vstack(conv_other), conv])
            for f in range(F):
                try:
                    mix[conv, :, f] = np.linalg.solve(hat_Rss[f].T, bis[f].T)
                except np.linalg.LinAlgError:
                    raise np.linalg.LinAlgError('Singular Matrix')
        for k, sc in self.spat_comps.items():
            if sc['frdm_prior'] == 'free':
                if sc['mix_type'] == 'inst':
                    sc['params'] = np.mean(mix[parts[k]], axis=2).T
                else:
                    sc['params'] = mix[parts[k]]

    # audioModel.py:1469-1978, NMF branch of TW_constr (GMM/HMM not restated)
    def update_spectral_components(self, hat_W):
        omega = self.nmfUpdateCoeff
        lam = self.lambdaCorr
        for k, comp in self.spec_comps.items():
            nfac = len(comp['factor'])
            j = comp['spat_comp_ind']
            if lam > 0:
                all_pow = np.maximum(self.comp_spat_cmps_powers(list(self.spat_comps.keys())), EPS)
                own = np.maximum(self.comp_spat_comp_power(j), EPS)
                minus = all_pow - own
                if np.all(minus >= 0):
                    minus = np.maximum(minus, EPS)
            for fi, fac in comp['factor'].items():
                others = [x for x in range(nfac) if x != fi]
                # N1: `others == []` means all factors of spec comp k
                other = np.maximum(self.comp_spat_comp_power(j, spec_comp_ind=[k],
                                                             factor_ind=others), EPS)
                if fac['FB_frdm_prior'] == 'free':
                    Vj = np.maximum(self.comp_spat_comp_power(j), EPS)
                    H = np.dot(fac['TW'], fac['TB']) if len(fac['TB']) else fac['TW']
                    FWH = np.dot(fac['FW'], H).T
                    pen = lam * minus / np.maximum(all_pow ** 2, EPS) if lam > 0 else 0.
                    den = np.dot(other * (1. / Vj + pen), FWH)
                    if lam > 0:
                        pen *= 2 * (Vj / all_pow)
                    num = np.dot((hat_W[j] / (Vj ** 2) + pen) * other, FWH)
                    fac['FB'] *= (num / np.maximum(den, EPS)) ** omega
                if fac['FW_frdm_prior'] == 'free':
                    Vj = np.maximum(self.comp_spat_comp_power(j, spec_comp_ind=[k]), EPS)
                    H = np.dot(fac['TW'], fac['TB']) if len(fac['TB']) else fac['TW']
                    pen = lam * np.maximum(minus, EPS) / np.maximum(all_pow ** 2, EPS) if lam > 0 else 0.
                    den = np.dot(fac['FB'].T, np.dot(other * (1. / Vj + pen), H.T))
                    if lam > 0:
                        pen *= 2 * (Vj / all_pow)
                    num = np.dot(fac['FB'].T, np.dot((hat_W[j] / (Vj ** 2) + pen) * other, H.T))
                    fac['FW'] *= (num / np.maximum(den, EPS)) ** omega
                if fac['TW_frdm_prior'] == 'free':
                    if fac['TW_constr'] != 'NMF':
                        raise NotImplementedError("only TW_constr='NMF' is restated")
                    Vj = np.maximum(self.comp_spat_comp_power(j, spec_comp_ind=[k]), EPS)
                    W = np.dot(fac['FB'], fac['FW'])
                    pen = lam * np.maximum(minus, EPS) / np.maximum(all_pow ** 2, EPS) if lam > 0 else 0.
                    if len(fac['TB']):
                        den = np.dot(W.T, np.dot(other * (1. / Vj + pen), fac['TB'].T))
                        if lam > 0:
                            pen *= 2 * (Vj / all_pow)
                        num = np.dot(W.T, np.dot((hat_W[j] / (Vj ** 2) + pen) * other, fac['TB'].T))
                    else:
                        den = np.dot(W.T, other * (1. / Vj + pen))
                        if lam > 0:
                            pen *= 2 * (Vj / all_pow)
                        num = np.dot(W.T, other * (hat_W[j] / (Vj ** 2) + pen))
                    fac['TW'] *= (num / np.maximum(den, EPS)) ** omega
                if len(fac['TB']) and fac['TB_frdm_prior'] == 'free':
                    Vj = np.maximum(self.comp_spat_comp_power(j, spec_comp_ind=[k]), EPS)
                    W = np.dot(np.dot(fac['FB'], fac['FW']), fac['TW'])
                    pen = lam * np.maximum(minus, EPS) / np.maximum(all_pow ** 2, EPS) if lam > 0 else 0.
                    den = np.dot(W.T, other * (1. / Vj + pen))
                    if lam > 0:
                        pen *= 2 * (Vj / all_pow)
                    num = np.dot(W.T, (hat_W[j] / np.maximum(Vj ** 2, EPS) + pen) * other)
                    fac['TB'] *= (num / np.maximum(den, EPS)) ** omega

    def comp_spat_cmps_powers(self, inds):
        V = 0
        for i in inds:
            V += self.comp_spat_comp_power(spat_comp_ind=i)
        return V

    # audioModel.py:1980-2040
    def renormalize_parameters(self, rng=np.random):
        energy = np.zeros(len(self.spat_comps))
        for j, sc in self.spat_comps.items():
            energy[j] = np.mean(np.abs(sc['params']) ** 2)
            sc['params'] /= np.sqrt(energy[j])
        self.restarted = []
        for k, comp in self.spec_comps.items():
            e = energy[comp['spat_comp_ind']]
            nfac = len(comp['factor'])
            for fi, fac in comp['factor'].items():
                fac['FB'] *= e
                w = fac['FB'].max(axis=0)
                w[w == 0] = 1.
                fac['FB'] /= w
                fac['FW'] *= w[:, None]
                if fac['TW_constr'] in ('GMM', 'HMM'):
                    raise NotImplementedError("Temporal discrete state mngmt not done yet. ")
                w = fac['FW'].mean(axis=0)
                w[w == 0] = 1.
                fac['FW'] /= w
                fac['TW'] *= w[:, None]
                if np.sum(fac['TW']) < EPS:
                    fac['TW'] = rng.randn(*fac['TW'].shape) ** 2
                    fac['TW'] *= 1e3 * EPS
                    self.restarted.append((k, fi))
                if len(fac['TB']):
                    w = fac['TB'].mean(axis=1)
                    w[w == 0] = 1.
                    fac['TB'] /= w[:, None]
                    fac['TW'] *= w
                ge = fac['TW'].mean()
                if fi < nfac - 1:
                    fac['TW'] /= ge

    # ---------------------------------------------------------------- Wiener
    # audioModel.py:1327-1372
    def compute_sigma_comp_2d(self, spat_ind, spec_comp_ind):
        P = self.comp_spat_comp_power(spat_comp_ind=spat_ind, spec_comp_ind=spec_comp_ind)
        sc = self.spat_comps[spat_ind]
        A = sc['params'].T if sc['mix_type'] == 'inst' else sc['params']
        r0 = np.atleast_1d((np.abs(A[:, 0]) ** 2).sum(axis=0))
        r1 = np.atleast_1d((np.abs(A[:, 1]) ** 2).sum(axis=0))
        ro = np.atleast_1d((A[:, 0] * np.conj(A[:, 1])).sum(axis=0))
        d = np.zeros([2, self.nbFreqsSigRepr, self.nbFramesSigRepr])
        d[0] = r0[:, None] * P
        d[1] = r1[:, None] * P
        return d, ro[:, None] * P

    # audioModel.py:1374-1394
    def compute_inv_sigma_mix_2d(self, sdiag, soff):
        d = sdiag.sum(axis=0)
        o = soff.sum(axis=0)
        for c in range(2):
            d[c] += self.noise['PSD'][:, None]
        isd, iso, _ = inv_herm_mat_2d(d, o)
        return isd, iso

    # audioModel.py:1396-1467
    @staticmethod
    def compute_Wiener_gain_2d(sd, so, isd, iso):
        WG = np.zeros((2, 2) + so.shape, dtype=complex)
        WG[0, 0] = so * np.conj(iso)
        WG[1, 1] = np.conj(WG[0, 0])
        WG[0, 0] += sd[0] * isd[0]
        WG[1, 1] += sd[1] * isd[1]
        WG[0, 1] = sd[0] * iso + so * isd[1]
        WG[1, 0] = np.conj(so) * isd[0] + sd[1] * np.conj(iso)
        return WG

    # audioModel.py:1063-1217 without the file I/O: returns the STFT-domain
    # images S[n, c] = sum_c2 WG_n[c, c2] X[c2] (parity quantity |S|).
    def separated_images(self, X, spec_comp_ind=None):
        if spec_comp_ind is None:
            spec_comp_ind = {}
            for j in range(len(self.spat_comps)):
                spec_comp_ind[j] = []
            for k, comp in self.spec_comps.items():
                spec_comp_ind[comp['spat_comp_ind']].append(k)
        nsrc = len(spec_comp_ind)
        F, T = self.nbFreqsSigRepr, self.nbFramesSigRepr
        sd = np.zeros([nsrc, 2, F, T])
        so = np.zeros([nsrc, F, T], dtype=complex)
        for n in range(nsrc):
            for s in np.unique([self.spec_comps[k]['spat_comp_ind'] for k in spec_comp_ind[n]]):
                d, o = self.compute_sigma_comp_2d(s, spec_comp_ind[n])
                sd[n] += d
                so[n] += o
        isd, iso = self.compute_inv_sigma_mix_2d(sd, so)
        S = np.zeros([nsrc, 2, F, T], dtype=complex)
        for n in range(nsrc):
            WG = self.compute_Wiener_gain_2d(sd[n], so[n], isd, iso)
            for c1 in range(2):
                for c2 in range(2):
                    S[n, c1] += WG[c1, c2] * X[c2]
        return S


# ----------------------------------------------------------------------------
# audioModel.py:2349-2393 : RNG order matters for parity of the initial state
def init_nmf_inst(model, nbComps, nbNMFComps, spatial_rank, rng=np.random):
    rank = np.atleast_1d(spatial_rank)
    if rank.size < nbComps:
        rank = [rank[0]] * nbComps
    model.rank = rank
    nc = model.channels
    model.spat_comps = {}
    model.spec_comps = {}
    F, T = model.nbFreqsSigRepr, model.nbFramesSigRepr
    for j in range(nbComps):
        sc = {'time_dep': 'indep', 'mix_type': 'inst', 'frdm_prior': 'free'}
        sc['params'] = rng.randn(nc, rank[j])
        if nc == 2:
            ang = (j + 1) * np.pi / (2. * (nbComps + 1))
            s0 = np.sin(ang) + rng.randn(rank[j]) * np.sqrt(0.01)
            s1 = np.cos(ang) + rng.randn(rank[j]) * np.sqrt(0.01)
            sc['params'] = np.array([s0, s1])
        model.spat_comps[j] = sc
        fac = {'FB': 0.75 * np.abs(rng.randn(F, nbNMFComps)) + 0.25,
               'FW': np.eye(nbNMFComps),
               'TW': 0.75 * np.abs(rng.randn(nbNMFComps, T)) + 0.25,
               'TB': [], 'FB_frdm_prior': 'free', 'FW_frdm_prior': 'fixed',
               'TW_frdm_prior': 'free', 'TB_frdm_prior': [], 'TW_constr': 'NMF'}
        model.spec_comps[j] = {'spat_comp_ind': j, 'factor': {0: fac}}
    model.renormalize_parameters(rng=rng)


# audioModel.py:2488-2508
def make_convolutive(model):
    for n, (j, sc) in enumerate(model.spat_comps.items()):
        if sc['mix_type'] != 'inst':
            continue
        sc['mix_type'] = 'conv'
        inst = sc['params']
        p = np.zeros([model.rank[n], model.channels, model.nbFreqsSigRepr], dtype=complex)
        for f in range(model.nbFreqsSigRepr):
            p[:, :, f] = inst.T
        sc['params'] = p


# audioModel.py:2224-2294, initMethod 'rand' (the DEMIX branch is out of scope)
def init_conv_rand(model, rng=np.random):
    nc, F, J = model.channels, model.nbFreqsSigRepr, len(model.spat_comps)
    for j, sc in model.spat_comps.items():
        sc['mix_type'] = 'conv'
    A = rng.randn(J, F, nc) + 1j * rng.randn(J, F, nc)
    for n, (j, sc) in enumerate(model.spat_comps.items()):
        sc['params'] = np.zeros([model.rank[n], nc, F], dtype=complex)
        for r in range(model.rank[n]):
            sc['params'][r] = A[j].T


# ----------------------------------------------------------------------------
# tools/nmf.py:24-61 (IS-NMF multiplicative updates)
def nmf_decomposition(SX, nbComps=10, niter=10, rng=np.random):
    nf, nt = SX.shape
    W = rng.randn(nf, nbComps) ** 2
    H = rng.randn(nbComps, nt) ** 2
    W /= W.sum(axis=0)
    for _ in range(niter):
        hat = np.dot(W, H)
        num = np.dot(SX / np.maximum(hat ** 2, EPS), H.T)
        den = np.dot(1 / np.maximum(hat, EPS), H.T)
        W *= num / np.maximum(den, EPS)
        s = W.sum(axis=0)
        s[s == 0] = 1.
        W /= s
        H *= s[:, None]
        hat = np.dot(W, H)
        num = np.dot(W.T, SX / np.maximum(hat ** 2, EPS))
        den = np.dot(W.T, 1 / np.maximum(hat, EPS))
        H *= num / np.maximum(den, EPS)
    return W, H


def nmf_decomp_init(SX, nbComps=10, niter=10, Winit=None, Hinit=None, updateW=True,
                    updateH=True, rng=np.random):
    """tools/nmf.py:63-159: frame-major H internally, returned transposed."""
    nf, nt = SX.shape
    if Winit is None or Winit.shape != (nf, nbComps):
        W = rng.randn(nf, nbComps) ** 2
    else:
        W = np.copy(Winit)
    if Hinit is not None:
        if Hinit.shape == (nbComps, nt):
            H = np.copy(Hinit.T)
        elif Hinit.shape == (nt, nbComps):
            H = np.copy(Hinit)
        else:
            raise AttributeError('Hinit not in the right shape.')
    else:
        H = rng.randn(nt, nbComps) ** 2
    if updateW:
        W /= W.sum(axis=0)
    for _ in range(niter):
        if updateW:
            hat = np.dot(W, H.T)
            num = np.dot(SX / np.maximum(hat ** 2, EPS), H)
            den = np.dot(1 / np.maximum(hat, EPS), H)
            W *= num / np.maximum(den, EPS)
            s = W.sum(axis=0)
            s[s == 0] = 1.
            W /= s
            H *= s
        if updateH:
            hat = np.dot(H, W.T)
            num = np.dot(SX.T / np.maximum(hat ** 2, EPS), W)
            den = np.dot(1 / np.maximum(hat, EPS), W)
            H *= num / np.maximum(den, EPS)
    return W, H.T


# ----------------------------------------------------------------------------
# audioModel.py:2091-2222: spectral components initialised by IS-NMF of the
# channel-averaged power Cx
def _mono_power(model):
    nc = 2
    Cx = np.copy(np.real(model.Cx[0]))
    Cx += np.real(model.Cx[2])
    return Cx / np.double(nc)


def init_nmf_indiv(model, niter=10, updateFreqBasis=True, updateTimeWeight=True,
                   rng=np.random):
    """initialize_all_spec_comps_with_NMF_indiv (audioModel.py:2118-2177)"""
    nb = [sc['factor'][0]['FB'].shape[1] for sc in model.spec_comps.values()]
    tot = int(np.sum(nb))
    FBinit = np.zeros([model.nbFreqsSigRepr, tot])
    TWinit = np.zeros([tot, model.nbFramesSigRepr])
    for k, sc in model.spec_comps.items():
        a = int(np.sum(nb[:k]))
        FBinit[:, a:a + nb[k]] = sc['factor'][0]['FB']
        TWinit[a:a + nb[k]] = sc['factor'][0]['TW']
    W, H = nmf_decomp_init(_mono_power(model), nbComps=tot, niter=niter, Winit=FBinit,
                           Hinit=TWinit, updateW=updateFreqBasis, updateH=updateTimeWeight,
                           rng=rng)
    for k, sc in model.spec_comps.items():
        a = int(np.sum(nb[:k]))
        if updateFreqBasis:
            sc['factor'][0]['FB'] = np.maximum(W[:, a:a + nb[k]], EPS)
        if updateTimeWeight:
            sc['factor'][0]['TW'] = np.maximum(H[a:a + nb[k]], EPS)
    model.renormalize_parameters(rng=rng)


def init_nmf_same(model, niter=10, rng=np.random):
    """initialize_all_spec_comps_with_NMF_same (audioModel.py:2179-2222)"""
    nb = [sc['factor'][0]['FB'].shape[1] for sc in model.spec_comps.values()]
    W, H = nmf_decomposition(_mono_power(model), nbComps=int(np.max(nb)), niter=niter, rng=rng)
    order = np.argsort(H.sum(axis=1))[::-1]
    W, H = W[:, order], H[order]
    for sc in model.spec_comps.values():
        n = sc['factor'][0]['FB'].shape[1]
        sc['factor'][0]['FB'][:] = W[:, :n]
        sc['factor'][0]['TW'][:] = H[:n]
    model.renormalize_parameters(rng=rng)


# ----------------------------------------------------------------------------
# BASELINE configs[1] (C2): per-source mono Wiener images of the IS-NMF model.
# The one-channel degenerate of compute_sigma_comp_2d (audioModel.py:1327-1372,
# mixing = 1), compute_inv_sigma_mix_2d (:1374-1394, the inv_herm_mat_2d guard
# of signalTools.py:177-188 on a 1 x 1 Sigma_x) and compute_Wiener_gain_2d
# (:1396-1467), image WG X as separate_comps (:1205-1214), with V_n the
# IS-NMF model of tools/nmf.py:24-61 restricted to source n's components.
# PARITY UNPINNED by reference code: the reference's FASST raises for mono
# signals (audioModel.py:394, :418-420, :605-607), so no
# reference output exists for this stage.
def mono_wiener_images(X, W, H, comp_ind, psd=None):
    F, T = X.shape
    nsrc = len(comp_ind)
    sd = np.zeros([nsrc, F, T])
    for n in range(nsrc):
        c = list(comp_ind[n])
        sd[n] = np.dot(W[:, c], H[c])
    d = sd.sum(axis=0)
    if psd is not None:
        d += np.asarray(psd)[:, None]
    det = np.sign(d + EPS) * np.maximum(np.abs(d), EPS)
    isd = 1. / det
    S = np.zeros([nsrc, F, T], dtype=complex)
    for n in range(nsrc):
        S[n] = (sd[n] * isd) * X
    return S
