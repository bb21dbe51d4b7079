"""Thin object wrapper over one device context of libfasst_hip.so.

All compute happens on the GPU; this module only moves NumPy arrays across
the C ABI (include/fasst_hip.h) and maps status codes to exceptions.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, dptr, iptr, lib


def wiener_gain(device, sdiag, soff, idiag, ioff):
    """compute_Wiener_gain_2d on the device (fasst_wiener_gain): WG [2, 2, *soff.shape]."""
    sdiag = np.ascontiguousarray(sdiag, dtype=np.float64)
    idiag = np.ascontiguousarray(idiag, dtype=np.float64)
    soff = np.ascontiguousarray(soff, dtype=np.complex128)
    ioff = np.ascontiguousarray(ioff, dtype=np.complex128)
    shp = soff.shape
    if sdiag.shape != (2,) + shp or idiag.shape != (2,) + shp or ioff.shape != shp:
        raise ValueError("Wiener gain operands %s %s %s %s"
                         % (sdiag.shape, shp, idiag.shape, ioff.shape))
    WG = np.empty((2, 2) + shp, dtype=np.complex128)
    check(lib.fasst_wiener_gain(int(device), int(soff.size), dptr(sdiag), dptr(soff),
                                dptr(idiag), dptr(ioff), dptr(WG)), "compute_Wiener_gain_2d")
    return WG


def colmask_words(masks):
    """Column sets (Python ints, bit k = NMF column k, K <= 128) as the C
    ABI's 128-bit form: uint64 [n][2] = (columns 0..63, columns 64..127)."""
    out = np.zeros((len(masks), 2), dtype=np.uint64)
    for i, m in enumerate(masks):
        m = int(m)
        if m < 0 or m >> 128:
            raise ValueError("column set beyond the HIP path's 128 NMF columns")
        out[i, 0] = m & 0xFFFFFFFFFFFFFFFF
        out[i, 1] = m >> 64
    return out


class Engine(object):
    """Device state of one FASST model: observation (Cx, STFT) + parameters."""

    def __init__(self, F, T, device=None):
        self.device = _lib.default_device() if device is None else int(device)
        self.F, self.T = int(F), int(T)
        h = ctypes.c_void_p()
        check(lib.fasst_create(self.device, self.F, self.T, ctypes.byref(h)), "fasst_create")
        self._h = h
        self.structure = None

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib.fasst_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def configure(self, ranks, Ks, conv):
        """conv: True / False for every source, or one flag per source (a
        model with both 'inst' and 'conv' spatial components)."""
        per = np.broadcast_to(np.asarray(conv, dtype=bool), (len(ranks),))
        key = (tuple(int(r) for r in ranks), tuple(int(k) for k in Ks),
               tuple(bool(c) for c in per))
        if key == self.structure:
            return
        r = np.ascontiguousarray(ranks, dtype=np.int32)
        k = np.ascontiguousarray(Ks, dtype=np.int32)
        c = np.ascontiguousarray(per, dtype=np.int32)
        check(lib.fasst_configure_types(self._h, len(r), iptr(r), iptr(k), iptr(c)),
              "fasst_configure_types")
        self.structure = key

    # ------------------------------------------------------------ observation
    def set_audio(self, data, window, nfft, hop):
        data = np.ascontiguousarray(data, dtype=np.float64)
        window = np.ascontiguousarray(window, dtype=np.float64)
        check(lib.fasst_set_audio(self._h, dptr(data), data.shape[0], dptr(window), window.size,
                                  int(nfft), int(hop)), "fasst_set_audio")

    def mix_psd(self):
        out = np.empty(self.F)
        check(lib.fasst_mix_psd(self._h, dptr(out)), "fasst_mix_psd")
        return out

    def set_cx(self, Cx):
        Cx = np.ascontiguousarray(Cx, dtype=np.complex128)
        if Cx.shape != (3, self.F, self.T):
            raise ValueError("Cx shape %s != (3, %d, %d)" % (Cx.shape, self.F, self.T))
        check(lib.fasst_set_cx(self._h, dptr(Cx)), "fasst_set_cx")

    def get_cx(self):
        out = np.empty((3, self.F, self.T), dtype=np.complex128)
        check(lib.fasst_get_cx(self._h, dptr(out)), "fasst_get_cx")
        return out

    def set_stft(self, X):
        X = np.ascontiguousarray(X, dtype=np.complex128)
        if X.shape != (2, self.F, self.T):
            raise ValueError("X shape %s != (2, %d, %d)" % (X.shape, self.F, self.T))
        check(lib.fasst_set_stft(self._h, dptr(X)), "fasst_set_stft")

    # ------------------------------------------------------------ parameters
    def set_spatial(self, j, params, free):
        p = np.ascontiguousarray(params, dtype=np.complex128)
        check(lib.fasst_set_spatial(self._h, int(j), dptr(p), int(bool(free))), "fasst_set_spatial")

    def get_spatial(self, j, shape):
        out = np.empty(shape, dtype=np.complex128)
        check(lib.fasst_get_spatial(self._h, int(j), dptr(out)), "fasst_get_spatial")
        return out

    def set_spectral(self, j, FB, FW, TW, fb_free, tw_free, fw_free=False):
        FB = np.ascontiguousarray(FB, dtype=np.float64)
        FW = np.ascontiguousarray(FW, dtype=np.float64)
        TW = np.ascontiguousarray(TW, dtype=np.float64)
        check(lib.fasst_set_spectral(self._h, int(j), dptr(FB), dptr(FW), dptr(TW),
                                     int(bool(fb_free)), int(bool(tw_free))), "fasst_set_spectral")
        check(lib.fasst_set_fw_prior(self._h, int(j), int(bool(fw_free))), "fasst_set_fw_prior")

    def set_blocks(self, j, kb, fb_free, fw_free, tw_free):
        """Spectral components of source j side by side in its columns
        [kb[b], kb[b + 1]) (fasst_set_blocks)."""
        kb = np.ascontiguousarray(kb, dtype=np.int32)
        fb = np.ascontiguousarray(fb_free, dtype=np.int32)
        fw = np.ascontiguousarray(fw_free, dtype=np.int32)
        tw = np.ascontiguousarray(tw_free, dtype=np.int32)
        check(lib.fasst_set_blocks(self._h, int(j), kb.size - 1, iptr(kb), iptr(fb), iptr(fw),
                                   iptr(tw)), "fasst_set_blocks")

    def set_corr(self, lam, seq_j=(), seq_b=()):
        """lambdaCorr and the spectral components' key order (fasst_set_corr)."""
        sj = np.ascontiguousarray(list(seq_j) or [0], dtype=np.int32)
        sb = np.ascontiguousarray(list(seq_b) or [0], dtype=np.int32)
        check(lib.fasst_set_corr(self._h, float(lam), len(seq_j), iptr(sj), iptr(sb)),
              "fasst_set_corr")

    def set_tb(self, j, b, TW=None, TB=None, tb_free=True):
        """Time blobs of component b of source j (fasst_set_tb): TW = the
        component's factor TW (rows x L), TB = L x T; TB None removes them."""
        if TB is None:
            check(lib.fasst_set_tb(self._h, int(j), int(b), 0, None, None, 0), "fasst_set_tb")
            return
        TW = np.ascontiguousarray(TW, dtype=np.float64)
        TB = np.ascontiguousarray(TB, dtype=np.float64)
        if TB.ndim != 2 or TB.shape[1] != self.T or TW.ndim != 2 or TW.shape[1] != TB.shape[0]:
            raise ValueError("time blobs: TW %s, TB %s (T = %d)" % (TW.shape, TB.shape, self.T))
        check(lib.fasst_set_tb(self._h, int(j), int(b), TB.shape[0], dptr(TW), dptr(TB),
                               int(bool(tb_free))), "fasst_set_tb")

    def get_tb(self, j, b, rows, L):
        TW = np.empty((rows, L))
        TB = np.empty((L, self.T))
        check(lib.fasst_get_tb(self._h, int(j), int(b), dptr(TW), dptr(TB)), "fasst_get_tb")
        return TW, TB

    def get_spectral(self, j, K):
        FB = np.empty((self.F, K))
        FW = np.empty((K, K))
        TW = np.empty((K, self.T))
        check(lib.fasst_get_spectral(self._h, int(j), dptr(FB), dptr(FW), dptr(TW)),
              "fasst_get_spectral")
        return FB, FW, TW

    # ------------------------------------------------------------ compute
    def renormalize(self):
        mask = ctypes.c_int(0)
        check(lib.fasst_renormalize(self._h, ctypes.byref(mask)), "fasst_renormalize")
        return mask.value

    def run(self, psd_rows, omega):
        """Run len(psd_rows) GEM iterations.  Returns (logliks, done, restart_mask)."""
        psd_rows = np.ascontiguousarray(psd_rows, dtype=np.float64)
        n = psd_rows.shape[0]
        if n and psd_rows.shape[1] != self.F:
            raise ValueError("psd rows must have F=%d columns" % self.F)
        ll = np.zeros(max(n, 1))
        mask = ctypes.c_int(0)
        done = ctypes.c_int(0)
        st = lib.fasst_run(self._h, n, dptr(psd_rows) if n else None, float(omega), dptr(ll),
                           ctypes.byref(mask), ctypes.byref(done))
        if st == _lib.FASST_TW_RESTART:
            return ll[:done.value], done.value, mask.value
        check(st, "fasst_run")
        return ll[:n], n, 0

    def set_profiling(self, on=True):
        check(lib.fasst_set_profiling(self._h, int(bool(on))), "fasst_set_profiling")

    def kernel_times(self):
        """{kernel name: (mean ms per launch, launches)} over the profiled iterations."""
        nk = 32
        ms = np.zeros(nk)
        cnt = (ctypes.c_long * nk)()
        n = lib.fasst_kernel_times(self._h, dptr(ms), cnt, nk)
        return {lib.fasst_kernel_name(i).decode(): (ms[i], cnt[i]) for i in range(n) if cnt[i]}

    def set_sources(self, sources):
        """Separation sources (fasst_set_sources): None = one per spatial
        component; else a list, per source, of (spatial component, column
        mask) terms."""
        if sources is None:
            check(lib.fasst_set_sources(self._h, 0, None, None, None), "fasst_set_sources")
            self.nsrc = None
            return
        off = np.cumsum([0] + [len(t) for t in sources]).astype(np.int32)
        tj = np.array([j for t in sources for j, _ in t] or [0], dtype=np.int32)
        tm = colmask_words([m for t in sources for _, m in t] or [0])
        check(lib.fasst_set_sources(self._h, len(sources), iptr(off), iptr(tj),
                                    tm.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))),
              "fasst_set_sources")
        self.nsrc = len(sources)

    def _nsrc(self):
        return getattr(self, 'nsrc', None) or len(self.structure[0])

    def separate_waveforms(self, psd, window, analysis_window, nfft, hop):
        """Wiener images + per-image iSTFT on the device: [nsrc, 2, len] float64."""
        psd = np.ascontiguousarray(psd, dtype=np.float64)
        w = np.ascontiguousarray(window, dtype=np.float64)
        aw = np.ascontiguousarray(analysis_window, dtype=np.float64)
        J = self._nsrc()
        n = int(hop) * (self.T - 1) + w.size - w.size // 2
        out = np.empty((J, 2, n))
        check(lib.fasst_separate_waveforms(self._h, dptr(psd), dptr(w), dptr(aw), w.size,
                                           int(nfft), int(hop), dptr(out)),
              "fasst_separate_waveforms")
        return out

    # ------------------------------------------------------------ step methods
    def source_powers(self, j0, nj, colmasks=None):
        """V [nj, F, T] of spatial components j0 .. j0+nj-1 (fasst_source_powers)."""
        out = np.empty((nj, self.F, self.T))
        mp = None
        if colmasks is not None:
            m = colmask_words(colmasks)
            mp = m.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))
        check(lib.fasst_source_powers(self._h, int(j0), int(nj), mp, dptr(out)),
              "fasst_source_powers")
        return out

    def suff_stat(self, V, mix, psd):
        """compute_suff_stat on the resident Cx (fasst_suff_stat):
        (hat_Rxx [3, F], hat_Rxs [F, 2, R], hat_Rss [F, R, R], hat_Ws [R, F, T], loglik)."""
        V = np.ascontiguousarray(V, dtype=np.float64)
        mix = np.ascontiguousarray(mix, dtype=np.complex128)
        psd = np.ascontiguousarray(np.broadcast_to(psd, (self.F,)), dtype=np.float64)
        R = V.shape[0]
        if V.shape != (R, self.F, self.T) or mix.shape != (R, 2, self.F):
            raise ValueError("spat_comp_powers %s / mix_matrix %s for F=%d, T=%d"
                             % (V.shape, mix.shape, self.F, self.T))
        rxx = np.empty((3, self.F), dtype=np.complex128)
        rxs = np.empty((self.F, 2, R), dtype=np.complex128)
        rss = np.empty((self.F, R, R), dtype=np.complex128)
        ws = np.empty((R, self.F, self.T))
        ll = np.zeros(1)
        check(lib.fasst_suff_stat(self._h, R, dptr(V), dptr(mix), dptr(psd), dptr(rxx), dptr(rxs),
                                  dptr(rss), dptr(ws), dptr(ll)), "compute_suff_stat")
        return rxx, rxs, rss, ws, ll[0]

    def mix_solve(self, rss, rxs, mix, kind):
        """update_mix_matrix's solves, mix [R, 2, F] complex128 updated in place."""
        rss = np.ascontiguousarray(rss, dtype=np.complex128)
        rxs = np.ascontiguousarray(rxs, dtype=np.complex128)
        k = np.ascontiguousarray(kind, dtype=np.int32)
        R = k.size
        if mix.dtype != np.complex128 or not mix.flags['C_CONTIGUOUS'] or \
                mix.shape != (R, 2, self.F):
            raise ValueError("mix_matrix must be a C-contiguous complex128 (%d, 2, %d) array"
                             % (R, self.F))
        check(lib.fasst_mix_solve(self.device, self.F, R, dptr(rss), dptr(rxs), dptr(mix),
                                  iptr(k)), "update_mix_matrix")

    def spectral_update(self, hat_W, omega):
        hat_W = np.ascontiguousarray(hat_W, dtype=np.float64)
        if hat_W.shape != (len(self.structure[0]), self.F, self.T):
            raise ValueError("hat_W shape %s" % (hat_W.shape,))
        check(lib.fasst_spectral_update(self._h, dptr(hat_W), float(omega)),
              "update_spectral_components")

    def sigma_comp(self, j, colmask):
        diag = np.empty((2, self.F, self.T))
        off = np.empty((self.F, self.T), dtype=np.complex128)
        m = colmask_words([colmask])
        check(lib.fasst_sigma_comp(self._h, int(j), m.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)),
                                   dptr(diag), dptr(off)),
              "compute_sigma_comp_2d")
        return diag, off

    def inv_sigma_mix(self, diag, off, psd):
        diag = np.ascontiguousarray(diag, dtype=np.float64)
        off = np.ascontiguousarray(off, dtype=np.complex128)
        n = diag.shape[0]
        if diag.shape != (n, 2, self.F, self.T) or off.shape != (n, self.F, self.T):
            raise ValueError("sigma_comps_diag %s / sigma_comps_off %s" % (diag.shape, off.shape))
        psd = np.ascontiguousarray(np.broadcast_to(psd, (self.F,)), dtype=np.float64)
        idiag = np.empty((2, self.F, self.T))
        ioff = np.empty((self.F, self.T), dtype=np.complex128)
        check(lib.fasst_inv_sigma_mix(self.device, n, self.F, self.T, dptr(diag), dptr(off),
                                      dptr(psd), dptr(idiag), dptr(ioff)),
              "compute_inv_sigma_mix_2d")
        return idiag, ioff

    def wiener_images(self, psd, X=None):
        psd = np.ascontiguousarray(psd, dtype=np.float64)
        J = self._nsrc()
        out = np.empty((J, 2, self.F, self.T), dtype=np.complex128)
        xp = None
        if X is not None:
            X = np.ascontiguousarray(X, dtype=np.complex128)
            xp = dptr(X)
        check(lib.fasst_wiener_images(self._h, dptr(psd), xp, dptr(out)), "fasst_wiener_images")
        return out
