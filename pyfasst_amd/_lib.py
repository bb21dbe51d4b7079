"""ctypes binding of libfasst_hip.so (declared in include/fasst_hip.h,
include/fasst_simm.h, include/fasst_nmf.h, include/fasst_cqt.h,
include/fasst_viterbi.h and include/fasst_dict.h).

The product path has no CPU fallback: if the HIP library is missing this
module raises at import time, and every compute call raises if the device
call fails.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FASST_HIP_LIB", os.path.join(_HERE, "libfasst_hip.so"))

FASST_OK = 0
FASST_ERR_SHAPE = 1
FASST_ERR_SINGULAR = 2
FASST_ERR_DEVICE = 3
FASST_ERR_OOM = 4
FASST_TW_RESTART = 5
FASST_ERR_UNSUPPORTED = 6

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "pyfasst_amd: HIP library %s not found; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` or "
        "`make -C pyfasst_amd/csrc` (hipcc --offload-arch=gfx950)" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p
_llp = ctypes.POINTER(ctypes.c_longlong)

# name -> (restype, argtypes); must match include/*.h exactly
SIGNATURES = {
    "fasst_abi_version": (ctypes.c_int, []),
    "fasst_last_error": (ctypes.c_char_p, []),
    "fasst_device_count": (ctypes.c_int, [_ip]),
    "fasst_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]),
    "fasst_configure": (ctypes.c_int, [_vp, ctypes.c_int, _ip, _ip, ctypes.c_int]),
    "fasst_configure_types": (ctypes.c_int, [_vp, ctypes.c_int, _ip, _ip, _ip]),
    "fasst_destroy": (ctypes.c_int, [_vp]),
    "fasst_set_audio": (ctypes.c_int, [_vp, _dp, ctypes.c_int, _dp, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int]),
    "fasst_mix_psd": (ctypes.c_int, [_vp, _dp]),
    "fasst_set_cx": (ctypes.c_int, [_vp, _dp]),
    "fasst_get_cx": (ctypes.c_int, [_vp, _dp]),
    "fasst_set_stft": (ctypes.c_int, [_vp, _dp]),
    "fasst_set_spatial": (ctypes.c_int, [_vp, ctypes.c_int, _dp, ctypes.c_int]),
    "fasst_get_spatial": (ctypes.c_int, [_vp, ctypes.c_int, _dp]),
    "fasst_set_spectral": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, _dp, ctypes.c_int,
                                          ctypes.c_int]),
    "fasst_get_spectral": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, _dp]),
    "fasst_set_fw_prior": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "fasst_set_blocks": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _ip, _ip, _ip, _ip]),
    "fasst_set_corr": (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_int, _ip, _ip]),
    "fasst_set_tb": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                    ctypes.c_int]),
    "fasst_get_tb": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _dp, _dp]),
    "fasst_renormalize": (ctypes.c_int, [_vp, _ip]),
    "fasst_run": (ctypes.c_int, [_vp, ctypes.c_int, _dp, ctypes.c_double, _dp, _ip, _ip]),
    "fasst_wiener_images": (ctypes.c_int, [_vp, _dp, _dp, _dp]),
    "fasst_set_sources": (ctypes.c_int, [_vp, ctypes.c_int, _ip, _ip,
                                         ctypes.POINTER(ctypes.c_ulonglong)]),
    "fasst_separate_waveforms": (ctypes.c_int, [_vp, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, _dp]),
    "fasst_stft": (ctypes.c_int, [ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, _dp, _ip]),
    "fasst_istft": (ctypes.c_int, [ctypes.c_int, _dp, ctypes.c_int, _dp, _dp, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, _dp]),
    "fasst_istft_simm": (ctypes.c_int, [ctypes.c_int, _dp, ctypes.c_int, _dp, _dp, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, _dp]),
    "fasst_set_profiling": (ctypes.c_int, [_vp, ctypes.c_int]),
    "fasst_kernel_times": (ctypes.c_int, [_vp, _dp, ctypes.POINTER(ctypes.c_long), ctypes.c_int]),
    "fasst_kernel_name": (ctypes.c_char_p, [ctypes.c_int]),
    "fasst_inv_herm_mat_2d": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, _dp,
                                             _dp]),
    "fasst_source_powers": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_ulonglong), _dp]),
    "fasst_suff_stat": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp,
                                       _dp]),
    "fasst_mix_solve": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp,
                                       _ip]),
    "fasst_spectral_update": (ctypes.c_int, [_vp, _dp, ctypes.c_double]),
    "fasst_sigma_comp": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong),
                                        _dp, _dp]),
    "fasst_inv_sigma_mix": (ctypes.c_int, [ctypes.c_int] * 4 + [_dp, _dp, _dp, _dp, _dp]),
    "fasst_wiener_gain": (ctypes.c_int, [ctypes.c_int, ctypes.c_long, _dp, _dp, _dp, _dp, _dp]),
    # include/fasst_simm.h
    "simm_create": (ctypes.c_int, [ctypes.c_int] * 8 + [ctypes.POINTER(_vp)]),
    "simm_destroy": (ctypes.c_int, [_vp]),
    "simm_set_data": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp]),
    "simm_set_params": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    "simm_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double, ctypes.c_int, _dp]),
    "simm_reco_error": (ctypes.c_int, [_vp, _dp]),
    "simm_separate": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _dp, _dp]),
    "simm_get_params": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    "simm_nf0_product_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_long),
                                               ctypes.POINTER(ctypes.c_long)]),
    # include/fasst_nmf.h
    "nmf_create": (ctypes.c_int, [ctypes.c_int] * 4 + [ctypes.POINTER(_vp)]),
    "nmf_destroy": (ctypes.c_int, [_vp]),
    "nmf_set_data": (ctypes.c_int, [_vp, _dp]),
    "nmf_set_params": (ctypes.c_int, [_vp, _dp, _dp]),
    "nmf_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "nmf_get_params": (ctypes.c_int, [_vp, _dp, _dp]),
    "nmf_wiener_images": (ctypes.c_int, [ctypes.c_int] * 4 + [_dp, _dp, ctypes.c_int, _ip, _dp,
                                                              _dp, _dp]),
    "nmf_wiener_waveforms": (ctypes.c_int, [ctypes.c_int] * 4 + [_dp, _dp, ctypes.c_int, _ip, _dp,
                                                                 _dp, _dp, _dp, ctypes.c_int,
                                                                 ctypes.c_int, ctypes.c_int, _dp]),
    # include/fasst_cqt.h
    "cqt_create": (ctypes.c_int, [ctypes.c_int] * 8 + [_dp, _dp, _dp, _dp] +
                   [ctypes.c_int] * 3 + [_dp, ctypes.POINTER(_vp)]),
    "cqt_destroy": (ctypes.c_int, [_vp]),
    "cqt_shape": (ctypes.c_int, [_vp, ctypes.c_long, _ip, _ip, _ip]),
    "cqt_forward": (ctypes.c_int, [_vp, _dp, ctypes.c_long, _dp]),
    "cqt_inverse": (ctypes.c_int, [_vp, _dp, ctypes.c_long, _dp]),
    "cqt_device_ms": (ctypes.c_int, [_vp, _dp, _dp]),
    "dict_wf0_cqt": (ctypes.c_int, [_vp, ctypes.c_int, _dp, _dp, _ip, ctypes.c_int, _dp,
                                    ctypes.c_double, ctypes.c_long, ctypes.c_int, _dp]),
    # include/fasst_viterbi.h
    "viterbi_tracking": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp,
                                        ctypes.c_long, _dp, _dp, ctypes.c_long, _llp]),
    "viterbi_last_timing": (ctypes.c_int, [_dp, _ip]),
    "viterbi_fallback_count": (ctypes.c_int, [_ip]),
    # include/fasst_dict.h
    "dict_wf0_stft": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _dp, _dp, _ip, ctypes.c_int, _dp,
                                     ctypes.c_double, ctypes.c_int, _dp, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_long, _dp]),
    "dict_last_ms": (ctypes.c_int, [_dp]),
    # include/fasst_nnls.h
    "nnls_columns": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int,
                                    _dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, _dp,
                                    _ip]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

# include/fasst_hip.h FASST_ABI_VERSION these signatures were written against
# (revision 2: 128-bit column sets in fasst_source_powers / fasst_sigma_comp)
ABI_VERSION = 2
if lib.fasst_abi_version() != ABI_VERSION:
    raise ImportError("pyfasst_amd: %s has ABI revision %d, this binding expects %d; rebuild it "
                      "(make -C pyfasst_amd/csrc)" % (LIB_PATH, lib.fasst_abi_version(), ABI_VERSION))


class FasstError(RuntimeError):
    pass


def last_error():
    msg = lib.fasst_last_error()
    return msg.decode() if msg else ""


def check(status, what=""):
    """Map a status code to the reference's exceptions."""
    if status == FASST_OK:
        return
    msg = "%s: %s" % (what, last_error())
    if status == FASST_ERR_SINGULAR:
        raise np.linalg.LinAlgError('Singular Matrix')
    if status == FASST_ERR_SHAPE:
        raise ValueError(msg)
    if status == FASST_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if status == FASST_ERR_OOM:
        raise MemoryError(msg)
    raise FasstError("%s (status %d)" % (msg, status))


def dptr(a):
    """float64 / complex128 C-contiguous array -> double*"""
    assert a.flags['C_CONTIGUOUS'] and a.dtype in (np.float64, np.complex128), (a.dtype, a.flags)
    return a.ctypes.data_as(_dp)


def iptr(a):
    assert a.flags['C_CONTIGUOUS'] and a.dtype == np.int32
    return a.ctypes.data_as(_ip)


def default_device():
    """Device index for this process: FASST_DEVICE, else LOCAL_RANK, else 0."""
    for var in ("FASST_DEVICE", "LOCAL_RANK"):
        if var in os.environ:
            return int(os.environ[var])
    return 0


def device_count():
    n = ctypes.c_int(0)
    check(lib.fasst_device_count(ctypes.byref(n)), "fasst_device_count")
    return n.value
