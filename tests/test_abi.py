"""The C-ABI library loads and exports every symbol declared in include/*.h.

CPU-only: no compute call is made (there is no GPU in the build container).
"""
import ctypes
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        syms |= set(re.findall(r"\b((?:fasst|simm|nmf|cqt|viterbi|dict|nnls)_\w+)\s*\(", src))
    return sorted(syms)


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("fasst_create", "fasst_configure", "fasst_run", "fasst_wiener_images",
              "fasst_stft", "fasst_istft", "fasst_inv_herm_mat_2d", "fasst_destroy",
              "simm_create", "simm_run", "simm_set_params", "simm_get_params"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from pyfasst_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # and the ctypes table binds exactly the declared set
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_library_is_gfx950_code_object():
    from pyfasst_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_step_abi_refuses_bad_shapes_before_touching_a_device():
    """The GEM step entry points validate their arguments on the host first:
    a free 'conv' rank next to other ranks (the reference's solve raises,
    audioModel.py:856-857) and a total rank above 16 return FASST_ERR_SHAPE
    with a message, no device call."""
    import numpy as np
    from pyfasst_amd import _lib
    F, R = 5, 3
    rss = np.zeros((F, R, R), complex)
    rxs = np.zeros((F, 2, R), complex)
    mix = np.zeros((R, 2, F), complex)
    kind = np.array([2, 0, 1], dtype=np.int32)
    st = _lib.lib.fasst_mix_solve(0, F, R, _lib.dptr(rss), _lib.dptr(rxs), _lib.dptr(mix),
                                  _lib.iptr(kind))
    assert st == _lib.FASST_ERR_SHAPE
    assert "conv" in _lib.last_error()
    st = _lib.lib.fasst_suff_stat(None, 17, *([None] * 8))
    assert st == _lib.FASST_ERR_SHAPE


def test_abi_revision_matches_header_and_binding():
    """The header's FASST_ABI_VERSION, the library's fasst_abi_version() and
    the binding's ABI_VERSION agree (the loader refuses a library of another
    revision: a revision-1 caller of fasst_source_powers passed one mask word
    per component where revision 2 reads two)."""
    from pyfasst_amd import _lib
    src = open(os.path.join(ROOT, "include", "fasst_hip.h")).read()
    hdr = int(re.search(r"#define FASST_ABI_VERSION (\d+)", src).group(1))
    assert _lib.lib.fasst_abi_version() == hdr == _lib.ABI_VERSION
