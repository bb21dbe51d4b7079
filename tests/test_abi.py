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
