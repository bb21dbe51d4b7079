"""`import pyfasst.<module>` (the reference's import name,
doc/source/description.rst:50-100) serves the MI355X package's modules."""
import importlib

import pytest


@pytest.mark.parametrize("name", ["audioModel", "audioObject", "tools.nmf", "tools.signalTools",
                                  "tftransforms.stft", "tftransforms.minqt",
                                  "SeparateLeadStereo.SIMM.SIMM",
                                  "SeparateLeadStereo.SeparateLeadStereoTF",
                                  "SeparateLeadStereo.tracking.tracking"])
def test_alias_is_same_module(name):
    a = importlib.import_module("pyfasst." + name)
    b = importlib.import_module("pyfasst_amd." + name)
    assert a is b
    assert b.__spec__.name == "pyfasst_amd." + name


def test_alias_classes_and_missing_modules():
    import pyfasst.audioModel as am
    import pyfasst_amd.audioModel as am2
    assert am.MultiChanNMFConv is am2.MultiChanNMFConv
    from pyfasst.tools import nmf
    assert callable(nmf.NMF_decomposition)
    with pytest.raises(ImportError):
        importlib.import_module("pyfasst.demixTF")   # out of scope
