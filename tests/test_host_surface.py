"""Host-side pieces of the class surface that need no GPU call."""
import pytest


def test_automatic_melody_and_separation_raises_as_reference():
    """The reference's un-chunked automaticMelodyAndSeparation starts with
    `raise warnings.warn(...)` (SeparateLeadStereoTF.py:1130-1140): a warning,
    then a TypeError (warn returns None), before any step runs."""
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    proc = SL.SeparateLeadProcess(SIMMParams={}, stftParams={})
    with pytest.warns(UserWarning):
        with pytest.raises(TypeError):
            proc.automaticMelodyAndSeparation()
