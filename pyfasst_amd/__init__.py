"""pyfasst_amd -- MI355X-native FASST EM engine (drop-in for pyfasst's hot path).

Modules mirror the reference layout: `audioModel` (FASST,
MultiChanNMFInst_FASST, MultiChanNMFConv), `audioObject`,
`tftransforms.stft`, `tools.signalTools`.  All compute runs in
libfasst_hip.so (HIP, gfx950); importing the package fails loudly if the
library is missing.
"""
from . import _lib  # noqa: F401  (raises ImportError when libfasst_hip.so is absent)

__version__ = "0.1.0"
