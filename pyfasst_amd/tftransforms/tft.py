"""Transform registry (tftransforms/tft.py:74-81): the abbreviated names
SeparateLeadProcess and FASST use to build their time-frequency transforms.
STFT, CQT and MinQT run on the GPU; the NSGT ('nsgmqt') is outside the
GPU path."""
from .minqt import CQTransfo, MinQTransfo, sqrt_blackmanharris  # noqa: F401
from .stft import STFT  # noqa: F401

tftransforms = {
    'stft': STFT,
    'mqt': MinQTransfo,
    'minqt': MinQTransfo,
    'cqt': CQTransfo}
"""A convenience dictionary, with abbreviated names for the transforms."""
