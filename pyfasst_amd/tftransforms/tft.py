"""Transform registry (tftransforms/tft.py).  Only the STFT is on the HIP
path; CQT / MinQT / NSGT are outside this round's scope."""
from .stft import STFT  # noqa: F401
