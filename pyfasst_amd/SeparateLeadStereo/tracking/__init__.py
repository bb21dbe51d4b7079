"""Viterbi melody tracking on the GPU (SeparateLeadStereo/tracking of the reference)."""
