"""mkids_sdr_amd — MI355X-native MKID channeliser + phase / photon-pulse trigger.

Hot path (HIP, gfx950, libmkidgpu.so through the C ABI of include/mkidgpu.h):
  PFB + FFT + bin select + DDC -> 26-tap IQ low-pass /2 -> centre + atan2 -> matched filter +
  baseline + threshold + peak -> 64-bit photon packets.
Host side (this package): the ChannelizerControls setup surface of the reference (LUTs, bins,
FIR taps, centres, thresholds) and an FpgaClient-compatible register shim.
"""
from . import _lib  # noqa: F401

__all__ = ['_lib']
