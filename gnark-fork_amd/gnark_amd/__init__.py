"""gnark_amd -- MI355X-native (gfx950) proving backend for gnark's Groth16 hot path.

Host-side mirror of gnark's icicle build-tag path over the C ABI in
include/gnark_amd.h (libgnark_amd.so).  Importing this package loads the HIP
library and fails loudly if it is missing: there is no CPU fallback.
"""
from ._lib import LIB_PATH, DeviceBuffer, GnarkAmdError, device_count, lib  # noqa: F401
from . import backend, fr, groth16, msm, ntt, witness  # noqa: F401

__all__ = ["backend", "fr", "groth16", "msm", "ntt", "DeviceBuffer", "GnarkAmdError",
           "device_count", "LIB_PATH"]
