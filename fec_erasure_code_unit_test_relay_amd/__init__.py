"""MI355X-native GF(2^8) streaming-erasure codec (drop-in for the coding path of
domanovi/FEC_Erasure_Code_Unit_Test_Relay).

The product is the in-tree HIP library ``libfec_amd.so`` (kernels for gfx950 + C ABI,
include/fec_amd.h) and the reference-named C++ classes in include/fec_amd_dropin.h.  This Python
package mirrors the reference's FEC_Encoder / FEC_Decoder interface and exposes the batched,
device-resident API used by bench.py and the tests.
"""
from ._lib import LIB_PATH, FecError, lib  # noqa: F401
from .codec import Codec, DecodeStream, FEC_Decoder, FEC_Encoder, StreamGroup, plan_host  # noqa: F401
from .payload import fill_payload  # noqa: F401

__all__ = ["Codec", "DecodeStream", "StreamGroup", "FEC_Encoder", "FEC_Decoder", "FecError", "plan_host", "fill_payload", "lib",
           "LIB_PATH"]
