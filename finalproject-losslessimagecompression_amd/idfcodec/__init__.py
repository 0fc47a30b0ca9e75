"""idfcodec -- MI355X-native (gfx950) integer-discrete-flow + rANS lossless image codec.

Native core: libidfcodec.so (HIP, C ABI in include/idf_codec.h).  This package
holds the host side: ctypes binding (_lib), weight packing (packing), the flow
engine (engine), the batched coder and bitstream container (codec), the
synthetic-weight recipe (synthetic) and the multi-GPU shard/gather (dist).
"""
import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    # the reference-API mirror modules (flows, coder, rans, ...) live next to this package
    sys.path.insert(0, _PKG_ROOT)

__version__ = "0.1.0"
