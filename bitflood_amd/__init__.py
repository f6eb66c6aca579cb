"""bitflood_amd -- MI355X-native chunk-hash path for bitflood.

Product pieces:
  bitflood_amd/csrc/      HIP kernels (gfx950) + C ABI  -> bitflood_amd/lib/liblbfhash.so
  bitflood_amd/host/      C++ libBitFlood layer (Encoder / FloodFile / verify) -> libbitflood.so
  include/                the public headers of both
  bitflood_amd/hashing.py Python binding used by tests and bench.py

See DESIGN.md for the path, the boundary and the kernels.
"""
from . import _capi  # noqa: F401  (imports torch first: one HIP runtime per process)
from .hashing import (ChunkHasher, DeviceBuffer, LbfError, b64_27, b64_27_decode,  # noqa: F401
                      chunk_table)

__version__ = "0.1.0"
