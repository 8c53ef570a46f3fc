"""ambry_amd -- MI355X-native engine for Ambry's blob CRC-32 path.

Layers:
  include/ambrycrc.h + ambry_amd/csrc/   C ABI and gfx950 kernels (libambrycrc.so)
  ambry_amd.crc32                        mirror of com.github.ambry.utils.Crc32 (host path)
  ambry_amd.device                       device-resident batch / verify over torch HBM
  ambry_amd.multi                        one-process-per-GPU sharding + RCCL all-gather
"""
from ._lib import EXPORTED, LIB_PATH, AmbryCrcError, lib  # noqa: F401
from .crc32 import Crc32, combine, crc32, zeros  # noqa: F401

__all__ = ["Crc32", "crc32", "combine", "zeros", "lib", "LIB_PATH", "EXPORTED", "AmbryCrcError"]
