"""ctypes binding of libambrycrc.so (the C ABI declared in include/ambrycrc.h).

The shared library is built in-tree (``make -C ambry_amd`` or
``__graft_entry__.build()``). There is no fallback: if the library is missing
or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# AMBRYCRC_LIBRARY names another build of the same library (A/B timing of two kernel builds on
# one box, tools/ab_cases.sh); default: the in-tree build.
LIB_PATH = os.environ.get("AMBRYCRC_LIBRARY") or os.path.join(_HERE, "libambrycrc.so")

AMBRYCRC_OK = 0
AMBRYCRC_EINVAL = -1
AMBRYCRC_EHIP = -2
AMBRYCRC_ENOMEM = -3
AMBRYCRC_ENOINIT = -4
AMBRYCRC_ENODEV = -5
AMBRYCRC_ECOMM = -6
AMBRYCRC_EPROBE = -7
UNIQUE_ID_BYTES = 128


class Shard(ctypes.Structure):
    """struct ambrycrc_shard (include/ambrycrc.h): one GPU's part of a multi-GPU batch."""
    _fields_ = [("device", ctypes.c_int), ("d_base", ctypes.c_void_p), ("d_off", ctypes.c_void_p),
                ("d_len", ctypes.c_void_p), ("d_crc_in", ctypes.c_void_p), ("n", ctypes.c_size_t),
                ("d_gathered", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


class PutDesc(ctypes.Structure):
    """struct ambrycrc_put_desc (include/ambrycrc.h): one PUT message to serialize (80 bytes)."""
    _fields_ = [("out_off", ctypes.c_uint64), ("key_src", ctypes.c_uint64), ("enckey_src", ctypes.c_uint64),
                ("props_src", ctypes.c_uint64), ("usermeta_src", ctypes.c_uint64), ("blob_src", ctypes.c_uint64),
                ("blob_len", ctypes.c_uint64), ("key_len", ctypes.c_uint32), ("enckey_len", ctypes.c_int32),
                ("props_len", ctypes.c_uint32), ("usermeta_len", ctypes.c_uint32), ("life_version", ctypes.c_int16),
                ("blob_type", ctypes.c_int16), ("compressed", ctypes.c_uint8), ("header_version", ctypes.c_uint8),
                ("reserved", ctypes.c_uint8 * 2)]


assert ctypes.sizeof(PutDesc) == 80

# (name, restype, argtypes) for every symbol include/ambrycrc.h declares.
_u8p = ctypes.c_void_p
_SIGNATURES = [
    ("ambrycrc_init", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_shutdown", ctypes.c_int, []),
    ("ambrycrc_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("ambrycrc_version", ctypes.c_char_p, []),
    ("ambrycrc_update", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    ("ambrycrc_update_byte", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_int]),
    ("ambrycrc_host_impl", ctypes.c_char_p, []),
    ("ambrycrc_update_iov", ctypes.c_uint32,
     [ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t]),
    ("ambrycrc_combine", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    ("ambrycrc_zeros", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint64]),
    ("ambrycrc_workspace_bytes", ctypes.c_size_t, [ctypes.c_size_t]),
    ("ambrycrc_batch_dev", ctypes.c_int,
     [_u8p, _u8p, _u8p, _u8p, _u8p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("ambrycrc_verify_dev", ctypes.c_int,
     [_u8p, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
      ctypes.c_void_p]),
    ("ambrycrc_messages_workspace_bytes", ctypes.c_size_t, [ctypes.c_size_t]),
    ("ambrycrc_verify_messages_dev", ctypes.c_int,
     [_u8p, ctypes.c_uint64, _u8p, ctypes.c_size_t, _u8p, _u8p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("ambrycrc_verify_messages_host", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
      ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_put_layout", ctypes.c_uint64, [ctypes.POINTER(PutDesc), ctypes.POINTER(ctypes.c_uint64)]),
    ("ambrycrc_serialize_put_host", ctypes.c_int,
     [ctypes.POINTER(PutDesc), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
      ctypes.POINTER(ctypes.c_uint32)]),
    ("ambrycrc_serialize_puts_workspace_bytes", ctypes.c_size_t, [ctypes.c_size_t]),
    ("ambrycrc_serialize_puts_dev", ctypes.c_int,
     [_u8p, ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("ambrycrc_transform_workspace_bytes", ctypes.c_size_t, [ctypes.c_size_t]),
    ("ambrycrc_transform_out_bound", ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_size_t]),
    ("ambrycrc_transform_messages_dev", ctypes.c_int,
     [_u8p, ctypes.c_uint64, _u8p, ctypes.c_size_t, _u8p, ctypes.c_int, _u8p, ctypes.c_uint64, _u8p, _u8p, _u8p,
      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("ambrycrc_transform_messages_host", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int,
      ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
      ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_trailed_workspace_bytes", ctypes.c_size_t, [ctypes.c_size_t]),
    ("ambrycrc_verify_trailed_dev", ctypes.c_int,
     [_u8p, _u8p, _u8p, _u8p, _u8p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("ambrycrc_verify_trailed_host", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint8),
      ctypes.c_size_t, ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_chain_messages_host", ctypes.c_size_t,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]),
    ("ambrycrc_verify_message_cpu", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32),
      ctypes.POINTER(ctypes.c_uint64)]),
    ("ambrycrc_transform_message_cpu", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
      ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]),
    ("ambrycrc_batch_host", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
      ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_batch_multi", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
      ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_batch_cpu", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
      ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_int]),
    ("ambrycrc_shard_by_bytes", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    ("ambrycrc_gather_layout", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int),
      ctypes.POINTER(ctypes.c_uint64)]),
    ("ambrycrc_gather_compact_host", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_void_p]),
    ("ambrycrc_unique_id", ctypes.c_int, [ctypes.POINTER(ctypes.c_uint8)]),
    ("ambrycrc_comm_init_all", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("ambrycrc_comm_init_rank", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("ambrycrc_comm_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("ambrycrc_comm_size", ctypes.c_int, [ctypes.c_void_p]),
    ("ambrycrc_batch_dev_multi", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Shard), ctypes.c_int]),
    ("ambrycrc_batch_dev_gather", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(Shard), ctypes.POINTER(ctypes.c_uint64)]),
    ("ambrycrc_put_crcs", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_void_p),
      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64),
      ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    ("ambrycrc_range_checksums_host", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
      ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
    ("ambrycrc_set_variant", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_get_variant", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_set_region_mode", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_get_region_mode", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_last_message_mode", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_last_transform_path", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_set_transform_verdict", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_set_put_stream_max", ctypes.c_long, [ctypes.c_int, ctypes.c_long]),
    ("ambrycrc_set_host_policy", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_host_rates", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    ("ambrycrc_last_host_path", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_set_host_cpu_threads", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_host_calibrate", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    ("ambrycrc_host_msg_rates", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    ("ambrycrc_set_grid", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_set_window", ctypes.c_int, [ctypes.c_int, ctypes.c_uint64]),
    ("ambrycrc_timing_enable", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("ambrycrc_timing_collect", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    ("ambrycrc_timing_collect_each", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    ("ambrycrc_grid_size", ctypes.c_int, [ctypes.c_int]),
    ("ambrycrc_fill_random_dev", ctypes.c_int,
     [_u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]),
    ("ambrycrc_debug_readbw_dev", ctypes.c_int, [_u8p, ctypes.c_uint64, _u8p, ctypes.c_int, ctypes.c_void_p]),
    ("ambrycrc_debug_table_image", ctypes.c_long, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]),
]

EXPORTED = [s[0] for s in _SIGNATURES]

_lock = threading.Lock()
_lib = None


class AmbryCrcError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})")


def lib() -> ctypes.CDLL:
    """Load libambrycrc.so (raises if it is absent: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not built; run `make -C {_HERE}` or __graft_entry__.build()")
            handle = ctypes.CDLL(LIB_PATH)
            for name, res, args in _SIGNATURES:
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def strerror(code: int) -> str:
    return lib().ambrycrc_strerror(code).decode()


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise AmbryCrcError(rc, what)
    return rc
