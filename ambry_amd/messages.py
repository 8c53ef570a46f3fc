"""PUT message serialization (the write side of Ambry's message path).

Mirrors PutMessageFormatInputStream (PutMessageFormatInputStream.java:60-124): a message is
described by its store key, optional encryption key, BlobPropertiesSerDe bytes, user metadata
and blob content, plus header version / life version / blob type / compression flag. The bytes
and every CRC trailer are produced by libambrycrc -- on the CPU for one message
(ambrycrc_serialize_put_host), on the GPU for a batch (ambrycrc_serialize_puts_dev).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import PutDesc, check, lib

# numpy mirror of struct ambrycrc_put_desc (80 bytes), for descriptor arrays copied to HBM
PUT_DESC_DTYPE = np.dtype([
    ("out_off", "<u8"), ("key_src", "<u8"), ("enckey_src", "<u8"), ("props_src", "<u8"), ("usermeta_src", "<u8"),
    ("blob_src", "<u8"), ("blob_len", "<u8"), ("key_len", "<u4"), ("enckey_len", "<i4"), ("props_len", "<u4"),
    ("usermeta_len", "<u4"), ("life_version", "<i2"), ("blob_type", "<i2"), ("compressed", "u1"),
    ("header_version", "u1"), ("reserved", "u1", (2,))])
assert PUT_DESC_DTYPE.itemsize == ctypes.sizeof(PutDesc) == 80

FIELDS = ("key", "enckey", "props", "usermeta", "blob")


@dataclass
class PutMessage:
    """One PUT: the arguments of PutMessageFormatInputStream's constructor, as bytes."""
    key: bytes                # StoreKey.toBytes()
    props: bytes              # BlobPropertiesSerDe bytes
    usermeta: bytes
    blob: bytes
    enckey: bytes | None = None
    header_version: int = 3   # MessageFormatRecord.headerVersionToUse
    life_version: int = 0
    blob_type: int = 0        # BlobType ordinal (0 = DataBlob)
    compressed: bool = False

    def desc(self, out_off: int = 0, src: dict | None = None) -> PutDesc:
        src = src or {}
        d = PutDesc()
        d.out_off = out_off
        d.key_src, d.enckey_src, d.props_src = src.get("key", 0), src.get("enckey", 0), src.get("props", 0)
        d.usermeta_src, d.blob_src = src.get("usermeta", 0), src.get("blob", 0)
        d.blob_len = len(self.blob)
        d.key_len, d.props_len, d.usermeta_len = len(self.key), len(self.props), len(self.usermeta)
        d.enckey_len = -1 if self.enckey is None else len(self.enckey)
        d.life_version, d.blob_type = self.life_version, self.blob_type
        d.compressed, d.header_version = 1 if self.compressed else 0, self.header_version
        return d


def layout(msg: PutMessage):
    """(message length, {field: offset from the message start}) -- ambrycrc_put_layout."""
    offs = (ctypes.c_uint64 * 5)()
    n = lib().ambrycrc_put_layout(ctypes.byref(msg.desc()), offs)
    if n == 0:
        raise ValueError("invalid PUT descriptor")
    return n, dict(zip(FIELDS, list(offs)))


def serialize_host(msg: PutMessage):
    """(message bytes, [header, enckey, props, usermeta, blob record CRCs]) on the CPU."""
    fields = b"".join([msg.key, msg.enckey or b"", msg.props, msg.usermeta])
    src = {"key": 0, "enckey": len(msg.key), "props": len(msg.key) + len(msg.enckey or b""),
           "usermeta": len(msg.key) + len(msg.enckey or b"") + len(msg.props), "blob": 0}
    n, _ = layout(msg)
    out = ctypes.create_string_buffer(max(n, 1))
    fb = ctypes.create_string_buffer(fields, max(len(fields), 1))
    bb = ctypes.create_string_buffer(msg.blob, max(len(msg.blob), 1))
    crcs = (ctypes.c_uint32 * 5)()
    check(lib().ambrycrc_serialize_put_host(ctypes.byref(msg.desc(0, src)), fb, bb, out, n, crcs),
          "ambrycrc_serialize_put_host")
    return out.raw[:n], list(crcs)


def pack_batch(msgs, out_align: int = 1, field_align: int = 1, gap: int = 0):
    """Host-side packing for ambrycrc_serialize_puts_dev: (descriptor array, fields bytes, blobs
    bytes, message offsets, total output bytes). Fields go back to back (each at field_align),
    blobs likewise, messages at out_align with `gap` spare bytes between them."""
    descs = np.zeros(len(msgs), dtype=PUT_DESC_DTYPE)
    fields, blobs = bytearray(), bytearray()
    offs, pos = [], 0
    for i, m in enumerate(msgs):
        src = {}
        for name in FIELDS[:4]:
            b = getattr(m, name) or b""
            fields += bytes((-len(fields)) % field_align)
            src[name] = len(fields)
            fields += b
        blobs += bytes((-len(blobs)) % field_align)
        src["blob"] = len(blobs)
        blobs += m.blob
        pos += (-pos) % out_align
        offs.append(pos)
        d = m.desc(pos, src)
        descs[i] = np.frombuffer(bytes(d), dtype=PUT_DESC_DTYPE)[0]
        pos += layout(m)[0] + gap
    return descs, bytes(fields), bytes(blobs), offs, pos


def serialize_dev(descs, out, fields=None, blobs=None, msg_len=None, stream=None):
    """ambrycrc_serialize_puts_dev: descs is a uint8 CUDA tensor holding the PUT_DESC_DTYPE array;
    fields / blobs uint8 CUDA tensors or None (bytes already in place in `out`)."""
    import torch

    from .device import _stream_handle

    if descs.dtype != torch.uint8 or not descs.is_cuda or descs.numel() % PUT_DESC_DTYPE.itemsize:
        raise TypeError("descs must be a uint8 CUDA tensor of 80-byte descriptors")
    m = descs.numel() // PUT_DESC_DTYPE.itemsize
    for name, t in (("out", out), ("fields", fields), ("blobs", blobs)):
        if t is not None and (t.dtype != torch.uint8 or not t.is_cuda or t.device != descs.device):
            raise TypeError(f"{name} must be a uint8 CUDA tensor on {descs.device}")
    if msg_len is not None and (msg_len.dtype != torch.int64 or msg_len.numel() != m or not msg_len.is_cuda):
        raise TypeError("msg_len must be an int64 CUDA tensor of m elements")
    ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    check(lib().ambrycrc_serialize_puts_dev(ptr(descs), m, ptr(fields), ptr(blobs), ptr(out), ptr(msg_len), None, 0,
                                            ctypes.c_void_p(_stream_handle(stream))), "ambrycrc_serialize_puts_dev")


def verify_message_cpu(region, off: int):
    """ambrycrc_verify_message_cpu: (AMBRYCRC_MSG_* status bits, message end or 0) for the message
    at `off` in a host buffer (bytes / bytearray / uint8 numpy array)."""
    buf = np.frombuffer(region, dtype=np.uint8) if not isinstance(region, np.ndarray) else region
    st, end = ctypes.c_uint32(0), ctypes.c_uint64(0)
    check(lib().ambrycrc_verify_message_cpu(buf.ctypes.data_as(ctypes.c_void_p), buf.size, off, ctypes.byref(st),
                                            ctypes.byref(end)), "ambrycrc_verify_message_cpu")
    return st.value, end.value


def transform_message_cpu(region, off: int, header_version: int = 3, life=None, out_cap=None):
    """ambrycrc_transform_message_cpu: (status bits, the re-serialized message or None)."""
    buf = np.frombuffer(region, dtype=np.uint8) if not isinstance(region, np.ndarray) else region
    # default: the ABI's bound (the stored bytes after off + TRANSFORM_GROWTH_MAX), never NO_ROOM
    cap = out_cap if out_cap is not None else out_bound(buf.size - min(off, buf.size), 1)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    st, n = ctypes.c_uint32(0), ctypes.c_uint64(0)
    check(lib().ambrycrc_transform_message_cpu(buf.ctypes.data_as(ctypes.c_void_p), buf.size, off,
                                               -1 if life is None else int(life), header_version,
                                               out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n),
                                               ctypes.byref(st)), "ambrycrc_transform_message_cpu")
    return st.value, (out[:n.value].tobytes() if st.value == 0 else None)


# status bits added by the transform (include/ambrycrc.h)
MSG_NOT_PUT = 1 << 10
MSG_BAD_RECORD = 1 << 11
MSG_NO_ROOM = 1 << 12
MSG_NOT_ENCODABLE = 1 << 13

# A transformed message is at most this many bytes longer than the stored one: header V1 -> V3 (+6),
# BlobProperties SerDe V1 -> V5 (+17), Blob_Format_V1 -> V3 head (+3) (AMBRYCRC_TRANSFORM_GROWTH_MAX).
TRANSFORM_GROWTH_MAX = 26


def out_bound(region_len: int, m: int) -> int:
    """ambrycrc_transform_out_bound: an output capacity that never yields MSG_NO_ROOM for m
    messages that share no bytes of a region_len-byte region."""
    return int(lib().ambrycrc_transform_out_bound(region_len, m))


def transform_dev(region, msg_off, header_version: int = 3, life_version=None, out=None, stream=None):
    """ambrycrc_transform_messages_dev -- ValidatingTransformer.transform for a batch of stored
    messages in HBM: every clean PUT re-serialized at `header_version` (and life version
    life_version[i], an int16 CUDA tensor, or the stored one), packed in order into `out` (a uint8
    CUDA tensor; default: out_bound(region bytes, m), enough for every message of a region whose
    messages do not overlap -- TRANSFORM_GROWTH_MAX = 26 B of growth per message).
    Returns (out, out_off int64[m], out_len int64[m], status int32[m])."""
    import torch

    from .device import _stream_handle

    if region.dtype != torch.uint8 or not region.is_cuda:
        raise TypeError("region must be a uint8 CUDA tensor")
    if msg_off.dtype != torch.int64 or not msg_off.is_cuda or not msg_off.is_contiguous() or \
            msg_off.device != region.device:
        raise TypeError("msg_off must be a contiguous int64 CUDA tensor on the region's device")
    m = msg_off.numel()
    if life_version is not None and (life_version.dtype != torch.int16 or life_version.numel() != m
                                     or not life_version.is_cuda or not life_version.is_contiguous()):
        raise TypeError("life_version must be a contiguous int16 CUDA tensor of m elements")
    if out is None:
        out = torch.empty(out_bound(region.numel(), m), dtype=torch.uint8, device=region.device)
    elif out.dtype != torch.uint8 or not out.is_cuda or not out.is_contiguous() or out.device != region.device:
        raise TypeError("out must be a contiguous uint8 CUDA tensor on the region's device")
    out_off = torch.empty(m, dtype=torch.int64, device=region.device)
    out_len = torch.empty(m, dtype=torch.int64, device=region.device)
    status = torch.empty(m, dtype=torch.int32, device=region.device)
    ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    check(lib().ambrycrc_transform_messages_dev(ptr(region), region.numel(), ptr(msg_off), m, ptr(life_version),
                                                header_version, ptr(out), out.numel(), ptr(out_off), ptr(out_len),
                                                ptr(status), None, 0, ctypes.c_void_p(_stream_handle(stream))),
          "ambrycrc_transform_messages_dev")
    return out, out_off, out_len, status


def transform_host(region, msg_off, header_version: int = 3, life_version=None, out_cap=None, device: int = 0,
                   pinned: bool = False):
    """ambrycrc_transform_messages_host: the batched transform of a region in host memory (bytes,
    bytearray, uint8 numpy array or uint8 CPU tensor; pinned=True for a pin_memory() tensor), staged
    through the pinned slabs. Returns (out bytes packed in message order, out_off int64[m] (-1: not
    transformed), out_len int64[m], status uint32[m])."""
    if hasattr(region, "data_ptr"):
        base, n = region.data_ptr(), region.numel()
        keep = region
    else:
        keep = np.frombuffer(region, dtype=np.uint8) if not isinstance(region, np.ndarray) else region
        base, n = keep.ctypes.data, keep.size
    offs = np.ascontiguousarray(np.asarray(msg_off, dtype=np.uint64))
    m = offs.size
    cap = out_bound(n, m) if out_cap is None else int(out_cap)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    life = None if life_version is None else np.ascontiguousarray(np.asarray(life_version, dtype=np.int16))
    oo = np.zeros(m, dtype=np.uint64)
    ol = np.zeros(m, dtype=np.uint64)
    st = np.zeros(m, dtype=np.uint32)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    check(lib().ambrycrc_transform_messages_host(
        ctypes.c_void_p(base), n, offs.ctypes.data_as(u64p), m, None if life is None else life.ctypes.data,
        header_version, out.ctypes.data, cap, oo.ctypes.data_as(u64p), ol.ctypes.data_as(u64p),
        st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), device, 1 if pinned else 0),
        "ambrycrc_transform_messages_host")
    del keep
    used = int((oo[st == 0] + ol[st == 0]).max()) if (st == 0).any() else 0
    return out[:used].tobytes(), oo.view(np.int64), ol.view(np.int64), st
