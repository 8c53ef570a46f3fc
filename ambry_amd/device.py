"""Device-resident batch API over torch-allocated HBM (thin layer on the C ABI).

Torch is only plumbing here: it allocates HBM and provides the stream; every
CRC is computed by libambrycrc's gfx950 kernels via ``ambrycrc_batch_dev`` /
``ambrycrc_verify_dev``. Offsets/lengths are int64 device tensors (uint64 in
the ABI), CRCs are int32 device tensors holding the uint32 bit patterns
(``.view(torch.uint32)`` / numpy ``.view(np.uint32)`` to read them).
"""
from __future__ import annotations

import ctypes

from ._lib import UNIQUE_ID_BYTES, Shard, check, lib


def _torch():
    import torch  # deferred: CPU-only tests import this module without a GPU

    return torch


def _stream_handle(stream=None) -> int:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _ptr(t) -> ctypes.c_void_p | None:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def init(device: int = 0) -> None:
    check(lib().ambrycrc_init(device), f"ambrycrc_init({device})")


def _check_batch(base, off, length, n):
    torch = _torch()
    if base.dtype != torch.uint8 or not base.is_cuda:
        raise TypeError("base must be a uint8 CUDA tensor")
    for name, t in (("off", off), ("len", length)):
        if t.dtype != torch.int64 or not t.is_cuda or t.numel() != n or not t.is_contiguous():
            raise TypeError(f"{name} must be a contiguous int64 CUDA tensor of {n} elements")
        if t.device != base.device:
            raise TypeError(f"{name} must be on {base.device}")


def _check_u32(name, t, n, device):
    """crc_in / out / expected: a contiguous int32 or uint32 CUDA tensor of n elements on `device`."""
    torch = _torch()
    if t is None:
        return
    if t.dtype not in (torch.int32, torch.uint32) or not t.is_cuda or t.numel() != n or not t.is_contiguous():
        raise TypeError(f"{name} must be a contiguous int32/uint32 CUDA tensor of {n} elements")
    if t.device != device:
        raise TypeError(f"{name} must be on {device}")


def _workspace(workspace, device):
    """(pointer, byte size) of a caller workspace (any dtype: its byte size is what counts)."""
    if workspace is None:
        return None, 0
    if not workspace.is_cuda or not workspace.is_contiguous() or workspace.device != device:
        raise TypeError(f"workspace must be a contiguous CUDA tensor on {device}")
    return _ptr(workspace), workspace.numel() * workspace.element_size()


def crc32_batch(base, off, length, crc_in=None, out=None, workspace=None, stream=None):
    """out[i] = crc32(crc_in[i] or 0, base[off[i]:off[i]+len[i]]) for every chunk i (on the GPU).
    out may be crc_in itself (an in-place continuation)."""
    torch = _torch()
    n = off.numel()
    _check_batch(base, off, length, n)
    _check_u32("crc_in", crc_in, n, base.device)
    _check_u32("out", out, n, base.device)
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    ws, ws_bytes = _workspace(workspace, base.device)
    check(lib().ambrycrc_batch_dev(_ptr(base), _ptr(off), _ptr(length), _ptr(crc_in), _ptr(out), n, ws, ws_bytes,
                                   ctypes.c_void_p(_stream_handle(stream))), "ambrycrc_batch_dev")
    return out


def crc32_verify(base, off, length, expected, crc_in=None, out=None, stream=None, mismatch=None,
                 count=True):
    """Returns (crc int32[n], mismatch uint8[n], mismatch_count int32[1] or None) computed on the GPU.
    mismatch: optional preallocated uint8[n]; count=False skips the counter (and its zeroing)."""
    torch = _torch()
    n = off.numel()
    _check_batch(base, off, length, n)
    for name, t in (("crc_in", crc_in), ("out", out), ("expected", expected)):
        _check_u32(name, t, n, base.device)
    if expected is None:
        raise TypeError("expected is required")
    if mismatch is not None and (mismatch.dtype != torch.uint8 or not mismatch.is_cuda or mismatch.numel() != n
                                 or not mismatch.is_contiguous() or mismatch.device != base.device):
        raise TypeError(f"mismatch must be a contiguous uint8 CUDA tensor of {n} elements on {base.device}")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    if mismatch is None:
        mismatch = torch.empty(n, dtype=torch.uint8, device=base.device)
    count = torch.zeros(1, dtype=torch.int32, device=base.device) if count else None
    check(lib().ambrycrc_verify_dev(_ptr(base), _ptr(off), _ptr(length), _ptr(crc_in), _ptr(expected), _ptr(out),
                                    _ptr(mismatch), _ptr(count), n, None, 0,
                                    ctypes.c_void_p(_stream_handle(stream))), "ambrycrc_verify_dev")
    return out, mismatch, count


def fill_random(buf, seed: int, stream_off: int = 0, stream=None) -> None:
    """Deterministic splitmix64 bytes (same stream as oracle_fill_splitmix)."""
    torch = _torch()
    if buf.dtype != torch.uint8 or not buf.is_cuda or not buf.is_contiguous():
        raise TypeError("buf must be a contiguous uint8 CUDA tensor")
    check(lib().ambrycrc_fill_random_dev(_ptr(buf), buf.numel(), seed & (2**64 - 1), stream_off,
                                         ctypes.c_void_p(_stream_handle(stream))), "ambrycrc_fill_random_dev")


def _host_chunks(chunks, crc_in):
    n = len(chunks)
    ptrs = (ctypes.c_void_p * n)()
    lens = (ctypes.c_uint64 * n)()
    for i, c in enumerate(chunks):
        if isinstance(c, tuple):
            ptrs[i], lens[i] = c
        else:
            ptrs[i], lens[i] = c.data_ptr(), c.numel()
    cin = None
    if crc_in is not None:
        cin = (ctypes.c_uint32 * n)(*[int(x) & 0xFFFFFFFF for x in crc_in])
    return n, ptrs, lens, cin


def crc32_batch_host(chunks, device: int = 0, pinned: bool = False, crc_in=None):
    """CRC of host buffers through pinned staging + hipMemcpyAsync (PCIe-inclusive path).

    ``chunks``: sequence of objects exposing ``data_ptr()``/``numel()`` (uint8
    CPU tensors) or (address, length) tuples.
    """
    n, ptrs, lens, cin = _host_chunks(chunks, crc_in)
    out = (ctypes.c_uint32 * n)()
    check(lib().ambrycrc_batch_host(ptrs, lens, cin, out, n, device, 1 if pinned else 0), "ambrycrc_batch_host")
    return list(out)


def crc32_batch_multi(chunks, devices, pinned: bool = False, crc_in=None):
    """ambrycrc_batch_multi: host chunks split by bytes over ``devices`` (one host thread each)."""
    n, ptrs, lens, cin = _host_chunks(chunks, crc_in)
    out = (ctypes.c_uint32 * n)()
    devs = (ctypes.c_int * len(devices))(*devices)
    check(lib().ambrycrc_batch_multi(ptrs, lens, cin, out, n, devs, len(devices), 1 if pinned else 0),
          "ambrycrc_batch_multi")
    return list(out)


def set_variant(device: int, variant: int) -> None:
    check(lib().ambrycrc_set_variant(device, variant), "ambrycrc_set_variant")


def get_variant(device: int = 0) -> int:
    return check(lib().ambrycrc_get_variant(device), "ambrycrc_get_variant")


def set_region_mode(device: int, mode) -> None:
    """Message verify form (ambrycrc_set_region_mode): 2 = region mode in two passes (the
    default), 1 / True = region mode in one pass, 0 / False = CRC jobs through the batch engine.
    The transform's one-pass fast path runs whenever region mode is on (1 or 2)."""
    m = int(mode) if not isinstance(mode, bool) else (1 if mode else 0)
    check(lib().ambrycrc_set_region_mode(device, m), "ambrycrc_set_region_mode")


def get_region_mode(device: int = 0) -> int:
    return check(lib().ambrycrc_get_region_mode(device), "ambrycrc_get_region_mode")


def last_message_mode(device: int = 0) -> int:
    """The form the device's last message verify took: 0 jobs, 1 region one-pass, 2 region two-pass
    (-1: none yet); ambrycrc_last_message_mode."""
    return lib().ambrycrc_last_message_mode(device)


def last_transform_path(device: int = 0) -> int:
    """The path the device's last transform took: 1 the one-pass fast path, 0 the general path
    (-1: none yet); ambrycrc_last_transform_path."""
    return lib().ambrycrc_last_transform_path(device)


def set_transform_verdict(device: int, host: bool) -> int:
    """How the transform learns whether its fast path took the batch (ambrycrc_set_transform_verdict):
    False = on the device, the call stays asynchronous (the default); True = read back by the
    calling thread (one stream synchronization, no gated dispatches). Returns the previous value."""
    return check(lib().ambrycrc_set_transform_verdict(device, 1 if host else 0), "ambrycrc_set_transform_verdict")


def set_put_stream_max(device: int, nbytes: int) -> int:
    """Serialize copy mode streams messages of at most nbytes (ambrycrc_set_put_stream_max; 6144 the default,
    0 = every message through the job path). Returns the previous value."""
    return check(lib().ambrycrc_set_put_stream_max(device, int(nbytes)), "ambrycrc_set_put_stream_max")


HOST_AUTO, HOST_GPU, HOST_CPU = 0, 1, 2


def set_host_policy(device: int, policy: int) -> int:
    """Host-resident dispatch of the *_host entries (ambrycrc_set_host_policy): HOST_AUTO (the
    default: the CPU leg for pageable bytes when the CPU threads beat the GPU host path), HOST_GPU,
    HOST_CPU. Returns the previous policy."""
    return check(lib().ambrycrc_set_host_policy(device, int(policy)), "ambrycrc_set_host_policy")


def host_rates(device: int = 0) -> dict:
    """The rates the auto policy compares (ambrycrc_host_rates) and the leg it takes for pageable bytes."""
    c, g, t = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    leg = check(lib().ambrycrc_host_rates(device, ctypes.byref(c), ctypes.byref(g), ctypes.byref(t)),
                "ambrycrc_host_rates")
    return {"cpu_gibps": c.value, "gpu_gibps": g.value, "cpu_threads": t.value, "auto_leg": "gpu" if leg else "cpu"}


def set_host_cpu_threads(device: int, threads: int) -> int:
    """The CPU leg's thread budget on `device` (-1: the process's; 0: the default, half this process's CPU
    share) -- ambrycrc_set_host_cpu_threads. Returns the previous setting (0 = default)."""
    return check(lib().ambrycrc_set_host_cpu_threads(device, int(threads)), "ambrycrc_set_host_cpu_threads")


def host_calibrate(device: int = -1) -> float:
    """Calibrates the CPU leg at `device`'s budget now (ambrycrc_host_calibrate); returns its GiB/s."""
    r = ctypes.c_double()
    check(lib().ambrycrc_host_calibrate(device, ctypes.byref(r)), "ambrycrc_host_calibrate")
    return r.value


def host_msg_rates(device: int = 0, op: str = "verify") -> dict:
    """The rates auto compares for the host message entries (op "verify" / "transform";
    ambrycrc_host_msg_rates) and the leg it takes for pageable bytes."""
    c, g = ctypes.c_double(), ctypes.c_double()
    leg = check(lib().ambrycrc_host_msg_rates(device, {"verify": 0, "transform": 1}[op], ctypes.byref(c),
                                              ctypes.byref(g)), "ambrycrc_host_msg_rates")
    return {"cpu_gibps": c.value, "gpu_gibps": g.value, "auto_leg": "gpu" if leg else "cpu"}


def last_host_path(device: int = 0) -> int:
    """The leg the device's last host call took: 0 CPU, 1 GPU (-1: none yet)."""
    return lib().ambrycrc_last_host_path(device)


def set_grid(device: int, workgroups: int) -> None:
    check(lib().ambrycrc_set_grid(device, workgroups), "ambrycrc_set_grid")


def set_window(device: int, nbytes: int) -> None:
    """Sweep rounds of at most nbytes (0 = one round); see ambrycrc_set_window."""
    check(lib().ambrycrc_set_window(device, nbytes), "ambrycrc_set_window")


def grid_size(device: int = 0) -> int:
    return lib().ambrycrc_grid_size(device)


def timing_enable(device: int, enable: bool = True) -> None:
    check(lib().ambrycrc_timing_enable(device, 1 if enable else 0), "ambrycrc_timing_enable")


def timing_collect(device: int = 0):
    """(sum of sweep-kernel ms, launches) since the last collect (HIP events on the launch stream)."""
    ms = ctypes.c_double()
    cnt = ctypes.c_int()
    check(lib().ambrycrc_timing_collect(device, ctypes.byref(ms), ctypes.byref(cnt)), "ambrycrc_timing_collect")
    return ms.value, cnt.value


def timing_collect_each(device: int = 0, cap: int = 4096):
    """Per-launch sweep-kernel durations (ms, launch order) since the last collect."""
    buf = (ctypes.c_float * cap)()
    cnt = ctypes.c_int()
    check(lib().ambrycrc_timing_collect_each(device, buf, cap, ctypes.byref(cnt)), "ambrycrc_timing_collect_each")
    return [buf[i] for i in range(min(cap, cnt.value))]


def workspace_bytes(n: int) -> int:
    """Bytes of caller workspace ambrycrc_batch_dev needs for n chunks."""
    return lib().ambrycrc_workspace_bytes(n)


def messages_workspace_bytes(m: int) -> int:
    return lib().ambrycrc_messages_workspace_bytes(m)


def verify_messages(region, msg_off, stream=None, want_end: bool = True):
    """GPU verify of every CRC of the messages starting at msg_off (int64 CUDA tensor) in `region`.

    Returns (status int32[m] of AMBRYCRC_MSG_* bits, msg_end int64[m] or None).
    """
    torch = _torch()
    if region.dtype != torch.uint8 or not region.is_cuda:
        raise TypeError("region must be a uint8 CUDA tensor")
    if msg_off.dtype != torch.int64 or not msg_off.is_cuda or not msg_off.is_contiguous() or \
            msg_off.device != region.device:
        raise TypeError(f"msg_off must be a contiguous int64 CUDA tensor on {region.device}")
    m = msg_off.numel()
    status = torch.empty(m, dtype=torch.int32, device=region.device)
    end = torch.empty(m, dtype=torch.int64, device=region.device) if want_end else None
    check(lib().ambrycrc_verify_messages_dev(_ptr(region), region.numel(), _ptr(msg_off), m, _ptr(status),
                                             _ptr(end), None, 0, ctypes.c_void_p(_stream_handle(stream))),
          "ambrycrc_verify_messages_dev")
    return status, end


def verify_trailed(base, off, length, stream=None):
    """CRC-trailered items on the GPU: item i = base[off[i]:off[i]+len[i]] ends in the big-endian
    8-B CRC of the bytes before it. Returns (mismatch uint8[n], count int32[1])."""
    torch = _torch()
    n = off.numel()
    _check_batch(base, off, length, n)
    mismatch = torch.empty(n, dtype=torch.uint8, device=base.device)
    count = torch.zeros(1, dtype=torch.int32, device=base.device)
    check(lib().ambrycrc_verify_trailed_dev(_ptr(base), _ptr(off), _ptr(length), _ptr(mismatch), _ptr(count), n,
                                            None, 0, ctypes.c_void_p(_stream_handle(stream))),
          "ambrycrc_verify_trailed_dev")
    return mismatch, count


def verify_trailed_host(buffers, device: int = 0, pinned: bool = False):
    """The same over host buffers (bytes-likes, e.g. whole files): returns a list of bools, True =
    the trailer does not match (IndexSegment.checkDataIntegrityInByteBufferWithCRC is False)."""
    import numpy as np

    arrs = [np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview)) else
            np.ascontiguousarray(b, dtype=np.uint8) for b in buffers]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data if a.nbytes else None for a in arrs])
    lens = (ctypes.c_uint64 * n)(*[a.nbytes for a in arrs])
    mism = (ctypes.c_uint8 * n)()
    check(lib().ambrycrc_verify_trailed_host(ptrs, lens, mism, n, device, 1 if pinned else 0),
          "ambrycrc_verify_trailed_host")
    return [bool(x) for x in mism]


def verify_messages_host(region, msg_off, device: int = 0, pinned: bool = False):
    """verify_messages for a region in host memory (bytes, numpy uint8, or a CPU uint8 tensor;
    pinned=True for a hipHostMalloc'd / pin_memory() buffer). Returns (status uint32[m],
    msg_end uint64[m]) as numpy arrays."""
    import numpy as np

    if hasattr(region, "data_ptr"):  # torch CPU tensor
        ptr, nbytes, keep = region.data_ptr(), region.numel(), region
    else:
        arr = np.frombuffer(region, dtype=np.uint8) if isinstance(region, (bytes, bytearray)) else \
            np.ascontiguousarray(region, dtype=np.uint8)
        ptr, nbytes, keep = arr.ctypes.data, arr.nbytes, arr
    offs = np.ascontiguousarray(np.asarray(msg_off, dtype=np.uint64))
    m = len(offs)
    status = np.zeros(m, dtype=np.uint32)
    end = np.zeros(m, dtype=np.uint64)
    check(lib().ambrycrc_verify_messages_host(
        ctypes.c_void_p(ptr), nbytes, offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), m,
        status.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), end.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
        device, 1 if pinned else 0), "ambrycrc_verify_messages_host")
    del keep
    return status, end


def chain_messages_host(region: bytes, start: int = 0, max_messages: int = 1 << 20):
    """Offsets of consecutive messages from `start` in a host buffer (BlobStoreRecovery's hop)."""
    import numpy as np

    arr = np.frombuffer(region, dtype=np.uint8) if isinstance(region, (bytes, bytearray, memoryview)) else \
        np.ascontiguousarray(region, dtype=np.uint8)  # no copy for bytes, mmaps and uint8 arrays
    offs = np.zeros(max_messages, dtype=np.uint64)
    n = lib().ambrycrc_chain_messages_host(ctypes.c_void_p(arr.ctypes.data if arr.nbytes else 0), arr.nbytes, start,
                                           offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), max_messages)
    return [int(x) for x in offs[:n]]


# ------------------------------------------------ multi-GPU batch + RCCL all-gather (§8e)

def shard_by_bytes(lengths, nshards: int):
    """ambrycrc_shard_by_bytes: contiguous chunk ranges [lo, hi) of about equal bytes per shard."""
    import numpy as np

    lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
    cuts = (ctypes.c_size_t * (nshards + 1))()
    check(lib().ambrycrc_shard_by_bytes(lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(lens), nshards,
                                        cuts), "ambrycrc_shard_by_bytes")
    return [(int(cuts[g]), int(cuts[g + 1])) for g in range(nshards)]


def crc32_batch_cpu(chunks, crc_in=None, threads: int = 0):
    """ambrycrc_batch_cpu: per-chunk CRCs of host buffers on `threads` CPU threads (0 = all allowed)."""
    n, ptrs, lens, cin = _host_chunks(chunks, crc_in)
    out = (ctypes.c_uint32 * n)()
    check(lib().ambrycrc_batch_cpu(ptrs, lens, cin, out, n, threads), "ambrycrc_batch_cpu")
    return list(out)


def unique_id() -> bytes:
    """ambrycrc_unique_id: the 128-byte RCCL id rank 0 sends to every rank."""
    buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES)()
    check(lib().ambrycrc_unique_id(buf), "ambrycrc_unique_id")
    return bytes(buf)


class Comm:
    """An ambrycrc_comm (RCCL communicator): Comm.all_devices([0, 1, ...]) for one process driving
    several GPUs, Comm.rank(uid, nranks, rank, device) for one process per GPU."""

    def __init__(self, handle: int, devices):
        self.handle = ctypes.c_void_p(handle)
        self.devices = list(devices)

    @classmethod
    def all_devices(cls, devices):
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        check(lib().ambrycrc_comm_init_all(devs, len(devices), ctypes.byref(h)), "ambrycrc_comm_init_all")
        return cls(h.value, devices)

    @classmethod
    def rank(cls, uid: bytes, nranks: int, rank: int, device: int):
        if len(uid) != UNIQUE_ID_BYTES:
            raise ValueError(f"unique id must be {UNIQUE_ID_BYTES} bytes")
        buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        check(lib().ambrycrc_comm_init_rank(buf, nranks, rank, device, ctypes.byref(h)), "ambrycrc_comm_init_rank")
        c = cls(h.value, [device])
        c.rank_id = rank
        return c

    def size(self) -> int:
        return check(lib().ambrycrc_comm_size(self.handle), "ambrycrc_comm_size")

    def destroy(self) -> None:
        if self.handle.value:
            check(lib().ambrycrc_comm_destroy(self.handle), "ambrycrc_comm_destroy")
            self.handle = ctypes.c_void_p()


def _shard(base, off, length, gathered, crc_in=None, stream=None):
    torch = _torch()
    n = off.numel()
    _check_batch(base, off, length, n)
    _check_u32("crc_in", crc_in, n, base.device)
    if gathered.dtype not in (torch.int32, torch.uint32) or not gathered.is_cuda or not gathered.is_contiguous() \
            or gathered.device != base.device:
        raise TypeError(f"gathered must be a contiguous int32/uint32 CUDA tensor on {base.device}")
    s = stream if stream is not None else torch.cuda.current_stream(base.device)
    return Shard(base.device.index, base.data_ptr(), off.data_ptr(), length.data_ptr(),
                 None if crc_in is None else crc_in.data_ptr(), n, gathered.data_ptr(), s.cuda_stream)


def crc32_batch_multi_dev(comm: Comm, shards):
    """ambrycrc_batch_dev_multi. shards: one dict per device of comm, in comm order, with keys
    base, off, len, gathered (int32[total chunks] on that device), optional crc_in and stream.
    Every device's `gathered` receives all CRCs (shard order). Asynchronous."""
    arr = (Shard * len(shards))(*[_shard(s["base"], s["off"], s["len"], s["gathered"], s.get("crc_in"),
                                         s.get("stream")) for s in shards])
    total = sum(int(s["off"].numel()) for s in shards)
    for s in shards:
        if s["gathered"].numel() != total:
            raise TypeError(f"gathered must hold all {total} CRCs")
    check(lib().ambrycrc_batch_dev_multi(comm.handle, arr, len(shards)), "ambrycrc_batch_dev_multi")


def crc32_batch_gather(comm: Comm, base, off, length, gathered, counts, crc_in=None, stream=None):
    """ambrycrc_batch_dev_gather: this rank's shard, then the all-gather into `gathered`
    (int32[sum(counts)]). counts: chunks per rank, the same on every rank. Asynchronous."""
    if gathered.numel() != sum(int(c) for c in counts):
        raise TypeError("gathered must hold sum(counts) CRCs")
    sh = _shard(base, off, length, gathered, crc_in, stream)
    cnt = (ctypes.c_uint64 * len(counts))(*[int(c) for c in counts])
    check(lib().ambrycrc_batch_dev_gather(comm.handle, ctypes.byref(sh), cnt), "ambrycrc_batch_dev_gather")
