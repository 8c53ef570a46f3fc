"""The JNI shim's argument checks and marshalling (ambry_amd/jni/ambrycrc_jni_core.c), driven
through ctypes: no JDK exists in this image, so ambrycrc_jni.c keeps only the JNI calls and every
decision it makes is made by these functions. Bounds follow java.util.zip.CRC32.update(byte[],
off, len) (ArrayIndexOutOfBoundsException unless 0 <= off, 0 <= len, off + len <= length) and
Crc32.update(ByteBuffer) (position..limit, Crc32.java:100-143). Errors never come back in the
CRC slot."""
import ctypes
import os
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORE = os.path.join(ROOT, "ambry_amd", "libambrycrc_jnicore.so")

AJC_OK, AJC_EBOUNDS, AJC_ENOTDIRECT, AJC_ESHORT, AJC_ENULL = 0, -100, -101, -102, -103


@pytest.fixture(scope="module")
def core(ambry):
    if not os.path.exists(CORE):
        import subprocess

        subprocess.run(["make", "-C", os.path.join(ROOT, "ambry_amd")], check=True, capture_output=True)
    L = ctypes.CDLL(CORE)
    i64, i32, u32 = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32
    L.ajc_range_ok.argtypes = [i64, i64, i64]
    L.ajc_update.argtypes = [u32, ctypes.c_void_p, i64, i64, i64, ctypes.POINTER(u32)]
    L.ajc_exception_class.restype = ctypes.c_char_p
    L.ajc_message.restype = ctypes.c_char_p
    L.ajc_batch_args.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(i64),
                                 ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_void_p),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_size_t)]
    L.ajc_iov_args.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(i64),
                               ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_void_p),
                               ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    L.ajc_batch_lengths.argtypes = [i64] * 5
    L.ajc_verify_lengths.argtypes = [i64] * 3
    return L


def test_range_checks_follow_java(core):
    ok = core.ajc_range_ok
    assert ok(10, 0, 10) and ok(10, 10, 0) and ok(0, 0, 0) and ok(10, 3, 7)
    for cap, off, ln in ((10, 0, 11), (10, -1, 1), (10, 1, -1), (10, 11, 0), (-1, 0, 0),
                         (2**31 - 1, 2**31 - 1, 2**31 - 1), (100, 2**62, 2**62)):
        assert not ok(cap, off, ln), (cap, off, ln)


def test_update_reports_out_of_band(core):
    data = np.frombuffer(os.urandom(1000), dtype=np.uint8)
    out = ctypes.c_uint32(0xDEAD)
    assert core.ajc_update(0, data.ctypes.data, 1000, 10, 500, ctypes.byref(out)) == AJC_OK
    assert out.value == zlib.crc32(data[10:510].tobytes())
    out.value = 0x1234
    # a bad range is a status; the CRC slot keeps its value (never a status code)
    assert core.ajc_update(7, data.ctypes.data, 1000, 900, 101, ctypes.byref(out)) == AJC_EBOUNDS
    assert out.value == 0x1234
    assert core.ajc_update(7, None, 0, 0, 0, ctypes.byref(out)) == AJC_OK and out.value == 7
    assert core.ajc_update(7, None, 5, 0, 5, ctypes.byref(out)) == AJC_ENULL
    # 0xFFFFFFFF is a legitimate CRC and comes back as a value
    assert core.ajc_update(0xFFFFFFFF, data.ctypes.data, 1000, 0, 0, ctypes.byref(out)) == AJC_OK
    assert out.value == 0xFFFFFFFF


def test_batch_and_iov_marshalling(core):
    bufs = [np.frombuffer(os.urandom(n), dtype=np.uint8) for n in (100, 4096, 1)]
    n = len(bufs)
    bases = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    caps = (ctypes.c_int64 * n)(*[b.nbytes for b in bufs])
    ptrs = (ctypes.c_void_p * n)()
    lens = (ctypes.c_uint64 * n)()
    bad = ctypes.c_size_t(99)
    pos = (ctypes.c_int32 * n)(0, 96, 1)
    ln = (ctypes.c_int32 * n)(100, 4000, 0)
    assert core.ajc_batch_args(n, bases, caps, pos, ln, ptrs, lens, ctypes.byref(bad)) == AJC_OK
    assert [ptrs[i] for i in range(n)] == [bufs[0].ctypes.data, bufs[1].ctypes.data + 96, bufs[2].ctypes.data + 1]
    assert list(lens) == [100, 4000, 0]
    ln[1] = 4001  # one byte past the capacity of buffer 1
    assert core.ajc_batch_args(n, bases, caps, pos, ln, ptrs, lens, ctypes.byref(bad)) == AJC_EBOUNDS
    assert bad.value == 1
    ln[1] = 4000
    bases[2] = None  # a heap buffer (no native address)
    assert core.ajc_batch_args(n, bases, caps, pos, ln, ptrs, lens, ctypes.byref(bad)) == AJC_ENOTDIRECT
    assert bad.value == 2
    bases[2] = bufs[2].ctypes.data
    szs = (ctypes.c_size_t * n)()
    lim = (ctypes.c_int32 * n)(100, 4096, 1)
    assert core.ajc_iov_args(n, bases, caps, pos, lim, ptrs, szs, ctypes.byref(bad)) == AJC_OK
    assert list(szs) == [100, 4000, 0]
    lim[0] = -1  # limit below position
    assert core.ajc_iov_args(n, bases, caps, pos, lim, ptrs, szs, ctypes.byref(bad)) == AJC_EBOUNDS
    lim[0] = 101  # limit past capacity
    assert core.ajc_iov_args(n, bases, caps, pos, lim, ptrs, szs, ctypes.byref(bad)) == AJC_EBOUNDS
    assert bad.value == 0


def test_array_length_checks(core):
    assert core.ajc_batch_lengths(3, 3, 3, -1, 3) == AJC_OK
    assert core.ajc_batch_lengths(3, 3, 3, 3, 4) == AJC_OK
    assert core.ajc_batch_lengths(3, 2, 3, -1, 3) == AJC_ESHORT
    assert core.ajc_batch_lengths(3, 3, 3, 2, 3) == AJC_ESHORT
    assert core.ajc_batch_lengths(3, 3, 3, 3, 2) == AJC_ESHORT
    assert core.ajc_verify_lengths(5, 5, -1) == AJC_OK
    assert core.ajc_verify_lengths(5, 4, -1) == AJC_ESHORT
    assert core.ajc_verify_lengths(5, 5, 4) == AJC_ESHORT


def test_exception_mapping(core):
    cls = lambda s: core.ajc_exception_class(s)  # noqa: E731
    assert cls(AJC_OK) is None
    assert cls(AJC_EBOUNDS) == b"java/lang/IndexOutOfBoundsException"
    assert cls(AJC_ENOTDIRECT) == b"java/lang/IllegalArgumentException"
    assert cls(AJC_ENULL) == b"java/lang/NullPointerException"
    assert cls(-1) == b"java/lang/IllegalArgumentException"
    assert cls(-3) == b"java/lang/OutOfMemoryError"
    for code in (-2, -4, -5, -6):
        assert cls(code) == b"java/lang/IllegalStateException"
    assert core.ajc_message(-4).decode().startswith("ambrycrc_init")


def _run_harness(tmp_path, *args):
    import subprocess

    amd = os.path.join(ROOT, "ambry_amd")
    exe = str(tmp_path / "jni_harness")
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "tests", "native", "jni_stub"), "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", "-o", exe, os.path.join(ROOT, "tests", "native", "jni_harness.c"),
                    os.path.join(amd, "jni", "ambrycrc_jni.c"), "-L", amd, "-lambrycrc_jnicore", "-lambrycrc",
                    "-Wl,-rpath," + amd], check=True, capture_output=True)
    out = subprocess.run([exe, *args], check=True, capture_output=True, text=True, timeout=120).stdout
    return {name: (int(val, 16), exc) for name, val, exc in (line.split() for line in out.splitlines())}


def test_jni_shim_against_fake_jvm(core, tmp_path):
    """ambrycrc_jni.c itself, compiled (-Wall -Wextra -Werror) against the JNI subset in
    tests/native/jni_stub/jni.h and run inside the fake JVM of tests/native/jni_harness.c: the
    exported Java_com_github_ambry_utils_NativeCrc32_* entries return zlib's CRCs, leave the CRC
    argument unchanged when they throw, and throw the exception class the core maps."""
    got = _run_harness(tmp_path)
    crc = lambda b: zlib.crc32(b)  # noqa: E731
    NPE, IOOBE = "java/lang/NullPointerException", "java/lang/IndexOutOfBoundsException"
    IAE, ISE = "java/lang/IllegalArgumentException", "java/lang/IllegalStateException"
    expect = {
        "array_full": (crc(b"123456789"), "-"), "array_tail": (crc(b"56789"), "-"),
        "array_bounds": (0x1234, IOOBE), "array_negative": (0x1234, IOOBE), "array_null": (0x1234, NPE),
        "direct_full": (crc(b"123456789"), "-"), "direct_bounds": (7, IOOBE), "direct_heap": (7, IAE),
        "direct_null": (7, NPE), "byte": (crc(b"1"), "-"), "combine": (crc(b"123456789"), "-"),
        "combine_negative": (0, IAE), "direct_all": (crc(b"123456789"), "-"), "direct_all_bounds": (0, IOOBE),
        "direct_all_heap": (0, IAE), "batch_short_out": (0, IAE), "batch_null": (0, NPE),
        "batch_bounds": (0, IOOBE), "verify_short_status": (0, IAE), "verify_heap": (0, IAE),
        "verify_null": (0, NPE), "xform_short_lens": (0, IAE), "xform_short_life": (0, IAE),
        "xform_null_out": (0, NPE), "xform_heap": (0, IAE),
        "xform_no_context": (0, "java/lang/IllegalStateException"),
        "chain_null": (0, NPE), "chain_heap": (0, IAE), "chain_negative": (0, IOOBE), "chain_none": (0, "-"),
        "policy_no_context": (0xFFFFFFFF, ISE), "rates_null": (0xFFFFFFFF, NPE), "rates_short": (0xFFFFFFFF, IAE),
        "rates_no_context": (0xFFFFFFFF, ISE), "last_path_no_context": (0xFFFFFFFF, ISE),
        "cpu_threads_set": (0, "-"), "cpu_threads_prev": (3, "-"), "cpu_threads_bad": (0xFFFFFFFF, IAE),
        "cpu_threads_no_context": (0xFFFFFFFF, ISE),
    }
    for name, want in expect.items():
        assert got[name] == want, name
    # without a GPU ambrycrc_init fails and nativeInit throws; with one it succeeds
    assert got["init_no_gpu"] in ((0, "java/lang/IllegalStateException"), (0, "-"))


@pytest.mark.gpu
def test_jni_shim_device_entries(core, tmp_path):
    """The shim's device entries on a GPU, in the fake JVM: nativeBatchDirect over three direct
    buffers at positions 0 / 2 / 1 (ambrycrc_batch_host), nativeVerifyMessages over a region
    holding no message (AMBRYCRC_MSG_BAD_VERSION at both offsets, ends 0)."""
    got = _run_harness(tmp_path, "gpu")
    assert got["gpu_init"] == (0, "-")
    assert got["gpu_batch_0"] == (zlib.crc32(b"123"), "-")
    assert got["gpu_batch_1"] == (zlib.crc32(b"456"), "-")
    assert got["gpu_batch_2"] == (zlib.crc32(b"89yy"), "-")
    assert got["gpu_verify_0"] == (1 << 8, "-") and got["gpu_verify_1"] == (1 << 8, "-")
    assert got["gpu_verify_end"] == (0, "-")
    # host-resident dispatch (nativeSetHostPolicy / nativeHostRates / nativeLastHostPath)
    assert got["gpu_rates_leg"] in ((0, "-"), (1, "-")) and got["gpu_rates_positive"] == (1, "-")
    assert got["gpu_policy_bad"] == (0xFFFFFFFF, "java/lang/IllegalArgumentException")
    assert got["gpu_policy_cpu"] == (1, "-")
    assert got["gpu_cpu_leg_batch_1"] == (zlib.crc32(b"456"), "-") and got["gpu_cpu_leg_path"] == (0, "-")
    assert got["gpu_policy_gpu"] == (2, "-")
    assert got["gpu_gpu_leg_batch_1"] == (zlib.crc32(b"456"), "-") and got["gpu_gpu_leg_path"] == (1, "-")


def test_jni_shim_message_entries(core, tmp_path):
    """nativeVerifyMessage / nativeTransformMessage (ambrycrc_verify_message_cpu /
    ambrycrc_transform_message_cpu) in the fake JVM on the C1 message: clean verify with its end,
    V3 -> V3 reproducing it, V1 re-serialized 6 B shorter (34-B header), NO_ROOM into 16 B, a
    blob flip flagged, and the argument errors thrown."""
    from c1_message import c1_message_bytes

    msg = c1_message_bytes()
    path = tmp_path / "msg.bin"
    path.write_bytes(msg)
    got = _run_harness(tmp_path, "msg", str(path))
    NPE = "java/lang/NullPointerException"
    IAE, ISE = "java/lang/IllegalArgumentException", "java/lang/IllegalStateException"
    assert got["msg_verify"] == (0, "-") and got["msg_verify_end"] == (len(msg), "-")
    assert got["msg_verify_heap"] == (0, IAE) and got["msg_verify_null"] == (0, NPE)
    assert got["msg_verify_short"] == (0, IAE)
    assert got["msg_verify_past"] == (1 << 9, "-")  # BAD_LAYOUT is data, not an error
    assert got["msg_transform_v3"] == (0, "-") and got["msg_transform_v3_len"] == (len(msg), "-")
    assert got["msg_transform_v3_same"] == (1, "-")
    assert got["msg_transform_v1"] == (0, "-") and got["msg_transform_v1_len"] == (len(msg) - 6, "-")
    assert got["msg_transform_small"] == (1 << 12, "-") and got["msg_transform_small_len"] == (0, "-")
    assert got["msg_transform_badver"][1] in (IAE, ISE)
    assert got["msg_verify_corrupt"] == (1 << 5, "-") and got["msg_transform_corrupt"] == (1 << 5, "-")


@pytest.mark.gpu
def test_jni_shim_batched_transform(core, tmp_path):
    """nativeTransformMessages (ambrycrc_transform_messages_host) in the fake JVM on the GPU: the C1
    message twice in a direct buffer, transformed at header V3 with life versions 0 -- the output
    reproduces the region, the second message packed right after the first -- then an output
    buffer of one message's capacity: the first transforms, the second gets MSG_NO_ROOM."""
    from c1_message import c1_message_bytes

    msg = c1_message_bytes()
    path = tmp_path / "msg.bin"
    path.write_bytes(msg)
    got = _run_harness(tmp_path, "gpumsg", str(path))
    assert got["gpumsg_init"] == (0, "-")
    assert got["gpumsg_xform_st"] == (0, "-") and got["gpumsg_xform_off1"] == (len(msg), "-")
    assert got["gpumsg_xform_len"] == (2 * len(msg), "-") and got["gpumsg_xform_same"] == (1, "-")
    assert got["gpumsg_xform_room0"] == (0, "-") and got["gpumsg_xform_room1"] == (1 << 12, "-")


def _sieve_response(mf):
    """One GetResponse as ReplicaThread hands it to MessageSievingInputStream: clean PUTs (header V1/V2/V3,
    some with an encryption key), one with a corrupt blob byte, one update record, and messages the
    index marks deleted or expired (read and skipped). Returns (bytes, [(size, flag, life)])."""
    import numpy as np

    from datagen import stream_bytes

    rng = np.random.default_rng(55)
    msgs, infos = [], []
    for i in range(40):
        blen = int(rng.choice([0, 5, 300, 4096, 9000]))
        v = 1 + i % 3
        enc = stream_bytes(i, 7, 32).tobytes() if v >= 2 and i % 4 == 1 else None
        if i == 17:
            m = mf.update_message(mf.store_key("upd"), version=3)
        else:
            m = mf.put_message(mf.store_key("sv-%d" % i), mf.blob_properties_bytes(blen), b"m" * (i % 5),
                               stream_bytes(300 + i, 0, blen).tobytes(), version=v, enc_key=enc, life=i % 3)
        if i == 23:
            m = bytearray(m)
            m[-12] ^= 0x40  # inside the blob content / record tail
            m = bytes(m)
        msgs.append(m)
        infos.append((len(m), 1 if i % 11 == 5 else 2 if i % 13 == 7 else 0, int(rng.integers(0, 5))))
    return b"".join(msgs), infos


@pytest.mark.gpu
def test_jni_sieve_call_sequence(core, tmp_path):
    """The replication sieve with ambry-messageformat-batch-sieve.patch, as its Java code calls the shim,
    run in the fake JVM: one direct buffer holding the whole response, NativeCrc32.transformMessages
    over the live messages at their response offsets (deleted / expired ones skipped, leaving gaps),
    then each result classified as applyOutput does. Every sieved message's bytes are the oracle's
    ValidatingTransformer output (length and CRC), the corrupt one is skipped as invalid, and the
    update record is the exception that fails the stream -- the reference's outcomes, message by
    message."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("message_format", os.path.join(ROOT, "oracle", "message_format.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    region, infos = _sieve_response(mf)
    (tmp_path / "resp.bin").write_bytes(region)
    (tmp_path / "infos.txt").write_text("".join("%d %d %d\n" % x for x in infos))
    got = _run_harness(tmp_path, "sieve", str(tmp_path / "resp.bin"), str(tmp_path / "infos.txt"))
    assert got["sieve_init"] == (0, "-") and got["sieve_transform"] == (0, "-")
    at, seen = 0, set()
    for i, (size, flag, life) in enumerate(infos):
        cls = got["sieve_%d" % i]
        if flag:
            assert cls == (0, "-"), i
        else:
            st, exp = mf.transform_message(region, at, life=life, version=3)
            if st == 0:
                assert cls == (1, "-"), i
                assert got["sieve_%d_len" % i] == (len(exp), "-"), i
                assert got["sieve_%d_crc" % i] == (zlib.crc32(exp), "-"), i
            else:
                want = 3 if i == 17 else 2  # the update record fails the stream; corruption skips one message
                assert cls == (want, "-"), (i, st)
            seen.add(cls[0])
        at += size
    assert seen == {1, 2, 3}


def _log_span(mf, corrupt_at=None, truncate=False):
    from datagen import stream_bytes

    msgs = []
    for i in range(30):
        if i % 6 == 4:
            m = mf.update_message(mf.store_key("lg-%d" % i), version=1 + i % 3, life=i % 2)
        else:
            blen = [0, 1, 700, 5000, 70000][i % 5]
            m = mf.put_message(mf.store_key("lg-%d" % i), mf.blob_properties_bytes(blen), b"u" * (i % 7),
                               stream_bytes(800 + i, 0, blen).tobytes(), version=1 + i % 3)
        msgs.append(m)
    if corrupt_at is not None:
        m = bytearray(msgs[corrupt_at])
        m[len(m) // 2] ^= 0x02
        msgs[corrupt_at] = bytes(m)
    span = b"".join(msgs)
    if truncate:
        span = span[:-100]
    return span, [len(m) for m in msgs]


def _oracle_recover(mf, span):
    """BlobStoreRecovery.recover's outcome (BlobStoreRecovery.java:43-110) by the oracle: messages from the
    span's start while each verifies, stopping at the first that does not (LogFileFormatError)."""
    pos, count = 0, 0
    while pos < len(span):
        st, end = mf.verify_message(span, pos)
        if st or not end:
            return count, pos, 1
        count, pos = count + 1, end
    return count, pos, 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["clean", "corrupt", "truncated"])
def test_jni_recovery_call_sequence(core, tmp_path, case):
    """Store recovery with ambry-messageformat-batch-recovery.patch, as NativeBlobStoreRecovery calls the
    shim, in the fake JVM: nativeChainMessages in batches of 7 offsets, nativeVerifyMessages per batch on
    the GPU, the first failure stopping the scan. Recovered count, reported startOffset and the
    LogFileFormatError equal the oracle's reading of the reference loop -- a clean span to its end, a
    corrupt blob byte in message 13, and a span whose last message is cut short."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("message_format", os.path.join(ROOT, "oracle", "message_format.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    span, _ = _log_span(mf, corrupt_at=13 if case == "corrupt" else None, truncate=case == "truncated")
    (tmp_path / "span.bin").write_bytes(span)
    got = _run_harness(tmp_path, "recover", str(tmp_path / "span.bin"), "7")
    count, stop, failed = _oracle_recover(mf, span)
    assert got["recover_init"] == (0, "-")
    assert (got["recover_count"][0], got["recover_stop"][0], got["recover_failed"][0]) == (count, stop, failed)
    assert failed == (case != "clean") and count == {"clean": 30, "corrupt": 13, "truncated": 29}[case]


def test_jni_putchunk_call_sequence(core, tmp_path):
    """com.github.ambry.utils.Crc32 with ambry-utils-crc32-native.patch, as PutOperation.PutChunk calls it, in the
    fake JVM: fillFrom's update(slice.nioBuffer()) per slice (PutOperation.java:1700-1703) -- slices of 256 B and
    more through nativeUpdateDirect on the inverted register, shorter ones through the class's own loop -- then
    verifyCRC's fresh Crc32 over nioBuffers() (:2033-2054). Both equal zlib's CRC of the 4 MiB chunk (the C3 chunk
    size), the slices are consumed, a byte mutated after the fill fails verifyCRC (PutOperationTest.java:629-679),
    and the post-compression reset + recompute (:1595-1599) sees the new bytes."""
    from datagen import stream_bytes

    chunk = bytearray(stream_bytes(0xC3, 0, 4 << 20).tobytes())
    (tmp_path / "chunk.bin").write_bytes(bytes(chunk))
    rng = __import__("numpy").random.default_rng(11)
    slices, left = [], len(chunk)
    while left:
        s = min(left, int(rng.choice([1, 7, 255, 256, 257, 4096, 65536, 1 << 20])))
        slices.append(s)
        left -= s
    slices = slices[:200] + [sum(slices[200:])] if len(slices) > 201 else slices
    got = _run_harness(tmp_path, "putchunk", str(tmp_path / "chunk.bin"), *map(str, slices))
    want = zlib.crc32(bytes(chunk))
    assert got["putchunk_fill"] == (want, "-") and got["putchunk_verify"] == (want, "-")
    assert got["putchunk_fill_consumed"] == (1, "-") and got["putchunk_verify_match"] == (1, "-")
    assert got["putchunk_mutated_match"] == (0, "-")
    chunk[len(chunk) // 2] ^= 0x10
    assert got["putchunk_recomputed"] == (zlib.crc32(bytes(chunk)), "-")


def _filestore_ranges(image, ranges):
    """FileStore.getChecksumsForRanges (FileStore.java:567-595) restated: each range read from `first` for
    `second - first` bytes by FileChannel.read, so cut at the end of the file and empty past it."""
    n = len(image)
    return [zlib.crc32(image[min(a, n):min(b, n)]) for a, b in ranges]


def _ranges_case(tmp_path, image, ranges, device):
    (tmp_path / "file.bin").write_bytes(image)
    (tmp_path / "ranges.txt").write_text("".join("%d %d\n" % r for r in ranges))
    return _run_harness(tmp_path, "ranges", str(tmp_path / "file.bin"), str(tmp_path / "ranges.txt"), str(device))


def _check_ranges(got, image, ranges):
    IAE, NPE = "java/lang/IllegalArgumentException", "java/lang/NullPointerException"
    assert got["ranges_call"] == (0, "-")
    for i, want in enumerate(_filestore_ranges(image, ranges)):
        assert got["range_%d" % i] == (want, "-"), i
    assert got["ranges_short"] == (0, IAE) and got["ranges_heap"] == (0, IAE) and got["ranges_null"] == (0, NPE)


def _file_and_ranges():
    from datagen import stream_bytes

    image = stream_bytes(0xF5, 0, 3 << 20).tobytes()
    n = len(image)
    # StoreFileCopyHandler.getChecksumRanges' shape (start, start + size - 1), plus empty, straddling and past-EOF
    ranges = [(i * (256 << 10), i * (256 << 10) + (256 << 10) - 1) for i in range(12)]
    ranges += [(0, 0), (5, 5), (1, 2), (n - 100, n + 100), (n, n + 10), (n + 50, n + 60), (7, n), (0, n)]
    return image, ranges


def test_jni_filestore_ranges_cpu(core, tmp_path):
    """ambry-store-filestore-ranges.patch's call, in the fake JVM on the library's CPU threads (device -1):
    nativeRangeChecksums over the file image equals FileStore's per-range reads -- the copy handler's ranges,
    empty ranges, ranges straddling and past the end of the file -- and an empty file image (capacity-0 mapping)
    gives 0 for every range, as the reference's empty reads do. An invalid range throws IllegalArgumentException
    and computes nothing."""
    image, ranges = _file_and_ranges()
    _check_ranges(_ranges_case(tmp_path, image, ranges, -1), image, ranges)
    got = _ranges_case(tmp_path, b"", [(0, 10), (3, 3)], -1)
    assert got["range_0"] == (0, "-") and got["range_1"] == (0, "-")
    got = _ranges_case(tmp_path, image, [(0, 10), (9, 3)], -1)
    assert got["ranges_call"] == (0, "java/lang/IllegalArgumentException")
    assert got["range_0"] == (0x5A5A5A5A, "-")  # nothing computed


@pytest.mark.gpu
def test_jni_filestore_ranges_gpu(core, tmp_path):
    """The same FileStore ranges through the library's host-resident dispatch on GPU 0 (nativeInit first)."""
    image, ranges = _file_and_ranges()
    got = _ranges_case(tmp_path, image, ranges, 0)
    assert got["ranges_init"] == (0, "-")
    _check_ranges(got, image, ranges)


def test_jni_put_crcs(core, tmp_path):
    """NativeCrc32.putCrcs (ambrycrc_put_crcs, §8f row 2) in the fake JVM: from each blob's CRC alone, the PutRequest
    wire CRC over the V5 fields and the blob (PutRequest.java:238-283) and the Blob_Format_V3 record CRC over its
    13-B prefix and the blob (MessageFormatRecord.java:1789-1795), equal to zlib over the concatenations; then the
    record CRCs alone, and the argument errors (a wire output without fields, a short output, a negative blob
    length, a heap field buffer, a limit past the capacity) thrown."""
    from ambry_amd.protocol import blob_record_prefix_v3
    from test_protocol import make_requests

    reqs = make_requests(n=12, seed=9)
    prefixes = [blob_record_prefix_v3(len(b), t, c) for _, b, c, t in reqs]
    blob = b"".join(b"%d %d %d\n" % (len(f), len(p), len(b)) + f + p + b for (f, b, _, _), p in zip(reqs, prefixes))
    (tmp_path / "puts.bin").write_bytes(blob)
    got = _run_harness(tmp_path, "putcrcs", str(tmp_path / "puts.bin"))
    assert got["putcrcs_call"] == (0, "-")
    for i, ((f, b, _, _), p) in enumerate(zip(reqs, prefixes)):
        assert got["wire_%d" % i] == (zlib.crc32(f + b), "-"), i
        assert got["record_%d" % i] == (zlib.crc32(p + b), "-"), i
    assert got["putcrcs_record_only_0"] == (zlib.crc32(prefixes[0] + reqs[0][1]), "-")
    NPE, IAE, IOOBE = ("java/lang/NullPointerException", "java/lang/IllegalArgumentException",
                       "java/lang/IndexOutOfBoundsException")
    assert got["putcrcs_wire_without_fields"] == (0, NPE) and got["putcrcs_short_out"] == (0, IAE)
    assert got["putcrcs_negative_len"] == (0, IAE) and got["putcrcs_heap_field"] == (0, IAE)
    assert got["putcrcs_field_bounds"] == (0, IOOBE)


def test_integration_patches_apply(tmp_path):
    """Every integration/*.patch applies to the reference tree (git apply --check; read-only). Skipped where the
    reference is absent (the GPU box)."""
    import glob
    import subprocess

    ref = "/root/reference"
    if not os.path.isdir(os.path.join(ref, "ambry-utils")):
        pytest.skip("reference tree not present")
    patches = sorted(glob.glob(os.path.join(ROOT, "integration", "*.patch")))
    assert len(patches) >= 5
    for p in patches:
        r = subprocess.run(["git", "apply", "--check", p], cwd=ref, capture_output=True, text=True)
        assert r.returncode == 0, (p, r.stderr)
