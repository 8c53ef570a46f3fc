"""C ABI: libambrycrc loads, exports every declared symbol, and its host primitives agree
with the oracle and golden vectors. No device compute here (CPU-only container)."""
import os
import re
import zlib

import numpy as np
import pytest
from datagen import stream_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "ambrycrc.h")).read()
    return sorted(set(re.findall(r"\b(ambrycrc_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol(ambry):
    lib = ambry.lib()
    decl = declared_symbols()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(ambry.EXPORTED) == decl


def test_version_and_errors(ambry):
    lib = ambry.lib()
    assert lib.ambrycrc_version().decode().startswith("ambrycrc")
    for code in (0, -1, -2, -3, -4, -5, -6, -7):
        assert lib.ambrycrc_strerror(code)


def test_product_build_has_no_knob_overrides(ambry):
    """The in-tree library is the product build: no A/B knob differs from build_knobs.h's defaults,
    it is not a probe build, and the split group kernel (variant 32) is not linked into it."""
    import subprocess

    v = ambry.lib().ambrycrc_version().decode()
    assert v == "ambrycrc 0.4.0 gfx950", v
    syms = subprocess.run(["nm", "-D", "--defined-only", ambry.LIB_PATH], capture_output=True, text=True).stdout
    assert "launch_group" not in syms and "crc32_group_kernel" not in syms


@pytest.mark.parametrize("flag", ["-DAMBRY_REGION_PROBE=1", "-DAMBRY_RUNS_PROBE=5", "-DAMBRYCRC_DIAGNOSTICS",
                                  "-DAMBRY_AB_SPLIT_GROUP"])
def test_probe_knobs_need_probe_build(flag):
    """A wrong-CRC probe knob does not compile without -DAMBRY_AB_PROBE_BUILD (tools/ab_build.sh)."""
    import subprocess

    hdr = os.path.join(ROOT, "ambry_amd", "csrc", "build_knobs.h")
    bad = subprocess.run(["cpp", flag, hdr], capture_output=True, text=True)
    assert bad.returncode != 0 and "AMBRY_AB_PROBE_BUILD" in bad.stderr
    ok = subprocess.run(["cpp", flag, "-DAMBRY_AB_PROBE_BUILD", hdr], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr


def test_probe_build_refused_and_reported(tmp_path):
    """A probe build names itself in ambrycrc_version() and its overridden knobs, and ambrycrc_init
    refuses it (AMBRYCRC_EPROBE, before any device call) unless AMBRYCRC_ALLOW_PROBE=1."""
    import glob
    import subprocess
    import sys

    d = os.path.join(ROOT, "ambry_amd")
    objs = [o for o in glob.glob(os.path.join(d, "build", "obj", "*.o")) if not o.endswith("ambrycrc.cpp.o")]
    if len(objs) < 6 or not os.path.exists(os.path.join(d, "host_crc.o")):
        pytest.skip("in-tree objects not built (make -C ambry_amd)")
    so = str(tmp_path / "libprobe.so")
    cc = ["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DAMBRY_AB_PROBE_BUILD",
          "-DAMBRY_REGION_PROBE=2", "-c", "-o", str(tmp_path / "a.o"), os.path.join(d, "csrc", "ambrycrc.cpp")]
    subprocess.run(cc, check=True, capture_output=True, timeout=600)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o", so, str(tmp_path / "a.o"),
                    os.path.join(d, "host_crc.o")] + objs + ["-ldl"], check=True, capture_output=True, timeout=600)
    code = ("import ctypes; l = ctypes.CDLL(%r); l.ambrycrc_version.restype = ctypes.c_char_p; "
            "print(l.ambrycrc_version().decode()); print(l.ambrycrc_init(0))" % so)
    env = {k: v for k, v in os.environ.items() if k != "AMBRYCRC_ALLOW_PROBE"}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    version, rc = r.stdout.split("\n")[:2]
    assert "ab-probe-build" in version and "AMBRY_REGION_PROBE=2" in version
    assert int(rc) == -7


def test_host_update_golden(ambry, vectors):
    for v in vectors["known_answers"] + vectors["message_headers"]:
        assert ambry.crc32(bytes.fromhex(v["hex"])) == int(v["crc"], 16), v["name"]
    for v in vectors["random"]:
        data = stream_bytes(int(v["seed"], 16), v["offset"], v["len"]).tobytes()
        assert ambry.crc32(data, int(v["crc_in"], 16)) == int(v["crc"], 16)


def test_host_update_vs_oracle(ambry, oracle):
    data = stream_bytes(3, 0, 10000)
    for n in list(range(0, 40)) + [999, 4096, 10000]:
        assert ambry.crc32(data[:n].tobytes()) == oracle.crc32(data[:n])


def test_crc32_object_mirrors_java(ambry):
    """Crc32Test.crcTest + update(int)/update(byte[],off,len)/update(ByteBuffer) semantics."""
    from ambry_amd.crc32 import ByteBufferLike, Crc32

    buf = bytearray(stream_bytes(42, 0, 4000).tobytes())
    c = Crc32()
    c.update(buf, 0, 4000)
    v1 = c.getValue()
    c = Crc32()
    c.update(buf, 0, 4000)
    assert c.getValue() == v1 == zlib.crc32(bytes(buf))
    buf[3999] = (~buf[3999]) & 0xFF
    c = Crc32()
    c.update(buf, 0, 4000)
    assert c.getValue() != v1
    # split: bytes, single ints, ByteBuffer (consumed: position == limit afterwards)
    c = Crc32()
    c.update(buf, 0, 10)
    for i in range(10, 20):
        c.update(buf[i])
    bb = ByteBufferLike(bytes(buf), position=20)
    c.update_buffer(bb)
    assert bb.position == bb.limit == 4000
    assert c.getValue() == zlib.crc32(bytes(buf))
    c.reset()
    assert c.getValue() == 0
    empty = ByteBufferLike(b"", 0)
    c.update_buffer(empty)
    assert c.getValue() == 0


def test_combine_and_zeros(ambry, oracle, vectors):
    data = stream_bytes(8, 0, 100000).tobytes()
    for cut in (0, 1, 15, 16, 4096, 99999, 100000):
        a, b = data[:cut], data[cut:]
        assert ambry.combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(data)
        assert ambry.combine(zlib.crc32(a), zlib.crc32(b), len(b)) == oracle.combine(zlib.crc32(a), zlib.crc32(b),
                                                                                      len(b))
    for v in vectors["zero_runs"]:
        assert ambry.zeros(0, v["len"]) == int(v["crc"], 16)
    assert ambry.zeros(0x12345678, 777) == zlib.crc32(bytes(777), 0x12345678)
    assert ambry.zeros(5, 0) == 5


def test_table_image_layout(ambry):
    """The LDS image's slice region holds T0..T3 at the v_perm-addressed, lane-replicated slots."""
    import ctypes

    from kernel_model import K_IMG_BYTES

    words = K_IMG_BYTES // 4
    buf = (ctypes.c_uint32 * words)()
    assert ambry.lib().ambrycrc_debug_table_image(buf, words) == words * 4
    img = np.frombuffer(buf, dtype=np.uint32)
    T = [[0] * 256 for _ in range(4)]
    for b in range(256):
        c = b
        for _ in range(8):
            c = (c >> 1) ^ 0xEDB88320 if c & 1 else c >> 1
        T[0][b] = c
    for j in range(1, 4):
        for b in range(256):
            T[j][b] = (T[j - 1][b] >> 8) ^ T[0][T[j - 1][b] & 0xFF]
    for j in range(4):
        for lane in (0, 5, 31):
            for b in (0, 1, 128, 255):
                addr = ((j >> 1) << 16) | (b << 8) | ((j & 1) << 7) | (lane << 2)
                assert img[addr >> 2] == T[j][b]


def test_batch_dev_without_init_fails_loudly(ambry):
    """No silent fallback: without a device context the device entry point errors."""
    import ctypes

    from ambry_amd._lib import AMBRYCRC_ENOINIT

    rc = ambry.lib().ambrycrc_batch_dev(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), None,
                                        ctypes.c_void_p(16), 1, None, 0, None)
    assert rc == AMBRYCRC_ENOINIT


def test_host_entry_points_without_init_fail_loudly(ambry):
    """The host-resident entry points (batch, messages, file ranges) return ENOINIT without a
    device context, and EINVAL for null arguments, before touching any memory."""
    import ctypes

    import numpy as np

    from ambry_amd._lib import AMBRYCRC_EINVAL, AMBRYCRC_ENOINIT

    lib = ambry.lib()
    data = np.zeros(64, dtype=np.uint8)
    offs = (ctypes.c_uint64 * 1)(0)
    st = (ctypes.c_uint32 * 1)()
    end = (ctypes.c_uint64 * 1)()
    ptr = ctypes.c_void_p(data.ctypes.data)
    assert lib.ambrycrc_verify_messages_host(ptr, 64, offs, 1, st, end, 0, 0) == AMBRYCRC_ENOINIT
    assert lib.ambrycrc_verify_messages_host(ptr, 64, None, 1, st, end, 0, 0) == AMBRYCRC_EINVAL
    assert lib.ambrycrc_verify_messages_host(ptr, 64, offs, 0, st, end, 0, 0) == 0  # nothing to do
    ptrs = (ctypes.c_void_p * 1)(data.ctypes.data)
    lens = (ctypes.c_uint64 * 1)(64)
    out = (ctypes.c_uint32 * 1)()
    assert lib.ambrycrc_batch_host(ptrs, lens, None, out, 1, 0, 0) == AMBRYCRC_ENOINIT
    first = (ctypes.c_int64 * 1)(0)
    second = (ctypes.c_int64 * 1)(-1)
    assert lib.ambrycrc_range_checksums_host(ptr, 64, first, second, 1, out, 0) == AMBRYCRC_EINVAL


def test_host_update_every_cpu_impl():
    """Each host implementation (slice-by-8, SSE PCLMULQDQ fold, AVX-512 VPCLMULQDQ fold) is
    bit-exact with zlib (java.util.zip.CRC32's function) at every length 0..1100 (crossing the
    64 B and 256 B dispatch points and every fold remainder), at unaligned offsets, with a
    running crc_in, and at large sizes. Each runs in its own process (the choice is per process)."""
    import subprocess
    import sys

    code = r"""
import sys, zlib
import numpy as np
import pytest
sys.path.insert(0, sys.argv[1])
import ambry_amd
rng = np.random.default_rng(7)
d = rng.integers(0, 256, (1 << 20) + 64, dtype=np.uint8).tobytes()
for n in list(range(0, 1101)) + [4095, 4096, 65535, 65536, 1 << 20]:
    for off in (0, 3, 13):
        b = d[off:off + n]
        for ci in (0, 0xDEADBEEF):
            assert ambry_amd.crc32(b, ci) == zlib.crc32(b, ci), (n, off, ci)
print(ambry_amd.lib().ambrycrc_host_impl().decode())
"""
    seen = []
    for impl in ("slice8", "pclmul", "vpclmul"):
        env = dict(os.environ, AMBRYCRC_HOST_IMPL=impl)
        r = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        seen.append(r.stdout.strip())
    assert seen[0] == "slice8"
    # a CPU without the feature keeps the best it has; this image's Xeon has both
    assert seen[1] in ("slice8", "pclmul") and seen[2] in ("slice8", "pclmul", "vpclmul")


def test_host_crc_loops_under_asan(tmp_path):
    """The CLMUL and slice-by-8 host loops under AddressSanitizer/UBSan (host code only), each
    implementation forced in turn: no out-of-bounds read at any length or alignment, and
    bit-exact with zlib."""
    import shutil
    import subprocess

    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = tmp_path / "host_crc_asan"
    src = os.path.join(ROOT, "tests", "native", "host_crc_asan.cpp")
    lib = os.path.join(ROOT, "ambry_amd", "csrc", "host_crc.cpp")
    subprocess.run(["g++", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-std=c++17", "-I" + os.path.join(ROOT, "ambry_amd", "csrc"),
                    src, lib, "-lz", "-o", str(exe)], check=True, timeout=300)
    for impl in ("slice8", "pclmul", "vpclmul"):
        r = subprocess.run([str(exe)], env=dict(os.environ, AMBRYCRC_HOST_IMPL=impl), capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "bad=0" in r.stdout


def test_chain_messages_host_under_asan(tmp_path):
    """ambrycrc_chain_messages_host parses untrusted log bytes: built with the library's host code
    under AddressSanitizer/UBSan (-Xarch_host, device code untouched) and run from every start
    offset and on every tail truncation of a region of mixed, partly corrupted messages."""
    import shutil
    import subprocess

    from test_message_format import build_region

    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc) or not shutil.which("g++"):
        pytest.skip("hipcc/g++ not available")
    region, _, _ = build_region(n=40, seed=5, corrupt_frac=0.2, big_every=10**9)
    rf = tmp_path / "region.bin"
    rf.write_bytes(region)
    exe = tmp_path / "chain_asan"
    csrc = os.path.join(ROOT, "ambry_amd", "csrc")
    host_o = tmp_path / "host_crc.o"
    subprocess.run(["g++", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fPIC",
                    "-std=c++17", "-c", os.path.join(csrc, "host_crc.cpp"), "-o", str(host_o)],
                   check=True, timeout=300)
    subprocess.run([hipcc, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950",
                    "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                    "-Xarch_host", "-fno-sanitize-recover=all", str(host_o),
                    os.path.join(ROOT, "tests", "native", "chain_asan.cpp"), os.path.join(csrc, "ambrycrc.cpp"),
                    os.path.join(csrc, "ambrycrc_multi.cpp"), os.path.join(csrc, "crc32_kernels.hip"),
                    os.path.join(csrc, "message_kernels.hip"), os.path.join(csrc, "ambrycrc_put.cpp"),
                    os.path.join(csrc, "put_kernels.hip"), os.path.join(csrc, "ambrycrc_msg_cpu.cpp"), "-ldl", "-o",
                    str(exe)], check=True, timeout=900)
    r = subprocess.run([str(exe), str(rf)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runs=" in r.stdout


def test_message_cpu_under_asan(ambry, tmp_path):
    """ambrycrc_verify_message_cpu / ambrycrc_transform_message_cpu parse untrusted bytes: built with
    ASan + UBSan (host side) and run over every message of a region, its truncations and byte
    flips in its header and record heads (tests/native/msg_cpu_asan.cpp)."""
    import shutil
    import subprocess

    from test_message_format import build_region

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    from test_gpu_transform import build_region as transform_region
    from test_message_format import MF, record_level_cases

    region, _, _ = build_region(n=30, seed=8, corrupt_frac=0.0, big_every=10**9)
    rf = tmp_path / "region.bin"
    rf.write_bytes(region)
    # properties at SerDe V1..V5 (non-canonical flags, non-ASCII strings) and the record-level cases:
    # the properties / update parsers walk data-dependent offsets
    r2, offs2 = transform_region(MF, 40, seed=5, corrupt=False)
    rf2 = tmp_path / "region2.bin"  # the messages back to back (the harness chains them from offset 0)
    rf2.write_bytes(b"".join(r2[o:MF.verify_message(r2, o)[1]] for o in offs2))
    rf3 = tmp_path / "region3.bin"
    rf3.write_bytes(b"".join(m for m, _ in record_level_cases()))
    exe = tmp_path / "msg_cpu_asan"
    csrc = os.path.join(ROOT, "ambry_amd", "csrc")
    host_o = tmp_path / "host_crc.o"
    subprocess.run(["g++", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fPIC",
                    "-std=c++17", "-c", os.path.join(csrc, "host_crc.cpp"), "-o", str(host_o)],
                   check=True, timeout=300)
    subprocess.run([hipcc, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950",
                    "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                    "-Xarch_host", "-fno-sanitize-recover=all", str(host_o),
                    os.path.join(ROOT, "tests", "native", "msg_cpu_asan.cpp"), os.path.join(csrc, "ambrycrc.cpp"),
                    os.path.join(csrc, "ambrycrc_multi.cpp"), os.path.join(csrc, "ambrycrc_put.cpp"),
                    os.path.join(csrc, "ambrycrc_msg_cpu.cpp"), os.path.join(csrc, "crc32_kernels.hip"),
                    os.path.join(csrc, "message_kernels.hip"), os.path.join(csrc, "put_kernels.hip"), "-ldl",
                    "-o", str(exe)], check=True, timeout=900)
    for f in (rf, rf2, rf3):
        r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        assert "runs=" in r.stdout


def test_update_iov_gather_list(ambry):
    """ambrycrc_update_iov == successive updates (PutChunk.verifyCRC over a CompositeByteBuf's
    nioBuffers, PutOperation.java:2041-2043), empty and NULL entries included; the Crc32 mirror's
    update_buffers consumes every buffer."""
    from ambry_amd.crc32 import ByteBufferLike, Crc32

    data = stream_bytes(21, 0, 300000).tobytes()
    cuts = [0, 0, 1, 17, 4096, 4096, 100000, 299999, 300000]
    slices = [ByteBufferLike(data[a:b]) for a, b in zip(cuts, cuts[1:])]
    c = Crc32()
    c.update(b"prefix", 0, 6)
    c.update_buffers(slices)
    assert c.getValue() == zlib.crc32(data, zlib.crc32(b"prefix"))
    assert all(s.position == s.limit for s in slices)
    import ctypes
    lib = ambry.lib()
    ptrs = (ctypes.c_void_p * 3)(None, None, None)
    lens = (ctypes.c_size_t * 3)(0, 0, 0)
    assert lib.ambrycrc_update_iov(0x1234, ptrs, lens, 3) == 0x1234


def test_batch_cpu_vs_oracle(ambry, oracle):
    """ambrycrc_batch_cpu (the host-resident many-record batch) on 1, 3 and all threads."""
    from ambry_amd import device as D

    rng = np.random.default_rng(9)
    mem = stream_bytes(31, 0, 3 << 20)
    n = 500
    ln = rng.integers(0, 20000, size=n)
    ln[:6] = [0, 1, 63, 64, 65, 1 << 20]
    off = rng.integers(0, (3 << 20) - (1 << 20), size=n)
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(mem, off, ln, crc_in=cin)
    base = mem.ctypes.data
    chunks = [(base + int(o), int(l)) for o, l in zip(off, ln)]
    for th in (1, 3, 0):
        assert D.crc32_batch_cpu(chunks, crc_in=cin, threads=th) == exp.tolist()
    assert D.crc32_batch_cpu([(0, 0), (base, 5)], threads=64) == [0, oracle.crc32(mem[:5])]


def test_multi_gpu_entries_validate_without_gpu(ambry):
    """The RCCL entry points reject bad arguments before touching a device or RCCL."""
    import ctypes

    lib = ambry.lib()
    h = ctypes.c_void_p()
    assert lib.ambrycrc_comm_init_all(None, 0, ctypes.byref(h)) == -1
    assert lib.ambrycrc_comm_init_rank(None, 2, 0, 0, ctypes.byref(h)) == -1
    assert lib.ambrycrc_batch_dev_multi(None, None, 1) == -1
    assert lib.ambrycrc_batch_dev_gather(None, None, None) == -1
    assert lib.ambrycrc_comm_destroy(None) == 0
    assert lib.ambrycrc_comm_size(None) == -1
    assert lib.ambrycrc_unique_id(None) == -1
