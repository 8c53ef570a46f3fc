"""Replication's ValidatingTransformer on the GPU (ambrycrc_transform_messages_dev): stored
messages of every header version, with and without encryption keys, blob records V1/V2/V3,
corrupted ones, update records and bad blob types, re-serialized at header V3, V2 and V1 with
every CRC recomputed. Byte-exact against oracle/message_format.py's transform_message, which
restates ValidatingTransformer.java:46-104; outputs packed in message order; every output
verifies clean."""
import struct
import zlib

import numpy as np
import pytest

from datagen import stream_bytes
from test_gpu_put import mf  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def _blob_v1_message(mf, key, props, um, content, version):
    """A PUT whose blob record is Blob_Format_V1 (stored by old servers)."""
    h = mf.HEADER_SIZE[version]
    pr, ur, bl = mf.props_record(props), mf.usermeta_record(um), mf.blob_record_v1(content)
    bp = h + len(key)
    return mf.header(version, len(pr) + len(ur) + len(bl), mf.INVALID, bp, mf.INVALID, bp + len(pr),
                     bp + len(pr) + len(ur), 0) + key + pr + ur + bl


def stored_props(mf, rng, blen, i):
    """BlobPropertiesSerDe bytes as servers of every version stored them (V1..V5), some with
    non-canonical private / encrypted bytes (read as `== 1`), a few with a non-ASCII string
    (the transform cannot re-encode those: NOT_ENCODABLE)."""
    v = int(rng.choice([1, 2, 3, 4, 5], p=[0.15, 0.15, 0.15, 0.15, 0.4]))
    odd = rng.random() < 0.15
    s = rng.random()
    owner = b"own\xc3\xa9r" if s < 0.03 else ("o%d" % (i % 5) if s < 0.8 else None)
    return mf.blob_properties_bytes(
        blen, service_id="s%d" % (i % 7), owner_id=owner, content_type=None if i % 9 == 0 else "application/x",
        ttl=int(rng.integers(-1, 10**6)), private=int(rng.choice([0, 1, 2])) if odd else bool(i % 2),
        encrypted=int(rng.choice([0, 1, 5])) if odd else bool(i % 3 == 0),
        content_encoding="gzip" if i % 4 == 0 else None, filename="file-%d.bin" % i if i % 5 else None,
        reserved="res%d" % i if i % 6 == 0 else None, account=int(rng.integers(-5, 30000)), container=i % 300,
        serde_version=v)


def build_region(mf, n, seed, corrupt=True):
    rng = np.random.default_rng(seed)
    msgs = []
    for i in range(n):
        kind = rng.random()
        v = int(rng.choice([1, 2, 3]))
        key = mf.store_key("rep-%d" % i)
        blen = int(rng.choice([0, 1, 100, 4096, 4109, 70000]))
        content = stream_bytes(seed + i, 0, blen).tobytes()
        um = stream_bytes(seed + i, 1 << 20, int(rng.choice([0, 7, 1000]))).tobytes()
        props = stored_props(mf, rng, blen, i)
        if kind < 0.08:
            m = mf.update_message(key, version=3)
        elif kind < 0.14:
            m = _blob_v1_message(mf, key, props, um, content, 1 if v == 1 else 2)
        else:
            enc = stream_bytes(seed, 9, 32).tobytes() if (v >= 2 and rng.random() < 0.4) else None
            bt = int(rng.choice([0, 1, 2], p=[0.6, 0.35, 0.05]))
            m = mf.put_message(key, props, um, content, version=v, enc_key=enc, life=int(rng.integers(0, 4)) if v == 3
                               else 0, blob_version=int(rng.choice([2, 3])), compressed=bool(rng.random() < 0.3),
                               blob_type=bt)
        m = bytearray(m)
        if rng.random() < 0.07 and corrupt:  # corrupt a byte somewhere
            m[int(rng.integers(0, len(m)))] ^= 0x40
        msgs.append(bytes(m))
    region, offs = bytearray(), []
    for m in msgs:
        region += bytes(int(rng.integers(0, 5)))  # gaps and odd alignment between messages
        offs.append(len(region))
        region += m
    return bytes(region), offs


def dense_old_region(mf, n, seed):
    """A dense, gap-free region of clean messages as old servers stored them -- header V1 (some
    V2), BlobProperties at SerDe V1 (some V2 / V3), Blob_Format_V1 -- so a transform to header V3
    grows nearly every message by the full 26 B (+6 header, +17 props, +3 blob head): an old
    replica being re-replicated (PutMessageFormatInputStream.java:88-90,122)."""
    rng = np.random.default_rng(seed)
    msgs = []
    for i in range(n):
        blen = int(rng.choice([0, 1, 100, 4096]))
        content = stream_bytes(seed + i, 0, blen).tobytes()
        um = stream_bytes(seed + i, 1 << 20, int(rng.choice([0, 5, 300]))).tobytes()
        sv = int(rng.choice([1, 2, 3], p=[0.7, 0.15, 0.15]))
        props = mf.blob_properties_bytes(blen, service_id="s%d" % (i % 7), owner_id="o%d" % (i % 3),
                                         private=bool(i % 2), serde_version=sv)
        hv = 1 if rng.random() < 0.8 else 2
        msgs.append(_blob_v1_message(mf, mf.store_key("old-%d" % i), props, um, content, hv))
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    return b"".join(msgs), offs


def test_transform_dense_old_region_default_out(gpu, mf):
    """The default `out` (ambrycrc_transform_out_bound) holds every message of a dense region of
    old messages grown by up to 26 B each: no MSG_NO_ROOM, every status 0, byte-exact output."""
    import torch

    from ambry_amd.messages import TRANSFORM_GROWTH_MAX, out_bound, transform_dev

    region, offs = dense_old_region(mf, 700, seed=5)
    assert out_bound(len(region), len(offs)) == len(region) + TRANSFORM_GROWTH_MAX * len(offs)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, out_off, out_len, status = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    st, oo, ol = status.cpu().numpy().view(np.uint32), out_off.cpu().numpy(), out_len.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    assert st.tolist() == [0] * len(offs)
    pos, grown = 0, 0
    for i, o in enumerate(offs):
        exp_st, exp = mf.transform_message(region, o, version=3)
        assert exp_st == 0
        assert oo[i] == pos and ol[i] == len(exp), i
        assert out_h[pos:pos + len(exp)] == exp, i
        pos += len(exp)
        grown += len(exp) - ((offs[i + 1] if i + 1 < len(offs) else len(region)) - o)
    assert grown > 20 * len(offs)  # the region really grows by ~26 B per message


@pytest.mark.parametrize("version", [3, 2, 1])
def test_transform_matches_oracle(gpu, mf, version):
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = build_region(mf, 600, seed=31 + version)
    m = len(offs)
    life = np.random.default_rng(version).integers(0, 9, size=m).astype(np.int16)
    use_life = version != 2  # V2 run: the stored life versions
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, out_off, out_len, status = transform_dev(
        dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), header_version=version,
        life_version=torch.from_numpy(life).cuda() if use_life else None)
    torch.cuda.synchronize()
    out_h = out.cpu().numpy().tobytes()
    st, oo, ol = status.cpu().numpy().view(np.uint32), out_off.cpu().numpy(), out_len.cpu().numpy()
    pos, kinds = 0, set()
    for i, o in enumerate(offs):
        exp_st, exp = mf.transform_message(region, o, life=int(life[i]) if use_life else None, version=version)
        assert int(st[i]) == exp_st, i
        kinds.add(exp_st)
        if exp is None:
            assert ol[i] == 0 and oo[i] == -1
            continue
        assert oo[i] == pos and ol[i] == len(exp), i
        assert out_h[pos:pos + len(exp)] == exp, i
        assert mf.verify_message(out_h, pos) == (0, pos + len(exp))
        pos += len(exp)
    assert 0 in kinds and mf.NOT_PUT in kinds and mf.BAD_RECORD in kinds and mf.NOT_ENCODABLE in kinds
    assert len(kinds) >= 5


def test_transform_out_of_room(gpu, mf):
    import torch

    from ambry_amd.messages import MSG_NO_ROOM, transform_dev

    msgs = [mf.put_message(mf.store_key("k%d" % i), mf.blob_properties_bytes(1000), b"u", bytes(1000))
            for i in range(10)]
    region = b"".join(msgs)
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    cap = len(msgs[0]) * 4 + 10  # room for four
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    _, out_off, out_len, status = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), out=out)
    torch.cuda.synchronize()
    st = status.cpu().numpy().tolist()
    assert st[:4] == [0] * 4 and all(s == MSG_NO_ROOM for s in st[4:])
    assert out_len.cpu().numpy().tolist() == [len(msgs[0])] * 4 + [0] * 6
    assert out.cpu().numpy().tobytes()[:4 * len(msgs[0])] == b"".join(msgs[:4])


def test_transform_large_batch_group_phase(gpu, mf):
    """3,500 messages: 17,500 CRC jobs engage the group phase in both the verify and the re-serialize."""
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = build_region(mf, 3500, seed=77)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, out_off, out_len, status = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint32)
    oo, ol = out_off.cpu().numpy(), out_len.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    for i in range(0, len(offs), 7):
        exp_st, exp = mf.transform_message(region, offs[i], version=3)
        assert int(st[i]) == exp_st
        if exp is not None:
            assert out_h[oo[i]:oo[i] + ol[i]] == exp
    good = np.nonzero(st == 0)[0]
    status2, _ = gpu.verify_messages(out, torch.from_numpy(oo[good]).cuda())
    torch.cuda.synchronize()
    assert int(status2.abs().sum().item()) == 0


@pytest.mark.parametrize("version", [3, 1])
def test_transform_speculative_pass(gpu, mf, version):
    """No message fails its CRCs (update records and bad blob types still do not transform): the
    two-pass speculative path alone produces the output -- the verify's copy-through places every
    kept record, the blob V1/V2 heads are rewritten as V3, the keys are copied -- packed and
    byte-exact against the oracle; then one flipped byte sends the same batch through the
    fallback pass, with the same result for every other message."""
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = build_region(mf, 400, seed=90 + version, corrupt=False)
    life = np.random.default_rng(7).integers(0, 9, size=len(offs)).astype(np.int16)

    def run(reg):
        dev = torch.frombuffer(bytearray(reg), dtype=torch.uint8).cuda()
        out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                                        header_version=version, life_version=torch.from_numpy(life).cuda())
        torch.cuda.synchronize()
        return out.cpu().numpy().tobytes(), oo.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy().view(np.uint32)

    for reg in (region, None):
        if reg is None:  # one stored-CRC failure: the fallback pass
            reg = bytearray(region)
            reg[offs[len(offs) // 2] + 60] ^= 0x01
            reg = bytes(reg)
        out, oo, ol, st = run(reg)
        pos = 0
        for i, o in enumerate(offs):
            exp_st, exp = mf.transform_message(reg, o, life=int(life[i]), version=version)
            assert int(st[i]) == exp_st, i
            if exp is None:
                assert ol[i] == 0 and oo[i] == -1
                continue
            assert oo[i] == pos and ol[i] == len(exp), i
            assert out[pos:pos + len(exp)] == exp, i
            pos += len(exp)


@pytest.mark.parametrize("version", [3, 1])
def test_transform_host_matches_dev_and_oracle(gpu, mf, version):
    """ambrycrc_transform_messages_host (the region in host memory, staged through the pinned slabs)
    gives the device call's outputs over the whole region -- packed in message order, byte-exact
    against the oracle -- on the mixed region (failures, updates, gaps) and on a dense old one."""
    import torch

    from ambry_amd.messages import transform_dev, transform_host

    for region, offs in (build_region(mf, 500, seed=140 + version), dense_old_region(mf, 300, seed=9)):
        life = np.random.default_rng(3).integers(0, 9, size=len(offs)).astype(np.int16)
        out, oo, ol, st = transform_host(region, offs, header_version=version, life_version=life)
        dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
        dout, doo, dol, dst = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                                            header_version=version, life_version=torch.from_numpy(life).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(st, dst.cpu().numpy().view(np.uint32))
        assert np.array_equal(oo, doo.cpu().numpy()) and np.array_equal(ol, dol.cpu().numpy())
        assert out == dout.cpu().numpy().tobytes()[:len(out)]
        pos = 0
        for i, o in enumerate(offs):
            exp_st, exp = mf.transform_message(region, o, life=int(life[i]), version=version)
            assert int(st[i]) == exp_st, i
            if exp is not None:
                assert oo[i] == pos and out[pos:pos + len(exp)] == exp, i
                pos += len(exp)


def test_transform_host_slabs_order_room_and_pinned(gpu, mf):
    """Many slabs (a 150 MiB region of 64 KiB-blob messages: three 64 MiB slabs), pinned and pageable
    sources, unsorted offsets (packing follows the message order, not the offsets), and a capacity
    that cuts the batch: the prefix that fits is placed, the rest get MSG_NO_ROOM (as the device
    call's exclusive scan of the lengths decides)."""
    import torch

    from ambry_amd.messages import MSG_NO_ROOM, transform_host

    msgs = [mf.put_message(mf.store_key("s%d" % i), mf.blob_properties_bytes(65536, serde_version=1 + i % 5),
                           b"m" * (i % 50), stream_bytes(i, 0, 65536).tobytes(), version=1 + i % 3)
            for i in range(16)]
    tmpl = b"".join(msgs)
    reps = 150
    region = tmpl * reps
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    all_offs = [r * len(tmpl) + o for r in range(reps) for o in offs]
    want = [mf.transform_message(region, o)[1] for o in all_offs[:16]]
    out, oo, ol, st = transform_host(region, all_offs)
    assert st.tolist() == [0] * len(all_offs)
    assert out == b"".join(want) * reps
    pinned = torch.frombuffer(bytearray(region), dtype=torch.uint8).pin_memory()
    out_p, oo_p, _, st_p = transform_host(pinned, all_offs, pinned=True)
    assert out_p == out and np.array_equal(oo_p, oo) and np.array_equal(st_p, st)
    # unsorted: message order decides the packing
    perm = np.random.default_rng(1).permutation(64)
    sub = [all_offs[j] for j in perm]
    out_u, oo_u, ol_u, st_u = transform_host(region, sub)
    pos = 0
    for k, j in enumerate(perm):
        exp = want[j % 16]
        assert oo_u[k] == pos and out_u[pos:pos + len(exp)] == exp
        pos += len(exp)
    # a cap that holds the first 20 of them
    cap = int(oo_u[20])
    _, oo_c, ol_c, st_c = transform_host(region, sub, out_cap=cap)
    assert st_c[:20].tolist() == [0] * 20 and all(s == MSG_NO_ROOM for s in st_c[20:])
    assert (oo_c[20:] == -1).all() and (ol_c[20:] == 0).all()


def test_transform_host_oversize_message(gpu, mf):
    """A message larger than a 64 MiB staging slab (a 70 MiB blob, Blob_Format_V1 under a V1 header)
    gets its own device buffers; the messages around it keep their order and bytes."""
    from ambry_amd.messages import transform_host

    big = _blob_v1_message(mf, mf.store_key("big"), mf.blob_properties_bytes(70 << 20, serde_version=1), b"meta",
                           stream_bytes(5, 0, 70 << 20).tobytes(), 1)
    small = mf.put_message(mf.store_key("s"), mf.blob_properties_bytes(10), b"", b"0123456789")
    region = small + big + small
    offs = [0, len(small), len(small) + len(big)]
    out, oo, ol, st = transform_host(region, offs)
    assert st.tolist() == [0, 0, 0]
    want = [mf.transform_message(region, o)[1] for o in offs]
    assert out == b"".join(want)
    assert len(want[1]) == len(big) + 26


def dense_v3_region(mf, n, seed, lead=0, trail=0):
    """Clean PUTs as a current server stores them -- header V3, BlobProperties at VERSION_5, a
    Blob_Format_V3 record, some with an encryption key -- back to back after `lead` junk bytes and
    before `trail` more: replication's common case, which the transform's one-pass fast path takes
    (the output is the messages' own bytes with each header's life version rewritten)."""
    rng = np.random.default_rng(seed)
    msgs = []
    for i in range(n):
        blen = int(rng.choice([0, 1, 100, 1000, 4096, 4109]))
        content = stream_bytes(seed + i, 0, blen).tobytes()
        um = stream_bytes(seed + i, 1 << 20, int(rng.choice([0, 7, 300]))).tobytes()
        props = mf.blob_properties_bytes(blen, service_id="s%d" % (i % 7), private=bool(i % 2),
                                         encrypted=bool(i % 3 == 0), filename="f%d" % i if i % 4 else None)
        enc = stream_bytes(seed, 9, 32).tobytes() if i % 5 == 0 else None
        msgs.append(mf.put_message(mf.store_key("v3-%d" % i), props, um, content, version=3, enc_key=enc,
                                   life=int(rng.integers(0, 3)), compressed=bool(i % 6 == 0),
                                   blob_type=int(i % 7 == 0)))
    junk = stream_bytes(seed, 1 << 30, lead + trail).tobytes()
    region = junk[:lead] + b"".join(msgs) + junk[lead:]
    offs = (lead + np.cumsum([0] + [len(x) for x in msgs[:-1]])).tolist()
    return region, offs


def fast_expected(region, offs, end, life=None):
    """What the fast path must produce for clean V3 PUTs back to back over region[offs[0]:end]: those
    bytes with each header's life version (bytes 2-3, big-endian) set from `life` and its CRC (the
    8-B big-endian trailer at 32, over bytes 0-31) recomputed (ValidatingTransformer.java:86-95 on a
    V3 PUT rewrites nothing else). Returns (bytes, out_off, out_len) for every message."""
    out = bytearray(region[offs[0]:end])
    oo = np.asarray(offs, dtype=np.int64) - offs[0]
    ol = np.diff(np.append(oo, end - offs[0]))
    if life is not None:
        for i, o in enumerate(oo.tolist()):
            out[o + 2:o + 4] = struct.pack(">h", int(life[i]))
            out[o + 32:o + 40] = struct.pack(">Q", zlib.crc32(bytes(out[o:o + 32])))
    return bytes(out), oo, ol


def assert_fast_output(out_h, oo, ol, region, offs, end, life=None):
    """Every byte and every (out_off, out_len) of a fast-path result against fast_expected."""
    exp, eoo, eol = fast_expected(region, offs, end, life)
    assert np.array_equal(oo, eoo) and np.array_equal(ol, eol)
    assert len(out_h) >= len(exp)
    if out_h[:len(exp)] != exp:
        a = np.frombuffer(out_h[:len(exp)], dtype=np.uint8)
        b = np.frombuffer(exp, dtype=np.uint8)
        bad = np.nonzero(a != b)[0]
        k = int(np.searchsorted(eoo, bad[0], side="right") - 1)
        raise AssertionError("%d bytes differ; first at output byte %d (message %d, byte %d): %#x vs %#x"
                             % (len(bad), bad[0], k, bad[0] - eoo[k], a[bad[0]], b[bad[0]]))


@pytest.mark.parametrize("n,lead,use_life", [(2000, 0, True), (1500, 13, False), (30000, 0, True)])
def test_transform_fast_path_dense_v3(gpu, mf, n, lead, use_life):
    """The one-pass fast path (region_fused_kernel's copy form): a dense clean V3 region -- at the
    region start or after junk, with and without index life versions, and (30,000 messages) with
    messages cut by CU share boundaries, which the tail kernel finishes -- transforms byte-exact
    against the oracle, packed from 0, every status 0."""
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = dense_v3_region(mf, n, seed=n + lead, lead=lead, trail=29)
    life = np.random.default_rng(4).integers(0, 9, size=n).astype(np.int16)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), header_version=3,
                                    life_version=torch.from_numpy(life).cuda() if use_life else None)
    torch.cuda.synchronize()
    st, oo, ol = st.cpu().numpy().view(np.uint32), oo.cpu().numpy(), ol.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    assert st.tolist() == [0] * n
    assert gpu.last_transform_path(0) == 1  # the fast path took the batch alone
    # every byte, then the oracle on a sample (which pins fast_expected itself)
    assert_fast_output(out_h, oo, ol, region, offs, len(region) - 29, life if use_life else None)
    for i in range(0, n, 1 if n <= 2000 else 29):
        o = offs[i]
        exp_st, exp = mf.transform_message(region, o, life=int(life[i]) if use_life else None, version=3)
        assert exp_st == 0
        assert oo[i] == o - offs[0] and ol[i] == len(exp), i
        assert out_h[oo[i]:oo[i] + len(exp)] == exp, i


@pytest.mark.parametrize("spoil", ["corrupt", "v1_props", "gap", "update", "order"])
def test_transform_fast_path_falls_back(gpu, mf, spoil):
    """One message the fast path cannot take -- a flipped byte, properties stored at SerDe V1 (a
    re-encode), a gap between two messages, an update record, two offsets swapped -- sends the
    batch through the general path; the result is the oracle's for every message."""
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = dense_v3_region(mf, 800, seed=3)
    region = bytearray(region)
    k = 400
    if spoil == "corrupt":
        region[offs[k] + 70] ^= 0x08
    elif spoil in ("v1_props", "gap", "update"):
        if spoil == "v1_props":
            new = mf.put_message(mf.store_key("x"), mf.blob_properties_bytes(10, serde_version=1), b"", b"0123456789")
        elif spoil == "update":
            new = mf.update_message(mf.store_key("x"), version=3)
        else:
            new = bytes(region[offs[k]:offs[k + 1]]) + b"\0\0\0"
        region = region[:offs[k]] + new + region[offs[k + 1]:]
        d = len(new) - (offs[k + 1] - offs[k])
        offs = offs[:k + 1] + [o + d for o in offs[k + 1:]]
    elif spoil == "order":
        offs[k], offs[k + 1] = offs[k + 1], offs[k]
    region = bytes(region)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    assert gpu.last_transform_path(0) == 0  # the general path redid the batch
    st, oo, ol = st.cpu().numpy().view(np.uint32), oo.cpu().numpy(), ol.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    pos = 0
    for i, o in enumerate(offs):
        exp_st, exp = mf.transform_message(region, o, version=3)
        assert int(st[i]) == exp_st, i
        if exp is None:
            assert ol[i] == 0 and oo[i] == -1
            continue
        assert oo[i] == pos and out_h[pos:pos + len(exp)] == exp, i
        pos += len(exp)


def test_transform_fast_path_long_messages(gpu, mf):
    """Long messages between small ones on the fast path (~2.5 KiB per message on average): two of
    3 MiB span many CU shares and go to the tail kernel, which takes each with a whole wave (a lane
    alone would walk its ~50,000 run sums one step at a time); 48 KiB blobs inside a share are the
    processors' long records (more than 512 runs), each verified once the stream has passed it."""
    import torch

    from ambry_amd.messages import transform_dev

    rng = np.random.default_rng(77)
    msgs = []
    for i in range(8000):
        if i in (1500, 6100):
            blen = (3 << 20) + 77 * i
        elif i % 250 == 7:
            blen = (48 << 10) + i
        else:
            blen = int(rng.integers(0, 3000))
        content = stream_bytes(500 + i, 0, blen).tobytes()
        msgs.append(mf.put_message(mf.store_key("long-%d" % i), mf.blob_properties_bytes(blen), b"um" * (i % 9),
                                   content, version=3))
    region = b"".join(msgs)
    assert len(region) <= 24576 * len(msgs)  # the fast path's cut-off
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), header_version=3)
    torch.cuda.synchronize()
    assert st.cpu().numpy().view(np.uint32).tolist() == [0] * len(msgs)
    assert gpu.last_transform_path(0) == 1
    oo, ol = oo.cpu().numpy(), ol.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    assert_fast_output(out_h, oo, ol, region, offs, len(region))
    for i in list(range(0, len(msgs), 97)) + [1500, 6100] + [i for i in range(len(msgs)) if i % 1000 == 7]:
        o = offs[i]
        exp_st, exp = mf.transform_message(region, o, version=3)
        assert exp_st == 0 and oo[i] == o and ol[i] == len(exp) and out_h[o:o + len(exp)] == exp, i


def test_transform_fast_path_32k_blobs(gpu, mf):
    """PUTs of ~32 KiB blobs (~33 KiB of region per message, under the 40 KiB cut-off) on the fast
    path: every blob is a long record (more than 512 runs) for a processor's wave, and a CU share of
    the region (~8 messages) ends inside a message each time -- its records past the share are
    hashed from the bytes (within kDirectSpan)."""
    import torch

    from ambry_amd.messages import transform_dev

    msgs = []
    for i in range(2000):
        blen = (32 << 10) - 500 + 7 * (i % 97)
        msgs.append(mf.put_message(mf.store_key("b32-%d" % i), mf.blob_properties_bytes(blen), b"u" * (i % 5),
                                   stream_bytes(900 + i, 0, blen).tobytes(), version=3))
    region = b"".join(msgs)
    assert 24576 * len(msgs) < len(region) <= 40960 * len(msgs)
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), header_version=3)
    torch.cuda.synchronize()
    assert st.cpu().numpy().view(np.uint32).tolist() == [0] * len(msgs)
    assert gpu.last_transform_path(0) == 1
    oo, ol = oo.cpu().numpy(), ol.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    assert_fast_output(out_h, oo, ol, region, offs, len(region))
    for i in list(range(0, len(msgs), 97)) + [len(msgs) - 1]:
        o = offs[i]
        exp_st, exp = mf.transform_message(region, o, version=3)
        assert exp_st == 0 and oo[i] == o and ol[i] == len(exp) and out_h[o:o + len(exp)] == exp, i


def test_transform_fast_path_share_boundaries(gpu, mf):
    """Messages placed against the one-pass kernel's CU share boundaries (a region of 48 KiB per
    CU: three 16 KiB groups per share): at each boundary B a message starts d bytes before it, for d
    from 1 to 3000 -- headers that cross into the next CU's share, and straddlers whose records
    lie past the share, finished by their own processor from the bytes; every header is patched by
    region_patch_kernel after the copy. Every output byte against fast_expected and every message
    against the oracle, life versions rewritten, the fast path alone."""
    import torch

    from ambry_amd.messages import transform_dev

    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    share = 3 * 16384
    total = ncu * share
    base_msg = lambda i, blen: mf.put_message(mf.store_key("sb-%d" % i), mf.blob_properties_bytes(blen),  # noqa: E731
                                              b"m" * (i % 5), stream_bytes(900 + i, 0, blen).tobytes(), version=3)
    ds = [1, 10, 39, 40, 41, 63, 64, 65, 100, 400, 3000]
    rng = np.random.default_rng(17)
    msgs, pos, i = [], 0, 0
    for b in range(1, ncu + 1):
        target = min(b * share - ds[b % len(ds)], total)
        while pos < target:
            rem = target - pos
            ovh = len(base_msg(i, 0))  # (the key's length varies with i)
            if ovh <= rem <= ovh + 6000:  # one message lands exactly on the target
                blen = rem - ovh
            else:
                blen = int(rng.integers(200, 3000))
                if rem - (ovh + blen) < ovh + 16:  # leave room for a landing message
                    blen = max(0, rem - 2 * ovh - 1000)
            m = base_msg(i, blen)
            msgs.append(m)
            pos += len(m)
            i += 1
    region = b"".join(msgs)
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    starts = set(offs)
    hit = [b * share - ds[b % len(ds)] in starts for b in range(1, ncu)]
    assert sum(hit) >= ncu // 2  # most boundaries got their placed message
    life = np.random.default_rng(5).integers(0, 9, size=len(msgs)).astype(np.int16)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    assert dev.data_ptr() % 64 == 0  # the shares are then exactly 48 KiB of the region
    out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"), header_version=3,
                                    life_version=torch.from_numpy(life).cuda())
    torch.cuda.synchronize()
    assert st.cpu().numpy().view(np.uint32).tolist() == [0] * len(msgs)
    assert gpu.last_transform_path(0) == 1
    oo, ol = oo.cpu().numpy(), ol.cpu().numpy()
    out_h = out.cpu().numpy().tobytes()
    assert_fast_output(out_h, oo, ol, region, offs, len(region), life)
    for k, o in enumerate(offs):
        exp_st, exp = mf.transform_message(region, o, life=int(life[k]), version=3)
        assert exp_st == 0 and oo[k] == o and out_h[o:o + len(exp)] == exp, k


def test_transform_graph_capture_and_replay(gpu, mf):
    """ambrycrc_transform_messages_dev only enqueues work (the fast path's verdict stays on the
    device, the general path behind its gate), so it can be captured into a HIP graph. Captured once
    over a clean V3 region (the fast path) and replayed: with new life versions (new header bytes),
    then after one message is corrupted in place (the general path, behind its device gate). Every
    replay gives every byte, offset and status the oracle gives."""
    import torch

    from ambry_amd.messages import transform_dev

    n = 600
    region, offs = dense_v3_region(mf, n, seed=41)
    life = np.random.default_rng(6).integers(0, 9, size=n).astype(np.int16)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    off_t = torch.tensor(offs, dtype=torch.int64, device="cuda")
    life_t = torch.from_numpy(life).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        transform_dev(dev, off_t, life_version=life_t)  # sizes the stream's default workspace
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out, oo, ol, st = transform_dev(dev, off_t, life_version=life_t)
    torch.cuda.synchronize()

    def replay():
        g.replay()
        torch.cuda.synchronize()
        return (out.cpu().numpy().tobytes(), oo.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy().view(np.uint32))

    out_h, oo_h, ol_h, st_h = replay()
    assert st_h.tolist() == [0] * n and gpu.last_transform_path(0) == 1
    assert_fast_output(out_h, oo_h, ol_h, region, offs, len(region), life)
    life2 = (life + 3).astype(np.int16)
    life_t.copy_(torch.from_numpy(life2).cuda())
    out_h, oo_h, ol_h, st_h = replay()
    assert st_h.tolist() == [0] * n and gpu.last_transform_path(0) == 1
    assert_fast_output(out_h, oo_h, ol_h, region, offs, len(region), life2)
    bad = bytearray(region)
    bad[offs[300] + 70] ^= 0x10
    dev.copy_(torch.frombuffer(bytes(bad), dtype=torch.uint8).cuda())
    out_h, oo_h, ol_h, st_h = replay()
    assert gpu.last_transform_path(0) == 0
    pos = 0
    for i, o in enumerate(offs):
        exp_st, exp = mf.transform_message(bytes(bad), o, life=int(life2[i]), version=3)
        assert int(st_h[i]) == exp_st, i
        if exp is None:
            assert ol_h[i] == 0 and oo_h[i] == -1
            continue
        assert oo_h[i] == pos and out_h[pos:pos + len(exp)] == exp, i
        pos += len(exp)
    assert st_h[300] != 0 and pos > 0


@pytest.mark.parametrize("clean", [True, False])
def test_transform_host_verdict(gpu, mf, clean):
    """ambrycrc_set_transform_verdict(device, 1): the call reads the fast path's verdict back (one
    stream synchronization) and enqueues the general path only when it must. Same outputs either
    way: a clean dense V3 batch (the fast path alone) and one with a corrupt message (the general
    path), against the oracle."""
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = dense_v3_region(mf, 700, seed=43)
    if not clean:
        region = bytearray(region)
        region[offs[350] + 60] ^= 0x01
        region = bytes(region)
    life = np.random.default_rng(8).integers(0, 9, size=len(offs)).astype(np.int16)
    prev = gpu.set_transform_verdict(0, True)
    try:
        dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
        out, oo, ol, st = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                                        life_version=torch.from_numpy(life).cuda())
        torch.cuda.synchronize()
        assert gpu.last_transform_path(0) == (1 if clean else 0)
    finally:
        gpu.set_transform_verdict(0, bool(prev))
    out_h, oo, ol, st = out.cpu().numpy().tobytes(), oo.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy().view(np.uint32)
    if clean:
        assert st.tolist() == [0] * len(offs)
        assert_fast_output(out_h, oo, ol, region, offs, len(region), life)
        return
    pos = 0
    for i, o in enumerate(offs):
        exp_st, exp = mf.transform_message(region, o, life=int(life[i]), version=3)
        assert int(st[i]) == exp_st, i
        if exp is None:
            continue
        assert oo[i] == pos and out_h[pos:pos + len(exp)] == exp, i
        pos += len(exp)


def test_transform_host_shared_bytes_matches_dev(gpu, mf):
    """Messages that share region bytes (every offset listed twice) through the host entry's staging
    slabs: their outputs sum past one slab's output buffer while their span fits one slab, so a run
    ends by output size -- the result equals one _dev call over the whole region, with the same cap
    (the slab's own cap could report NO_ROOM the whole-region call would not)."""
    import torch

    from ambry_amd.messages import transform_dev, transform_host

    msgs = [mf.put_message(mf.store_key("dup-%d" % i), mf.blob_properties_bytes(9 << 20), b"u" * i,
                           stream_bytes(70 + i, 0, 9 << 20).tobytes(), version=3) for i in range(5)]
    region = b"".join(msgs)
    base = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    offs = [o for o in base for _ in range(2)]
    cap = 2 * len(region) + 26 * len(offs)
    out_h, oo_h, ol_h, st_h = transform_host(region, offs, out_cap=cap)
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    out_d, oo_d, ol_d, st_d = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                                            out=torch.empty(cap, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    assert st_h.tolist() == [0] * len(offs) == st_d.cpu().numpy().view(np.uint32).tolist()
    assert np.array_equal(ol_h.astype(np.int64), ol_d.cpu().numpy())
    assert np.array_equal(oo_h.astype(np.int64), oo_d.cpu().numpy())
    total = int(oo_h[-1] + ol_h[-1])
    assert out_h[:total] == out_d.cpu().numpy().tobytes()[:total]
    for i in (0, 1, 9):
        exp_st, exp = mf.transform_message(region, offs[i], version=3)
        assert exp_st == 0 and out_h[oo_h[i]:oo_h[i] + ol_h[i]] == exp


@pytest.mark.parametrize("dense", [True, False])
def test_transform_negative_life_versions_device_and_cpu_leg(gpu, mf, dense):
    """Index life versions below zero (MessageInfo.LIFE_VERSION_FROM_FRONTEND = -1) are written unchanged by
    the device batch (the fast path declines them, the general path writes them) and by the host entry's CPU
    leg alike, so the auto policy's choice of leg never changes a byte: both against the oracle."""
    import torch

    from ambry_amd.messages import transform_dev, transform_host

    region, offs = dense_v3_region(mf, 80, seed=31) if dense else build_region(mf, 150, seed=32)
    life = np.random.default_rng(9).integers(-2, 4, size=len(offs)).astype(np.int16)
    life[::4] = -1
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    dout, doo, dol, dst = transform_dev(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                                        header_version=3, life_version=torch.from_numpy(life).cuda())
    torch.cuda.synchronize()
    cout, coo, col, cst = transform_host(region, offs, header_version=3, life_version=life, device=-1)
    assert np.array_equal(cst, dst.cpu().numpy().view(np.uint32))
    assert np.array_equal(coo, doo.cpu().numpy()) and np.array_equal(col, dol.cpu().numpy())
    assert cout == dout.cpu().numpy().tobytes()[:len(cout)]
    pos = 0
    for i, o in enumerate(offs):
        exp_st, exp = mf.transform_message(region, o, life=int(life[i]), version=3)
        assert int(cst[i]) == exp_st, i
        if exp is not None:
            assert coo[i] == pos and cout[pos:pos + len(exp)] == exp, i
            pos += len(exp)


def test_transform_back_to_back_verdicts_one_stream(gpu, mf):
    """The device verdict's side stream: 40 transforms enqueued back to back on one
    stream -- more than the 32 gate slots -- every third one with a corrupted message (the general path
    redoes that batch on the side stream while later calls' fast paths run), then ONE synchronize of
    the caller's stream only: every call's outputs are the oracle's (the clean ones byte-exact with
    fast_expected), so no side chain read a later call's verdict and the stream waited for every
    general path it needed."""
    import torch

    from ambry_amd.messages import transform_dev

    region, offs = dense_v3_region(mf, 120, seed=77)
    k = 60
    bad = bytearray(region)
    bad[offs[k] + 70] ^= 0x08
    s = torch.cuda.Stream()
    regions = [torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda(),
               torch.frombuffer(bytearray(bad), dtype=torch.uint8).cuda()]
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    results = []
    with torch.cuda.stream(s):
        for call in range(40):
            spoiled = call % 3 == 2
            results.append((spoiled, transform_dev(regions[int(spoiled)], d_off, stream=s)))
    s.synchronize()
    clean_exp = fast_expected(region, offs, len(region))
    bad_exp = [mf.transform_message(bytes(bad), o, version=3) for o in offs]
    for call, (spoiled, (out, oo, ol, st)) in enumerate(results):
        st, oo, ol = st.cpu().numpy().view(np.uint32), oo.cpu().numpy(), ol.cpu().numpy()
        out_h = out.cpu().numpy().tobytes()
        if not spoiled:
            assert st.tolist() == [0] * len(offs), call
            assert np.array_equal(oo, clean_exp[1]) and np.array_equal(ol, clean_exp[2]), call
            assert out_h[:len(clean_exp[0])] == clean_exp[0], call
            continue
        pos = 0
        for i, (exp_st, exp) in enumerate(bad_exp):
            assert int(st[i]) == exp_st, (call, i)
            if exp is None:
                assert ol[i] == 0 and oo[i] == -1, (call, i)
                continue
            assert oo[i] == pos and out_h[pos:pos + len(exp)] == exp, (call, i)
            pos += len(exp)
