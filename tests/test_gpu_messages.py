"""GPU parity for ambrycrc_verify_messages_dev against oracle/message_format.py (§8f next #1).

Bit-exact per-message status and message-end offsets on log regions mixing PUT
messages (header V1/V2/V3, with and without encryption-key records, blobs from
0 B to ~300 KB) and update messages, with random single-bit corruptions, an
unknown header version and a message truncated by the region end."""
import struct

import numpy as np
import pytest

from test_message_format import MF, build_region

pytestmark = pytest.mark.gpu


MODES = {"region": 1, "region2": 2, "jobs": 0}


@pytest.fixture(autouse=True, params=list(MODES))
def msg_mode(request, gpu):
    """Every test runs in every message-verify form: region mode in one pass (the region swept
    once into 64-B run sums while each CU's processor waves take its messages), region mode in two
    passes (the default), and CRC jobs through the batch engine. Region mode engages for
    regions of <= 6 KiB per message."""
    gpu.set_region_mode(0, MODES[request.param])
    yield request.param
    gpu.set_region_mode(0, 2)


def run(gpu, region: bytes, offs, shift: int = 0):
    """Verify on the GPU; shift > 0 places the region `shift` bytes into its allocation."""
    import torch

    buf = np.zeros(len(region) + shift, dtype=np.uint8)
    buf[shift:] = np.frombuffer(region, dtype=np.uint8)
    r = torch.from_numpy(buf).cuda()[shift:]
    o = torch.tensor(np.asarray(offs, dtype=np.int64), device="cuda")
    status, end = gpu.verify_messages(r, o)
    torch.cuda.synchronize()
    return status.cpu().numpy().view(np.uint32).tolist(), end.cpu().numpy().tolist()


@pytest.mark.parametrize("shift", [0, 1, 13, 48, 63])
def test_small_messages_unaligned_region(gpu, msg_mode, shift):
    """Small PUT / update messages (region mode engages: < 6 KiB per message) with 8 % corrupted,
    the region starting at every kind of offset from a 64-B boundary, so record ends fall on every
    residue of the run grid; status and ends bit-exact vs the oracle."""
    region, offs, expect = build_region(n=700, seed=40 + shift, corrupt_frac=0.08, big_every=10**9)
    assert len(region) <= 6144 * len(offs)
    st, end = run(gpu, region, offs, shift)
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert sum(1 for s in st if s) >= 40


def test_region_mode_sparse_and_overlapping_offsets(gpu, msg_mode):
    """Messages listed out of order, one listed twice, gaps of junk between them, offsets past the
    region end: region mode sweeps every byte and still reads each record's own runs."""
    region, offs, _ = build_region(n=300, seed=77, corrupt_frac=0.05, big_every=10**9)
    junk = bytes(range(256)) * 3
    spaced, offs2 = bytearray(), []
    for i, o in enumerate(offs):
        e = offs[i + 1] if i + 1 < len(offs) else len(region)
        if i % 7 == 3:
            spaced += junk[: (i * 37) % 700]
        offs2.append(len(spaced))
        spaced += region[o:e]
    spaced = bytes(spaced)
    order = list(reversed(offs2)) + [offs2[5], len(spaced) + 3, len(spaced) - 1]
    expect = [MF.verify_message(spaced, o) if o + 2 <= len(spaced) else (MF.BAD_LAYOUT, 0) for o in order]
    st, end = run(gpu, spaced, order, shift=9)
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_region_status_matches_oracle(gpu, seed):
    region, offs, expect = build_region(n=600, seed=seed, corrupt_frac=0.1)
    st, end = run(gpu, region, offs)
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert sum(1 for s in st if s) >= 30


def test_many_small_messages_group_phase(gpu):
    """4,000 messages = 20,000 record jobs (>= 16,384): the small records take the group phase."""
    region, offs, expect = build_region(n=4000, seed=11, corrupt_frac=0.05, big_every=10**9)
    st, end = run(gpu, region, offs)
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert sum(1 for s in st if s) >= 150


def test_bad_version_truncated_and_out_of_range(gpu):
    region, offs, _ = build_region(n=50, seed=9, corrupt_frac=0.0)
    junk = struct.pack(">h", 7) + bytes(60)  # unknown header version
    region2 = region + junk
    last_msg = MF.put_message(MF.store_key("tail"), MF.blob_properties_bytes(5000), b"m" * 10, bytes(5000))
    truncated = region2 + last_msg[:-100]
    offs2 = offs + [len(region), len(region2), len(truncated) - 1, len(truncated) + 10]
    expect = [MF.verify_message(truncated, o) if o + 2 <= len(truncated) else (MF.BAD_LAYOUT, 0) for o in offs2]
    st, end = run(gpu, truncated, offs2)
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert st[-4] == MF.BAD_VERSION and st[-3] == MF.BAD_LAYOUT


def test_each_record_kind_flagged(gpu):
    key = MF.store_key("id1")
    msg = MF.put_message(key, MF.blob_properties_bytes(4096), b"u" * 1000, bytes(range(256)) * 16, version=3,
                         enc_key=b"k" * 100)
    upd = MF.update_message(key)
    h, kl = 40, len(key)
    enc_at = h + kl + 10
    props_at = h + kl + len(MF.enckey_record(b"k" * 100)) + 10
    um_at = len(msg) - len(MF.blob_record(bytes(4096))) - 500
    blob_at = len(msg) - 1000
    cases = [(msg, 5, MF.HEADER_CRC), (msg, enc_at, MF.ENCKEY_CRC), (msg, props_at, MF.PROPS_CRC),
             (msg, um_at, MF.USERMETA_CRC), (msg, blob_at, MF.BLOB_CRC), (upd, h + kl + 3, MF.UPDATE_CRC),
             (msg, len(msg) - 2, MF.BLOB_CRC)]
    region, offs = bytearray(), []
    for base, pos, _ in cases:
        b = bytearray(base)
        b[pos] ^= 0x01
        offs.append(len(region))
        region += b
    st, _ = run(gpu, bytes(region), offs)
    assert st == [bit for _, _, bit in cases]


@pytest.mark.parametrize("variant", [0, 29])
def test_stored_crc_bytes_corrupted_group_phase(gpu, variant):
    """Flips inside the stored 8-B CRCs themselves, upper word (a CRC-32 has none: always a
    mismatch) and lower word, on every record kind, in a batch large enough for the group
    phase (4,000 messages). Variant 29 reads the stored CRCs of group-phase records inside the
    sweep (SweepArgs::exp_fill); variant 0 reads all of them in the parse kernel."""
    region, offs, expect = build_region(n=4000, seed=21, corrupt_frac=0.0, big_every=97)
    assert all(s == 0 for s, _ in expect)
    region = bytearray(region)
    rng = np.random.default_rng(5)
    for i in rng.choice(len(offs), size=400, replace=False):
        off = offs[i]
        v, total, rel = MF.parse_header(bytes(region[off:off + 64]), 0)
        present = [r for r in rel if r != MF.INVALID]
        end = present[0] + total
        ends = present[1:] + [end]
        e = ends[int(rng.integers(0, len(ends)))]
        pos = off + e - 8 + int(rng.integers(0, 8))  # either word of the stored CRC
        region[pos] ^= 1 << int(rng.integers(0, 8))
    region = bytes(region)
    expect = [MF.verify_message(region, o) for o in offs]
    prev = gpu.get_variant(0)
    gpu.set_variant(0, variant)
    try:
        st, end = run(gpu, region, offs)
    finally:
        gpu.set_variant(0, prev)
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert sum(1 for s in st if s) == 400


def _host_case(n_msgs, seed):
    """Region > one 64 MiB staging slab, messages listed out of order, with offsets at and past
    the region end, a message truncated by the region end and one whose header claims a size
    past it."""
    region, offs, _ = build_region(n=n_msgs, seed=seed, corrupt_frac=0.05, big_every=3)
    region = bytearray(region)
    # a header whose total size runs past the region end (layout error, header-only read)
    huge = bytearray(MF.put_message(MF.store_key("huge"), MF.blob_properties_bytes(10), b"u", bytes(10)))
    offs.append(len(region))
    region += huge
    last = MF.put_message(MF.store_key("cut"), MF.blob_properties_bytes(3000), b"m" * 10, bytes(3000))
    offs.append(len(region))
    region += last[:-50]  # truncated by the region end
    region = bytes(region)
    offs += [len(region), len(region) + 7]
    rng = np.random.default_rng(seed)
    perm = rng.permutation(len(offs))
    offs = [offs[i] for i in perm]
    expect = [MF.verify_message(region, o) if o + 2 <= len(region) else (MF.BAD_LAYOUT, 0) for o in offs]
    return region, offs, expect


@pytest.mark.parametrize("pinned", [False, True])
def test_verify_messages_host_matches_oracle(gpu, pinned):
    """ambrycrc_verify_messages_host (host region staged through the pinned slabs) gives the
    oracle's status and message end for every message, across slab boundaries."""
    import torch

    region, offs, expect = _host_case(1500, 31)
    assert len(region) > (64 << 20)
    if pinned:
        host = torch.from_numpy(np.frombuffer(region, dtype=np.uint8).copy()).pin_memory()
    else:
        host = region
    st, end = gpu.verify_messages_host(host, offs, device=0, pinned=pinned)
    assert st.tolist() == [s for s, _ in expect]
    assert end.tolist() == [e for _, e in expect]
    assert sum(1 for s in st if s) >= 70


def test_verify_messages_host_oversize_message(gpu):
    """A message larger than a staging slab (a 70 MB blob) takes its own staging buffer."""
    big = MF.put_message(MF.store_key("big"), MF.blob_properties_bytes(70 << 20), b"meta", bytes(70 << 20))
    small = MF.put_message(MF.store_key("s"), MF.blob_properties_bytes(100), b"x", bytes(range(100)))
    bad = bytearray(big)
    bad[len(bad) // 2] ^= 4
    region = small + big + bytes(bad) + small
    offs = [0, len(small), len(small) + len(big), len(small) + 2 * len(big)]
    expect = [MF.verify_message(region, o) for o in offs]
    st, end = gpu.verify_messages_host(region, offs)
    assert st.tolist() == [s for s, _ in expect]
    assert end.tolist() == [e for _, e in expect]
    assert st[2] == MF.BLOB_CRC and st[1] == 0


def test_hard_deleted_messages_verify_clean(gpu):
    """Messages hard-deleted in place (HardDeleteMessageFormatInputStream.java:58-124: zeroed user
    metadata and blob, CRCs from ambrycrc_zeros) verify clean on the device, group phase engaged."""
    from ambry_amd.protocol import hard_delete_records

    region, offs = bytearray(), []
    rng = np.random.default_rng(13)
    for i in range(4000):
        size = int(rng.integers(0, 20000))
        um_len = int(rng.integers(0, 1200))
        msg = bytearray(MF.put_message(MF.store_key(f"hd{i}"), MF.blob_properties_bytes(size), bytes([7]) * um_len,
                                       bytes([i & 255]) * size))
        if i % 2:
            v, total, rel = MF.parse_header(bytes(msg), 0)
            um, bl = hard_delete_records(um_len, size)
            msg[rel[3]:rel[3] + len(um)] = um
            msg[rel[4]:rel[4] + len(bl)] = bl
        offs.append(len(region))
        region += msg
    region = bytes(region)
    st, end = run(gpu, region, offs)
    assert st == [0] * len(offs)
    assert end == [MF.verify_message(region, o)[1] for o in offs]


def test_verify_messages_host_many_small_messages(gpu):
    """70,000 update messages (~90 B each): more messages than one staging slab takes
    (65,536), so the host path cuts slabs by count as well as by bytes."""
    one = MF.update_message(MF.store_key("u"), version=3, kind="delete")
    bad = bytearray(one)
    bad[len(bad) - 12] ^= 0x40  # inside the update record
    msgs = [bytes(bad) if i % 997 == 0 else one for i in range(70000)]
    offs, pos = [], 0
    for m in msgs:
        offs.append(pos)
        pos += len(m)
    region = b"".join(msgs)
    st, end = gpu.verify_messages_host(region, offs)
    exp_one, exp_bad = MF.verify_message(one, 0)[0], MF.verify_message(bytes(bad), 0)[0]
    assert exp_one == 0 and exp_bad != 0
    assert st.tolist() == [exp_bad if i % 997 == 0 else 0 for i in range(70000)]
    assert end.tolist() == [o + len(one) for o in offs]


def test_verify_log_tool(gpu, tmp_path):
    """tools/verify_log.py over a log segment file (LogSegment header + messages): the chain, the
    per-message status and the header check agree with the oracle; a corrupt header stops the
    chain where BlobStoreRecovery would stop."""
    import importlib.util
    import os

    from ambry_amd import store_files

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("verify_log", os.path.join(root, "tools", "verify_log.py"))
    vl = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(vl)
    region, offs, expect = build_region(n=300, seed=4, corrupt_frac=0.0, big_every=50)
    region = bytearray(region)
    for i in (7, 99, 200):  # record corruption: still chained, flagged
        v, total, rel = MF.parse_header(bytes(region[offs[i]:offs[i] + 64]), 0)
        region[offs[i] + rel[-1] + 3] ^= 0x08
    hdr = store_files.log_segment_header(1 << 30)
    path = tmp_path / "0_0_log"
    path.write_bytes(hdr + bytes(region))
    r = vl.verify_log(str(path))
    assert r["log_header_intact"] and r["messages"] == 300
    exp = [MF.verify_message(bytes(region), o)[0] for o in offs]
    assert r["corrupt"] == sum(1 for s in exp if s) == 3
    assert [x["offset"] for x in r["first_corrupt"]] == [len(hdr) + offs[i] for i in (7, 99, 200)]
    assert r["unscanned_tail_bytes"] == 0
    # a corrupt message header ends the chain there (BlobStoreRecovery stops at the first bad header)
    region[offs[150] + 5] ^= 0x01
    path.write_bytes(hdr + bytes(region))
    r = vl.verify_log(str(path))
    assert r["messages"] == 150 and r["chain_end"] == len(hdr) + offs[150]


def test_record_level_checks(gpu):
    """Messages whose CRCs are all valid but whose record versions / size fields / blob type are
    not what the reference's deserializers accept: BAD_VERSION / BAD_RECORD, as the oracle says."""
    from test_message_format import record_level_cases

    cases = record_level_cases()
    region, offs = bytearray(), []
    for msg, _ in cases:
        region += bytes(3)  # odd alignment
        offs.append(len(region))
        region += msg
    st, end = run(gpu, bytes(region), offs)
    assert st == [want for _, want in cases]
    assert end == [o + len(m) for o, (m, _) in zip(offs, cases)]


def _expect_mode(gpu, msg_mode, region_len, m):
    if region_len <= 6144 * m:
        assert gpu.last_message_mode(0) == MODES[msg_mode]
    else:
        assert gpu.last_message_mode(0) == 0


def test_many_shares_boundary_messages(gpu, msg_mode):
    """30,000 small messages (~90 MB): every CU share boundary cuts a message, which the one-pass
    kernel defers to the tail kernel; status and ends bit-exact, and the call took the form asked."""
    region, offs, expect = build_region(n=30000, seed=5, corrupt_frac=0.02, big_every=10**9)
    st, end = run(gpu, region, offs, shift=7)
    _expect_mode(gpu, msg_mode, len(region), len(offs))
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]


def test_long_records_inside_region_mode(gpu, msg_mode):
    """A region of small messages around long records: one 4 MiB blob (crossing many
    CU shares: deferred, then taken by a whole wave in the tail kernel) and 48 KiB blobs (768 runs:
    taken by the whole wave, inside a share in the one-pass kernel or deferred when they cross one),
    corrupted and clean; region mode still engages (<= 6 KiB per message on average)."""
    rng = np.random.default_rng(8)
    msgs = []
    for i in range(20000):
        if i == 1500:
            size = 4 << 20
        elif i % 400 == 17:
            size = 48 << 10
        else:
            size = int(rng.integers(0, 1500))
        from datagen import stream_bytes

        content = stream_bytes(i, 0, size).tobytes()
        msgs.append(MF.put_message(MF.store_key("L%d" % i), MF.blob_properties_bytes(size), b"m" * (i % 30), content,
                                   version=3))
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    region = bytearray(b"".join(msgs))
    for i in (1500, 17, 417):  # flip a byte deep inside each long blob
        region[offs[i] + len(msgs[i]) - 5000] ^= 0x10
    region = bytes(region)
    expect = [MF.verify_message(region, o) for o in offs]
    assert len(region) <= 6144 * len(offs)
    st, end = run(gpu, region, offs)
    _expect_mode(gpu, msg_mode, len(region), len(offs))
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert st[1500] == MF.BLOB_CRC and st[17] == MF.BLOB_CRC and st[817] == 0


def test_unsorted_offsets_take_the_tail(gpu, msg_mode):
    """Offsets in random order over a region large enough for every CU: the one-pass kernel finds
    its messages by binary search of sorted offsets, sees they are not, and the tail kernel redoes
    every message; results identical to the sorted call's, reordered."""
    region, offs, expect = build_region(n=6000, seed=12, corrupt_frac=0.05, big_every=10**9)
    perm = np.random.default_rng(2).permutation(len(offs))
    st, end = run(gpu, region, [offs[j] for j in perm])
    assert st == [expect[j][0] for j in perm]
    assert end == [expect[j][1] for j in perm]


def test_long_records_split_over_the_grid(gpu, msg_mode):
    """Several multi-MiB blobs among small PUTs (tools/probes/long_mix.py's shape, scaled down): in
    region mode each is split into 64 KiB pieces that waves across the GPU hash from the run sums;
    the wave that finishes a record's last piece folds them (region_long_kernel, long_fold). Flips
    land in the first piece, on the last byte of one piece and the first byte of another, and in the
    last 64-B run of a blob; a 3 MiB + 1 B blob (an uneven last piece) and a 32 KiB + 1 B one (a
    single piece) stay clean. Every status and end equals the oracle's."""
    from datagen import stream_bytes

    sizes = {300: (4 << 20) + 13, 900: (3 << 20) + 1, 1400: (32 << 10) + 1, 2100: (5 << 20) - 7, 2500: 9 << 20}
    msgs = []
    for i in range(6000):
        size = sizes.get(i, 200 + (i * 37) % 1700)
        msgs.append(MF.put_message(MF.store_key("G%d" % i), MF.blob_properties_bytes(size), b"q" * (i % 11),
                                   stream_bytes(7000 + i, 0, size).tobytes(), version=1 + i % 3))
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    region = bytearray(b"".join(msgs))
    blob_at = {i: offs[i] + len(msgs[i]) - 8 - sizes[i] for i in sizes}  # blob content start
    # (record = 13-B head + content + 8-B CRC; piece p = record bytes [p * 64 KiB, (p + 1) * 64 KiB))
    flips = {300: 100, 2100: 3 * 65536 - 13 - 1, 2500: (9 << 20) - 3}  # 2100: piece 2's last byte
    for i, d in flips.items():
        region[blob_at[i] + d] ^= 0x04
    region[blob_at[2100] + 7 * 65536 - 13] ^= 0x80  # piece 7's first byte
    region = bytes(region)
    expect = [MF.verify_message(region, o) for o in offs]
    assert len(region) <= 6144 * len(offs)  # region mode engages
    st, end = run(gpu, region, offs, shift=3)
    _expect_mode(gpu, msg_mode, len(region), len(offs))
    assert st == [s for s, _ in expect]
    assert end == [e for _, e in expect]
    assert st[300] == st[2100] == st[2500] == MF.BLOB_CRC and st[900] == st[1400] == 0


def test_verify_graph_capture_and_replay(gpu, msg_mode):
    """ambrycrc_verify_messages_dev only enqueues work (the form is chosen on the host from the
    region's size, the long-record list is reset on the device by pass 1), so it can be captured
    into a HIP graph. Captured once over small PUTs with two multi-MiB blobs and replayed after the
    bytes change -- a flip in a small message, then one in a long blob's middle piece: every
    replay's statuses and ends equal the oracle's."""
    import torch

    from datagen import stream_bytes

    sizes = {200: (3 << 20) + 5, 700: (2 << 20) + 77}
    msgs = []
    for i in range(1500):
        size = sizes.get(i, 100 + (i * 53) % 2500)
        msgs.append(MF.put_message(MF.store_key("C%d" % i), MF.blob_properties_bytes(size), b"m" * (i % 7),
                                   stream_bytes(9100 + i, 0, size).tobytes(), version=1 + i % 3))
    offs = np.cumsum([0] + [len(x) for x in msgs[:-1]]).tolist()
    region = bytearray(b"".join(msgs))
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    o = torch.tensor(np.asarray(offs, dtype=np.int64), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gpu.verify_messages(dev, o)  # sizes the stream's default workspace outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            st, end = gpu.verify_messages(dev, o)
    torch.cuda.synchronize()

    def replay_check(b):
        dev.copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda())
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        expect = [MF.verify_message(bytes(b), x) for x in offs]
        assert st.cpu().numpy().view(np.uint32).tolist() == [e for e, _ in expect]
        assert end.cpu().numpy().tolist() == [e for _, e in expect]
        return expect

    assert all(e == 0 for e, _ in replay_check(region))
    region[offs[50] + len(msgs[50]) - 20] ^= 0x01
    assert replay_check(region)[50][0] != 0
    blob200 = offs[200] + len(msgs[200]) - 8 - sizes[200]
    region[blob200 + 21 * 65536 + 5] ^= 0x40
    got = replay_check(region)
    assert got[200][0] == MF.BLOB_CRC and got[700][0] == 0


def test_long_record_list_overflow(gpu, msg_mode):
    """More long records than region mode's grid-wide list holds (4,096): 4,200 PUTs with 33 KiB blobs
    (528 runs each, over the 512-run cut) among 100,800 small PUTs, so the records listed past the
    list's capacity fall back to their wave's queue (and past that to their own thread). One long
    record in ten has a flipped content bit, spread over the whole region (which records reach the
    list is decided by the device's atomics). Statuses and ends against the construction, and a
    sample of messages against the oracle."""
    import torch

    from datagen import stream_bytes

    small = MF.put_message(MF.store_key("s"), MF.blob_properties_bytes(300), b"u" * 200,
                           stream_bytes(77, 0, 300).tobytes(), version=3)
    longs = []
    for j in range(4200):
        blob = stream_bytes(50000 + j, 0, 33 << 10).tobytes()
        longs.append(MF.put_message(MF.store_key("L%d" % j), MF.blob_properties_bytes(len(blob)), b"", blob,
                                    version=1 + j % 3))
    parts, offs, is_long = [], [], []
    pos = 0
    for j in range(4200):
        for _ in range(24):
            parts.append(small)
            offs.append(pos)
            is_long.append(-1)
            pos += len(small)
        parts.append(longs[j])
        offs.append(pos)
        is_long.append(j)
        pos += len(longs[j])
    region = bytearray(b"".join(parts))
    flipped = set(range(3, 4200, 10))
    for j in flipped:
        i = 25 * j + 24
        region[offs[i] + len(longs[j]) - 8 - 1000] ^= 0x02  # inside the blob content
    region = bytes(region)
    assert len(region) <= 6144 * len(offs)
    r = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    o = torch.tensor(np.asarray(offs, dtype=np.int64), device="cuda")
    st, end = gpu.verify_messages(r, o)
    torch.cuda.synchronize()
    st = st.cpu().numpy().view(np.uint32)
    end = end.cpu().numpy()
    want_st = np.array([MF.BLOB_CRC if k in flipped else 0 for k in is_long], dtype=np.uint32)
    lens = np.array([len(small) if k < 0 else len(longs[k]) for k in is_long], dtype=np.int64)
    assert np.array_equal(st, want_st)
    assert np.array_equal(end, np.asarray(offs, dtype=np.int64) + lens)
    for i in list(range(0, len(offs), 997)) + [25 * j + 24 for j in (3, 4095, 4096, 4193, 4199)]:
        assert (int(st[i]), int(end[i])) == MF.verify_message(region, offs[i]), i
