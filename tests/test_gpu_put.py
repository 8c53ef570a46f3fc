"""GPU write path (ambrycrc_serialize_puts_dev): batches of PUT messages laid out in HBM with every
CRC trailer filled, byte-exact against oracle/message_format.py's layouts (zlib CRCs), then
verified by ambrycrc_verify_messages_dev (round trip). Copy mode (fields and blobs gathered from
their own buffers, at any alignment) and in-place mode (bytes already at ambrycrc_put_layout's
offsets); batches under and over the group-phase threshold; 4 MiB blobs."""
import numpy as np
import pytest

from test_put_serialize import expected, random_messages

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mf():
    import importlib.util
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("message_format", os.path.join(root, "oracle", "message_format.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(autouse=True, params=["stream", "jobs"])
def put_form(request, gpu):
    """Every case in both copy-mode forms: messages of at most 6 KiB streamed (put_stream_kernel, the
    default) and every message through the job path (ambrycrc_set_put_stream_max(dev, 0))."""
    prev = gpu.set_put_stream_max(0, 6144 if request.param == "stream" else 0)
    yield request.param
    gpu.set_put_stream_max(0, prev)


def _dev(b):
    import torch

    return torch.frombuffer(bytearray(b if len(b) else b"\0"), dtype=torch.uint8).cuda()


def _far(b, at):
    """b in device memory `at` bytes into a larger allocation (a view whose buffer starts lower)."""
    import torch

    d = _dev(b)
    big = torch.full((d.numel() + at,), 0x5A, dtype=torch.uint8, device="cuda")
    big[at:] = d
    return big[at:]


def _run(gpu, mf, msgs, out_align, field_align, gap, in_place=False, place=("key", "enckey", "props", "usermeta",
                                                                           "blob"), far=0):
    import torch

    from ambry_amd.messages import layout, pack_batch, serialize_dev

    descs, fields, blobs, offs, total = pack_batch(msgs, out_align=out_align, field_align=field_align, gap=gap)
    host_out = bytearray(b"\xAA" * total)  # filler: gaps must stay untouched
    if in_place:
        for m, o in zip(msgs, offs):
            _, fo = layout(m)
            for name in place:
                b = getattr(m, name)
                if b:
                    host_out[o + fo[name]:o + fo[name] + len(b)] = b
    out = _dev(bytes(host_out))
    mlen = torch.empty(len(msgs), dtype=torch.int64, device="cuda")
    dev_in = (lambda b: _far(b, far)) if far else _dev
    fields_in = None if in_place and "key" in place else dev_in(fields)
    blobs_in = None if in_place and "blob" in place else dev_in(blobs)
    serialize_dev(_dev(descs.tobytes()), out, fields_in, blobs_in, msg_len=mlen)
    torch.cuda.synchronize()
    got = out.cpu().numpy().tobytes()
    exp = bytearray(b"\xAA" * total)
    for m, o in zip(msgs, offs):
        e = expected(mf, m)
        exp[o:o + len(e)] = e
    assert got == bytes(exp)
    assert mlen.cpu().numpy().tolist() == [len(expected(mf, m)) for m in msgs]
    status, end = gpu.verify_messages(out, torch.tensor(offs, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    # BlobType has two values: a type-2 blob record fails the reader's check (AMBRYCRC_MSG_BAD_RECORD)
    assert status.cpu().numpy().tolist() == [mf.BAD_RECORD if m.blob_type >= 2 else 0 for m in msgs]
    assert end.cpu().numpy().tolist() == [o + len(expected(mf, m)) for o, m in zip(offs, msgs)]


@pytest.mark.parametrize("out_align,field_align,gap", [(1, 1, 0), (16, 16, 0), (1, 7, 3), (4096, 1, 0)])
def test_serialize_batch_copy_mode(gpu, mf, out_align, field_align, gap):
    _run(gpu, mf, random_messages(mf, 400, seed=100 + out_align + field_align), out_align, field_align, gap)


def test_serialize_batch_in_place(gpu, mf):
    _run(gpu, mf, random_messages(mf, 300, seed=7), 1, 1, 5, in_place=True)


def test_serialize_group_phase_batch(gpu, mf):
    """4,000 messages = 20,000 CRC jobs (>= 16,384: the group phase takes the small records)."""
    _run(gpu, mf, random_messages(mf, 4000, seed=9, max_blob=9000), 1, 3, 0)


@pytest.mark.parametrize("far", [(64 << 20) + 3, (1 << 30) + 11])
def test_serialize_class0_heavy_far_sources(gpu, mf, far):
    """Round-2 fault regression (an experimental class-0 tail load read the sweep's base block, and the
    copy-through then passed base = null): 6,000 PUTs whose every field is <= 256 B (30,000 jobs, all
    in group class 0 of the copy-through sweep), sources placed `far` bytes into their allocations.
    The copy-through's base is now the lowest source buffer (PutArgs::src_base)."""
    from ambry_amd.messages import PutMessage

    from datagen import stream_bytes

    rng = np.random.default_rng(far & 0xFFFF)
    msgs = []
    for i in range(6000):
        blen = int(rng.integers(0, 200))
        enc = stream_bytes(i, 5, int(rng.integers(0, 64))).tobytes() if i % 3 else None
        msgs.append(PutMessage(key=mf.store_key("c0-%d" % i), props=mf.blob_properties_bytes(blen, service_id="s%d" % i),
                               usermeta=stream_bytes(i, 7 << 20, int(rng.integers(0, 120))).tobytes(),
                               blob=stream_bytes(i ^ 77, 0, blen).tobytes(), enckey=enc, header_version=3,
                               life_version=i % 4))
    _run(gpu, mf, msgs, 1, 1, 0, far=far)


def test_serialize_large_blobs(gpu, mf):
    from ambry_amd.messages import PutMessage
    from datagen import stream_bytes

    msgs = [PutMessage(key=mf.store_key("big%d" % i), props=mf.blob_properties_bytes(4 << 20),
                       usermeta=b"m" * 1000, blob=stream_bytes(50 + i, 0, (4 << 20) - (i % 3)).tobytes(),
                       header_version=3) for i in range(12)]
    _run(gpu, mf, msgs, 1, 1, 0)


@pytest.mark.parametrize("place", [("blob",), ("key", "enckey", "props", "usermeta")])
def test_serialize_batch_mixed(gpu, mf, place):
    """One source buffer given, the other slots already in place: the copy-through sweep copies
    the given fields and re-reads the in-place ones where they lie."""
    _run(gpu, mf, random_messages(mf, 300, seed=13), 1, 5, 2, in_place=True, place=place)


def test_serialize_large_blobs_copy_through(gpu, mf):
    """Blobs of 4-17 MiB at ragged lengths: the copy-through sweep splits each over several waves'
    byte shares (segments that start mid-blob, nontemporal body stores, the trailing bytes), so
    every segment boundary's head piece and tail must land exactly."""
    from ambry_amd.messages import PutMessage

    from datagen import stream_bytes

    sizes = [4 << 20, (4 << 20) + 13, (17 << 20) + 5, 3, (1 << 20) + 4109, 65536 + 1, 9 << 20]
    msgs = []
    for i, blen in enumerate(sizes * 2):
        msgs.append(PutMessage(key=mf.store_key("big-%d" % i), props=mf.blob_properties_bytes(blen),
                               usermeta=stream_bytes(i, 3 << 20, 1000 + i).tobytes(),
                               blob=stream_bytes(i, 0, blen).tobytes(), header_version=3, life_version=i % 3))
    _run(gpu, mf, msgs, 1, 7, 5)


def test_serialize_6k_messages(gpu, mf):
    """Messages of 6,100 to 6,200 bytes, byte by byte (round 4's whole-message assembly cut-off, 6,144
    B; round 6's streamed form has the same cut-off, kStreamPutMax), under header versions 1-3,
    with and without an encryption key, at unaligned output offsets: every byte as the oracle lays
    it out."""
    from ambry_amd.messages import PutMessage, layout
    from datagen import stream_bytes

    msgs = []
    for i, want in enumerate(range(6100, 6201)):
        v = 1 + i % 3
        enc = b"k" * (i % 17) if v >= 2 and i % 2 else None
        base = PutMessage(key=mf.store_key("cut-%d" % i), props=mf.blob_properties_bytes(10), usermeta=b"u" * (i % 7),
                          blob=b"", enckey=enc, header_version=v, life_version=i % 4 if v == 3 else 0)
        L0, _ = layout(base)
        blen = want - L0
        props = mf.blob_properties_bytes(blen)
        m = PutMessage(key=base.key, props=props, usermeta=base.usermeta, blob=stream_bytes(i, 3, blen).tobytes(),
                       enckey=enc, header_version=v, life_version=base.life_version)
        assert layout(m)[0] == want
        msgs.append(m)
    _run(gpu, mf, msgs, 1, 3, 5)


def test_serialize_graph_capture_and_replay(gpu, mf):
    """ambrycrc_serialize_puts_dev only enqueues work, so it can be captured into a HIP graph:
    captured once over 300 PUTs in copy mode and replayed after every blob's bytes change (same
    sizes); each replay's output is the oracle's layout of the current bytes, every CRC trailer
    included."""
    import dataclasses

    import torch

    from ambry_amd.messages import pack_batch, serialize_dev
    from datagen import stream_bytes

    msgs = random_messages(mf, 300, seed=21, max_blob=9000)
    descs, fields, blobs, offs, total = pack_batch(msgs, out_align=1, field_align=3, gap=2)
    d, f, b = _dev(descs.tobytes()), _dev(fields), _dev(blobs)
    out = _dev(b"\xAA" * total)
    mlen = torch.empty(len(msgs), dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        serialize_dev(d, out, f, b, msg_len=mlen)  # sizes the stream's default workspace outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            serialize_dev(d, out, f, b, msg_len=mlen)
    torch.cuda.synchronize()

    def check(ms):
        g.replay()
        torch.cuda.synchronize()
        exp = bytearray(b"\xAA" * total)
        for m, o in zip(ms, offs):
            e = expected(mf, m)
            exp[o:o + len(e)] = e
        assert out.cpu().numpy().tobytes() == bytes(exp)
        assert mlen.cpu().numpy().tolist() == [len(expected(mf, m)) for m in ms]

    check(msgs)
    msgs2 = [dataclasses.replace(m, blob=stream_bytes(500 + i, 11, len(m.blob)).tobytes()) if m.blob else m
             for i, m in enumerate(msgs)]
    _, _, blobs2, offs2, total2 = pack_batch(msgs2, out_align=1, field_align=3, gap=2)
    assert offs2 == offs and total2 == total and len(blobs2) == len(blobs)
    b.copy_(_dev(blobs2))
    check(msgs2)


def test_serialize_descriptors_out_of_output_order(gpu, mf):
    """Descriptors in an order unrelated to their output offsets (a permutation; messages back to back,
    so neighbours share 16-B pieces and 64-B runs but sit at distant indices, taken by different waves
    and workgroups): every message lands at its own offset byte-exact, gaps untouched, msg_len in
    descriptor order."""
    import torch

    from ambry_amd.messages import pack_batch, serialize_dev

    msgs = random_messages(mf, 500, seed=31, max_blob=7000)
    descs, fields, blobs, offs, total = pack_batch(msgs, out_align=1, field_align=1, gap=0)
    perm = np.random.default_rng(5).permutation(len(msgs))
    out = _dev(b"\xAA" * total)
    mlen = torch.empty(len(msgs), dtype=torch.int64, device="cuda")
    serialize_dev(_dev(descs[perm].tobytes()), out, _dev(fields), _dev(blobs), msg_len=mlen)
    torch.cuda.synchronize()
    exp = bytearray(b"\xAA" * total)
    for m, o in zip(msgs, offs):
        e = expected(mf, m)
        exp[o:o + len(e)] = e
    assert out.cpu().numpy().tobytes() == bytes(exp)
    assert mlen.cpu().numpy().tolist() == [len(expected(mf, msgs[i])) for i in perm]


def test_serialize_streamed_after_job_batch(gpu, mf):
    """The streamed messages' job entries are only zeroed when the job path runs (a gated clear launch,
    put_layout_kernel with clear_short): a batch of long messages fills the stream's workspace with job
    entries, then a batch of the same size, mostly short with a few long, reuses it -- every byte as the
    oracle lays it out, so no stale entry of the first batch is copied or hashed into the second."""
    import dataclasses

    from datagen import stream_bytes

    n = 200
    longs = random_messages(mf, n, seed=41, max_blob=9000)
    longs = [dataclasses.replace(m, blob=stream_bytes(900 + i, 1, 7000 + i).tobytes(),
                                 props=mf.blob_properties_bytes(7000 + i)) for i, m in enumerate(longs)]
    _run(gpu, mf, longs, 1, 1, 0)
    mixed = random_messages(mf, n, seed=43, max_blob=3000)
    mixed = [dataclasses.replace(m, blob=stream_bytes(700 + i, 2, 8000).tobytes(),
                                 props=mf.blob_properties_bytes(8000)) if i % 37 == 5 else m
             for i, m in enumerate(mixed)]
    _run(gpu, mf, mixed, 1, 3, 1)


def test_serialize_back_to_back_one_stream(gpu, mf):
    """The streamed form's job path runs on the stream's side stream (ring slot per call, the caller's
    stream waiting on the done signal): 40 calls on one stream -- past the 32 ring slots -- every third
    batch with long messages (the job path runs), each into its own output, then one synchronize of
    that stream only. Every output is the oracle's layout."""
    import dataclasses

    import torch

    from ambry_amd.messages import pack_batch, serialize_dev
    from datagen import stream_bytes

    s = torch.cuda.Stream()
    cases = []
    with torch.cuda.stream(s):
        for c in range(40):
            msgs = random_messages(mf, 60, seed=300 + c, max_blob=2000)
            if c % 3 == 1:
                msgs = [dataclasses.replace(m, blob=stream_bytes(c * 97 + i, 4, 6500 + i).tobytes(),
                                            props=mf.blob_properties_bytes(6500 + i)) if i % 7 == 2 else m
                        for i, m in enumerate(msgs)]
            descs, fields, blobs, offs, total = pack_batch(msgs, out_align=1, field_align=1, gap=1)
            d = torch.frombuffer(bytearray(descs.tobytes()), dtype=torch.uint8).to("cuda", non_blocking=False)
            f = torch.frombuffer(bytearray(fields), dtype=torch.uint8).to("cuda")
            b = torch.frombuffer(bytearray(blobs if len(blobs) else b"\0"), dtype=torch.uint8).to("cuda")
            out = torch.full((total,), 0xAA, dtype=torch.uint8, device="cuda")
            serialize_dev(d, out, f, b)
            cases.append((msgs, offs, total, out, (d, f, b)))
    s.synchronize()
    for msgs, offs, total, out, _ in cases:
        exp = bytearray(b"\xAA" * total)
        for m, o in zip(msgs, offs):
            e = expected(mf, m)
            exp[o:o + len(e)] = e
        assert out.cpu().numpy().tobytes() == bytes(exp)
