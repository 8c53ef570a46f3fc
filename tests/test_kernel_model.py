"""CPU replay of the gfx950 sweep kernel's arithmetic (tests/kernel_model.py) against the oracle.

Catches LDS-layout / GF(2) / tiling mistakes without a GPU; the real kernel is
checked by tests/test_gpu_parity.py on the MI355X."""
import numpy as np
import pytest

from datagen import stream_bytes
from kernel_model import KernelModel


@pytest.fixture(scope="module")
def model(ambry):
    return KernelModel()


CASES = [(0, 0), (0, 1), (3, 5), (16, 16), (5, 15), (5, 16), (5, 17), (0, 1024), (7, 1024), (1, 3000),
         (100, 70000), (13, 65536 + 7), (64, 200000), (4095, 4097), (1, 1)]


@pytest.mark.parametrize("nwaves", [1, 2, 3, 7, 64, 4096])
def test_model_matches_oracle(model, oracle, nwaves):
    mem = stream_bytes(123, 0, 300000)
    off = [c[0] for c in CASES]
    ln = [c[1] for c in CASES]
    got = model.batch(mem, off, ln, nwaves=nwaves)
    exp = list(oracle.batch(mem, off, ln))
    assert got == exp
    assert model.batch(mem, off, ln, nwaves=nwaves, min_share=16384, group=(16, 32)) == exp  # kernel defaults


@pytest.mark.parametrize("run", [2, 4, -4])
def test_model_lane_runs(model, oracle, run):
    """R-piece lane runs (variants 8-11) and the quad-transposed 64-B runs (run=-4, variant 12)."""
    mem = stream_bytes(321, 0, 300000)
    off = [c[0] for c in CASES]
    ln = [c[1] for c in CASES]
    exp = list(oracle.batch(mem, off, ln))
    for nw in (1, 3, 64):
        assert model.batch(mem, off, ln, nwaves=nw, run=run) == exp


def test_model_crc_in(model, oracle):
    mem = stream_bytes(77, 0, 100000)
    off = [c[0] for c in CASES[:10]]
    ln = [c[1] for c in CASES[:10]]
    cin = np.array([(i * 0x9E3779B9) & 0xFFFFFFFF for i in range(10)], dtype=np.uint32)
    for nw in (1, 5, 300):
        assert model.batch(mem, off, ln, crc_in=cin, nwaves=nw) == list(oracle.batch(mem, off, ln, crc_in=cin))


def test_model_cut_points_everywhere(model, oracle):
    """Wave cuts landing in every residue of a chunk (incl. its last 15 bytes) must tile it exactly."""
    mem = stream_bytes(5, 0, 20000)
    for cs, ln in ((3, 4000), (16, 4096), (1, 1040), (0, 17)):
        for nw in range(2, 12):
            assert model.batch(mem, [cs], [ln], nwaves=nw, quantum=16) == list(oracle.batch(mem, [cs], [ln]))


def test_model_large_shift_slow_path(model):
    """shift_bytes beyond the 2^36-byte table range takes the gf2 fallback; compare with the host ABI."""
    import ambry_amd

    for n in (1 << 36, (1 << 37) + 12345, (1 << 40) - 1):
        assert model.shift_bytes(0xFFFFFFFF ^ 0x1234, n) ^ 0xFFFFFFFF == ambry_amd.zeros(0x1234, n)


@pytest.mark.parametrize("group", [(16, 8), (16, 16), (32, 8)])
def test_model_group_mode(model, oracle, group):
    """Group mode: whole small chunks, 64/G at a time, init register folded into the data.
    Lengths 0..~4 KiB at every end/start residue, mixed with chunks too big for a group."""
    G, nbmax = group
    rng = np.random.default_rng(G * 100 + nbmax)
    mem = stream_bytes(17, 0, 400000)
    smax = 16 * G * nbmax
    ln = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 255, 256, 257, 1000, smax - 1, smax, smax + 1, 20000]
    ln += [int(x) for x in rng.integers(0, smax + 1, size=40)]
    off = [int(x) for x in rng.integers(0, 380000, size=len(ln))]
    off[:5] = [0, 1, 15, 17, 33]
    cin = np.array([(i * 0x9E3779B9 + 5) & 0xFFFFFFFF for i in range(len(ln))], dtype=np.uint32)
    exp = list(oracle.batch(mem, off, ln, crc_in=cin))
    for nw, ms in ((1, 0), (3, 0), (7, 32768)):
        assert model.batch(mem, off, ln, crc_in=cin, nwaves=nw, group=group, min_share=ms) == exp
    assert model.batch(mem, off, ln, nwaves=2, group=group) == list(oracle.batch(mem, off, ln))


@pytest.mark.parametrize("nwaves,window", [(3, 50000), (7, 100000), (64, 20000), (5, 300000)])
def test_model_sweep_rounds(model, oracle, nwaves, window):
    """Sweep rounds (SweepArgs::window): shares w, w + nwaves, ... over R rounds cut chunks at
    round boundaries too; the XOR of the segment results is still each chunk's CRC."""
    mem = stream_bytes(77, 0, 300000)
    off = [c[0] for c in CASES]
    ln = [c[1] for c in CASES]
    exp = list(oracle.batch(mem, off, ln))
    assert model.batch(mem, off, ln, nwaves=nwaves, window=window, run=-4) == exp
    assert model.batch(mem, off, ln, nwaves=nwaves, window=window, min_share=16384) == exp


def test_region_model_matches_zlib(ambry):
    """Region mode's algebra (64-B run sums, head / tail runs from the bytes with the initial
    register folded in, four Horner streams, x^(-8d) un-shift) against zlib, on jobs that start and
    end at every residue mod 64 (and 1-3 B jobs), in regions whose start is not 64-aligned."""
    import random
    import zlib

    from kernel_model import RegionModel, table_image

    rm = RegionModel(table_image())
    rng = random.Random(7)
    for reg0 in (0, 5, 63):
        mem = stream_bytes(900 + reg0, 0, 1500).tobytes()
        rk = rm.runs(mem, reg0)
        jobs = [(0, len(mem)), (0, 1), (1, 2), (2, 3), (len(mem) - 3, 3), (len(mem) - 4, 4)]
        jobs += [(a, ln) for a in (0, 1, 58, 59, 60, 61, 62, 63, 64) for ln in (4, 5, 6, 7, 63, 64, 65, 127, 128, 129, 700)]
        jobs += [(rng.randrange(0, 1000), rng.randrange(0, 500)) for _ in range(60)]
        for a, ln in jobs:
            if a + ln > len(mem):
                continue
            assert rm.job_crc(mem, reg0, rk, a, ln) == zlib.crc32(mem[a:a + ln]), (reg0, a, ln)
            assert rm.job_crc_aux(mem, reg0, rk, a, ln) == zlib.crc32(mem[a:a + ln]), (reg0, a, ln)


def test_region_wave_model_matches_zlib(ambry):
    """The whole-wave form of a long record's CRC (region_crc.h record_crc_runs_wave: rounds of 64
    run sums aligned to the record's last run, folded by x^(8*4096), merged by the x^(8*64*2^k) DPP
    tree, un-shifted to the record's end) against zlib, on records of one to ~15 rounds starting
    and ending at odd offsets, in a region whose start is not 64-aligned."""
    import zlib

    from kernel_model import RegionModel, table_image

    rm = RegionModel(table_image())
    reg0 = 37
    mem = stream_bytes(4242, 0, 60000).tobytes()
    rk = rm.runs(mem, reg0)
    for a, ln in ((0, 33000), (5, 16411), (63, 40000), (1000, 17000), (3, 59990), (129, 257 * 64)):
        assert rm.job_crc_wave(mem, reg0, rk, a, ln) == zlib.crc32(mem[a:a + ln]), (a, ln)


def test_assembly_model_matches_zlib(ambry):
    """Round 4's whole-message assembly (tools/probes/put_assemble.hip until round 6): a record's
    CRC from the message's pieces on the output's 16-B grid -- per-lane piece hashes folded over the
    wave's 1 KiB chunks, the lanes rotated so the record's last piece comes last, the x^(8*16*2^k)
    tree, the x^(-8d) un-shift -- against zlib, for records of 2 B to ~6 KiB at every message
    alignment mod 16."""
    import random
    import zlib

    from kernel_model import RegionModel, table_image

    rm = RegionModel(table_image())
    rng = random.Random(11)
    msg = stream_bytes(777, 0, 6200).tobytes()
    cases = [(0, 2), (0, 3), (5, 9), (17, 4), (40, 6 + 1000), (1063, 13 + 4096), (3, 6144)]
    cases += [(rng.randrange(0, 6000), rng.choice([2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 1024, 1040])) for _ in range(20)]
    for a0 in (0, 1, 7, 15):
        for s, ln in cases:
            e = min(s + ln, len(msg))
            assert rm.assembly_crc(msg, a0, s, e) == zlib.crc32(msg[s:e]), (a0, s, ln)


def test_direct_record_model_matches_zlib(ambry):
    """The tail kernel's wave-wide record CRC straight from the region's bytes (region_proc.h
    record_crc_direct: end-aligned 64-B runs, a fold by x^(8*4096) over rounds, the x^(8*64*2^k)
    tree) against zlib, for records of 4 B to ~9 KiB (one and three rounds) at odd offsets."""
    import zlib

    from kernel_model import RegionModel, table_image

    rm = RegionModel(table_image())
    mem = stream_bytes(4343, 0, 12000).tobytes()
    for reg0 in (0, 13):
        for a, ln in ((0, 4), (1, 5), (63, 64), (7, 65), (100, 1006), (33, 4109), (5, 4096), (9, 9000)):
            assert rm.direct_crc(mem, reg0, a, ln) == zlib.crc32(mem[a:a + ln]), (reg0, a, ln)


def test_long_fold_model_matches_zlib(ambry):
    """region_long_kernel's fold of a long record's 64 KiB piece CRCs (message_kernels.hip long_fold:
    rounds of 64 lanes, the DPP tree by x^(8*2^(16+k)), the last piece's length) against zlib, for
    1, 2, 64, 65 and 130 pieces and last pieces of 1 B, a few bytes and a full 64 KiB."""
    import zlib

    from kernel_model import RegionModel, table_image

    rm = RegionModel(table_image())
    P = 64 << 10
    for npieces, last in ((1, 5), (2, 1), (2, P), (64, P), (65, 3), (130, 777)):
        ln = (npieces - 1) * P + last
        mem = stream_bytes(npieces * 31 + last, 0, ln).tobytes()
        sl = [zlib.crc32(mem[i:i + P]) for i in range(0, ln, P)]
        assert len(sl) == npieces
        assert rm.long_fold(sl, last) == zlib.crc32(mem), (npieces, last)
