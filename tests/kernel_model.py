"""CPU model of the gfx950 sweep kernel (ambry_amd/csrc/crc32_kernels.hip).

Test infrastructure: it replays the kernel's arithmetic -- the LDS image built
by libambrycrc (ambrycrc_debug_table_image), v_perm_b32 address formation,
slice-by-4 steps, nibble-table multiplies, the per-lane 1 KiB block hop, the
6-level wave tree and the byte-balanced wave/segment decomposition -- lane by lane in numpy,
so that layout or algebra mistakes show up on the CPU before a GPU run. It is
checked against zlib/the oracle in tests/test_kernel_model.py.
"""
from __future__ import annotations

import bisect
import ctypes

import numpy as np

K_SLICE_BYTES = 128 * 1024
K_NIB_BASE = K_SLICE_BYTES
K_NIB_SET = 512
K_FOLD_OFF = 0
K_TREE_OFF = K_FOLD_OFF + K_NIB_SET
K_POW_OFF = K_TREE_OFF + 6 * K_NIB_SET
K_POW_TABLES = 36
K_LDS_BYTES = K_NIB_BASE + K_POW_OFF + K_POW_TABLES * K_NIB_SET
K_IMG_INV_OFF = K_LDS_BYTES + 256  # nibble sets of x^(-8*2^k), k = 0..5 (crc32_layout.h)
K_INV_SETS = 6
K_IMG_REG_OFF = K_IMG_INV_OFF + K_INV_SETS * K_NIB_SET  # region pass 2's words (crc32_layout.h)
K_REG_H0, K_REG_GE, K_REG_LT, K_REG_AUX = 0, 64, 72, 80
K_REG_BYTE = 1024
K_REG_UN = 16 * (K_NIB_SET // 4)
K_IMG_BYTES = K_IMG_REG_OFF + 4 * (K_REG_AUX + K_REG_BYTE + K_REG_UN)
BLOCK = 1024
LANES = np.arange(64, dtype=np.uint32)


def table_image():
    from ambry_amd._lib import lib

    words = K_IMG_BYTES // 4
    buf = (ctypes.c_uint32 * words)()
    nbytes = lib().ambrycrc_debug_table_image(buf, words)
    assert nbytes == words * 4, nbytes
    return np.frombuffer(buf, dtype=np.uint32).copy()


class KernelModel:
    def __init__(self, img=None):
        self.img = table_image() if img is None else img
        self.xpow2 = self.img[K_LDS_BYTES // 4:K_LDS_BYTES // 4 + 64]
        col = (LANES & 31) << 2
        self.L = [((j >> 1) << 16) | ((j & 1) << 7) | col for j in range(4)]

    def lds(self, addr):
        return self.img[np.asarray(addr, dtype=np.int64) >> 2]

    @staticmethod
    def perm(L, x, k):
        # v_perm_b32(L, x, 0x0C06_k_04): byte0 = L.b0, byte1 = x.b_k, byte2 = L.b2, byte3 = 0
        return (L & 0xFF) | (((x >> (8 * k)) & 0xFF) << 8) | (((L >> 16) & 0xFF) << 16)

    def slice4(self, x, xin):
        t = (self.lds(self.perm(self.L[3], x, 0)) ^ self.lds(self.perm(self.L[2], x, 1)) ^
             self.lds(self.perm(self.L[1], x, 2)) ^ self.lds(self.perm(self.L[0], x, 3)))
        return (t ^ xin).astype(np.uint32)

    def rpiece(self, w, xin):
        s = self.slice4(w[:, 0], w[:, 1])
        s = self.slice4(s, w[:, 2])
        s = self.slice4(s, w[:, 3])
        return self.slice4(s, xin)

    def nib_mul(self, v, set_off):
        v = np.asarray(v, dtype=np.uint32)
        r = np.zeros_like(v)
        for n in range(8):
            r ^= self.lds(K_NIB_BASE + set_off + 64 * n + (((v >> (4 * n)) & 15) << 2))
        return r

    def shift_bytes(self, v, n):
        v = np.uint32(v)
        k = 0
        while n:
            if n & 1:
                if k < K_POW_TABLES:
                    v = self.nib_mul(np.array([v], dtype=np.uint32), K_POW_OFF + K_NIB_SET * k)[0]
                else:
                    v = np.uint32(gf2_mul(int(v), int(self.xpow2[k])))
            n >>= 1
            k += 1
        return int(v)

    def body_crc(self, mem: np.ndarray, bs: int, be: int, run: int = 1) -> int:
        """Raw CRC of [bs, be): lane l owns the run of `run` 16-B pieces at 16*run*l of every
        super-block of 1024*run bytes; the lane state hops one super-block per run
        (x^(8*1024*run) = POW[10+log2 run]); tree level l shifts by 16*run*2^l (POW[4+log2 run+l])."""
        lr = run.bit_length() - 1
        sb = BLOCK * run
        nb = (be - bs + sb - 1) // sb
        if nb == 0:
            return 0
        v0 = be - nb * sb
        s = np.zeros(64, dtype=np.uint32)
        for b in range(nb):
            w = np.zeros((run, 64, 4), dtype=np.uint32)
            for r in range(run):
                p = v0 + b * sb + 16 * run * LANES.astype(np.int64) + 16 * r
                for lane in range(64):
                    if p[lane] + 16 > bs:
                        # the kernel's load-address invariant: inside [floor16(bs), be)
                        assert (bs & ~15) <= p[lane] and p[lane] + 16 <= be, (bs, be, p[lane])
                        raw = bytearray(mem[p[lane]:p[lane] + 16].tobytes())
                        cut = bs - p[lane]
                        for i in range(max(0, cut)):
                            raw[i] = 0
                        w[r, lane] = np.frombuffer(bytes(raw), dtype="<u4")
            fold = (self.nib_mul(s, K_POW_OFF + K_NIB_SET * (10 + lr)) if b
                    else np.zeros(64, dtype=np.uint32))
            x = w[0][:, 0]
            words = [w[r][:, i] for r in range(run) for i in range(4)]
            for i in range(1, 4 * run):
                x = self.slice4(x, words[i])
            s = self.slice4(x, fold)
        for lvl in range(6):
            o = s[LANES ^ (1 << lvl)]
            sh = self.nib_mul(o, K_POW_OFF + K_NIB_SET * (4 + lr + lvl))
            s = np.where((LANES & (1 << lvl)) != 0, s ^ sh, s).astype(np.uint32)
        return int(s[63])

    def tail_crc(self, mem, p0: int, t: int) -> int:
        """Lane-parallel tail (kernel tail_crc): lane j: T_{k&3}[b_j] * x^(32*(k>>2)), k = t-1-j; XOR."""
        acc = 0
        for lane in range(t):
            b = int(mem[p0 + lane])
            k = t - 1 - lane
            j = k & 3
            v = int(self.lds(((j >> 1) << 16) | (b << 8) | ((j & 1) << 7) | ((lane & 31) << 2)))
            if k & 4:
                v = int(self.nib_mul(np.array([v], dtype=np.uint32), K_POW_OFF + K_NIB_SET * 2)[0])
            if k & 8:
                v = int(self.nib_mul(np.array([v], dtype=np.uint32), K_POW_OFF + K_NIB_SET * 3)[0])
            acc ^= v
        return acc

    def body_crc_t4(self, mem: np.ndarray, bs: int, be: int) -> int:
        """Coalesced loads + 4x4 quad transpose (sweep variant 12): per 4 KiB super-block, lane
        l = 4m+j loads piece l of each of the 4 blocks, then the quad transpose gives it the 64-B run
        [64m, 64m+64) of block j; fold x^(8*4096) once per run; tree over lane bits 2,3,4,5
        (shifts 64..512 B) then 0,1 (1024, 2048 B)."""
        sb = 4096
        nb = (be - bs + sb - 1) // sb
        if nb == 0:
            return 0
        v0 = be - nb * sb
        s = np.zeros(64, dtype=np.uint32)
        for b in range(nb):
            X = np.zeros((4, 64, 4), dtype=np.uint32)  # X[i][lane] = block i, piece lane
            for i in range(4):
                for lane in range(64):
                    p = v0 + b * sb + 1024 * i + 16 * lane
                    if p + 16 > bs:
                        assert (bs & ~15) <= p and p + 16 <= be, (bs, be, p)
                        raw = bytearray(mem[p:p + 16].tobytes())
                        for t in range(max(0, bs - p)):
                            raw[t] = 0
                        X[i, lane] = np.frombuffer(bytes(raw), dtype="<u4")
            # quad transpose: lane (m, j) element t <- lane (m, t) element j
            Y = np.zeros_like(X)
            for lane in range(64):
                m, j = lane >> 2, lane & 3
                for t in range(4):
                    Y[t, lane] = X[j, 4 * m + t]
            fold = self.nib_mul(s, K_POW_OFF + K_NIB_SET * 12) if b else np.zeros(64, dtype=np.uint32)
            words = [Y[t][:, c] for t in range(4) for c in range(4)]
            x = words[0]
            for c in range(1, 16):
                x = self.slice4(x, words[c])
            s = self.slice4(x, fold)
        for bit, k in ((2, 6), (3, 7), (4, 8), (5, 9), (0, 10), (1, 11)):
            o = s[LANES ^ (1 << bit)]
            sh = self.nib_mul(o, K_POW_OFF + K_NIB_SET * k)
            s = np.where((LANES & (1 << bit)) != 0, s ^ sh, s).astype(np.uint32)
        return int(s[63])

    def group_crc(self, mem: np.ndarray, segs, G: int, nbmax: int):
        """Group mode (sweep kernel group_crc): 64/G whole small chunks at once, lane gl of group gi
        owning bytes [16gl, 16gl+16) of every 16G-byte block of chunk gi, the initial register
        ~crc_in XORed into the chunk's first 4 bytes (r0 XOR'd into data, plus r0 >> 8len when
        len < 4), fold x^(8*16G) = POW[log2 16G], a log2(G)-level tree, the < 16-B tail
        lane-parallel. segs: [(cs, len, cin)] with len <= 16G*nbmax. Returns finalized CRCs."""
        BB = 16 * G
        lg = BB.bit_length() - 1
        out = []
        for cs, ln, cin in segs:
            assert len(segs) <= 64 // G
            rinit = (~cin) & 0xFFFFFFFF
            ce = cs + ln
            cb = max(cs, ce & ~15)
            nb = (cb - cs + BB - 1) // BB
            assert nb <= nbmax
            v0 = cb - nb * BB
            gl = np.arange(G, dtype=np.int64)

            def init_bytes(addr, nbytes):
                """XOR mask of the init register over bytes [addr, addr+nbytes) (little-endian)."""
                m = 0
                for i in range(nbytes):
                    o = addr + i - cs
                    if 0 <= o < 4:
                        m |= ((rinit >> (8 * o)) & 0xFF) << (8 * i)
                return m

            s = np.zeros(G, dtype=np.uint32)
            for b in range(nb):
                w = np.zeros((G, 4), dtype=np.uint32)
                for lane in range(G):
                    p = v0 + b * BB + 16 * lane
                    if p + 16 > cs:
                        assert (cs & ~15) <= p and p + 16 <= cb
                        raw = int.from_bytes(mem[p:p + 16].tobytes(), "little") ^ init_bytes(p, 16)
                        raw &= ~((1 << (8 * max(0, cs - p))) - 1)  # bytes before cs read as zero
                        w[lane] = np.frombuffer(raw.to_bytes(16, "little"), dtype="<u4")
                fold = self.nib_mul(s, K_POW_OFF + K_NIB_SET * lg) if b else np.zeros(G, dtype=np.uint32)
                L = [x[:G] for x in self.L]
                save = self.L
                self.L = L
                x = self.slice4(w[:, 0], w[:, 1])
                x = self.slice4(x, w[:, 2])
                x = self.slice4(x, w[:, 3])
                s = self.slice4(x, fold)
                self.L = save
            for lvl in range(G.bit_length() - 1):
                o = s[gl ^ (1 << lvl)]
                sh = self.nib_mul(o, K_TREE_OFF + K_NIB_SET * lvl)
                s = np.where((gl & (1 << lvl)) != 0, s ^ sh, s).astype(np.uint32)
            body = int(s[G - 1])
            t = ce - cb
            for bit in range(4):
                if (t >> bit) & 1:
                    body = int(self.nib_mul(np.array([body], dtype=np.uint32), K_POW_OFF + K_NIB_SET * bit)[0])
            tail = 0
            for lane in range(t):
                bval = int(mem[cb + lane]) ^ init_bytes(cb + lane, 1)
                k = t - 1 - lane
                j = k & 3
                v = int(self.lds(((j >> 1) << 16) | (bval << 8) | ((j & 1) << 7) | ((lane & 31) << 2)))
                if k & 4:
                    v = int(self.nib_mul(np.array([v], dtype=np.uint32), K_POW_OFF + K_NIB_SET * 2)[0])
                if k & 8:
                    v = int(self.nib_mul(np.array([v], dtype=np.uint32), K_POW_OFF + K_NIB_SET * 3)[0])
                tail ^= v
            crc = body ^ tail ^ 0xFFFFFFFF
            if ln < 4:
                crc ^= rinit >> (8 * ln)
            out.append(crc & 0xFFFFFFFF)
        return out

    def batch(self, mem: np.ndarray, off, length, crc_in=None, nwaves: int = 4096, quantum: int = 1024,
              run: int = 1, group=None, min_share: int = 0, window: int = 0):
        """Replays plan + sweep kernels with `nwaves` waves; returns the list of CRCs.
        group=(G, nbmax): runs of whole chunks of <= 16*G*nbmax bytes inside a 64-descriptor
        window go through group_crc, up to 64/G at a time, as the kernel's group mode does.
        window: sweep rounds (SweepArgs::window) -- a batch of more than `window` bytes is cut
        into R rounds of nwaves equal shares; wave w takes shares w, w + nwaves, ..."""
        n = len(off)
        off = [int(x) for x in off]
        length = [int(x) for x in length]
        byte_start = [0]
        for ln in length:
            byte_start.append(byte_start[-1] + ln)
        total = byte_start[n]
        out = [0 if length[c] else (0 if crc_in is None else int(crc_in[c])) for c in range(n)]
        share = ((total + nwaves - 1) // nwaves + quantum - 1) // quantum * quantum
        share = max(share, min_share)
        step = 0
        if window and total > window:
            rounds = (total + window - 1) // window
            share = ((total + rounds * nwaves - 1) // (rounds * nwaves) + quantum - 1) // quantum * quantum
            share = max(share, min_share)
            step = nwaves * share
        shares = []
        for w in range(nwaves):
            g0 = w * share
            while share and g0 < total:
                shares.append((g0, min(total, g0 + share)))
                if not step:
                    break
                g0 += step
        for g0, g1 in shares:
            c = bisect.bisect_right(byte_start, g0, 0, n) - 1
            win_end = c + 64
            while c < n:
                bsc = byte_start[c]
                if bsc >= g1:
                    break
                if c >= win_end:
                    win_end += 64
                if group is not None:
                    G, nbmax = group

                    def small(i):
                        return (i < min(n, win_end) and byte_start[i] < g1 and length[i] <= 16 * G * nbmax
                                and byte_start[i] >= g0 and byte_start[i] + length[i] <= g1)

                    if small(c):
                        run_ = [c]
                        while len(run_) < 64 // G and small(run_[-1] + 1):
                            run_.append(run_[-1] + 1)
                        segs = [(off[i], length[i], 0 if crc_in is None else int(crc_in[i])) for i in run_]
                        for i, v in zip(run_, self.group_crc(mem, segs, G, nbmax)):
                            out[i] = v  # whole chunk: plain store
                        c = run_[-1] + 1
                        continue
                ln = length[c]
                if ln == 0:
                    c += 1
                    continue
                cs = off[c]
                ce = cs + ln
                cb = max(cs, ce & ~15)
                r0 = snap_cut(cs, ln, g0 - bsc) if g0 > bsc else 0
                r1 = snap_cut(cs, ln, g1 - bsc) if g1 - bsc < ln else ln
                if r0 >= r1:
                    c += 1
                    continue
                sa, se = cs + r0, cs + r1
                be = cb if se == ce else se
                assert be % 16 == 0 or be == cs, (sa, se, be)
                r = 0
                if sa < be:
                    body = self.body_crc_t4(mem, sa, be) if run == -4 else self.body_crc(mem, sa, be, run)
                    r = self.shift_bytes(body, ce - be)
                if se == ce and ce > cb:
                    r ^= self.tail_crc(mem, max(sa, cb), ce - max(sa, cb))
                if r0 == 0:
                    cin = 0 if crc_in is None else int(crc_in[c])
                    r ^= self.shift_bytes((~cin) & 0xFFFFFFFF, ln) ^ 0xFFFFFFFF
                out[c] ^= r
                c += 1
        return [x & 0xFFFFFFFF for x in out]


class RegionModel:
    """Region mode of the message verify (crc32_kernels.hip region_runs_kernel, region_crc.h
    record_crc), scalar: run sums of the 64-B runs from base = region start rounded down
    to 64 B, then each job's CRC from its head / tail runs' bytes, the run sums between, four
    Horner streams and the x^(-8d) un-shift, with the image's one-copy slice tables and nibble
    sets exactly as the kernel addresses them."""

    def __init__(self, img):
        self.img = img
        self.T = [[int(img[(((j >> 1) << 16) | (b << 8) | ((j & 1) << 7)) >> 2]) for b in range(256)]
                  for j in range(4)]

    def _nib(self, v, byte_off):
        r = 0
        for n in range(8):
            r ^= int(self.img[(byte_off + 64 * n + 4 * ((v >> (4 * n)) & 15)) >> 2])
        return r

    def pow_(self, v, k):  # v * x^(8*2^k)
        return self._nib(v, K_NIB_BASE + K_POW_OFF + K_NIB_SET * k)

    def inv(self, v, k):  # v * x^(-8*2^k)
        return self._nib(v, K_IMG_INV_OFF + K_NIB_SET * k)

    def step4(self, x):
        T = self.T
        return T[3][x & 0xFF] ^ T[2][(x >> 8) & 0xFF] ^ T[1][(x >> 16) & 0xFF] ^ T[0][x >> 24]

    def runs(self, mem: bytes, reg0: int):
        """Pass 1: rk[k] = raw CRC of bytes [64k, 64k + 64) of base (zeros outside the region)."""
        nruns = (reg0 + len(mem) + 63) // 64
        buf = bytes(reg0) + mem + bytes(nruns * 64 - reg0 - len(mem))
        out = []
        for k in range(nruns):
            s = 0
            for w in range(16):
                s = self.step4(s ^ int.from_bytes(buf[64 * k + 4 * w:64 * k + 4 * w + 4], "little"))
            out.append(s)
        return out

    def run_bytes(self, buf, r0, lo, hi, ninit):
        """hash_run: four 4-step piece chains merged by x^(8*16), x^(8*32)."""
        p = []
        for q in range(4):
            s = 0
            for w in range(4 * q, 4 * q + 4):
                v = 0
                for b in range(4):
                    o = 4 * w + b
                    x = buf[r0 + o] if lo <= o < hi else 0
                    if lo <= o < lo + ninit:
                        x ^= 0xFF
                    v |= x << (8 * b)
                s = self.step4(s ^ v)
            p.append(s)
        return self.pow_(self.pow_(p[0], 4) ^ p[1], 5) ^ self.pow_(p[2], 4) ^ p[3]

    def direct_crc(self, mem: bytes, reg0: int, off: int, ln: int) -> int:
        """region_proc.h record_crc_direct: the wave on one record straight from the bytes -- 64-B
        runs aligned to the record's end, run R - 64(V - v) + l in lane l of round v (bytes before
        the record zeroed, its first four XORed with 0xFF), folded by x^(8*4096), merged by the
        x^(8*64*2^k) tree (POW[6..11]); lane 63 ends at the record's end."""
        buf = bytes(reg0) + mem
        pa, pb = reg0 + off, reg0 + off + ln
        R = (ln + 63) // 64
        V = (R + 63) // 64
        acc = [0] * 64
        for v in range(V):
            for l in range(64):
                j = R - 64 * (V - v) + l
                c = 0
                if j >= 0:
                    o = pb - 64 * (R - j)
                    for w in range(16):
                        x = 0
                        for b in range(4):
                            pos = o + 4 * w + b
                            y = buf[pos] if pa <= pos < pb else 0
                            if pa <= pos < pa + 4:
                                y ^= 0xFF
                            x |= y << (8 * b)
                        c = self.step4(c ^ x)
                acc[l] = self.pow_(acc[l], 12) ^ c
        for k in range(6):
            acc = [acc[l] ^ self.pow_(acc[l - (1 << k)], 6 + k) if l & (1 << k) else acc[l] for l in range(64)]
        return acc[63] ^ 0xFFFFFFFF

    def assembly_crc(self, msg: bytes, a0: int, s: int, e: int) -> int:
        """Round 4's put_assemble_kernel's record CRC (removed in round 6 for put_stream_kernel; git
        history, tools/probes/put_assemble.hip): the message on the output's 16-B grid
        (piece p = bytes [16p - a0, 16p - a0 + 16)), each lane's pieces l, l + 64, ... up to q (the
        piece of byte e - 1) hashed from zero with bytes outside [s, e) zeroed and the first four
        XORed with 0xFF, folded by x^(8*1024); lanes rotated so that lane q mod 64 is last, merged by
        the 6-level x^(8*16*2^k) tree, un-shifted by d = 16(q + 1) - a0 - e bytes."""
        fold = lambda v: self._nib(v, K_NIB_BASE + K_FOLD_OFF)  # noqa: E731
        tree = lambda v, k: self._nib(v, K_NIB_BASE + K_TREE_OFF + K_NIB_SET * k)  # noqa: E731
        q = (e - 1 + a0) // 16
        d = 16 * (q + 1) - a0 - e
        ni = min(4, e - s)
        acc = [0] * 64
        for p in range(q + 1):
            c = 0
            for w in range(4):
                v = 0
                for b in range(4):
                    pos = 16 * p - a0 + 4 * w + b
                    x = msg[pos] if s <= pos < e else 0
                    if s <= pos < s + ni:
                        x ^= 0xFF
                    v |= x << (8 * b)
                c = self.step4(c ^ v)
            acc[p % 64] = fold(acc[p % 64]) ^ c
        t = [acc[(v + q + 1) % 64] for v in range(64)]  # virtual lane v
        for k in range(6):
            t = [t[v] ^ tree(t[v - (1 << k)], k) if v & (1 << k) else t[v] for v in range(64)]
        V = t[63]
        for k in range(4):
            if d & (1 << k):
                V = self.inv(V, k)
        if e - s < 4:
            V ^= 0xFFFFFFFF >> (8 * (e - s))
        return V ^ 0xFFFFFFFF

    def job_crc(self, mem: bytes, reg0: int, rk, off: int, ln: int) -> int:
        if ln == 0:
            return 0
        nruns = len(rk)
        buf = bytes(reg0) + mem + bytes(nruns * 64 - reg0 - len(mem))
        pa = reg0 + off
        pb = pa + ln
        if ln < 4:
            c = 0xFFFFFFFF
            for i in range(pa, pb):
                c = self.T[0][(c ^ buf[i]) & 0xFF] ^ (c >> 8)
            return c ^ 0xFFFFFFFF
        A0, B1 = pa & ~63, (pb + 63) & ~63
        n, k0 = (B1 - A0) >> 6, A0 >> 6
        lo, hi = pa - A0, min(pb - A0, 64)
        tin = hi - lo
        H = self.run_bytes(buf, A0, lo, hi, min(tin, 4))
        if tin < 4:
            H ^= 0xFFFFFFFF >> (8 * tin)
        tail = n >= 2 and pb & 63 != 0
        T = self.run_bytes(buf, B1 - 64, 0, pb - (B1 - 64), 0) if tail else 0
        ng = (n + 3) >> 2
        e0, elast = k0 + n - 4 * ng, k0 + n - 1
        s = [0, 0, 0, 0]  # s[3]: updated last
        for e in range(e0, e0 + 4 * ng):
            v = 0 if e < k0 else H if e == k0 else T if (e == elast and tail) else rk[e]
            nv = self.pow_(s[0], 8) ^ v
            s = [s[1], s[2], s[3], nv]
        V = s[3] ^ self.pow_(s[2], 6) ^ self.pow_(s[1], 7) ^ self.pow_(self.pow_(s[0], 6), 7)
        d = B1 - pb
        for k in range(K_INV_SETS):
            if d >> k & 1:
                V = self.inv(V, k)
        return V ^ 0xFFFFFFFF


    def job_crc_aux(self, mem: bytes, reg0: int, rk, off: int, ln: int) -> int:
        """record_crc with region_msg_kernel's Aux words (region_crc.h): head / tail runs masked by
        the image's GE / LT words and no initial-register bytes, H0[lo] XORed into the head run,
        group 0 patched (padding zero, head run H), Horner by the x^(8*256) byte tables with the
        raw last-run sum swapped for T afterwards, streams merged by x^(8*64) three times, and the
        un-shift as x^(-8 (d & 7)) then x^(-64 (d >> 3)) from the 16 un-shift sets."""
        if ln == 0:
            return 0
        if ln < 4:
            return self.job_crc(mem, reg0, rk, off, ln)
        reg = self.img[K_IMG_REG_OFF // 4:]
        bt = reg[K_REG_AUX:K_REG_AUX + K_REG_BYTE]
        un = K_IMG_REG_OFF + 4 * (K_REG_AUX + K_REG_BYTE)

        def bmul(v):
            return int(bt[v & 0xFF] ^ bt[256 + ((v >> 8) & 0xFF)] ^ bt[512 + ((v >> 16) & 0xFF)] ^ bt[768 + (v >> 24)])

        def masked(buf, r0, lo, hi):
            p = []
            for q in range(4):
                s = 0
                for d in range(4):
                    w = 4 * q + d
                    c = 16 * w
                    v = int.from_bytes(buf[r0 + 4 * w:r0 + 4 * w + 4], "little")
                    v &= int(reg[K_REG_LT + (min(max(4 * hi, c), c + 16) - c) // 4])
                    v &= int(reg[K_REG_GE + (min(max(4 * lo, c), c + 16) - c) // 4])
                    s = self.step4(s ^ v)
                p.append(s)
            return self.pow_(self.pow_(p[0], 4) ^ p[1], 5) ^ self.pow_(p[2], 4) ^ p[3]

        nruns = len(rk)
        buf = bytes(reg0) + mem + bytes(nruns * 64 - reg0 - len(mem))
        pa = reg0 + off
        pb = pa + ln
        A0, B1 = pa & ~63, (pb + 63) & ~63
        n, k0 = (B1 - A0) >> 6, A0 >> 6
        lo, hi = pa - A0, min(pb - A0, 64)
        tin = hi - lo
        tail = n >= 2 and pb & 63 != 0
        H = masked(buf, A0, lo, hi) ^ int(reg[K_REG_H0 + lo])
        if tin < 4:
            H ^= 0xFFFFFFFF >> (8 * tin)
        T = masked(buf, B1 - 64, 0, pb - (B1 - 64)) if tail else 0
        ng = (n + 3) >> 2
        e0 = k0 + n - 4 * ng
        vals = [rk[e] if e >= 0 else 0 for e in range(e0, e0 + 4 * ng)]
        rb = n - 4 * ng
        for q in range(4):
            vals[q] = 0 if rb + q < 0 else H if rb + q == 0 else vals[q]
        s = [0, 0, 0, 0]
        for v in vals:
            s = [s[1], s[2], s[3], bmul(s[0]) ^ v]
        if tail:
            s[3] ^= T ^ rk[k0 + n - 1]
        V = s[3] ^ self.pow_(s[2] ^ self.pow_(s[1] ^ self.pow_(s[0], 6), 6), 6)
        d = B1 - pb
        V = self._nib(self._nib(V, un + K_NIB_SET * (d & 7)), un + K_NIB_SET * (8 + (d >> 3)))
        return V ^ 0xFFFFFFFF

    def long_fold(self, sl, last: int) -> int:
        """message_kernels.hip long_fold: a long record's CRC from its 64 KiB pieces' CRCs sl (the
        last piece `last` bytes) -- full pieces in rounds of 64 lanes aligned so that the last full
        piece is lane 63's, folded in-lane by POW[22] over rounds, the DPP tree (lane l takes lane
        l - 2^k's value times POW[16 + k]; lane 63 read), x^(8 last), plus the last piece's CRC."""
        np_ = len(sl)
        M = np_ - 1
        acc = 0
        if M:
            V = (M + 63) // 64
            lanes = [0] * 64
            for v in range(V):
                for l in range(64):
                    j = 64 * v + l - (64 * V - M)
                    x = sl[j] if j >= 0 else 0
                    lanes[l] = (self.pow_(lanes[l], 22) if v else 0) ^ x
            for k in range(6):
                lanes = [lanes[l] ^ self.pow_(lanes[l - (1 << k)], 16 + k) if l & (1 << k) else lanes[l]
                         for l in range(64)]
            acc = lanes[63]
            for k in range(17):
                if last >> k & 1:
                    acc = self.pow_(acc, k)
        return acc ^ sl[np_ - 1]

    def job_crc_wave(self, mem: bytes, reg0: int, rk, off: int, ln: int) -> int:
        """region_crc.h record_crc_runs_wave: a long record by the whole wave from the run sums --
        the record's runs [A0, B1) (head and tail runs from the bytes, as job_crc), run
        n - 64(V - v) + l in lane l of round v, folded over rounds by x^(8*4096) (POW[12]), merged by
        the tree over 256-B lane slices (POW[8 + k]), lane 63 ending at B1, then the x^(-8d) un-shift."""
        nruns = len(rk)
        buf = bytes(reg0) + mem + bytes(nruns * 64 - reg0 - len(mem))
        pa = reg0 + off
        pb = pa + ln
        A0, B1 = pa & ~63, (pb + 63) & ~63
        n, k0 = (B1 - A0) // 64, A0 // 64
        lo, hi = pa - A0, min(pb - A0, 64)
        tin = hi - lo
        tail_bytes = n >= 2 and (pb & 63) != 0
        H = self.run_bytes(buf, A0, lo, hi, min(tin, 4))
        if tin < 4:
            H ^= 0xFFFFFFFF >> (8 * tin)
        T = self.run_bytes(buf, B1 - 64, 0, pb - (B1 - 64), 0) if tail_bytes else 0
        V = ((n + 255) // 256 + 3) & ~3  # 256-run rounds padded at the front; round v -> stream v mod 4
        st = [[0] * 4 for _ in range(64)]
        for v in range(V):
            for l in range(64):
                x = 0
                for j in range(4):  # lane l: runs 4l .. 4l + 3 of the round, folded by x^(8*64)
                    r = n - 256 * (V - v) + 4 * l + j
                    val = 0 if r < 0 else H if r == 0 else T if (r == n - 1 and tail_bytes) else rk[k0 + r]
                    x = self.pow_(x, 6) ^ val if j else val
                st[l][v % 4] = self.pow_(st[l][v % 4], 16) ^ x
        acc = [self.pow_(self.pow_(self.pow_(s[0], 14) ^ s[1], 14) ^ s[2], 14) ^ s[3] for s in st]
        for k in range(6):
            acc = [acc[l] ^ self.pow_(acc[l - (1 << k)], 8 + k) if l & (1 << k) else acc[l] for l in range(64)]
        x = acc[63]
        d = B1 - pb
        for k in range(6):
            if d & (1 << k):
                x = self.inv(x, k)
        return x ^ 0xFFFFFFFF

def snap_cut(cs: int, ln: int, r: int) -> int:
    a = (cs + r + 15) & ~15
    return min(a - cs, ln)


def gf2_mul(a: int, b: int) -> int:
    p = 0
    for i in range(32):
        if (a >> (31 - i)) & 1:
            p ^= b
        b = (b >> 1) ^ (0xEDB88320 if b & 1 else 0)
    return p
