"""Minimal FLAC encoder -- TEST INFRASTRUCTURE ONLY (written for
tests/test_cpu_flac.py from the FLAC format specification, RFC 9639).

It emits the stream features the LibriSpeech fixtures never exercise, so the
native decoder (csrc/flac.cpp) is checked on them too: stereo decorrelation
(left/side, side/right, mid/side), wasted bits, CONSTANT / VERBATIM / FIXED
(orders 0-4) subframes, Rice and Rice2 residual coding with several partition
orders and escape partitions, 8/12/16/20/24-bit samples, frame-header sample
size codes, and a short final block.  Not compressed well; not used by the
product.
"""
import hashlib

import numpy as np


class BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.bits.append((int(v) >> i) & 1)

    def sput(self, v, n):
        self.put(int(v) & ((1 << n) - 1), n)

    def unary(self, q):
        self.bits.extend([0] * int(q))
        self.bits.append(1)

    def align(self):
        while len(self.bits) % 8:
            self.bits.append(0)

    def tobytes(self):
        assert len(self.bits) % 8 == 0
        b = np.packbits(np.array(self.bits, dtype=np.uint8))
        return bytes(b)


def crc8(d):
    c = 0
    for x in d:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(d):
    c = 0
    for x in d:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _fixed_residual(x, order):
    x = x.astype(np.int64)
    r = x.copy()
    if order == 1:
        r[1:] = x[1:] - x[:-1]
    elif order == 2:
        r[2:] = x[2:] - 2 * x[1:-1] + x[:-2]
    elif order == 3:
        r[3:] = x[3:] - 3 * x[2:-1] + 3 * x[1:-2] - x[:-3]
    elif order == 4:
        r[4:] = x[4:] - 4 * x[3:-1] + 6 * x[2:-2] - 4 * x[1:-3] + x[:-4]
    return r[order:]


def _residual(w, res, bs, order, method, porder, escape_every):
    w.put(method, 2)
    w.put(porder, 4)
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    parts = 1 << porder
    i = 0
    for p in range(parts):
        cnt = (bs >> porder) - (order if p == 0 else 0)
        seg = res[i:i + cnt]
        i += cnt
        if escape_every and p % escape_every == 0:
            nb = max(1, int(max(abs(int(v)) for v in seg).bit_length() + 1)) if len(seg) else 1
            w.put(esc, pbits)
            w.put(nb, 5)
            for v in seg:
                w.sput(v, nb)
            continue
        mean = float(np.mean(np.abs(seg))) if len(seg) else 0.0
        k = max(0, min(esc - 1, int(np.log2(mean + 1))))
        w.put(k, pbits)
        for v in seg:
            u = (int(v) << 1) ^ (int(v) >> 63) if v >= 0 else ((-int(v)) << 1) - 1
            w.unary(u >> k)
            w.put(u & ((1 << k) - 1), k)


def _subframe(w, x, bps, kind, order, method, porder, escape_every):
    x = np.asarray(x, dtype=np.int64)
    wasted = 0
    if kind != "constant" and np.any(x):
        while not np.any(x & ((1 << (wasted + 1)) - 1)) and wasted < bps - 1:
            wasted += 1
    w.put(0, 1)
    if kind == "constant":
        w.put(0, 6)
    elif kind == "verbatim":
        w.put(1, 6)
    else:
        w.put(8 + order, 6)
    if wasted:
        w.put(1, 1)
        w.unary(wasted - 1)
    else:
        w.put(0, 1)
    xs = x >> wasted
    eb = bps - wasted
    if kind == "constant":
        w.sput(xs[0], eb)
    elif kind == "verbatim":
        for v in xs:
            w.sput(v, eb)
    else:
        for v in xs[:order]:
            w.sput(v, eb)
        _residual(w, _fixed_residual(xs, order), len(xs), order, method, porder, escape_every)


def encode(pcm, sample_rate, bps, block=1024, chmode="independent", kind="fixed", order=2,
           method=0, porder=2, escape_every=0, ss_code_in_header=True):
    """pcm: int [frames, channels] -> FLAC bytes."""
    pcm = np.asarray(pcm, dtype=np.int64)
    n, nch = pcm.shape
    nb = (bps + 7) // 8
    raw = b"".join(int(v).to_bytes(4, "little", signed=True)[:nb] for v in pcm.reshape(-1))
    md5 = hashlib.md5(raw).digest()
    out = bytearray(b"fLaC")
    si = BitWriter()
    si.put(block, 16)
    si.put(block, 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(sample_rate, 20)
    si.put(nch - 1, 3)
    si.put(bps - 1, 5)
    si.put(n, 36)
    out += bytes([0x80, 0, 0, 34]) + si.tobytes() + md5
    ss_codes = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}
    fno = 0
    for s0 in range(0, n, block):
        x = pcm[s0:s0 + block]
        bs = len(x)
        w = BitWriter()
        w.put(0x3FFE, 14)
        w.put(0, 1)
        w.put(0, 1)
        w.put(7, 4)                       # 16-bit blocksize-1 follows
        w.put(0, 4)                       # sample rate from STREAMINFO
        code = {"independent": nch - 1, "left_side": 8, "side_right": 9, "mid_side": 10}[chmode]
        w.put(code, 4)
        w.put(ss_codes[bps] if ss_code_in_header else 0, 3)
        w.put(0, 1)
        assert fno < 128
        w.put(fno, 8)                     # UTF-8 frame number (one byte)
        w.put(bs - 1, 16)
        hdr = w.tobytes()
        w.put(crc8(hdr), 8)
        if chmode == "independent":
            chans = [(x[:, c], bps) for c in range(nch)]
        else:
            L, R = x[:, 0], x[:, 1]
            if chmode == "left_side":
                chans = [(L, bps), (L - R, bps + 1)]
            elif chmode == "side_right":
                chans = [(L - R, bps + 1), (R, bps)]
            else:
                chans = [((L + R) >> 1, bps), (L - R, bps + 1)]
        po = porder
        while po and (bs % (1 << po) or (bs >> po) < order):
            po -= 1
        for c, (v, b) in enumerate(chans):
            k = kind
            if k == "constant" and np.any(v != v[0]):
                k = "verbatim"
            _subframe(w, v, b, k, min(order, bs), method, po, escape_every)
        w.align()
        body = w.tobytes()
        out += body + crc16(body).to_bytes(2, "big")
        fno += 1
    return bytes(out)
