"""A small FLAC encoder for round-trip tests of the host FLAC decoder (vasr_flac_decode).

Test infrastructure only.  It writes the format as RFC 9639 specifies it and deliberately
exercises every decoder path the reference's inputs can take (LibriSpeech FLAC, torchaudio.load
in reference audio.py:47): CONSTANT / VERBATIM / FIXED 0-4 / LPC 1-32 subframes, wasted bits,
Rice and Rice2 residuals with partition orders and escape partitions, the four stereo
decorrelation modes, fixed and variable blocking, block-size and sample-rate header codes,
CRC-8 / CRC-16.  Encoding choices are explicit per frame (no search), so a test names the
feature it covers.
"""

from __future__ import annotations

import numpy as np

_SR_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
             48000: 10, 96000: 11}
_BPS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


class BitWriter:
    def __init__(self):
        self.buf = bytearray()
        self.acc = 0
        self.n = 0

    def write(self, v: int, bits: int):
        if bits == 0:
            return
        self.acc = (self.acc << bits) | (v & ((1 << bits) - 1))
        self.n += bits
        while self.n >= 8:
            self.n -= 8
            self.buf.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def unary(self, q: int):
        while q >= 32:
            self.write(0, 32)
            q -= 32
        self.write(1, q + 1)

    def align(self):
        if self.n:
            self.write(0, 8 - self.n)

    def bytes(self) -> bytes:
        assert self.n == 0
        return bytes(self.buf)


def crc8(d: bytes) -> int:
    c = 0
    for x in d:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(d: bytes) -> int:
    c = 0
    for x in d:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _utf8_num(v: int) -> bytes:
    if v < 0x80:
        return bytes([v])
    for nb in range(2, 8):
        if v < (1 << (5 * nb + 1)):
            break
    out = []
    for _ in range(nb - 1):
        out.append(0x80 | (v & 0x3F))
        v >>= 6
    lead = ((0xFF << (8 - nb)) & 0xFF) | v
    return bytes([lead] + out[::-1])


def _rice(w: BitWriter, res, k: int, escape_bits=None, method=0):
    pb = 4 if method == 0 else 5
    if escape_bits is not None:
        w.write((1 << pb) - 1, pb)
        w.write(escape_bits, 5)
        for r in res:
            w.write(int(r), escape_bits)
        return
    w.write(k, pb)
    for r in res:
        r = int(r)
        u = (-2 * r - 1) if r < 0 else 2 * r
        w.unary(u >> k)
        w.write(u & ((1 << k) - 1), k)


def _residual(w: BitWriter, res, order: int, bs: int, porder: int, k, method: int = 0, escape=()):
    """k: Rice parameter per partition (int or list); escape: partitions stored raw."""
    w.write(method, 2)
    w.write(porder, 4)
    parts = 1 << porder
    ks = k if isinstance(k, (list, tuple)) else [k] * parts
    pos = 0
    for p in range(parts):
        cnt = (bs >> porder) - (order if p == 0 else 0)
        seg = res[pos:pos + cnt]
        pos += cnt
        if p in escape:
            need = max([int(abs(int(v))).bit_length() + 1 for v in seg] + [0]) if len(seg) else 0
            _rice(w, seg, 0, escape_bits=need, method=method)
        else:
            _rice(w, seg, ks[p], method=method)


def _fixed_residual(x, order):
    x = x.astype(np.int64)
    if order == 0:
        return x.copy()
    d = x.copy()
    for _ in range(order):
        d = np.diff(d)
    return d


def lpc_coeffs(x, order: int, precision: int):
    """Quantised LPC coefficients (autocorrelation + Levinson-Durbin), FLAC style."""
    xf = x.astype(np.float64)
    win = np.hanning(len(xf) + 2)[1:-1] if len(xf) > 2 else np.ones(len(xf))
    xw = xf * win
    ac = np.array([np.dot(xw[:len(xw) - i], xw[i:]) for i in range(order + 1)])
    ac[0] *= 1.0 + 1e-9
    a = np.zeros(order)
    err = ac[0] if ac[0] > 0 else 1.0
    for i in range(order):
        acc = ac[i + 1] - np.dot(a[:i], ac[i:0:-1][:i])
        kk = acc / err
        a_new = a.copy()
        a_new[i] = kk
        a_new[:i] = a[:i] - kk * a[:i][::-1]
        a = a_new
        err *= (1 - kk * kk)
        if err <= 0:
            err = 1e-9
    cmax = np.max(np.abs(a)) if order else 1.0
    lim = (1 << (precision - 1)) - 1
    shift = precision - 1 - (int(np.floor(np.log2(cmax))) + 1 if cmax > 0 else 0)
    shift = max(0, min(15, shift))
    q = np.clip(np.round(a * (1 << shift)), -lim - 1, lim).astype(np.int64)
    return q, shift


def _lpc_residual(x, q, shift):
    x = x.astype(np.int64)
    order = len(q)
    res = np.empty(len(x) - order, np.int64)
    for i in range(order, len(x)):
        acc = int(np.dot(q, x[i - order:i][::-1]))
        res[i - order] = x[i] - (acc >> shift)
    return res


def subframe(w: BitWriter, x, bps: int, kind: str = "fixed", order: int = 2, k=None, porder: int = 0,
             wasted: int = 0, method: int = 0, escape=(), precision: int = 12):
    """One subframe of samples x (int64) at sample size bps."""
    x = np.asarray(x, np.int64)
    bs = len(x)
    w.write(0, 1)
    codes = {"constant": 0, "verbatim": 1}
    if kind in codes:
        w.write(codes[kind], 6)
    elif kind == "fixed":
        w.write(8 + order, 6)
    elif kind == "lpc":
        w.write(31 + order, 6)
    else:
        raise ValueError(kind)
    if wasted:
        assert np.all((x & ((1 << wasted) - 1)) == 0)
        w.write(1, 1)
        w.unary(wasted - 1)
        x = x >> wasted
        bps -= wasted
    else:
        w.write(0, 1)
    if kind == "constant":
        assert np.all(x == x[0])
        w.write(int(x[0]), bps)
        return
    if kind == "verbatim":
        for v in x:
            w.write(int(v), bps)
        return
    for v in x[:order]:
        w.write(int(v), bps)
    if kind == "fixed":
        res = _fixed_residual(x, order)
    else:
        q, shift = lpc_coeffs(x, order, precision)
        w.write(precision - 1, 4)
        w.write(shift, 5)
        for c in q:
            w.write(int(c), precision)
        res = _lpc_residual(x, q, shift)
    if k is None:
        mean = float(np.mean(np.abs(res))) if len(res) else 0.0
        k = max(0, min(14 if method == 0 else 30, int(np.log2(mean + 1))))
    _residual(w, res, order, bs, porder, k, method, escape)


def frame(number: int, chans, bps: int, sample_rate: int, mode: str = "independent", variable: bool = False,
          sub=None, bs_explicit: bool = False, sr_explicit: bool = False) -> bytes:
    """One frame.  chans: list of int64 arrays (equal length).  mode: independent | left_side |
    side_right | mid_side.  sub: per-channel subframe kwargs."""
    bs = len(chans[0])
    nch = len(chans)
    sub = sub or [{}] * nch
    w = BitWriter()
    w.write(0x3FFE, 14)
    w.write(0, 1)
    w.write(1 if variable else 0, 1)
    common = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
              8192: 13, 16384: 14, 32768: 15}
    if bs in common and not bs_explicit:
        bcode, btail = common[bs], None
    elif bs <= 256:
        bcode, btail = 6, (bs - 1, 8)
    else:
        bcode, btail = 7, (bs - 1, 16)
    w.write(bcode, 4)
    if sr_explicit:
        if sample_rate % 10 == 0 and sample_rate // 10 < 65536:
            scode, stail = 14, (sample_rate // 10, 16)
        else:
            scode, stail = 13, (sample_rate, 16)
    else:
        scode, stail = _SR_CODES.get(sample_rate, 0), None
    w.write(scode, 4)
    ch_code = {"independent": nch - 1, "left_side": 8, "side_right": 9, "mid_side": 10}[mode]
    w.write(ch_code, 4)
    w.write(_BPS_CODES.get(bps, 0), 3)
    w.write(0, 1)
    for byte in _utf8_num(number):
        w.write(byte, 8)
    if btail:
        w.write(*btail)
    if stail:
        w.write(*stail)
    hdr = w.bytes()
    w.write(crc8(hdr), 8)
    xs = [np.asarray(c, np.int64) for c in chans]
    if mode == "left_side":
        xs, sizes = [xs[0], xs[0] - xs[1]], [bps, bps + 1]
    elif mode == "side_right":
        xs, sizes = [xs[0] - xs[1], xs[1]], [bps + 1, bps]
    elif mode == "mid_side":
        xs, sizes = [(xs[0] + xs[1]) >> 1, xs[0] - xs[1]], [bps, bps + 1]
    else:
        sizes = [bps] * nch
    for c in range(nch):
        subframe(w, xs[c], sizes[c], **sub[c])
    w.align()
    body = w.bytes()
    return body + crc16(body).to_bytes(2, "big")


def streaminfo(sample_rate: int, channels: int, bps: int, total: int, min_bs: int = 16, max_bs: int = 65535) -> bytes:
    w = BitWriter()
    w.write(min_bs, 16)
    w.write(max_bs, 16)
    w.write(0, 24)
    w.write(0, 24)
    w.write(sample_rate, 20)
    w.write(channels - 1, 3)
    w.write(bps - 1, 5)
    w.write(total, 36)
    w.write(0, 128)  # MD5 unset
    return w.bytes()


def encode(chans, sample_rate: int, bps: int, block: int = 4096, frame_kw=None, extra_meta: bool = True,
           id3: bool = False, total=None) -> bytes:
    """Whole stream.  chans: list of int arrays (one per channel).  frame_kw(i, start, n) -> kwargs
    for frame() (mode, sub, variable, ...)."""
    chans = [np.asarray(c, np.int64) for c in chans]
    n = len(chans[0])
    info = streaminfo(sample_rate, len(chans), bps, n if total is None else total)
    meta = bytearray()
    blocks = [(0, info)]
    if extra_meta:
        blocks.append((4, (7).to_bytes(4, "little") + b"vasrenc" + (0).to_bytes(4, "little")))  # VORBIS_COMMENT
        blocks.append((1, b"\0" * 16))  # PADDING
    for i, (typ, data) in enumerate(blocks):
        last = i == len(blocks) - 1
        meta += bytes([(0x80 if last else 0) | typ]) + len(data).to_bytes(3, "big") + data
    out = bytearray()
    if id3:
        out += b"ID3\x03\x00\x00" + bytes([0, 0, 0, 10]) + b"\0" * 10
    out += b"fLaC" + meta
    start, idx = 0, 0
    while start < n:
        kw = dict(frame_kw(idx, start, n) if frame_kw else {})
        bs = min(kw.pop("block", block), n - start)
        variable = kw.get("variable", False)
        out += frame(start if variable else idx, [c[start:start + bs] for c in chans], bps, sample_rate, **kw)
        start += bs
        idx += 1
    return bytes(out)
