"""Deterministic synthetic PNG / JPEG files for the texture-decoder tests.

Test infrastructure: a PNG writer (every colour type and bit depth, the five
row filters, Adam7, tRNS, split IDATs, stored/fixed/dynamic deflate through
Python's zlib) and a small baseline JPEG writer (numpy DCT, Annex K Huffman
tables; 4:4:4, 4:2:2, 4:2:0, 4:4:0, 4:1:1, grey, 'RGB' ids, Adobe CMYK,
restart intervals, non-interleaved scans, 16-bit quantisers).  The decoded
RGBA8 of every variant by stb_image v2.28 (the reference's decoder, built by
oracle/Makefile.ref) is recorded as a SHA-256 in tests/golden/textures.json
by tests/golden/make_texture_golden.py.
"""
import struct
import zlib

import numpy as np


def _pattern(h, w, c, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), ((x + y) * 7) % 256,
                     ((x ^ y) * 13) % 256], axis=-1)[..., :c].astype(np.int32)
    noise = rng.integers(-40, 41, size=(h, w, c))
    edge = ((x // 5 + y // 3) % 2)[..., None] * 90
    return np.clip(base + noise + edge, 0, 255).astype(np.int64)


# ------------------------------------------------------------------ PNG
def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def _filter_rows(rows, bpp, filters):
    """rows: list of uint8 arrays (one scanline each); returns filtered bytes."""
    out = bytearray()
    prior = np.zeros_like(rows[0], dtype=np.int32) if rows else None
    for k, r in enumerate(rows):
        f = filters[k % len(filters)]
        cur = r.astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]]) if len(cur) > bpp else np.zeros_like(cur)
        if len(cur) <= bpp:
            a = np.zeros_like(cur)
        c = np.concatenate([np.zeros(bpp, np.int32), prior[:-bpp]]) if len(cur) > bpp else np.zeros_like(cur)
        b = prior
        pred = [np.zeros_like(cur), a, b, (a + b) >> 1, _paeth(a, b, c)][f]
        out.append(f)
        out += ((cur - pred) & 255).astype(np.uint8).tobytes()
        prior = cur
    return bytes(out)


def _pack(samples, depth):
    """one scanline of samples (ints) -> bytes at `depth` bits per sample."""
    if depth == 16:
        return np.asarray(samples, dtype=">u2").view(np.uint8)
    if depth == 8:
        return np.asarray(samples, dtype=np.uint8)
    bits = np.unpackbits(np.asarray(samples, dtype=np.uint8)[:, None], axis=1)[:, 8 - depth:].reshape(-1)
    return np.packbits(bits)


def png(w, h, color, depth, interlace=False, trns=False, filters=(0, 1, 2, 3, 4), level=6, idat_split=1,
        seed=1):
    """Returns PNG bytes."""
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[color]
    maxv = (1 << depth) - 1
    img = _pattern(h, w, ch, seed)
    if color == 3:
        img = (img[..., 0] * 7 + img[..., :1].sum(-1)) % (min(256, maxv + 1))
        img = img[..., None]
    elif depth == 16:
        img = img * 257 + (np.arange(w)[None, :, None] % 3)
    elif depth < 8:
        img = img >> (8 - depth)
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, int(interlace)))
    if color == 3:
        n = min(256, maxv + 1)
        pal = np.stack([np.arange(n) * 37 % 256, np.arange(n) * 91 % 256, 255 - np.arange(n)], -1).astype(np.uint8)
        out += _chunk(b"PLTE", pal.tobytes())
        if trns:
            out += _chunk(b"tRNS", bytes((i * 53) % 256 for i in range(max(1, n // 2))))
    elif trns and color in (0, 2):
        key = [int(v) for v in img[h // 2, w // 2, :ch]]
        out += _chunk(b"tEXt", b"Comment\x00ancillary chunk")  # skipped by decoders
        out += _chunk(b"tRNS", b"".join(struct.pack(">H", v) for v in key))
    bpp = max(1, ch * depth // 8)
    passes = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
    raw = b""
    for (x0, y0, dx, dy) in (passes if interlace else [(0, 0, 1, 1)]):
        sub = img[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        rows = [_pack(sub[y].reshape(-1), depth) for y in range(sub.shape[0])]
        raw += _filter_rows(rows, bpp, filters)
    z = zlib.compress(raw, level)
    step = max(1, len(z) // idat_split + 1)
    for k in range(0, len(z), step):
        out += _chunk(b"IDAT", z[k:k + step])
    return out + _chunk(b"IEND", b"")


PNG_VARIANTS = {
    "grey1": dict(w=37, h=23, color=0, depth=1),
    "grey2_adam7": dict(w=37, h=23, color=0, depth=2, interlace=True),
    "grey4_trns": dict(w=33, h=17, color=0, depth=4, trns=True),
    "grey8": dict(w=64, h=40, color=0, depth=8, level=0),
    "grey8_trns_adam7": dict(w=29, h=31, color=0, depth=8, trns=True, interlace=True),
    "grey16_trns": dict(w=21, h=19, color=0, depth=16, trns=True),
    "rgb8": dict(w=53, h=41, color=2, depth=8, idat_split=4),
    "rgb8_trns": dict(w=40, h=12, color=2, depth=8, trns=True, level=1),
    "rgb16_adam7": dict(w=19, h=27, color=2, depth=16, interlace=True),
    "pal1": dict(w=45, h=9, color=3, depth=1),
    "pal2_trns": dict(w=30, h=30, color=3, depth=2, trns=True),
    "pal4_adam7": dict(w=17, h=13, color=3, depth=4, interlace=True),
    "pal8_trns": dict(w=61, h=35, color=3, depth=8, trns=True, filters=(4,)),
    "greya8": dict(w=26, h=26, color=4, depth=8, filters=(3, 1)),
    "greya16": dict(w=15, h=33, color=4, depth=16),
    "rgba8_adam7": dict(w=50, h=50, color=6, depth=8, interlace=True),
    "rgba16": dict(w=23, h=11, color=6, depth=16, filters=(2,)),
    "rgba8_1x1": dict(w=1, h=1, color=6, depth=8),
    "rgb8_3x2_adam7": dict(w=3, h=2, color=2, depth=8, interlace=True),
}

# -------------------------------------------------------------------- JPEG
_ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                    13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
                    45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
_QL = np.array([16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56, 14, 17,
                22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92, 49, 64,
                78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99])
_QC = np.array([17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99, 47, 66,
                99, 99, 99, 99, 99, 99] + [99] * 32)
# Annex K.3 tables: (bits[16], values)
_DC_L = ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12)))
_DC_C = ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12)))
_AC_L = ([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d], [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71, 0x14,
    0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09,
    0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a,
    0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65,
    0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88,
    0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9,
    0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])
_AC_C = ([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77], [
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22, 0x32,
    0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16,
    0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39,
    0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86,
    0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8,
    0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9,
    0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])


def _codes(spec):
    bits, vals = spec
    code, k, table = 0, 0, {}
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            table[vals[k]] = (code, length)
            code += 1
            k += 1
        code <<= 1
    return table


class _BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, code, length):
        self.acc = (self.acc << length) | (code & ((1 << length) - 1))
        self.n += length
        while self.n >= 8:
            b = (self.acc >> (self.n - 8)) & 255
            self.out.append(b)
            if b == 0xFF:
                self.out.append(0)
            self.n -= 8

    def flush(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)
        self.acc = 0


def _dct_matrix():
    m = np.zeros((8, 8))
    for k in range(8):
        for n in range(8):
            m[k, n] = (np.sqrt(1 / 8) if k == 0 else np.sqrt(2 / 8)) * np.cos((2 * n + 1) * k * np.pi / 16)
    return m


_D = _dct_matrix()


def _magnitude(v):
    a = abs(int(v))
    s = a.bit_length()
    return s, (v if v >= 0 else v + (1 << s) - 1)


def jpeg(w, h, sampling=((1, 1), (1, 1), (1, 1)), quality=75, restart=0, interleaved=True, kind="ycc",
         q16=False, seed=2, progressive=False):
    """Returns baseline (or progressive) JPEG bytes.  kind: 'ycc' (JFIF), 'grey', 'rgb' (ids R,G,B, no JFIF),
    'cmyk' (Adobe 0)."""
    nc = {"ycc": 3, "grey": 1, "rgb": 3, "cmyk": 4}[kind]
    sampling = list(sampling)[:nc] + [(1, 1)] * max(0, nc - len(sampling))
    img = _pattern(h, w, 4, seed).astype(np.float64)
    if kind == "ycc":
        r, g, b = img[..., 0], img[..., 1], img[..., 2]
        planes = [0.299 * r + 0.587 * g + 0.114 * b, -0.168736 * r - 0.331264 * g + 0.5 * b + 128,
                  0.5 * r - 0.418688 * g - 0.081312 * b + 128]
    else:
        planes = [img[..., k] for k in range(nc)]
    scale = 5000 / quality if quality < 50 else 200 - 2 * quality
    qt = [np.clip((_QL * scale + 50) // 100, 1, 65535 if q16 else 255),
          np.clip((_QC * scale + 50) // 100, 1, 65535 if q16 else 255)]
    if q16:
        qt = [np.clip(q * 3 + 300, 1, 65535) for q in qt]  # exercise 16-bit tables
    hmax = max(s[0] for s in sampling)
    vmax = max(s[1] for s in sampling)
    mcux, mcuy = -(-w // (8 * hmax)), -(-h // (8 * vmax))
    comps = []
    for k in range(nc):
        hs, vs = sampling[k]
        cw, chh = mcux * hs * 8, mcuy * vs * 8
        p = planes[k]
        fx, fy = hmax // hs, vmax // vs
        # down-sample by averaging fx x fy boxes, edge-replicate to the MCU-padded size
        pw, ph = -(-w // fx) * fx, -(-h // fy) * fy
        p = np.pad(p, ((0, ph - h), (0, pw - w)), mode="edge")
        p = p.reshape(ph // fy, fy, pw // fx, fx).mean(axis=(1, 3))
        p = np.pad(p, ((0, chh - p.shape[0]), (0, cw - p.shape[1])), mode="edge")
        q = qt[0 if k == 0 or kind in ("rgb", "cmyk") else 1]
        blocks = p.reshape(chh // 8, 8, cw // 8, 8).transpose(0, 2, 1, 3) - 128
        coef = np.einsum("ij,abjk,lk->abil", _D, blocks, _D)
        coef = np.round(coef.reshape(chh // 8, cw // 8, 64) / q.reshape(64)).astype(np.int64)
        comps.append(dict(h=hs, v=vs, q=0 if q is qt[0] else 1, coef=coef))
    dc_t = [_codes(_DC_L), _codes(_DC_C)]
    ac_t = [_codes(_AC_L), _codes(_AC_C)]
    tsel = [0 if k == 0 or kind in ("rgb", "cmyk") else 1 for k in range(nc)]

    def seg(m, data):
        return bytes([0xFF, m]) + struct.pack(">H", len(data) + 2) + data

    out = b"\xff\xd8"
    if kind in ("ycc", "grey"):
        out += seg(0xE0, b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00")
    if kind == "cmyk":
        out += seg(0xEE, b"Adobe\x00\x64\x00\x00\x00\x00\x00")
    out += seg(0xFE, b"synthetic test image")
    for t in range(2 if nc > 1 and kind == "ycc" else 1):
        if q16:
            out += seg(0xDB, bytes([0x10 | t]) + b"".join(struct.pack(">H", int(v)) for v in qt[t][_ZIGZAG]))
        else:
            out += seg(0xDB, bytes([t]) + bytes(int(v) for v in qt[t][_ZIGZAG]))
    ids = [ord("R"), ord("G"), ord("B")] if kind == "rgb" else list(range(1, nc + 1))
    sof = struct.pack(">BHHB", 8, h, w, nc)
    for k in range(nc):
        sof += bytes([ids[k], (sampling[k][0] << 4) | sampling[k][1], comps[k]["q"]])
    if progressive:
        return out + seg(0xC2, sof) + _progressive_scans(comps, ids, w, h, hmax, vmax, mcux, mcuy, seg) + b"\xff\xd9"
    out += seg(0xC0, sof)
    for t in range(2 if kind == "ycc" else 1):
        for cls, spec in ((0, (_DC_L, _DC_C)[t]), (1, (_AC_L, _AC_C)[t])):
            out += seg(0xC4, bytes([(cls << 4) | t]) + bytes(spec[0]) + bytes(spec[1]))
    if restart:
        out += seg(0xDD, struct.pack(">H", restart))

    def block(bw, c, pred, blk):
        k = c["coef"][blk]
        t = tsel[c["idx"]]
        diff = int(k[0]) - pred
        s, v = _magnitude(diff)
        bw.put(*dc_t[t][s])
        if s:
            bw.put(v, s)
        zz = k[_ZIGZAG]
        run = 0
        for i in range(1, 64):
            a = int(zz[i])
            if a == 0:
                run += 1
                continue
            while run > 15:
                bw.put(*ac_t[t][0xF0])
                run -= 16
            s, v = _magnitude(a)
            bw.put(*ac_t[t][(run << 4) | s])
            bw.put(v, s)
            run = 0
        if run:
            bw.put(*ac_t[t][0x00])
        return int(k[0])

    for k, c in enumerate(comps):
        c["idx"] = k

    def scan(members, units):
        """units: list of lists of (comp, (by, bx)) per MCU."""
        data = struct.pack(">B", len(members))
        for k in members:
            t = tsel[k]
            data += bytes([ids[k], (t << 4) | t])
        data += b"\x00\x3f\x00"
        body = _BitWriter()
        pred = {k: 0 for k in members}
        rst = 0
        for mi, unit in enumerate(units):
            if restart and mi and mi % restart == 0:
                body.flush()
                body.out += bytes([0xFF, 0xD0 + rst])
                rst = (rst + 1) % 8
                pred = {k: 0 for k in members}
            for k, b in unit:
                pred[k] = block(body, comps[k], pred[k], b)
        body.flush()
        return seg(0xDA, data) + bytes(body.out)

    if interleaved and nc > 1:
        units = []
        for my in range(mcuy):
            for mx in range(mcux):
                u = []
                for k, c in enumerate(comps):
                    for y in range(c["v"]):
                        for x in range(c["h"]):
                            u.append((k, (my * c["v"] + y, mx * c["h"] + x)))
                units.append(u)
        out += scan(list(range(nc)), units)
    else:
        for k, c in enumerate(comps):
            cx = -(-(-(-w * c["h"] // hmax)) // 8)
            cy = -(-(-(-h * c["v"] // vmax)) // 8)
            out += scan([k], [[(k, (by, bx))] for by in range(cy) for bx in range(cx)])
    return out + b"\xff\xd9"


# progressive coding (ITU T.81 G.1.2; the encoder side of libjpeg's
# jcphuff.c restated): one DC table (categories 0-11, 4-bit codes) and one AC
# table holding every run/size symbol plus EOB0-EOB14 and ZRL (8-bit codes)
_P_DC = ([0, 0, 0, 12] + [0] * 12, list(range(12)))
_P_AC_SYMS = [r << 4 for r in range(16)] + [(r << 4) | s for r in range(16) for s in range(1, 11)]
_P_AC = ([0] * 7 + [len(_P_AC_SYMS)] + [0] * 8, _P_AC_SYMS)


def _pt(v, al):
    """point transform of an AC coefficient: magnitude >> al, sign kept"""
    return -((-v) >> al) if v < 0 else v >> al


def _progressive_scans(comps, ids, w, h, hmax, vmax, mcux, mcuy, seg):
    dc_t, ac_t = _codes(_P_DC), _codes(_P_AC)
    out = seg(0xC4, bytes([0x00]) + bytes(_P_DC[0]) + bytes(_P_DC[1]))
    out += seg(0xC4, bytes([0x10]) + bytes(_P_AC[0]) + bytes(_P_AC[1]))
    nc = len(comps)
    zz = [c["coef"][..., _ZIGZAG].astype(np.int64) for c in comps]  # [by, bx, 64] in zigzag order

    def blocks_of(k):  # a non-interleaved scan covers the component's own blocks only
        c = comps[k]
        cx = -(-(-(-w * c["h"] // hmax)) // 8)
        cy = -(-(-(-h * c["v"] // vmax)) // 8)
        return [(by, bx) for by in range(cy) for bx in range(cx)]

    def header(members, ss, se, ah, al):
        d = struct.pack(">B", len(members))
        for k in members:
            d += bytes([ids[k], 0x00])
        return d + bytes([ss, se, (ah << 4) | al])

    def dc_scan(ah, al):
        bw = _BitWriter()
        pred = [0] * nc
        for my in range(mcuy):
            for mx in range(mcux):
                for k, c in enumerate(comps):
                    for y in range(c["v"]):
                        for x in range(c["h"]):
                            v = int(zz[k][my * c["v"] + y, mx * c["h"] + x, 0])
                            if ah == 0:
                                t = v >> al  # DC point transform: arithmetic shift
                                s, m = _magnitude(t - pred[k])
                                bw.put(*dc_t[s])
                                if s:
                                    bw.put(m, s)
                                pred[k] = t
                            else:
                                bw.put((v >> al) & 1, 1)
        bw.flush()
        return seg(0xDA, header(list(range(nc)), 0, 0, ah, al)) + bytes(bw.out)

    def ac_first(k, ss, se, al):
        bw = _BitWriter()
        st = {"eobrun": 0}

        def flush():
            if st["eobrun"]:
                n = st["eobrun"].bit_length() - 1
                bw.put(*ac_t[n << 4])
                if n:
                    bw.put(st["eobrun"] & ((1 << n) - 1), n)
                st["eobrun"] = 0

        for b in blocks_of(k):
            v = [_pt(int(x), al) for x in zz[k][b][ss:se + 1]]
            r = 0
            for t in v:
                if t == 0:
                    r += 1
                    continue
                flush()
                while r > 15:
                    bw.put(*ac_t[0xF0])
                    r -= 16
                s, m = _magnitude(t)
                bw.put(*ac_t[(r << 4) | s])
                bw.put(m, s)
                r = 0
            if r:
                st["eobrun"] += 1
                if st["eobrun"] == 0x7FFF:
                    flush()
        flush()
        bw.flush()
        return seg(0xDA, header([k], ss, se, 0, al)) + bytes(bw.out)

    def ac_refine(k, ss, se, al):
        bw = _BitWriter()
        st = {"eobrun": 0, "be": []}

        def flush():
            if st["eobrun"]:
                n = st["eobrun"].bit_length() - 1
                bw.put(*ac_t[n << 4])
                if n:
                    bw.put(st["eobrun"] & ((1 << n) - 1), n)
                st["eobrun"] = 0
                for bit in st["be"]:
                    bw.put(bit, 1)
                st["be"] = []

        for b in blocks_of(k):
            coefs = [int(x) for x in zz[k][b][ss:se + 1]]
            absv = [abs(x) >> al for x in coefs]
            eob = max([i for i, a in enumerate(absv) if a == 1], default=-1)
            r, br = 0, []
            for i, t in enumerate(absv):
                if t == 0:
                    r += 1
                    continue
                while r > 15 and i <= eob:
                    flush()
                    bw.put(*ac_t[0xF0])
                    r -= 16
                    for bit in br:
                        bw.put(bit, 1)
                    br = []
                if t > 1:
                    br.append(t & 1)  # correction bit of a previously nonzero coefficient
                    continue
                flush()
                bw.put(*ac_t[(r << 4) | 1])
                bw.put(1 if coefs[i] > 0 else 0, 1)
                for bit in br:
                    bw.put(bit, 1)
                br, r = [], 0
            if r > 0 or br:
                st["eobrun"] += 1
                st["be"] += br
                if st["eobrun"] == 0x7FFF or len(st["be"]) > 900:
                    flush()
        flush()
        bw.flush()
        return seg(0xDA, header([k], ss, se, al + 1, al)) + bytes(bw.out)

    out += dc_scan(0, 1)
    out += ac_first(0, 1, 5, 2)
    for k in range(1, nc):
        out += ac_first(k, 1, 63, 1)
    out += ac_first(0, 6, 63, 2)
    out += ac_refine(0, 1, 63, 1)
    out += dc_scan(1, 0)
    for k in range(1, nc):
        out += ac_refine(k, 1, 63, 0)
    out += ac_refine(0, 1, 63, 0)
    return out


JPEG_VARIANTS = {
    "ycc444": dict(w=40, h=24),
    "ycc422_odd": dict(w=37, h=23, sampling=((2, 1), (1, 1), (1, 1))),
    "ycc420_odd": dict(w=45, h=29, sampling=((2, 2), (1, 1), (1, 1)), quality=90),
    "ycc440": dict(w=32, h=34, sampling=((1, 2), (1, 1), (1, 1))),
    "ycc411_generic": dict(w=50, h=16, sampling=((4, 1), (1, 1), (1, 1))),
    "ycc420_restart": dict(w=70, h=38, sampling=((2, 2), (1, 1), (1, 1)), restart=3),
    "ycc420_noninterleaved": dict(w=33, h=35, sampling=((2, 2), (1, 1), (1, 1)), interleaved=False),
    "ycc420_1x1": dict(w=1, h=1, sampling=((2, 2), (1, 1), (1, 1))),
    "ycc420_w1": dict(w=1, h=19, sampling=((2, 2), (1, 1), (1, 1))),
    "ycc_q100": dict(w=24, h=24, quality=100),
    "ycc_q16": dict(w=24, h=16, q16=True),
    "grey": dict(w=31, h=17, kind="grey"),
    "grey_restart": dict(w=64, h=8, kind="grey", restart=2),
    "rgb_ids": dict(w=20, h=20, kind="rgb"),
    "cmyk": dict(w=18, h=22, kind="cmyk"),
    "prog_ycc420": dict(w=45, h=29, sampling=((2, 2), (1, 1), (1, 1)), quality=90, progressive=True),
    "prog_ycc444_q100": dict(w=24, h=24, quality=100, progressive=True),
    "prog_grey": dict(w=37, h=21, kind="grey", progressive=True),
    "prog_ycc422_big": dict(w=130, h=70, sampling=((2, 1), (1, 1), (1, 1)), quality=60, progressive=True, seed=5),
}


def variants():
    """name -> file bytes for every synthetic variant."""
    out = {}
    for k, v in PNG_VARIANTS.items():
        out["png_" + k] = png(**v)
    for k, v in JPEG_VARIANTS.items():
        out["jpeg_" + k] = jpeg(**v)
    return out
