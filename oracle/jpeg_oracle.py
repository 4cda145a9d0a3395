"""CPU oracle for the frame decode in front of the hot path.

TEST INFRASTRUCTURE ONLY (the checker): only `tests/` may import it; the product path
(vcap.jpeg -> vcap_jpeg_decode_batch) never does and has no CPU fallback.

The reference reads each sampled frame with PIL: `Image.open(path).convert("RGB")`
(core/preprocessing/frame_loader.py:42-44), i.e. libjpeg-turbo's decompressor (Pillow 12.2 here)
with its defaults.  This is a restatement of what that decoder computes for baseline sequential
Huffman JPEGs (SOF0 / SOF1, 8-bit, 1 or 3 components, sampling factors 1 or 2, restart markers):
  * entropy decode (ITU T.81 F.2.2: DC differences, AC run/size, EXTEND, byte stuffing, RSTn);
  * jidctint.c `jpeg_idct_islow`: the 13-bit fixed-point LL&M IDCT with PASS1_BITS 2, its
    column pass with dequantisation, its row pass and the post-IDCT range-limit table
    (values wrap mod 1024 before the clamp, exactly as `& RANGE_MASK` indexes it);
  * jdsample.c fancy upsampling (`h2v1_fancy_upsample`, `h2v2_fancy_upsample`: the triangle
    filter with its 8 / 7 rounding biases, first / last column special cases, the top and bottom
    image rows replicated as context as jdmainct.c does);
  * jdcolor.c `ycc_rgb_convert` with its 16-bit fixed-point tables.
Pinned bit-exact against Pillow's own decode of generated JPEGs (tests/test_cpu_jpeg.py).
"""
from __future__ import annotations

import numpy as np

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
    21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60,
    61, 54, 47, 55, 62, 63], dtype=np.int64)


class JpegError(ValueError):
    pass


def parse(data: bytes) -> dict:
    """Markers -> frame header, tables and the entropy-coded segment of the single scan."""
    if data[:2] != b"\xff\xd8":
        raise JpegError("not a JPEG (no SOI)")
    i, qt, ht, info = 2, {}, {}, {"restart": 0}
    while i < len(data):
        if data[i] != 0xFF:
            raise JpegError(f"marker expected at {i}")
        while data[i] == 0xFF:
            i += 1
        m = data[i]
        i += 1
        if m == 0xD9:
            break
        seg_len = int.from_bytes(data[i:i + 2], "big")
        seg = data[i + 2:i + seg_len]
        if m == 0xDB:                                   # DQT
            p = 0
            while p < len(seg):
                pq, tq = seg[p] >> 4, seg[p] & 15
                n = 128 if pq else 64
                vals = (np.frombuffer(seg[p + 1:p + 1 + n], ">u2") if pq else np.frombuffer(seg[p + 1:p + 65], "u1"))
                q = np.zeros(64, np.int64)
                q[ZIGZAG] = vals.astype(np.int64)       # natural order
                qt[tq] = q
                p += 1 + n
        elif m in (0xC0, 0xC1):                         # SOF0 / SOF1
            if seg[0] != 8:
                raise JpegError("only 8-bit samples")
            info["height"] = int.from_bytes(seg[1:3], "big")
            info["width"] = int.from_bytes(seg[3:5], "big")
            nc = seg[5]
            info["comps"] = [dict(id=seg[6 + 3 * k], h=seg[7 + 3 * k] >> 4, v=seg[7 + 3 * k] & 15, tq=seg[8 + 3 * k])
                             for k in range(nc)]
        elif 0xC2 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            raise JpegError(f"unsupported frame type SOF{m - 0xC0}")
        elif m == 0xC4:                                 # DHT
            p = 0
            while p < len(seg):
                tc, th = seg[p] >> 4, seg[p] & 15
                counts = list(seg[p + 1:p + 17])
                nsym = sum(counts)
                syms = list(seg[p + 17:p + 17 + nsym])
                code, k, table = 0, 0, {}
                for length in range(1, 17):
                    for _ in range(counts[length - 1]):
                        table[(length, code)] = syms[k]
                        k += 1
                        code += 1
                    code <<= 1
                ht[(tc, th)] = table
                p += 17 + nsym
        elif m == 0xDD:                                 # DRI
            info["restart"] = int.from_bytes(seg[0:2], "big")
        elif m == 0xDA:                                 # SOS: the scan runs to the next non-RST marker
            ns = seg[0]
            if ns != len(info["comps"]):
                raise JpegError("only single-scan (interleaved) images")
            for k in range(ns):
                cid, tdta = seg[1 + 2 * k], seg[2 + 2 * k]
                c = next(c for c in info["comps"] if c["id"] == cid)
                c["td"], c["ta"] = tdta >> 4, tdta & 15
            j = i + seg_len
            e = j
            while True:
                e = data.index(b"\xff", e)
                if data[e + 1] == 0x00 or 0xD0 <= data[e + 1] <= 0xD7:
                    e += 2
                    continue
                break
            info["scan"] = data[j:e]
            i = e
            continue
        i += seg_len
    info["qt"], info["ht"] = qt, ht
    return info


class _Bits:
    def __init__(self, b: bytes):
        self.b, self.p, self.acc, self.n = b, 0, 0, 0

    def bit(self) -> int:
        if self.n == 0:
            v = self.b[self.p] if self.p < len(self.b) else 0
            self.p += 1
            if v == 0xFF:
                nxt = self.b[self.p] if self.p < len(self.b) else 0
                if nxt == 0x00:
                    self.p += 1
                else:           # a marker: libjpeg feeds zeros past it
                    self.p -= 1
                    v = 0
            self.acc, self.n = v, 8
        self.n -= 1
        return (self.acc >> self.n) & 1

    def bits(self, k: int) -> int:
        v = 0
        for _ in range(k):
            v = (v << 1) | self.bit()
        return v

    def restart(self):
        """byte-align and step over the RSTn marker"""
        self.n = 0
        while self.p < len(self.b) - 1 and not (self.b[self.p] == 0xFF and 0xD0 <= self.b[self.p + 1] <= 0xD7):
            self.p += 1
        self.p += 2


def _huff(bits: _Bits, table: dict) -> int:
    code = 0
    for length in range(1, 17):
        code = (code << 1) | bits.bit()
        s = table.get((length, code))
        if s is not None:
            return s
    raise JpegError("bad Huffman code")


def _extend(v: int, s: int) -> int:
    return v - (1 << s) + 1 if s and v < (1 << (s - 1)) else v


def coefficients(info: dict) -> list:
    """Entropy decode -> per component [blocks_y, blocks_x, 64] int64 quantised coefficients
    (natural order), block grids padded to whole MCUs."""
    comps = info["comps"]
    hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
    mx = -(-info["width"] // (8 * hmax))
    my = -(-info["height"] // (8 * vmax))
    out = [np.zeros((my * c["v"], mx * c["h"], 64), np.int64) for c in comps]
    bits = _Bits(info["scan"])
    pred = [0] * len(comps)
    ri = info["restart"]
    for mcu in range(mx * my):
        if ri and mcu and mcu % ri == 0:
            bits.restart()
            pred = [0] * len(comps)
        by0, bx0 = divmod(mcu, mx)
        for k, c in enumerate(comps):
            dct, act = info["ht"][(0, c["td"])], info["ht"][(1, c["ta"])]
            for v in range(c["v"]):
                for h in range(c["h"]):
                    blk = np.zeros(64, np.int64)
                    s = _huff(bits, dct)
                    pred[k] += _extend(bits.bits(s), s)
                    blk[0] = pred[k]
                    z = 1
                    while z < 64:
                        rs = _huff(bits, act)
                        r, s = rs >> 4, rs & 15
                        if s == 0:
                            if r != 15:
                                break
                            z += 16
                            continue
                        z += r
                        blk[ZIGZAG[z]] = _extend(bits.bits(s), s)
                        z += 1
                    out[k][by0 * c["v"] + v, bx0 * c["h"] + h] = blk
    return out


# jidctint.c constants (CONST_BITS 13)
F0298, F0390, F0541, F0765, F0899, F1175 = 2446, 3196, 4433, 6270, 7373, 9633
F1501, F1847, F1961, F2053, F2562, F3072 = 12299, 15137, 16069, 16819, 20995, 25172
CB, P1 = 13, 2


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _idct_1d(d0, d1, d2, d3, d4, d5, d6, d7):
    """One even/odd butterfly of jpeg_idct_islow on int64 arrays; returns the 8 outputs before the
    pass's descale (out[i] = tmp + tmp')."""
    z2, z3 = d2, d6
    z1 = (z2 + z3) * F0541
    tmp2 = z1 + z3 * (-F1847)
    tmp3 = z1 + z2 * F0765
    tmp0 = (d0 + d4) << CB
    tmp1 = (d0 - d4) << CB
    tmp10, tmp13, tmp11, tmp12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    t0, t1, t2, t3 = d7, d5, d3, d1
    z1, z2, z3, z4 = t0 + t3, t1 + t2, t0 + t2, t1 + t3
    z5 = (z3 + z4) * F1175
    t0, t1, t2, t3 = t0 * F0298, t1 * F2053, t2 * F3072, t3 * F1501
    z1, z2, z3, z4 = z1 * (-F0899), z2 * (-F2562), z3 * (-F1961), z4 * (-F0390)
    z3 = z3 + z5
    z4 = z4 + z5
    t0, t1, t2, t3 = t0 + z1 + z3, t1 + z2 + z4, t2 + z2 + z3, t3 + z1 + z4
    return (tmp10 + t3, tmp11 + t2, tmp12 + t1, tmp13 + t0, tmp13 - t0, tmp12 - t1, tmp11 - t2, tmp10 - t3)


def _range_limit(v):
    """post-IDCT range_limit[v & RANGE_MASK] (jdmaster.c prepare_range_limit_table)"""
    y = v & 1023
    return np.where(y < 128, y + 128, np.where(y < 512, 255, np.where(y < 896, 0, y - 896))).astype(np.uint8)


def idct_plane(coef: np.ndarray, q: np.ndarray) -> np.ndarray:
    """[by, bx, 64] quantised coefficients -> [by*8, bx*8] uint8 samples (jpeg_idct_islow)."""
    by, bx = coef.shape[:2]
    c = coef.reshape(by * bx, 8, 8) * q.reshape(1, 8, 8)   # dequantised, [blk, row(u), col(v)]
    # pass 1: columns (the all-AC-zero shortcut gives the same numbers: dc << PASS1_BITS)
    cols = _idct_1d(*[c[:, r, :] for r in range(8)])        # each [blk, 8 cols]
    ws = np.stack([_descale(o, CB - P1) for o in cols], axis=1)  # [blk, row, col]
    # pass 2: rows (the zero-row shortcut is the same arithmetic)
    rows = _idct_1d(*[ws[:, :, k] for k in range(8)])        # each [blk, 8 rows]
    px = np.stack([_range_limit(_descale(o, CB + P1 + 3)) for o in rows], axis=2)  # [blk, row, col]
    return px.reshape(by, bx, 8, 8).transpose(0, 2, 1, 3).reshape(by * 8, bx * 8)


def _upsample(plane: np.ndarray, dw: int, dh: int, fh: int, fv: int, W: int, H: int) -> np.ndarray:
    p = plane[:dh, :dw].astype(np.int64)
    if fh == 1 and fv == 1:
        return p[:H, :W]
    if fh == 2 and fv == 1 and dw > 2:                       # h2v1_fancy_upsample
        left = np.concatenate([p[:, :1], p[:, :-1]], axis=1)
        right = np.concatenate([p[:, 1:], p[:, -1:]], axis=1)
        even = (3 * p + left + 1) >> 2
        odd = (3 * p + right + 2) >> 2
        even[:, 0] = p[:, 0]
        odd[:, -1] = p[:, -1]
        out = np.stack([even, odd], axis=2).reshape(p.shape[0], 2 * dw)
        return out[:H, :W]
    if fh == 2 and fv == 2 and dw > 2:                       # h2v2_fancy_upsample
        up = np.concatenate([p[:1], p[:-1]], axis=0)         # row above (top row replicated)
        dn = np.concatenate([p[1:], p[-1:]], axis=0)         # row below (bottom row replicated)
        rows = []
        for nb in (up, dn):                                   # v = 0 uses the row above, v = 1 below
            cs = 3 * p + nb
            last = np.concatenate([cs[:, :1], cs[:, :-1]], axis=1)
            nxt = np.concatenate([cs[:, 1:], cs[:, -1:]], axis=1)
            even = (3 * cs + last + 8) >> 4
            odd = (3 * cs + nxt + 7) >> 4
            even[:, 0] = (4 * cs[:, 0] + 8) >> 4
            odd[:, -1] = (4 * cs[:, -1] + 7) >> 4
            rows.append(np.stack([even, odd], axis=2).reshape(p.shape[0], 2 * dw))
        out = np.stack(rows, axis=1).reshape(2 * dh, 2 * dw)
        return out[:H, :W]
    raise JpegError(f"unsupported upsampling {fh}x{fv} (downsampled width {dw})")


def _fix(x: float) -> int:
    return int(x * 65536 + 0.5)


def decode(data: bytes) -> np.ndarray:
    """JPEG bytes -> [H, W, 3] uint8 RGB, as PIL Image.open(...).convert("RGB") gives."""
    info = parse(data)
    W, H, comps = info["width"], info["height"], info["comps"]
    if len(comps) not in (1, 3):
        raise JpegError("1 or 3 components only")
    hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
    coef = coefficients(info)
    planes = []
    for c, cf in zip(comps, coef):
        pl = idct_plane(cf, info["qt"][c["tq"]])
        dw, dh = -(-W * c["h"] // hmax), -(-H * c["v"] // vmax)
        planes.append(_upsample(pl, dw, dh, hmax // c["h"], vmax // c["v"], W, H))
    if len(comps) == 1:
        return np.repeat(planes[0].astype(np.uint8)[:, :, None], 3, axis=2)
    y, cb, cr = planes
    x_cb, x_cr = cb - 128, cr - 128
    crr = (_fix(1.40200) * x_cr + (1 << 15)) >> 16
    cbb = (_fix(1.77200) * x_cb + (1 << 15)) >> 16
    g_off = ((-_fix(0.34414)) * x_cb + (1 << 15) + (-_fix(0.71414)) * x_cr) >> 16
    rgb = np.stack([y + crr, y + g_off, y + cbb], axis=2)
    return np.clip(rgb, 0, 255).astype(np.uint8)
