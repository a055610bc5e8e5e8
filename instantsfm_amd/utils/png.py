"""Single-channel PNG reader for depth maps (stdlib ``zlib`` + numpy).

The reference reads depth maps with ``cv2.imread(f, cv2.IMREAD_UNCHANGED)`` (controllers/data_reader.py:136-144);
OpenCV is not part of this framework.  ScanNet-style depth maps are 16-bit grayscale PNGs (millimetres), for which
IMREAD_UNCHANGED returns the stored samples as a [H, W] uint16 array; this reader returns the same array for
grayscale PNGs of bit depth 8 or 16 (uint8 / uint16), non-interlaced, any of the five row filters.  Other colour
types, bit depths and Adam7 interlacing raise ValueError (a depth map is one channel).
"""
import struct
import zlib

import numpy as np

__all__ = ["read_png_gray"]

_SIG = b"\x89PNG\r\n\x1a\n"


def _unfilter(raw, height, stride, bpp):
    """Undo the per-row PNG filters (filter byte + stride bytes per row) -> [height, stride] uint8."""
    rows = np.frombuffer(raw, dtype=np.uint8)
    if rows.size != height * (stride + 1):
        raise ValueError(f"PNG data is {rows.size} bytes, expected {height * (stride + 1)}")
    rows = rows.reshape(height, stride + 1)
    out = np.zeros((height, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int64)
    for r in range(height):
        ft, line = int(rows[r, 0]), rows[r, 1:].astype(np.int64)
        if ft == 0:      # None
            cur = line
        elif ft == 1:    # Sub: running sum per byte lane of a pixel
            cur = np.cumsum(line.reshape(-1, bpp), axis=0).reshape(-1) & 255
        elif ft == 2:    # Up
            cur = (line + prev) & 255
        elif ft in (3, 4):  # Average / Paeth: sequential in x
            cur = line.copy()
            up = prev
            for i in range(stride):
                a = int(cur[i - bpp]) if i >= bpp else 0
                b = int(up[i])
                if ft == 3:
                    pred = (a + b) >> 1
                else:
                    c = int(up[i - bpp]) if i >= bpp else 0
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[i] = (int(line[i]) + pred) & 255
        else:
            raise ValueError(f"unknown PNG filter type {ft} in row {r}")
        out[r] = cur
        prev = cur
    return out


def read_png_gray(path):
    """[H, W] uint8 / uint16 samples of a grayscale PNG (what cv2.IMREAD_UNCHANGED returns for one)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != _SIG:
        raise ValueError(f"{path}: not a PNG file")
    pos, ihdr, idat = 8, None, []
    while pos + 8 <= len(data):
        (n,), kind = struct.unpack(">I", data[pos:pos + 4]), data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if kind == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat.append(body)
        elif kind == b"IEND":
            break
    if ihdr is None or not idat:
        raise ValueError(f"{path}: missing IHDR or IDAT")
    width, height, depth, ctype, _, _, interlace = ihdr
    if ctype != 0 or depth not in (8, 16) or interlace != 0:
        raise ValueError(f"{path}: only non-interlaced 8/16-bit grayscale PNGs are supported "
                         f"(bit depth {depth}, colour type {ctype}, interlace {interlace})")
    bpp = depth // 8
    px = _unfilter(zlib.decompress(b"".join(idat)), height, width * bpp, bpp)
    if depth == 8:
        return px
    return px.reshape(height, width, 2).view(">u2").reshape(height, width).astype(np.uint16)
