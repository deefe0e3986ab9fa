"""Independent PNG reader for tests (zlib + numpy; 8-bit RGB/RGBA, non-interlaced):
checks the product's atlas decoder (rt_scene_load_atlas) and feeds the oracle."""
import struct
import zlib

import numpy as np


def read_png_rgba8(path):
    d = open(path, "rb").read()
    assert d[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    pos, idat, w = 8, b"", None
    while pos < len(d):
        n, = struct.unpack(">I", d[pos:pos + 4])
        t, body = d[pos + 4:pos + 8], d[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
            assert depth == 8 and ctype in (2, 6) and interlace == 0
            bpp = 4 if ctype == 6 else 3
        elif t == b"IDAT":
            idat += body
        elif t == b"IEND":
            break
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * bpp)
    img = np.zeros((h, w * bpp), np.int32)
    for y in range(h):
        f, src = raw[y, 0], raw[y, 1:].astype(np.int32)
        up = img[y - 1] if y else np.zeros(w * bpp, np.int32)
        row = np.zeros(w * bpp, np.int32)
        for x in range(w * bpp):                      # sequential: each byte may depend on the previous pixel
            a = row[x - bpp] if x >= bpp else 0
            b = up[x]
            c = up[x - bpp] if x >= bpp else 0
            if f == 0:
                v = src[x]
            elif f == 1:
                v = src[x] + a
            elif f == 2:
                v = src[x] + b
            elif f == 3:
                v = src[x] + (a + b) // 2
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                v = src[x] + (a if pa <= pb and pa <= pc else (b if pb <= pc else c))
            row[x] = v & 255
        img[y] = row
    img = img.astype(np.uint8).reshape(h, w, bpp)
    if bpp == 3:
        img = np.concatenate([img, np.full((h, w, 1), 255, np.uint8)], 2)
    return img
