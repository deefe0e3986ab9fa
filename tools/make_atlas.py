"""Synthetic texture atlas with the shape of the reference's atlas (285 x 377, 8-bit RGBA,
non-interlaced PNG): deterministic tiles of gradients and checkers, written with our own
minimal PNG encoder (zlib).  Output: scenes/assets/atlas_synth.png.  The textured scene
variants (scenes/*_tex.json) name it as their "atlas"."""
import os
import struct
import zlib

import numpy as np

W, H = 285, 377


def atlas():
    y, x = np.mgrid[0:H, 0:W]
    img = np.zeros((H, W, 4), np.uint8)
    img[..., 0] = (x * 255 // (W - 1)).astype(np.uint8)
    img[..., 1] = (y * 255 // (H - 1)).astype(np.uint8)
    img[..., 2] = np.where(((x // 16) + (y // 16)) % 2 == 0, 220, 40).astype(np.uint8)
    img[..., 3] = 255
    # a few solid tiles (exact texel values are easy to spot in frames)
    img[0:64, 0:64] = (255, 32, 32, 255)
    img[64:128, 64:128] = (32, 255, 32, 255)
    img[128:192, 128:192] = (32, 32, 255, 255)
    return img


def png_bytes(img, filters=(0, 1, 2, 3, 4)):
    """RGBA8 PNG; rows cycle through all five filter types so decoders are exercised on each."""
    h, w, _ = img.shape
    raw = bytearray()
    a = img.astype(np.int32)
    for r in range(h):
        f = filters[r % len(filters)]
        row = a[r].reshape(-1)
        left = np.concatenate([np.zeros(4, np.int32), row[:-4]])
        up = a[r - 1].reshape(-1) if r else np.zeros_like(row)
        ul = np.concatenate([np.zeros(4, np.int32), up[:-4]])
        if f == 0:
            out = row
        elif f == 1:
            out = row - left
        elif f == 2:
            out = row - up
        elif f == 3:
            out = row - (left + up) // 2
        else:
            p = left + up - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
            out = row - pred
        raw.append(f)
        raw += (out & 255).astype(np.uint8).tobytes()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(bytes(raw), 9)) + chunk(b"IEND", b""))


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes", "assets", "atlas_synth.png")
    open(out, "wb").write(png_bytes(atlas()))
    print(out)
