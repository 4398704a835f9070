"""Test helpers: synthetic images, a baseline TIFF writer, decoders, PSNR.

Decoding uses OpenJPEG (opj_decompress from /opt/conda/bin, or Pillow's bundled
OpenJPEG) -- the "reference decoder" north_star names for parity; nothing here
is part of the product.
"""
from __future__ import annotations

import hashlib
import io
import os
import shutil
import struct
import subprocess
import tempfile

import numpy as np

OPJ_DIR = "/opt/conda/bin"


def opj(tool: str) -> str | None:
    p = os.path.join(OPJ_DIR, tool)
    if os.path.exists(p):
        return p
    return shutil.which(tool)


def synth_rgb8(h, w, seed=1234, noise=6.0):
    """C2-style content: sinusoids + checker patch + gaussian noise.
    (Row / column terms are broadcast, not evaluated on the full grid: the
    same float64 operations in the same order, so the same pixels.)"""
    rng = np.random.default_rng(seed)
    x = np.arange(w, dtype=np.float64)[None, :]
    y = np.arange(h, dtype=np.float64)[:, None]
    d = 20 * np.sin((x + y) / 11.0)
    img = np.empty((h, w, 3))
    for c in range(3):
        img[..., c] = 128 + 40 * np.sin(x / 37.0 + c) + 30 * np.cos(y / 23.0 - c) + d
    del d
    ys, xs = slice(h // 5, 2 * h // 5), slice(w // 5, 7 * w // 15)
    chk = 50 * ((np.floor(x[:, xs] / 16) + np.floor(y[ys, :] / 16)) % 2 - 0.5)
    img[ys, xs, :] += chk[..., None]
    img += rng.normal(0, noise, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def testjpx_tiled(pix: np.ndarray, h=4000, w=6000) -> np.ndarray:
    """SURVEY.md 8(d)'s second C2 content class: the RGB channels of the
    test.jpx pixels (a real scan), mirror-tiled to h x w."""
    rgb = np.ascontiguousarray(pix[..., :3])
    H, W = rgb.shape[:2]
    return np.ascontiguousarray(np.pad(rgb, ((0, max(0, h - H)), (0, max(0, w - W)), (0, 0)),
                                       mode="symmetric")[:h, :w])


def synth_u16(h, w, comps=3, seed=2):
    """C3/C5-style 16-bit content scaled to [0, 65535] plus N(0, 400)."""
    rng = np.random.default_rng(seed)
    x = np.arange(w, dtype=np.float64)[None, :]
    y = np.arange(h, dtype=np.float64)[:, None]
    d = 6000 * np.sin((x - y) / 17.0)
    out = np.empty((h, w, comps))
    for c in range(comps):
        out[..., c] = 32768 + 12000 * np.sin(x / 53.0 + c) + 9000 * np.cos(y / 31.0 - 2 * c) + d
    del d
    out += rng.normal(0, 400, out.shape)
    out = np.clip(out, 0, 65535).astype(np.uint16)
    return out if comps > 1 else out[..., 0]


def synth_gray16_rows(row0, row1, w, seed=5, band=512):
    """C5 content (40000x30000 Gray16) for image rows
    [row0, row1) only: synth_u16's sinusoids in global coordinates, noise
    seeded per `band` rows (seed, row // band), so any split of the image
    into bands of whole `band`-row groups yields the same pixels."""
    out = np.empty((row1 - row0, w), np.uint16)
    x = np.arange(w, dtype=np.float32)
    sx = (32768 + 12000 * np.sin(x / 53.0)).astype(np.float32)
    g = row0
    while g < row1:
        e = min(row1, (g // band + 1) * band)
        rng = np.random.default_rng([seed, g // band])
        skip = g - (g // band) * band  # noise rows of this group before g
        if skip:
            rng.standard_normal((skip, w), dtype=np.float32)
        y = np.arange(g, e, dtype=np.float32)[:, None]
        v = sx[None, :] + 9000 * np.cos(y / 31.0) + 6000 * np.sin((x[None, :] - y) / 17.0)
        v += 400 * rng.standard_normal((e - g, w), dtype=np.float32)
        out[g - row0:e - row0] = np.clip(v, 0, 65535).astype(np.uint16)
        g = e
    return out


def lzw_encode(data: bytes, clear_every: int | None = None, clear_when_full: bool = True) -> bytes:
    """TIFF 6.0 LZW (MSB-first, early width change) of one strip -- test
    fixture generator for encoder variants libtiff does not produce: a Clear
    every `clear_every` codes (libtiff clears only when the dictionary is
    full; libtiff decodes both, checked against Pillow in test_oracle.py).
    clear_when_full=False writes no Clear at all, a stream libtiff rejects."""
    def width(k):  # the k-th code after a Clear (the decoder's rule)
        return 9 if k < 254 else 10 if k < 766 else 11 if k < 1790 else 12

    acc, nacc, out = 0, 0, bytearray()

    def put(code, w):
        nonlocal acc, nacc
        acc = (acc << w) | code
        nacc += w
        while nacc >= 8:
            nacc -= 8
            out.append((acc >> nacc) & 0xFF)
        acc &= (1 << nacc) - 1

    table, k = {}, 0
    put(256, 9)
    cur = b""
    for byte in data:
        nxt = cur + bytes([byte])
        if not cur or nxt in table:
            cur = nxt
            continue
        put(cur[0] if len(cur) == 1 else table[cur], width(k))
        if 258 + k <= 4095:
            table[nxt] = 258 + k
        k += 1
        full = 258 + k > 4095
        if (clear_every and k >= clear_every) or (full and clear_when_full):
            put(256, width(k))
            table, k = {}, 0
        cur = bytes([byte])
    if cur:
        put(cur[0] if len(cur) == 1 else table[cur], width(k))
        k += 1
    put(257, width(k))
    if nacc:
        out.append((acc << (8 - nacc)) & 0xFF)
    return bytes(out)


def tiff_bytes(img: np.ndarray, rows_per_strip=64, planar=False, big_endian=False,
               alpha=None, strip_codec=None, compression=1) -> bytes:
    """Baseline TIFF (strips), 8/16-bit, 1-4 samples; uncompressed, or each
    strip passed through `strip_codec` (then tagged `compression`)."""
    if img.ndim == 2:
        img = img[..., None]
    h, w, nc = img.shape
    bits = img.dtype.itemsize * 8
    e = ">" if big_endian else "<"
    rps = min(rows_per_strip, h)
    nstrip = (h + rps - 1) // rps
    planes = [img[..., c] for c in range(nc)] if planar else [img]
    strips = []
    for pl in planes:
        for s in range(nstrip):
            blk = np.ascontiguousarray(pl[s * rps:(s + 1) * rps])
            strips.append(blk.astype(blk.dtype.newbyteorder(e)).tobytes())
    if strip_codec is not None:
        strips = [strip_codec(x) for x in strips]
    ntags = 11 + (1 if nc in (2, 4) else 0)
    ifd_off = 8
    ifd_size = 2 + 12 * ntags + 4
    extra = bytearray()
    extra_base = ifd_off + ifd_size

    def arr(vals, typ):
        nonlocal extra
        off = extra_base + len(extra)
        fmt = "H" if typ == 3 else "I"
        extra += struct.pack(e + fmt * len(vals), *vals)
        if len(extra) % 2:
            extra += b"\0"
        return off

    data_base_placeholder = []
    nst = len(strips)
    bps_off = arr([bits] * nc, 3) if nc > 2 else None
    so_off = arr([0] * nst, 4) if nst > 1 else None
    sbc_off = arr([len(s) for s in strips], 4) if nst > 1 else None
    data_base = extra_base + len(extra)
    offs = []
    pos = data_base
    for s in strips:
        offs.append(pos)
        pos += len(s)
    if nst > 1:
        extra[so_off - extra_base:so_off - extra_base + 4 * nst] = struct.pack(e + "I" * nst, *offs)
    tags = []

    def tag(t, typ, cnt, val_or_off, inline=True):
        if inline and typ == 3 and cnt == 1:
            v = struct.pack(e + "HH", val_or_off, 0)
        elif inline and typ == 3 and cnt == 2:
            v = struct.pack(e + "HH", *val_or_off)
        else:
            v = struct.pack(e + "I", val_or_off)
        tags.append((t, struct.pack(e + "HHI", t, typ, cnt) + v))

    tag(256, 4, 1, w)
    tag(257, 4, 1, h)
    if nc == 1:
        tag(258, 3, 1, bits)
    elif nc == 2:
        tag(258, 3, 2, (bits, bits))
    else:
        tag(258, 3, nc, bps_off, inline=False)
    tag(259, 3, 1, compression)
    tag(262, 3, 1, 2 if nc >= 3 else 1)
    tag(273, 4, nst, offs[0] if nst == 1 else so_off, inline=(nst == 1))
    tag(277, 3, 1, nc)
    tag(278, 4, 1, rps)
    tag(279, 4, nst, len(strips[0]) if nst == 1 else sbc_off, inline=(nst == 1))
    tag(284, 3, 1, 2 if planar else 1)
    if nc in (2, 4):
        tag(338, 3, 1, 2 if alpha is None else alpha)
    tag(339, 3, 1, 1)
    tags.sort(key=lambda t: t[0])
    assert len(tags) == ntags
    hdr = (b"MM\0*" if big_endian else b"II*\0") + struct.pack(e + "I", ifd_off)
    ifd = struct.pack(e + "H", ntags) + b"".join(t[1] for t in tags) + struct.pack(e + "I", 0)
    del data_base_placeholder
    return hdr + ifd + bytes(extra) + b"".join(strips)


def decode_opj(data: bytes, ext=".jpx", area=None, layers=None, reduce=None) -> np.ndarray:
    """Decode with opj_decompress (exact for 16-bit RGB, unlike Pillow);
    area = (x0, y0, x1, y1) decodes only that window (-d); layers = the
    first n quality layers only (-l); reduce = drop the r highest
    resolutions (-r), the views a IIIF image server serves."""
    tool = opj("opj_decompress")
    if tool is None:
        raise RuntimeError("opj_decompress not available")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "in" + (".jp2" if ext in (".jpx", ".jp2") else ".j2k"))
        dst = os.path.join(d, "out.tif")
        with open(src, "wb") as f:
            f.write(data)
        cmd = [tool, "-i", src, "-o", dst]
        if area is not None:
            cmd += ["-d", ",".join(str(int(v)) for v in area)]
        if layers is not None:
            cmd += ["-l", str(int(layers))]
        if reduce is not None:
            cmd += ["-r", str(int(reduce))]
        r = subprocess.run(cmd, capture_output=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr.decode() + r.stdout.decode())
        return read_tiff(open(dst, "rb").read())


def read_tiff(data: bytes) -> np.ndarray:
    """Minimal TIFF reader for opj_decompress output (uncompressed strips)."""
    le = data[:2] == b"II"
    e = "<" if le else ">"
    ifd = struct.unpack(e + "I", data[4:8])[0]
    n = struct.unpack(e + "H", data[ifd:ifd + 2])[0]
    tags = {}
    for i in range(n):
        t, typ, cnt, val = struct.unpack(e + "HHI4s", data[ifd + 2 + 12 * i: ifd + 14 + 12 * i])
        sz = {3: 2, 4: 4, 1: 1}.get(typ, 1)
        fmt = {3: "H", 4: "I", 1: "B"}.get(typ, "B")
        if sz * cnt <= 4:
            vals = struct.unpack(e + fmt * cnt, val[:sz * cnt])
        else:
            off = struct.unpack(e + "I", val)[0]
            vals = struct.unpack(e + fmt * cnt, data[off:off + sz * cnt])
        tags[t] = vals
    w, h = tags[256][0], tags[257][0]
    bits = tags[258][0]
    spp = tags.get(277, (1,))[0]
    planar = tags.get(284, (1,))[0]
    assert tags.get(259, (1,))[0] == 1
    dt = np.dtype(np.uint8 if bits == 8 else np.uint16).newbyteorder(e)
    raw = b"".join(data[o:o + c] for o, c in zip(tags[273], tags[279]))
    a = np.frombuffer(raw, dtype=dt).astype(dt.newbyteorder("="))
    if planar == 2:
        a = a.reshape(spp, h, w).transpose(1, 2, 0)
    else:
        a = a.reshape(h, w, spp)
    return a if spp > 1 else a[..., 0]


def decode_pillow(data: bytes) -> np.ndarray:
    from PIL import Image
    return np.array(Image.open(io.BytesIO(data)))


def psnr(a: np.ndarray, b: np.ndarray, bits=8) -> float:
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    peak = (1 << bits) - 1
    return float("inf") if mse == 0 else 10 * np.log10(peak * peak / mse)


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def markers(cs: bytes):
    """(offset, marker) list of the main header + the count of SOP/SOT/PLT markers."""
    i = cs.find(b"\xff\x4f")
    return i


def main_header_segments(cs: bytes) -> dict:
    """SIZ/COD/QCD segment bytes of a J2K codestream (possibly inside a JP2/JPX)."""
    i = cs.find(b"\xff\x4f\xff\x51")
    assert i >= 0, "no SOC+SIZ"
    out = {}
    p = i + 2
    while True:
        m = cs[p:p + 2]
        if m == b"\xff\x90":
            break
        L = struct.unpack(">H", cs[p + 2:p + 4])[0]
        out.setdefault(m.hex(), cs[p:p + 2 + L])
        p += 2 + L
    return out


def codestream(data: bytes) -> bytes:
    i = data.find(b"\xff\x4f\xff\x51")
    return data[i:]


def count_marker(cs: bytes, marker: bytes) -> int:
    return cs.count(marker)


def tile_parts(cs: bytes):
    """Walk SOT markers: list of (Isot, Psot, TPsot, TNsot)."""
    out = []
    p = cs.find(b"\xff\x90")
    while p >= 0 and cs[p:p + 2] == b"\xff\x90":
        isot, psot, tp, tn = struct.unpack(">HIBB", cs[p + 4:p + 12])
        out.append((isot, psot, tp, tn))
        if psot == 0:
            break
        p += psot
    return out


def tiff_set_tag(data: bytes, tag: int, value: int) -> bytes:
    """Classic or BigTIFF (either byte order): overwrite the first (inline)
    value of IFD entry `tag` -- malformed-file fixtures for the parser tests."""
    b = bytearray(data)
    e = "<" if b[:2] == b"II" else ">"
    big = struct.unpack(e + "H", b[2:4])[0] == 43
    ifd = struct.unpack(e + "Q", b[8:16])[0] if big else struct.unpack(e + "I", b[4:8])[0]
    n = struct.unpack(e + ("Q" if big else "H"), b[ifd:ifd + (8 if big else 2)])[0]
    base, size = ifd + (8 if big else 2), (20 if big else 12)
    for i in range(n):
        p = base + i * size
        t, typ = struct.unpack(e + "HH", b[p:p + 4])
        if t != tag:
            continue
        v = p + (12 if big else 8)
        fmt = {3: "H", 4: "I", 16: "Q"}[typ]
        b[v:v + struct.calcsize(fmt)] = struct.pack(e + fmt, value)
        return bytes(b)
    raise KeyError(tag)


def tiff_bytes_compressed(img: np.ndarray, compression: str, predictor: bool = False, rows_per_strip: int = 16) -> bytes:
    """LZW ("tiff_lzw"), Deflate ("tiff_adobe_deflate" = 8, "tiff_deflate" =
    32946) or PackBits ("packbits") strip TIFF written by Pillow's
    libtiff (test fixture generator only), optionally with Predictor 2."""
    import io
    from PIL import Image, TiffImagePlugin
    kw = {}
    if predictor:
        ti = TiffImagePlugin.ImageFileDirectory_v2()
        ti[317] = 2
        kw["tiffinfo"] = ti
    row = img.shape[1] * (img.shape[2] if img.ndim == 3 else 1) * img.dtype.itemsize
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="TIFF", compression=compression, strip_size=row * rows_per_strip, **kw)
    data = b.getvalue()
    if compression == "tiff_deflate":  # libtiff writes 8 for both; keep the old code's value in the tag
        tag = struct.pack("<HHIHH", 259, 3, 1, 8, 0)
        i = data.find(tag)
        assert i > 0
        data = data[:i] + struct.pack("<HHIHH", 259, 3, 1, 32946, 0) + data[i + len(tag):]
    return data


def bigtiff_bytes(img: np.ndarray, rows_per_strip=64, big_endian=False, strip_codec=None, compression=1) -> bytes:
    """Chunky BigTIFF (version 43, LONG8 strip offsets / counts); uncompressed,
    or each strip passed through `strip_codec` (then tagged `compression`)."""
    if img.ndim == 2:
        img = img[..., None]
    h, w, nc = img.shape
    bits = img.dtype.itemsize * 8
    e = ">" if big_endian else "<"
    rps = min(rows_per_strip, h)
    nst = (h + rps - 1) // rps
    strips = [np.ascontiguousarray(img[s * rps:(s + 1) * rps]) for s in range(nst)]
    strips = [b.astype(b.dtype.newbyteorder(e)).tobytes() for b in strips]
    if strip_codec is not None:
        strips = [strip_codec(x) for x in strips]
    ntags = 10
    ifd_off = 16
    arr_off = ifd_off + 8 + 20 * ntags + 8
    so_off, sbc_off = arr_off, arr_off + 8 * nst
    data = sbc_off + 8 * nst
    offs = []
    for s in strips:
        offs.append(data)
        data += len(s)

    def ent(t, typ, cnt, vals):
        fmt = {3: "H", 4: "I", 16: "Q"}[typ]
        raw = struct.pack(e + fmt * len(vals), *vals)
        return struct.pack(e + "HHQ", t, typ, cnt) + (raw + b"\0" * 8)[:8]

    tags = [ent(256, 4, 1, [w]), ent(257, 4, 1, [h]), ent(258, 3, nc, [bits] * nc), ent(259, 3, 1, [compression]),
            ent(262, 3, 1, [2 if nc >= 3 else 1]),
            ent(273, 16, nst, [offs[0]] if nst == 1 else [so_off]), ent(277, 3, 1, [nc]), ent(278, 4, 1, [rps]),
            ent(279, 16, nst, [len(strips[0])] if nst == 1 else [sbc_off]), ent(284, 3, 1, [1])]
    hdr = (b"MM" if big_endian else b"II") + struct.pack(e + "HHHQ", 43, 8, 0, ifd_off)
    ifd = struct.pack(e + "Q", ntags) + b"".join(tags) + struct.pack(e + "Q", 0)
    arrays = struct.pack(e + "Q" * nst, *offs) + struct.pack(e + "Q" * nst, *[len(s) for s in strips])
    return hdr + ifd + arrays + b"".join(strips)


def packbits_encode(raw: bytes) -> bytes:
    """PackBits with literal runs only (valid, if not small)."""
    out = bytearray()
    for i in range(0, len(raw), 128):
        chunk = raw[i:i + 128]
        out.append(len(chunk) - 1)
        out += chunk
    return bytes(out)


def tiled_tiff_bytes(img: np.ndarray, tile=(32, 48), planar=False, big_endian=False, packbits=False,
                     deflate=False) -> bytes:
    """Classic tiled TIFF (TileWidth/TileLength/TileOffsets/TileByteCounts),
    uncompressed, PackBits or Deflate (zlib levels 0 / 1 / 9 in turn, so
    stored, fixed-Huffman and dynamic-Huffman blocks all occur); edge tiles
    padded with zeros as TIFF requires."""
    import zlib
    if img.ndim == 2:
        img = img[..., None]
    h, w, nc = img.shape
    tw, th = tile
    bits = img.dtype.itemsize * 8
    e = ">" if big_endian else "<"
    across, down = (w + tw - 1) // tw, (h + th - 1) // th
    planes = [img[..., c:c + 1] for c in range(nc)] if planar else [img]
    tiles = []
    for pl in planes:
        for ty in range(down):
            for tx in range(across):
                t = np.zeros((th, tw, pl.shape[2]), img.dtype)
                part = pl[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw]
                t[:part.shape[0], :part.shape[1]] = part
                raw = t.astype(t.dtype.newbyteorder(e)).tobytes()
                if deflate:
                    tiles.append(zlib.compress(raw, (0, 1, 9)[len(tiles) % 3]))
                else:
                    tiles.append(packbits_encode(raw) if packbits else raw)
    nt = len(tiles)
    ntags = 13
    ifd_off = 8
    extra_base = ifd_off + 2 + 12 * ntags + 4
    bps_off = extra_base
    to_off = bps_off + 2 * max(nc, 2)
    tbc_off = to_off + 4 * nt
    data = tbc_off + 4 * nt
    offs = []
    for t in tiles:
        offs.append(data)
        data += len(t)

    def ent(tag, typ, cnt, val):
        v = struct.pack(e + "HH", val, 0) if (typ == 3 and cnt == 1) else struct.pack(e + "I", val)
        return struct.pack(e + "HHI", tag, typ, cnt) + v

    tags = [ent(256, 4, 1, w), ent(257, 4, 1, h), ent(258, 3, nc, bps_off) if nc > 1 else ent(258, 3, 1, bits),
            ent(259, 3, 1, 8 if deflate else 32773 if packbits else 1), ent(262, 3, 1, 2 if nc >= 3 else 1), ent(277, 3, 1, nc),
            ent(284, 3, 1, 2 if planar else 1), ent(322, 4, 1, tw), ent(323, 4, 1, th),
            ent(324, 4, nt, to_off if nt > 1 else offs[0]), ent(325, 4, nt, tbc_off if nt > 1 else len(tiles[0])),
            ent(339, 3, 1, 1), ent(338, 3, 1, 2) if nc in (2, 4) else ent(305, 2, 1, 0)]
    tags.sort(key=lambda t: struct.unpack(e + "H", t[:2])[0])
    hdr = (b"MM\0*" if big_endian else b"II*\0") + struct.pack(e + "I", ifd_off)
    ifd = struct.pack(e + "H", ntags) + b"".join(tags) + struct.pack(e + "I", 0)
    extra = struct.pack(e + "H" * max(nc, 2), *([bits] * max(nc, 2)))
    extra += struct.pack(e + "I" * nt, *offs) + struct.pack(e + "I" * nt, *[len(t) for t in tiles])
    return hdr + ifd + extra + b"".join(tiles)


# ---- a fixed-Huffman Deflate writer for crafted token streams (RFC 1951 3.2.6) ----
_LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131,
             163, 195, 227, 258]
_LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
_DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049,
              3073, 4097, 6145, 8193, 12289, 16385, 24577]
_DIST_EXTRA = [0, 0, 0, 0] + [k for k in range(1, 14) for _ in (0, 1)]


class _Bits:
    def __init__(self):
        self.buf, self.acc, self.n = bytearray(), 0, 0

    def put(self, v, n):  # LSB first
        self.acc |= v << self.n
        self.n += n
        while self.n >= 8:
            self.buf.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def put_code(self, code, n):  # Huffman codes go MSB first
        self.put(int(format(code, f"0{n}b")[::-1], 2), n)

    def done(self):
        if self.n:
            self.buf.append(self.acc & 0xFF)
        return bytes(self.buf)


def _fixed_litlen(bw, v):
    if v < 144:
        bw.put_code(0x30 + v, 8)
    elif v < 256:
        bw.put_code(0x190 + v - 144, 9)
    elif v < 280:
        bw.put_code(v - 256, 7)
    else:
        bw.put_code(0xC0 + v - 280, 8)


def deflate_tokens(tokens) -> tuple[bytes, bytes]:
    """zlib stream of one fixed-Huffman block coding `tokens` -- ints (a
    literal byte) or (length, distance) matches -- exactly as given, and the
    bytes it decodes to.  Lets a test pick every match distance and length
    (zlib picks its own)."""
    import zlib
    out = bytearray()
    bw = _Bits()
    bw.put(1, 1)  # BFINAL
    bw.put(1, 2)  # BTYPE 01: fixed codes
    for t in tokens:
        if isinstance(t, int):
            _fixed_litlen(bw, t)
            out.append(t)
            continue
        length, dist = t
        assert 3 <= length <= 258 and 1 <= dist <= min(32768, len(out))
        i = max(k for k in range(29) if _LEN_BASE[k] <= length) if length < 258 else 28
        _fixed_litlen(bw, 257 + i)
        if _LEN_EXTRA[i]:
            bw.put(length - _LEN_BASE[i], _LEN_EXTRA[i])
        j = max(k for k in range(30) if _DIST_BASE[k] <= dist)
        bw.put_code(j, 5)
        if _DIST_EXTRA[j]:
            bw.put(dist - _DIST_BASE[j], _DIST_EXTRA[j])
        for _ in range(length):
            out.append(out[-dist])
    _fixed_litlen(bw, 256)  # end of block
    body = bw.done()
    stream = b"\x78\x01" + body + struct.pack(">I", zlib.adler32(bytes(out)))
    return stream, bytes(out)


def crafted_match_tokens(seed=7):
    """Every match distance 1..70 with lengths 3..258 (overlapping copies,
    dist < length), then long distances up to 32768, between random
    literals: the decoded data runs over many 4096-byte window flushes."""
    rng = np.random.default_rng(seed)
    toks, n = [], 0
    for _ in range(300):
        toks.append(int(rng.integers(0, 256)))
        n += 1
    lens = (3, 4, 5, 7, 10, 31, 63, 64, 65, 100, 127, 128, 129, 200, 257, 258)
    for d in list(range(1, 71)) + [100, 255, 256, 1000, 4095, 4096, 4097, 20000, 32767, 32768]:
        for L in lens:
            for _ in range(int(rng.integers(0, 3))):
                toks.append(int(rng.integers(0, 256)))
                n += 1
            if d <= n:
                toks.append((L, d))
                n += L
    return toks


def packet_bytes_by_layer(cs: bytes, layers: int, tiles=None) -> list:
    """Bytes of the packets of each quality layer (SOP through the packet
    body) in a raw code-stream written with SOP markers and a
    layer-innermost progression (RPCL / LRCP-free recipes: Nsop mod layers
    is the layer), summed over ``tiles`` (all when None). This is what a
    decoder reading the first l layers receives, unlike Kakadu's
    Kdu-Layer-Info L column, which projects its first flush."""
    out = [0] * layers
    p = cs.find(b"\xff\x90")
    while p >= 0 and cs[p:p + 2] == b"\xff\x90":
        isot = struct.unpack(">H", cs[p + 4:p + 6])[0]
        end = p + struct.unpack(">I", cs[p + 6:p + 10])[0]
        if tiles is None or isot in tiles:
            body = cs[cs.find(b"\xff\x93", p) + 2:end]
            sops, j = [], body.find(b"\xff\x91")
            while j >= 0:
                sops.append(j)
                j = body.find(b"\xff\x91", j + 6)
            for a, b in zip(sops, sops[1:] + [len(body)]):
                out[struct.unpack(">H", body[a + 4:a + 6])[0] % layers] += b - a
        p = end
    return out
