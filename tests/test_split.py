"""Tile-split path: one image, contiguous bands of tile
rows per rank, one exchange step (global PCRD thresholds by all-reduce).

CPU tests pin the exchange rule: jp2hip_split_thresholds over any partition of
the hull segments across ranks (threads, or gloo processes) must give the
thresholds the oracle's select_threshold (oracle/jp2_oracle.c:1053-1067) gives
on the union.  GPU tests assert that the parts of 1..4 ranks, concatenated in
rank order, are byte-identical to the single-GPU file and to the oracle.
"""
import os
import threading

import numpy as np
import pytest

import imaging as im
import jp2hip
from jp2hip import split as js

K_NONE = 0x7FF0000000000001  # "include nothing" (csrc/split.cpp)


def select_threshold(keys, dr, budget):
    """Restatement of oracle/jp2_oracle.c:1053-1067 on (key, bytes) segments:
    walk equal-key groups in decreasing key order while the total fits."""
    order = np.argsort(-keys.astype(np.float64), kind="stable")
    ks, ds = keys[order], dr[order]
    acc, K, i, n = 0, None, 0, len(ks)
    while i < n:
        j, grp = i, 0
        while j < n and ks[j] == ks[i]:
            grp += int(ds[j])
            j += 1
        if acc + grp > budget:
            break
        acc += grp
        K = int(ks[i])
        i = j
    return K


def included(keys, dr, K):
    return int(dr[keys >= np.uint64(K)].sum()) if K is not None else 0


def _segments(rng, n, ties=True):
    # positive finite doubles' bit patterns, as slope_key() produces
    vals = rng.uniform(1e-3, 1e4, size=n)
    if ties:
        vals[rng.integers(0, n, n // 3)] = vals[rng.integers(0, n, n // 3)]
    keys = vals.astype(np.float64).view(np.uint64)
    dr = rng.integers(1, 4000, size=n).astype(np.int64)
    return keys, dr


def _rank_arrays(keys, dr):
    o = np.argsort(-keys.astype(np.float64), kind="stable")
    return keys[o], np.cumsum(dr[o]).astype(np.int64)


def test_split_rows_cover_every_row_once():
    """Bands are whole -flush_period stripes (so each rank's tile-parts are one
    contiguous run of the file) and balanced to within one stripe."""
    for h, th, fp in ((30000, 512, 1024), (1, 512, 1024), (1000, 512, 1024), (2048, 512, 1024),
                      (700, 256, 1024), (30000, 512, 0), (5000, 768, 1024), (8000, 1024, 1024)):
        nty = (h + th - 1) // th
        stripe = max(1, fp // th) if fp > 0 else 1
        for world in (1, 2, 3, 4, 7, 8, 64):
            bands = [js.split_rows(h, th, r, world, fp) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == h
            for (a0, a1), (b0, b1) in zip(bands, bands[1:]):
                assert a1 == b0 and a0 <= a1
            for r0, r1 in bands:
                assert r0 % th == 0
                assert r1 == h or r1 % th == 0
                if fp > 0 and r1 < h:
                    assert r1 % fp == 0 or (r1 // fp) > ((r1 - th) // fp), (h, th, fp, r1)  # ends a flush
            sizes = [-(-(r1 - r0) // th) if r1 > r0 else 0 for r0, r1 in bands]
            assert max(sizes) - min(sizes) <= 2 * stripe or nty < world * stripe


def test_thresholds_world1_match_oracle_rule():
    rng = np.random.default_rng(7)
    keys, dr = _segments(rng, 5000)
    k, c = _rank_arrays(keys, dr)
    total = int(dr.sum())
    budgets = [0, 1, 17, total // 64, total // 3, total // 2, total - 1, total, total * 4]
    for chunk in (budgets[:6], budgets[6:]):
        K = js.thresholds(k, c, chunk)
        for b, kk in zip(chunk, K):
            want = select_threshold(keys, dr, b)
            # same included set (the oracle names the last key taken, the
            # bisection the least key with the same set)
            assert included(keys, dr, int(kk)) == included(keys, dr, want)
            if want is None:
                assert int(kk) == K_NONE or included(keys, dr, int(kk)) == 0


def test_thresholds_empty_rank_and_no_segments():
    K = js.thresholds(np.zeros(0, np.uint64), np.zeros(0, np.int64), [0, 100])
    assert list(K) == [0, 0]  # S(0) = 0 fits every budget


def test_thresholds_threads_equal_world1():
    rng = np.random.default_rng(11)
    keys, dr = _segments(rng, 3000)
    total = int(dr.sum())
    budgets = np.array([total >> (5 - l) for l in range(6)], np.int64)
    want = js.thresholds(*_rank_arrays(keys, dr), budgets)
    for world in (2, 3, 5):
        owner = rng.integers(0, world, len(keys))
        owner[:world] = np.arange(world)
        g = js.ThreadGroup(world)
        out = [None] * world

        def work(r):
            m = owner == r
            out[r] = js.thresholds(*_rank_arrays(keys[m], dr[m]), budgets, g.member(r))

        th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for r in range(world):
            assert np.array_equal(out[r], want), (world, r)


def _gloo_worker(rank, world, port, keys, dr, owner, budgets, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = owner == rank
        K = js.thresholds(*_rank_arrays(keys[m], dr[m]), budgets, js.TorchGroup())
        q.put((rank, K.tolist()))
    finally:
        dist.destroy_process_group()


def test_thresholds_gloo_world2_equal_world1():
    import socket

    import torch.multiprocessing as mp
    rng = np.random.default_rng(3)
    keys, dr = _segments(rng, 2000)
    total = int(dr.sum())
    budgets = np.array([total >> (5 - l) for l in range(6)], np.int64)
    want = js.thresholds(*_rank_arrays(keys, dr), budgets).tolist()
    owner = (np.arange(len(keys)) * 7919) % 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, keys, dr, owner, budgets, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == want and res[1] == want


def test_band_strips_rebases_offsets():
    img = im.synth_rgb8(300, 170, seed=2)
    for kw in ({}, {"planar": True}, {"rows_per_strip": 7}):
        tif = im.tiff_bytes(img, **kw)
        lay, offs = jp2hip.tiff_layout(tif)
        rps = lay.rows_per_strip
        buf, blay, boffs = js.band_strips(tif, lay, offs, 128, 256)
        planes = 3 if kw.get("planar") else 1
        per_plane = (lay.height + rps - 1) // rps
        row_bytes = lay.width * (1 if planes == 3 else 3)
        for p in range(planes):
            for s in range(128 // rps, -(-256 // rps)):
                i = p * per_plane + s
                n = (min(lay.height, (s + 1) * rps) - s * rps) * row_bytes
                assert buf[boffs[i]:boffs[i] + n] == tif[offs[i]:offs[i] + n]


def test_band_units_pack_compressed_strips_and_tiles():
    """Compressed strips and tiles of a band are packed whole with their byte
    counts (offsets, then counts, as tiff_layout returns them)."""
    img = im.synth_rgb8(300, 170, seed=2)
    for tif in (im.tiff_bytes(img, rows_per_strip=48, strip_codec=im.lzw_encode, compression=5),
                im.tiff_bytes(img, rows_per_strip=7, planar=True, strip_codec=im.packbits_encode, compression=32773),
                im.tiled_tiff_bytes(img, tile=(32, 48)),
                im.tiled_tiff_bytes(img, tile=(32, 48), planar=True, deflate=True)):
        lay, offs = jp2hip.tiff_layout(tif)
        n = lay.nstrips
        buf, blay, boffs = js.band_strips(tif, lay, offs, 128, 256)
        assert blay.compression == lay.compression and blay.tile_width == lay.tile_width
        uh = lay.tile_height if lay.tile_width else lay.rows_per_strip
        across = -(-lay.width // lay.tile_width) if lay.tile_width else 1
        per_plane = across * -(-lay.height // uh)
        planes = 3 if lay.planar == 2 else 1
        seen = 0
        for p in range(planes):
            for u in range(128 // uh, -(-256 // uh)):
                for x in range(across):
                    i = p * per_plane + u * across + x
                    nb = offs[n + i]
                    assert boffs[n + i] == nb and blay.strip_bytes[i] == nb
                    assert buf[boffs[i]:boffs[i] + nb] == tif[offs[i]:offs[i] + nb]
                    seen += nb
        assert seen == len(buf)


def test_exports_split_symbols():
    from jp2hip import _lib
    L = _lib.lib()
    for s in ("jp2hip_split_rows", "jp2hip_encode_device_split", "jp2hip_split_thresholds"):
        assert hasattr(L, s)


# --------------------------------------------------------------------------
# GPU: parts concatenate to the single-GPU file
# --------------------------------------------------------------------------

def _encode_world(tif, conv, rc, world, band_only=False):
    """Ranks as threads, each with its own context on cuda:0."""
    from devmem import DeviceBytes
    lay, offs = jp2hip.tiff_layout(tif)
    g = js.ThreadGroup(world)
    parts, errs = [None] * world, []

    def work(r):
        try:
            enc = jp2hip.Encoder(0)
            try:
                if band_only:
                    r0, r1 = js.split_rows(lay.height, rc.tile_h, r, world, rc.flush_period)
                    buf, blay, keep = js.band_strips(tif, lay, offs, r0, r1)
                    src, use = (buf or b"\0"), blay
                else:
                    src, use = tif, lay
                d = DeviceBytes(src)
                member = g.member(r)
                try:
                    parts[r] = enc.encode_device_split(d.ptr, d.nbytes, use, conv, member.split(), rc)
                finally:
                    d.free()
            finally:
                enc.close()
        except Exception as e:  # keep the other ranks from waiting forever
            errs.append(e)
            g.abort()

    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    if errs:
        raise errs[0]
    data = b"".join(p[0] for p in parts)
    off = 0
    for p in parts:
        assert p[1] == off and p[2] == len(data)
        off += len(p[0])
    return data, parts


SPLIT_CASES = [
    # h, w, nc, bits, lossless, levels, tile, worlds
    (1300, 700, 3, 8, False, 6, 256, (1, 2, 3, 6)),
    (1300, 700, 3, 8, True, 6, 256, (2, 4)),
    (1100, 900, 1, 16, False, 7, 256, (1, 3, 5)),
    (1100, 900, 1, 16, True, 7, 256, (2,)),
    (200, 300, 3, 8, False, 6, 512, (2,)),  # one tile row: rank 1 has nothing
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", SPLIT_CASES,
                         ids=[f"{c[0]}x{c[1]}x{c[2]}_{c[3]}b_{'ll' if c[4] else 'ly'}_T{c[6]}" for c in SPLIT_CASES])
def test_split_parts_concatenate_to_single_gpu_file(encoder, case):
    import oracle_lib as ol
    h, w, nc, bits, lossless, levels, tile, worlds = case
    img = im.synth_u16(h, w, comps=nc, seed=h + w) if bits == 16 else im.synth_rgb8(h, w, seed=h + w)
    conv = jp2hip.LOSSLESS if lossless else jp2hip.LOSSY
    rc = jp2hip.recipe(conv, levels=levels, tile_w=tile, tile_h=tile)
    tif = im.tiff_bytes(img)
    single, _ = encoder.encode_tiff(tif, conv, rc)
    assert single == ol.encode(img, ol.copy_recipe(rc))
    for world in worlds:
        got, _ = _encode_world(tif, conv, rc, world)
        assert got == single, world


@pytest.mark.gpu
def test_split_slope_prediction_is_global(encoder):
    """Gray16 at 1 bpp: slope prediction skips planes, and its histogram is
    summed over ranks, so every world size reproduces the single-GPU file."""
    import oracle_lib as ol
    img = im.synth_u16(1100, 900, comps=1, seed=12)
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=7, tile_w=256, tile_h=256, rate_bpp=1.0)
    tif = im.tiff_bytes(img)
    single, st = encoder.encode_tiff(tif, jp2hip.LOSSY, rc)
    assert single == ol.encode(img, ol.copy_recipe(rc))
    _, st0 = encoder.encode_tiff(tif, jp2hip.LOSSY, jp2hip.recipe(jp2hip.LOSSY, levels=7, tile_w=256, tile_h=256,
                                                                  rate_bpp=1.0, slope_skip=0))
    assert st.t1_bytes < st0.t1_bytes
    for world in (2, 3):
        got, _ = _encode_world(tif, jp2hip.LOSSY, rc, world)
        assert got == single, world


@pytest.mark.gpu
def test_split_band_only_upload(encoder):
    img = im.synth_u16(1500, 800, comps=1, seed=8)
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=7, tile_w=256, tile_h=256)
    tif = im.tiff_bytes(img, rows_per_strip=48)
    single, _ = encoder.encode_tiff(tif, jp2hip.LOSSY, rc)
    got, _ = _encode_world(tif, jp2hip.LOSSY, rc, 3, band_only=True)
    assert got == single


def _packed_masters():
    """(name, TIFF bytes, conversion) of compressed / tiled masters of one
    1300x700 image: band boundaries (256-row tile rows) fall inside strips
    and tiles (48-row units)."""
    rgb = im.synth_rgb8(1300, 700, seed=21)
    g16 = im.synth_u16(1300, 700, comps=1, seed=22)
    return [
        ("lzw48", im.tiff_bytes(rgb, rows_per_strip=48, strip_codec=im.lzw_encode, compression=5), rgb),
        ("lzw_pred_pillow", im.tiff_bytes_compressed(rgb, "tiff_lzw", predictor=True, rows_per_strip=16), rgb),
        ("deflate_pillow", im.tiff_bytes_compressed(rgb, "tiff_adobe_deflate", rows_per_strip=40), rgb),
        ("packbits_planar", im.tiff_bytes(rgb, rows_per_strip=48, planar=True, strip_codec=im.packbits_encode,
                                          compression=32773), rgb),
        ("tiled", im.tiled_tiff_bytes(rgb, tile=(64, 48)), rgb),
        ("tiled_deflate_planar", im.tiled_tiff_bytes(rgb, tile=(64, 48), planar=True, deflate=True), rgb),
        ("bigtiff_lzw_gray16", im.bigtiff_bytes(g16, rows_per_strip=48, strip_codec=im.lzw_encode, compression=5),
         g16),
    ]


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(7), ids=["lzw48", "lzw_pred_pillow", "deflate_pillow", "packbits_planar",
                                               "tiled", "tiled_deflate_planar", "bigtiff_lzw_gray16"])
def test_split_compressed_and_tiled_masters(encoder, idx):
    """SURVEY.md 8(f) row 3 on the C5 route: LZW / Deflate / PackBits strips,
    tiled TIFFs and an LZW BigTIFF split over 2 and 3 ranks -- each rank
    decoding only its band's strips or tiles, from the whole file or from a
    band-only upload -- concatenate to the single-GPU file of the same pixels
    from an uncompressed TIFF."""
    name, tif, img = _packed_masters()[idx]
    lossless = idx % 2 == 1
    conv = jp2hip.LOSSLESS if lossless else jp2hip.LOSSY
    rc = jp2hip.recipe(conv, levels=6, tile_w=256, tile_h=256)
    want, _ = encoder.encode_tiff(im.tiff_bytes(img), conv, rc)
    single, _ = encoder.encode_tiff(tif, conv, rc)
    assert single == want, name
    for world, band_only in ((2, False), (3, True)):
        got, _ = _encode_world(tif, conv, rc, world, band_only=band_only)
        assert got == want, (name, world, band_only)


@pytest.mark.gpu
def test_split_truncated_band_fails_on_every_rank(encoder):
    """one rank's band-only upload of a compressed master is cut
    short (its last strip's bytes past the buffer): that rank fails on its
    own, and every other rank fails too (the failure flag of the exchanges)
    instead of writing a part of a file that cannot be whole."""
    from devmem import DeviceBytes
    img = im.synth_rgb8(1300, 700, seed=23)
    tif = im.tiff_bytes(img, rows_per_strip=48, strip_codec=im.lzw_encode, compression=5)
    rc = jp2hip.recipe(jp2hip.LOSSY, tile_w=256, tile_h=256)
    lay, offs = jp2hip.tiff_layout(tif)
    world = 3
    g = js.ThreadGroup(world)
    errs = [None] * world

    def work(r):
        enc = jp2hip.Encoder(0)
        try:
            r0, r1 = js.split_rows(lay.height, rc.tile_h, r, world, rc.flush_period)
            buf, blay, keep = js.band_strips(tif, lay, offs, r0, r1)
            if r == 1:
                buf = buf[:len(buf) - 100]  # the band's last strip runs past the upload
            d = DeviceBytes(buf or b"\0")
            try:
                enc.encode_device_split(d.ptr, d.nbytes, blay, jp2hip.LOSSY, g.member(r).split(), rc)
            finally:
                d.free()
        except Exception as e:
            errs[r] = e
        finally:
            enc.close()

    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert all(isinstance(e, jp2hip.Jp2hipError) for e in errs), errs
    assert "outside the source buffer" in str(errs[1])
    # the others stop at their next exchange: through the group's failure
    # flag, or -- a rank already waiting in the exchange the failing rank
    # never joined -- through that aborted exchange
    assert all("another rank failed" in str(errs[r]) or "exchange failed" in str(errs[r]) for r in (0, 2)), errs


@pytest.mark.gpu
def test_split_c5_shape_on_rate_and_identical(encoder):
    """C5's recipe (Gray16, 7 levels, 6 layers, lossy 3 bpp, 512^2 tiles) on a
    6000x4000 crop: 4 ranks == single GPU, within rate, decodes at a sane PSNR.
    (This synthetic Gray16 content holds ~2.5 bpp at the irreversible base
    step -- golden.json "synth_gray16_1024", opj agrees -- so 3 bpp is a cap,
    not a target it reaches.)"""
    img = im.synth_u16(4000, 6000, comps=1, seed=5)
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=7)
    tif = im.tiff_bytes(img)
    single, _ = encoder.encode_tiff(tif, jp2hip.LOSSY, rc)
    got, parts = _encode_world(tif, jp2hip.LOSSY, rc, 4)
    assert got == single
    cs = im.codestream(got)
    assert 2.0 * 6000 * 4000 / 8 <= len(cs) <= 3.0 * 6000 * 4000 / 8
    assert im.psnr(img, im.decode_opj(got), 16) > 40


@pytest.mark.gpu
def test_split_write_parts_to_one_file(encoder, tmp_path):
    img = im.synth_rgb8(1100, 600, seed=4)
    rc = jp2hip.recipe(jp2hip.LOSSLESS, tile_w=256, tile_h=256)
    tif = im.tiff_bytes(img)
    data, parts = _encode_world(tif, jp2hip.LOSSLESS, rc, 3)
    tmp = tmp_path / "x.jpx.part"
    for p in reversed(parts):  # any order
        js.write_part(str(tmp), p[0], p[1], p[2])
    os.replace(tmp, tmp_path / "x.jpx")
    assert (tmp_path / "x.jpx").read_bytes() == data
    assert np.array_equal(im.decode_pillow(data), img)


@pytest.mark.gpu
def test_split_c5_full_size(encoder, golden):
    """C5 at its configured size: 40000x30000 Gray16, lossy 3 bpp, 7 levels,
    512^2 tiles (1.2 GP, 4 661 tiles, 350 701 code-blocks).  The single-GPU
    file is the oracle's (SHA-256 committed by make_golden.py); the
    tile-split encode at world 1 and world 2 (ranks as threads on cuda:0)
    equals it, stays within rate, and decodes (opj_decompress on three
    1024^2 windows) at the expected PSNR."""
    from concurrent.futures import ThreadPoolExecutor
    from devmem import DeviceBytes
    w, h, rps = 40000, 30000, 64
    buf = np.empty((h, w), "<u2")

    def fill(g):
        buf[g:min(h, g + 512)] = im.synth_gray16_rows(g, min(h, g + 512), w, seed=5, band=512)

    with ThreadPoolExecutor(16) as ex:
        list(ex.map(fill, range(0, h, 512)))
    nstrips = (h + rps - 1) // rps
    from ctypes import POINTER, c_uint64, cast
    offs = (c_uint64 * nstrips)(*[s * rps * w * 2 for s in range(nstrips)])
    from jp2hip._lib import Layout
    lay = Layout(w, h, 1, 16, 1, 0, rps, nstrips, cast(offs, POINTER(c_uint64)))
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=7)
    d = DeviceBytes(buf)
    try:
        single, st = encoder.encode_device(d.ptr, d.nbytes, lay, jp2hip.LOSSY, rc)
        assert st.codeblocks == 350701
        # the oracle's file for the same pixels (tests/golden/make_golden.py c5_full)
        import hashlib
        assert len(single) == golden["c5_full"]["oracle_bytes"]
        assert hashlib.sha256(single).hexdigest() == golden["c5_full"]["oracle_sha256"]
        cs = im.codestream(single)
        assert len(cs) <= 3.0 * w * h / 8
        assert len(im.tile_parts(cs)) == 4661 * 8
        for world in (1, 2):
            g = js.ThreadGroup(world)
            parts, errs = [None] * world, []

            def work(r):
                try:
                    e = jp2hip.Encoder(0)
                    try:
                        parts[r] = e.encode_device_split(d.ptr, d.nbytes, lay, jp2hip.LOSSY, g.member(r).split(), rc)
                    finally:
                        e.close()
                except Exception as ex:
                    errs.append(ex)
                    g.abort()

            th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=600)
            assert not errs, errs
            assert b"".join(p[0] for p in parts) == single, world
    finally:
        d.free()
    # decoded windows (opj_decompress -d) against the source rows
    for (x0, y0) in ((0, 0), (19456, 14336), (38976, 28976)):
        x1, y1 = min(w, x0 + 1024), min(h, y0 + 1024)
        dec = im.decode_opj(single, ".jpx", area=(x0, y0, x1, y1))
        assert dec.shape[:2] == (y1 - y0, x1 - x0)
        assert im.psnr(buf[y0:y1, x0:x1], dec.reshape(y1 - y0, x1 - x0), 16) > 40
