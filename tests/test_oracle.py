"""Pin the CPU oracle before trusting it (runs without a GPU).

* the reference's golden artifact test.jpx: our decoder
  path reproduces its pixel hash, and the oracle's lossless encode of those
  pixels reproduces its SIZ/COD/QCD bytes, packet and tile-part structure,
  decodes bit-exact, and passes KakaduConverterTest.java:107 (size > 30000);
* the lossy yardstick: opj_compress at the same bpp (tests/golden/golden.json,
  made by tests/golden/make_golden.py) -- PSNR within 0.1 dB;
* edge cases the reference path meets: ragged tiles, tiny images, 1/2/4
  components, 16-bit, levels 0..7, JP2/JPX wrappers.
"""
import os

import numpy as np
import pytest

import imaging as im
import oracle_lib as ol


def test_golden_decoder_pins_testjpx(testjpx_pixels, golden):
    g = golden["testjpx"]
    assert list(testjpx_pixels.shape) == g["shape"]
    assert im.sha256(testjpx_pixels) == g["sha256"]


def test_testjpx_structure_matches_survey(testjpx_bytes, golden):
    g = golden["testjpx"]
    assert len(testjpx_bytes) == 303886
    assert g["sop"] == 3840 and g["tileparts"] == 112


def test_oracle_lossless_reproduces_testjpx_main_header(testjpx_pixels, golden):
    g = golden["testjpx"]
    cs = ol.encode(testjpx_pixels, ol.recipe(True, format=0))
    seg = im.main_header_segments(cs)
    assert seg["ff51"].hex() == g["siz"]
    assert seg["ff52"].hex() == g["cod"]
    assert seg["ff5c"].hex() == g["qcd"]
    assert im.count_marker(cs, b"\xff\x91") == g["sop"]
    tps = im.tile_parts(cs)
    assert len(tps) == g["tileparts"]
    # ORGtparts=R + -flush_period 1024: Kakadu's order in test.jpx -- tiles
    # 0-7 res 0, tiles 0-7 res 1, ..., res 6, then tiles 8-15 -- with TNsot
    # written only on each tile's last tile-part
    assert [[t[0], t[2], t[3]] for t in tps] == g["tp_order"]
    assert len(cs) > g["min_size_assert"]
    assert abs(len(cs) - g["size"]) / g["size"] < 0.02   # Kakadu: 303,886 B
    assert np.array_equal(im.decode_pillow(cs), testjpx_pixels)


def test_oracle_com_markers_follow_kakadu_layout(testjpx_pixels, testjpx_bytes):
    """test.jpx's main header ends in two COMs: a version string and
    Kdu-Layer-Info (one "%6.1f, %8.1e" line per layer, -192.0 on the lossless
    last layer, bytes through that layer).  The oracle writes the same
    layout (its own version string; slopes in its own units)."""
    def coms(cs):
        seg, p = [], cs.find(b"\xff\x64")
        while cs[p:p + 2] == b"\xff\x64":
            n = int.from_bytes(cs[p + 2:p + 4], "big")
            seg.append(cs[p + 4:p + 2 + n])
            p += 2 + n
        return seg
    ref = coms(testjpx_bytes)
    cs = ol.encode(testjpx_pixels, ol.recipe(True, format=0))
    got = coms(cs)
    assert len(got) == len(ref) == 2
    assert got[0][:2] == ref[0][:2] == b"\x00\x01"
    hdr = b"Kdu-Layer-Info: log_2{Delta-D(squared-error)/Delta-L(bytes)}, L(bytes)\n"
    for seg in (ref[1], got[1]):
        assert seg[:2] == b"\x00\x01" and seg[2:2 + len(hdr)] == hdr
        lines = seg[2 + len(hdr):].decode().splitlines()
        assert len(lines) == 6 and all(len(x) == 16 for x in lines)
        assert lines[-1].startswith("-192.0,")
        nbytes = [float(x.split(",")[1]) for x in lines]
        assert nbytes == sorted(nbytes)
    assert len(got[1]) == len(ref[1])
    last = float(got[1].decode("latin-1").splitlines()[-1].split(",")[1])
    assert abs(last - len(cs)) / len(cs) < 0.05


_KDU_VIEWS = {}


def _kdu_view(testjpx_bytes, layers=None, reduce=None):
    key = (layers, reduce)
    if key not in _KDU_VIEWS:
        _KDU_VIEWS[key] = im.decode_opj(testjpx_bytes, ext=".j2k", layers=layers, reduce=reduce)
    return _KDU_VIEWS[key]


def check_testjpx_views(cs, testjpx_bytes, testjpx_pixels):
    """SURVEY.md 8(f) row 4, what a IIIF image server reads from a lossless
    file (BatchJobStatusHandler.java:161-171 builds its URL): a lossless
    encode of test.jpx's pixels decodes, through OpenJPEG, to

    * test.jpx's own image at every reduced resolution, bit for bit
      (opj_decompress -r 0..6): not fitted, it follows from lossless 5/3
      with the same levels;
    * test.jpx's RGB PSNR within 0.3 dB at every quality layer
      (opj_decompress -l 1..5): the five lossless layer fractions are
      fitted to these five numbers (tests/tools/fit_layers.py), so this is a
      FIT CHECK; layer quality is unpinned for other images;
    * cross-check, not fitted: the first flush stripe's (tiles 0-7) packet
      bytes through layers 1-4 within 8 % of test.jpx's (the bytes
      Kakadu's Kdu-Layer-Info L column projects).
    Returns the per-layer PSNR pairs."""
    for r in range(7):
        assert np.array_equal(im.decode_opj(cs, ext=".j2k", reduce=r), _kdu_view(testjpx_bytes, reduce=r)), r
    pairs = []
    for l in range(1, 6):
        ref = im.psnr(_kdu_view(testjpx_bytes, layers=l)[..., :3], testjpx_pixels[..., :3])
        got = im.psnr(im.decode_opj(cs, ext=".j2k", layers=l)[..., :3], testjpx_pixels[..., :3])
        pairs.append((got, ref))
    assert all(abs(g - r) < 0.3 for g, r in pairs), pairs
    kt = np.cumsum(im.packet_bytes_by_layer(testjpx_bytes, 6, tiles=range(8)))
    ot = np.cumsum(im.packet_bytes_by_layer(cs, 6, tiles=range(8)))
    assert all(abs(ot[l] / kt[l] - 1) < 0.08 for l in range(4)), (ot, kt)
    return pairs


def test_oracle_lossless_layer_views_match_testjpx(testjpx_pixels, testjpx_bytes):
    """Quality layers and reduced resolutions of the oracle's lossless file
    against Kakadu's on the reference fixture (check_testjpx_views)."""
    cs = ol.encode(testjpx_pixels, ol.recipe(True, format=0))
    check_testjpx_views(cs, testjpx_bytes, testjpx_pixels)


def test_kakadu_layer_info_is_a_first_flush_projection(testjpx_bytes, golden):
    """Why round 5's fit to the Kdu-Layer-Info L column missed Kakadu's
    quality: in test.jpx that column (5.1e4, 6.9e4, 8.7e4, 1.1e5, 1.8e5) is
    the first 1024-line flush stripe's packet bytes scaled to the 2000-line
    image (within 6 %), while a decoder of the first l layers reads far more
    (79.8e3 B of packets in layer 1: the second stripe's layers are much
    larger, 54.2e3 B against the first stripe's 25.6e3 B)."""
    ref_l = [b for _, b in golden["testjpx"]["kdu_layer_info"]]
    top = np.cumsum(im.packet_bytes_by_layer(testjpx_bytes, 6, tiles=range(8)))
    allp = np.cumsum(im.packet_bytes_by_layer(testjpx_bytes, 6))
    for l in range(5):
        assert abs(top[l] * 2000 / 1024 / ref_l[l] - 1) < 0.06, (l, top[l], ref_l[l])
        assert allp[l] > 1.05 * ref_l[l]
    assert top[0] == 25633 and allp[0] == 79804


def tile_part_bytes(cs):
    """{(tile, TPsot): tile-part bytes} of a raw code-stream."""
    out, p = {}, cs.find(b"\xff\x90")
    while p >= 0 and cs[p:p + 2] == b"\xff\x90":
        n = int.from_bytes(cs[p + 6:p + 10], "big")
        out[(int.from_bytes(cs[p + 4:p + 6], "big"), cs[p + 10])] = cs[p:p + n]
        p += n
    return out


@pytest.mark.parametrize("flush", [1024, 512, 0])
def test_oracle_lossless_stripes_are_independent(flush):
    """-flush_period incremental flushing (KakaduConverter.java:40): a
    lossless stripe's layers come from its own tier-1 bytes, so changing the
    pixels of one flush stripe leaves every other stripe's tile-parts
    byte-identical (SOT, PLT, packet headers and bodies)."""
    img = im.synth_rgb8(1300, 700, seed=21)
    img2 = img.copy()
    img2[1100:1250, 100:600] ^= 0x5A  # inside tile row 2 (rows 1024..1299)
    rc = ol.recipe(True, format=0, tile_w=256, tile_h=256, flush_period=flush)
    a, b = tile_part_bytes(ol.encode(img, rc)), tile_part_bytes(ol.encode(img2, rc))
    ntx = 3  # 700 / 256
    changed = {t for t in a if a[t] != b[t]}
    assert changed and all(t[0] // ntx >= 4 for t in changed)  # the stripe of tile rows 4..5 only
    if flush == 0:  # a stripe per tile row: tile row 4 alone
        assert {t[0] // ntx for t in changed} == {4}


def test_oracle_ignores_experiment_environment(monkeypatch):
    """the parity oracle reads no environment variable (the
    experiment hooks exist only in the -DORACLE_EXPERIMENTS build)."""
    img = im.synth_rgb8(300, 400, seed=9)
    want = ol.encode(img, ol.recipe(False, format=0))
    monkeypatch.setenv("ORACLE_SKIP_MARGIN", "-40")
    monkeypatch.setenv("ORACLE_LAYER_FRACS", "1,1,1,1,1")
    assert ol.encode(img, ol.recipe(False, format=0)) == want


def _golden_lossy_names():
    import json
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return [c["name"] for c in json.load(f)["lossy"]]


@pytest.mark.parametrize("name", _golden_lossy_names())
def test_oracle_lossy_within_0p1db_of_opj(name, golden, testjpx_pixels):
    """The lossy yardstick (north_star): PSNR within 0.1 dB of opj_compress at
    the same bytes -- 1024-class crops, full-size C2 in both SURVEY.md 8(d)
    content classes (synthetic scan, test.jpx pixels mirror-tiled) and a
    4096^2 window of C5's Gray16 map scan at C5's 7-level recipe."""
    import hashlib
    from conftest import golden_image
    c = [x for x in golden["lossy"] if x["name"] == name][0]
    img = golden_image(c["name"], testjpx_pixels)
    cs = ol.encode(img, ol.recipe(False, levels=c["levels"], format=0))
    assert len(cs) == c["oracle_bytes"]            # deterministic
    assert hashlib.sha256(cs).hexdigest() == c["oracle_sha256"]
    dec = im.decode_opj(cs, ".j2k") if c["bits"] == 16 else im.decode_pillow(cs)
    ps = im.psnr(img, dec, c["bits"])
    assert abs(ps - c["oracle_psnr"]) < 1e-3
    if c["bpp"] > 2.9:  # on the rate target: opj was asked for the same bytes
        assert abs(c["opj_bytes"] - len(cs)) / len(cs) < 0.01
    else:  # every pass fits under 3 bpp: opj's output is no larger than ours
        assert c["opj_bytes"] <= len(cs) * 1.01
    assert ps >= c["opj_psnr"] - 0.1
    if "oracle_at_opj_bytes" in c:
        # opj's all-pass file is >= 1 % smaller than ours: compare at equal
        # bytes too -- the oracle with its rate target set to opj's size
        # (the margin must not be bought with bytes)
        at = c["oracle_at_opj_bytes"]
        assert at["bytes"] <= c["opj_bytes"] and at["psnr"] >= c["opj_psnr"] - 0.1
        if img.shape[0] * img.shape[1] <= 2_000_000:
            rate = 8.0 * c["opj_bytes"] / (img.shape[0] * img.shape[1])
            cs2 = ol.encode(img, ol.recipe(False, levels=c["levels"], format=0, rate_bpp=rate))
            assert len(cs2) == at["bytes"]


def test_oracle_lossy_meets_rate():
    img = im.synth_rgb8(600, 1000, seed=7)
    cs = ol.encode(img, ol.recipe(False, format=0))
    target = int(3.0 * 600 * 1000 / 8)
    assert target * 0.97 <= len(cs) <= target


@pytest.mark.parametrize("shape", [(1, 1, 3), (1, 9, 1), (9, 1, 3), (13, 17, 3), (65, 129, 4),
                                   (200, 513, 2), (517, 700, 3)])
def test_oracle_lossless_roundtrip_shapes(shape):
    h, w, nc = shape
    img = im.synth_rgb8(h, w, seed=h * 31 + w)
    if nc == 1:
        img = img[..., 0].copy()
    elif nc == 2:
        img = np.dstack([img[..., 0], img[..., 1]])
    elif nc == 4:
        img = np.dstack([img, img[..., 2] // 2])
    cs = ol.encode(img, ol.recipe(True, format=0))
    assert np.array_equal(im.decode_opj(cs, ".j2k"), img)


@pytest.mark.parametrize("levels,tile", [(0, 512), (1, 64), (3, 256), (5, 1024), (7, 512)])
def test_oracle_lossless_levels_tiles(levels, tile):
    img = im.synth_rgb8(300, 420, seed=levels)
    cs = ol.encode(img, ol.recipe(True, levels=levels, tile_w=tile, tile_h=tile, format=0))
    assert np.array_equal(im.decode_opj(cs, ".j2k"), img)


def test_oracle_lossless_16bit_rgb_and_gray():
    rgb = im.synth_u16(150, 230, comps=3, seed=3)
    cs = ol.encode(rgb, ol.recipe(True, format=0))
    assert np.array_equal(im.decode_opj(cs, ".j2k"), rgb)
    gray = im.synth_u16(150, 230, comps=1, seed=4)
    cs = ol.encode(gray, ol.recipe(True, levels=7, format=0))
    assert np.array_equal(im.decode_opj(cs, ".j2k"), gray)


@pytest.mark.parametrize("fmt", [1, 2])
def test_oracle_file_wrappers_decode(fmt):
    img = im.synth_rgb8(100, 120, seed=11)
    data = ol.encode(img, ol.recipe(True, format=fmt))
    assert data[4:8] == b"jP  "
    assert data[20:24] == (b"jpx " if fmt == 2 else b"jp2 ")
    assert np.array_equal(im.decode_pillow(data), img)
    assert np.array_equal(im.decode_opj(data, ".jpx"), img)


def test_oracle_tiff_input_matches_pixels():
    img = im.synth_rgb8(70, 90, seed=2)
    r = ol.recipe(True)
    want = ol.encode(img, r)
    for kw in ({}, {"planar": True}, {"big_endian": True}, {"rows_per_strip": 5}):
        assert ol.encode_tiff(im.tiff_bytes(img, **kw), r) == want


def test_oracle_t1_empty_and_single_sample():
    z = np.zeros((64, 64), np.int32)
    b, r, d, P = ol.t1_encode(z, 1, True)
    assert P == 0 and len(r) == 0 and b == b""
    one = z.view(np.uint32).copy()
    one[5, 7] = 1 | (1 << 31)
    b, r, d, P = ol.t1_encode(one.view(np.int32), 3, True)
    assert P == 1 and len(r) == 1 and d[0] > 0 and r[-1] == len(b)


def test_oracle_slope_prediction_skips_planes_not_quality():
    """Slope prediction (rate-driven only): fewer MQ decisions, same rate, no
    PSNR loss against coding every pass (oracle predict_and_code)."""
    img = im.synth_rgb8(512, 1024, seed=11)
    L = ol.lib()
    res = {}
    for skip in (0, 1):
        L.oracle_debug_decisions()
        cs = ol.encode(img, ol.recipe(False, format=0, slope_skip=skip))
        res[skip] = (L.oracle_debug_decisions(), len(cs), im.psnr(img, im.decode_pillow(cs)))
    assert res[1][0] < 0.8 * res[0][0]
    target = int(3.0 * 512 * 1024 / 8)
    assert target * 0.97 <= res[1][1] <= target
    assert res[1][2] >= res[0][2] - 0.02


def test_oracle_slope_prediction_inactive_for_lossless():
    img = im.synth_rgb8(200, 300, seed=3)
    a = ol.encode(img, ol.recipe(True, format=0, slope_skip=1))
    b = ol.encode(img, ol.recipe(True, format=0, slope_skip=0))
    assert a == b


@pytest.mark.parametrize("clear_every", [1, 700, 3000, None])
def test_lzw_fixture_encoder_decodes_in_libtiff(clear_every):
    """The LZW encoder variants the GPU tests feed (imaging.lzw_encode) are
    valid TIFF LZW: Pillow's libtiff decodes them to the source pixels."""
    import io
    from PIL import Image
    img = im.synth_rgb8(150, 200, seed=5)
    data = im.tiff_bytes(img, rows_per_strip=64, compression=5,
                         strip_codec=lambda x: im.lzw_encode(x, clear_every=clear_every))
    assert np.array_equal(np.array(Image.open(io.BytesIO(data))), img)
