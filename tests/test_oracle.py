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
    # ORGtparts=R: 7 tile-parts per tile, TPsot = resolution
    assert [t[2] for t in tps[:7]] == list(range(7))
    assert len(cs) > g["min_size_assert"]
    assert abs(len(cs) - g["size"]) / g["size"] < 0.02   # Kakadu: 303,886 B
    assert np.array_equal(im.decode_pillow(cs), testjpx_pixels)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_oracle_lossy_within_0p1db_of_opj(case, golden, testjpx_pixels):
    c = golden["lossy"][case]
    if c["name"].startswith("synth_rgb8"):
        img = im.synth_rgb8(1024, 1536, seed=1234)
    elif c["name"].startswith("testjpx"):
        img = testjpx_pixels[:1024, :1024, :3].copy()
    else:
        img = im.synth_u16(1024, 1024, comps=1, seed=5)
    cs = ol.encode(img, ol.recipe(False, levels=c["levels"], format=0))
    assert len(cs) == c["oracle_bytes"]            # deterministic
    dec = im.decode_opj(cs, ".j2k") if c["bits"] == 16 else im.decode_pillow(cs)
    ps = im.psnr(img, dec, c["bits"])
    assert abs(ps - c["oracle_psnr"]) < 1e-3
    assert abs(c["opj_bytes"] - len(cs)) / len(cs) < 0.01
    assert ps >= c["opj_psnr"] - 0.1


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
