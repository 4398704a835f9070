"""GPU parity: libjp2hip (through the C ABI) against the CPU oracle.

Bit-exact is the bar for both conversions: the integer path (5/3, RCT, tier-1,
tier-2) is deterministic, and the 9/7 / ICT path is computed in fp32 with the
oracle's operation order and no FMA contraction, so the whole code-stream must
match byte for byte.  Lossless output must also decode (OpenJPEG) to the
source pixels; lossy quality is pinned through the oracle's opj yardstick
(tests/golden/golden.json).
"""
import os
import threading

import numpy as np
import pytest

import imaging as im
import jp2hip
import oracle_lib as ol

pytestmark = pytest.mark.gpu


def _img(h, w, nc, bits, seed):
    if bits == 16:
        return im.synth_u16(h, w, comps=nc, seed=seed)
    a = im.synth_rgb8(h, w, seed=seed)
    if nc == 1:
        return a[..., 0].copy()
    if nc == 2:
        return np.dstack([a[..., 0], a[..., 2]])
    if nc == 4:
        return np.dstack([a, (a[..., 1] // 3 + 40).astype(np.uint8)])
    return a


CASES = [
    # h, w, nc, bits, lossless, levels, tile
    (200, 300, 3, 8, True, 6, 512),
    (200, 300, 3, 8, False, 6, 512),
    (1, 1, 3, 8, True, 6, 512),
    (3, 130, 1, 8, False, 6, 512),
    (130, 3, 1, 8, True, 6, 512),
    (517, 1030, 3, 8, True, 6, 512),
    (517, 1030, 3, 8, False, 6, 512),
    (300, 260, 4, 8, True, 6, 512),
    (300, 260, 4, 8, False, 6, 512),
    (257, 333, 2, 8, True, 5, 256),
    (700, 900, 3, 16, True, 6, 1024),
    (700, 900, 3, 16, False, 6, 512),
    (600, 777, 1, 16, False, 7, 512),
    (600, 777, 1, 16, True, 7, 512),
    (150, 250, 3, 8, True, 0, 512),
    (450, 350, 3, 8, False, 2, 128),
    # tiles wider than 1024: DWT level 1 by the windowed kernel (k_dwt_l1, one
    # component fits its LDS) or per component (k_dwt_band<INGEST>)
    (520, 2100, 1, 8, False, 6, 2048),
    (300, 2100, 1, 16, True, 6, 2048),
    (520, 2100, 3, 8, True, 6, 2048),
    (520, 2100, 3, 8, False, 6, 2048),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}_{c[3]}b_{'ll' if c[4] else 'ly'}_L{c[5]}_T{c[6]}"
                                             for c in CASES])
def test_codestream_identical_to_oracle(encoder, case):
    h, w, nc, bits, lossless, levels, tile = case
    img = _img(h, w, nc, bits, seed=h * 7 + w)
    conv = jp2hip.LOSSLESS if lossless else jp2hip.LOSSY
    rc = jp2hip.recipe(conv, levels=levels, tile_w=tile, tile_h=tile)
    got, st = encoder.encode_tiff(im.tiff_bytes(img), conv, rc)
    want = ol.encode(img, ol.copy_recipe(rc))
    assert got == want
    if lossless:
        assert np.array_equal(im.decode_opj(got), img)


def test_testjpx_pixels_lossless(encoder, testjpx_pixels, testjpx_bytes, golden):
    """C1: the reference fixture's pixels through the GPU converter path."""
    rc = jp2hip.recipe(jp2hip.LOSSLESS, format=jp2hip.FORMAT_J2K)
    got, st = encoder.encode_tiff(im.tiff_bytes(testjpx_pixels), jp2hip.LOSSLESS, rc)
    assert got == ol.encode(testjpx_pixels, ol.copy_recipe(rc))
    g = golden["testjpx"]
    seg = im.main_header_segments(got)
    assert (seg["ff51"].hex(), seg["ff52"].hex(), seg["ff5c"].hex()) == (g["siz"], g["cod"], g["qcd"])
    assert im.count_marker(got, b"\xff\x91") == g["sop"]
    assert len(im.tile_parts(got)) == g["tileparts"]
    # Kakadu's -flush_period 1024 tile-part order and TNsot, as in test.jpx
    assert [[t[0], t[2], t[3]] for t in im.tile_parts(got)] == g["tp_order"]
    assert np.array_equal(im.decode_pillow(got), testjpx_pixels)
    assert len(got) > g["min_size_assert"]
    # the views a IIIF server reads: every reduced
    # resolution equals test.jpx's decode bit for bit, every quality layer
    # within 0.3 dB of test.jpx's PSNR (test_oracle.check_testjpx_views)
    from test_oracle import check_testjpx_views
    check_testjpx_views(got, testjpx_bytes, testjpx_pixels)


def _golden_lossy_names():
    import json
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return [c["name"] for c in json.load(f)["lossy"]]


@pytest.mark.parametrize("name", _golden_lossy_names())
def test_golden_lossy_cases(encoder, golden, testjpx_pixels, name):
    """Every lossy golden case (1024-class crops, full-size C2 in both
    content classes, a 4096^2 window of C5's Gray16 map scan at C5's
    7-level recipe): the GPU file's SHA-256 is the oracle file's (committed
    by tests/golden/make_golden.py), and its PSNR is within 0.1 dB of
    opj_compress at the same bytes."""
    import hashlib
    from conftest import golden_image
    c = [x for x in golden["lossy"] if x["name"] == name][0]
    img = golden_image(c["name"], testjpx_pixels)
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=c["levels"], format=jp2hip.FORMAT_J2K)
    got, st = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSY, rc)
    assert len(got) == c["oracle_bytes"]
    assert hashlib.sha256(got).hexdigest() == c["oracle_sha256"]
    dec = im.decode_opj(got, ".j2k") if c["bits"] == 16 else im.decode_pillow(got)
    ps = im.psnr(img, dec, c["bits"])
    assert abs(ps - c["oracle_psnr"]) < 1e-3
    assert ps >= c["opj_psnr"] - 0.1


@pytest.mark.parametrize("levels", [6, 0])
@pytest.mark.parametrize("rate", [3.0, 0.0])
def test_fine_quantiser_32bit_index_plane(encoder, levels, rate):
    """An irreversible step fine enough that some band needs more than 15
    magnitude bit-planes: the DWT (or, with no decomposition, the ingest)
    writes 32-bit quantisation indices instead of 16-bit ones (QuantTab::q16,
    csrc/plan.cpp quant_tab) -- byte-identical to the oracle either way, rate
    driven or not."""
    img = _img(260, 390, 3, 8, seed=17)
    rc = jp2hip.recipe(jp2hip.LOSSY, qstep=1.0 / 65536, levels=levels, rate_bpp=rate)
    got, st = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSY, rc)
    assert got == ol.encode(img, ol.copy_recipe(rc))


@pytest.mark.parametrize("cblk", [4, 5])
@pytest.mark.parametrize("lossless", [True, False])
def test_small_codeblocks_identical_to_oracle(encoder, cblk, lossless):
    """Cblk={16,16} / {32,32}: precincts of up to 192 / 48 code-blocks -- tier-2's
    serial per-precinct kernel (k_t2_code + k_apply, more than 64 blocks) and
    the wave-per-precinct one (k_t2_wave) -- byte-identical to the oracle."""
    img = _img(300, 420, 3, 8, seed=5)
    conv = jp2hip.LOSSLESS if lossless else jp2hip.LOSSY
    rc = jp2hip.recipe(conv, cblk_w_log2=cblk, cblk_h_log2=cblk)
    got, st = encoder.encode_tiff(im.tiff_bytes(img), conv, rc)
    assert got == ol.encode(img, ol.copy_recipe(rc))
    if lossless:
        assert np.array_equal(im.decode_pillow(got), img)


@pytest.mark.parametrize("rate", [3.0, 1.0])
def test_slope_prediction_on_off_both_identical_to_oracle(encoder, rate):
    """Slope prediction (recipe.slope_skip, default on for rate-driven
    encodes) codes fewer bit-planes; with it on or off the GPU output equals
    the oracle's, and the rate is met either way."""
    img = _img(517, 1030, 3, 8, seed=41)
    tif = im.tiff_bytes(img)
    mq = {}
    for skip in (0, 1):
        rc = jp2hip.recipe(jp2hip.LOSSY, rate_bpp=rate, slope_skip=skip)
        got, st = encoder.encode_tiff(tif, jp2hip.LOSSY, rc)
        assert got == ol.encode(img, ol.copy_recipe(rc)), skip
        assert len(im.codestream(got)) <= rate * 517 * 1030 / 8
        mq[skip] = st.t1_bytes
    assert mq[1] < 0.8 * mq[0]


def test_c2_full_size_jpx_on_rate(encoder, golden):
    """C2 at full size with the default recipe (JPX file): on the 3 bpp target
    and, inside the JPX boxes, the oracle's code-stream (golden SHA-256)."""
    import hashlib
    img = im.synth_rgb8(4000, 6000, seed=1234)
    rc = jp2hip.recipe(jp2hip.LOSSY)
    got, st = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSY, rc)
    cs = im.codestream(got)
    assert 0.97 * 3.0 * 6000 * 4000 / 8 <= len(cs) <= 3.0 * 6000 * 4000 / 8
    c = [x for x in golden["lossy"] if x["name"] == "c2_synth_rgb8_6000x4000"][0]
    assert hashlib.sha256(cs).hexdigest() == c["oracle_sha256"]
    # the rate loop runs on the device: one wait for the final size, one for
    # the bytes (a third batch of rate iterations would add one)
    assert st.host_waits <= 2, st.host_waits


def test_c3_full_size_lossless_roundtrip(encoder, golden):
    """C3 at full size: 10000x8000 RGB16 lossless, 1024^2 tiles -> decode
    exact, and the file equals the oracle's (SHA-256 committed by
    tests/golden/make_golden.py c3_full)."""
    import hashlib
    img = im.synth_u16(8000, 10000, comps=3, seed=2)
    rc = jp2hip.recipe(jp2hip.LOSSLESS, tile_w=1024, tile_h=1024)
    got, st = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSLESS, rc)
    assert hashlib.sha256(got).hexdigest() == golden["c3_full"]["oracle_sha256"]
    assert np.array_equal(im.decode_opj(got), img)
    assert st.host_waits <= 2, st.host_waits


def test_deterministic_and_reusable_context(encoder):
    img = _img(333, 444, 3, 8, seed=9)
    tif = im.tiff_bytes(img)
    a, _ = encoder.encode_tiff(tif, jp2hip.LOSSY)
    big = im.tiff_bytes(_img(900, 1300, 3, 8, seed=10))
    encoder.encode_tiff(big, jp2hip.LOSSLESS)
    b, _ = encoder.encode_tiff(tif, jp2hip.LOSSY)
    assert a == b


def test_tiff_variants_same_output(encoder):
    img = _img(190, 270, 3, 8, seed=4)
    ref, _ = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSLESS)
    for kw in ({"planar": True}, {"big_endian": True}, {"rows_per_strip": 1}, {"rows_per_strip": 190}):
        got, _ = encoder.encode_tiff(im.tiff_bytes(img, **kw), jp2hip.LOSSLESS)
        assert got == ref, kw
    g16 = _img(190, 270, 1, 16, seed=5)
    a, _ = encoder.encode_tiff(im.tiff_bytes(g16), jp2hip.LOSSLESS)
    b, _ = encoder.encode_tiff(im.tiff_bytes(g16, big_endian=True), jp2hip.LOSSLESS)
    assert a == b


@pytest.mark.parametrize("comp,pred,kind", [("tiff_lzw", False, "rgb8"), ("tiff_lzw", True, "rgb8"),
                                            ("packbits", False, "rgb8"), ("tiff_lzw", True, "gray16"),
                                            ("packbits", False, "gray16"), ("tiff_adobe_deflate", False, "rgb8"),
                                            ("tiff_adobe_deflate", True, "gray16"), ("tiff_deflate", True, "rgb8")])
def test_compressed_strips_same_output(encoder, comp, pred, kind):
    """LZW / Deflate / PackBits (+ Predictor 2) strips decoded on the GPU: the file equals
    the encode of the same pixels from an uncompressed TIFF (and the oracle)."""
    img = im.synth_rgb8(301, 517, seed=9) if kind == "rgb8" else im.synth_u16(301, 517, comps=1, seed=9)
    for conv in (jp2hip.LOSSLESS, jp2hip.LOSSY):
        rc = jp2hip.recipe(conv)
        plain, _ = encoder.encode_tiff(im.tiff_bytes(img), conv, rc)
        got, _ = encoder.encode_tiff(im.tiff_bytes_compressed(img, comp, predictor=pred, rows_per_strip=24), conv, rc)
        assert got == plain
    assert plain == ol.encode(img, ol.copy_recipe(rc))


def test_bigtiff_same_output(encoder):
    img = im.synth_u16(230, 410, comps=3, seed=6)
    for conv in (jp2hip.LOSSLESS, jp2hip.LOSSY):
        a, _ = encoder.encode_tiff(im.tiff_bytes(img, rows_per_strip=32), conv)
        b, _ = encoder.encode_tiff(im.bigtiff_bytes(img, rows_per_strip=32, big_endian=True), conv)
        assert a == b


@pytest.mark.parametrize("kw,kind", [({}, "rgb8"), ({"packbits": True}, "rgb8"),
                                     ({"planar": True, "big_endian": True}, "rgb16"),
                                     ({"packbits": True, "big_endian": True}, "gray16"),
                                     ({"deflate": True}, "rgb8"), ({"deflate": True, "planar": True}, "rgb16")])
def test_tiled_tiff_same_output(encoder, kw, kind):
    """Tiled TIFFs (edge tiles padded) are untiled in HBM: same file as the
    strip TIFF of the same pixels."""
    if kind == "rgb8":
        img = im.synth_rgb8(301, 517, seed=5)
    else:
        img = im.synth_u16(301, 517, comps=3 if kind == "rgb16" else 1, seed=5)
    for conv in (jp2hip.LOSSLESS, jp2hip.LOSSY):
        a, _ = encoder.encode_tiff(im.tiff_bytes(img), conv)
        b, _ = encoder.encode_tiff(im.tiled_tiff_bytes(img, tile=(64, 48), **kw), conv)
        assert a == b


def test_corrupt_compressed_strip_fails_loudly(encoder):
    img = im.synth_rgb8(64, 64, seed=1)
    data = bytearray(im.tiff_bytes_compressed(img, "packbits", rows_per_strip=64))
    lay, keep = jp2hip.tiff_layout(bytes(data))
    o, n = lay.strip_offsets[0], lay.strip_bytes[0]
    data[o:o + n] = bytes([0x80]) * n  # PackBits no-ops only: the strip decodes short
    with pytest.raises(jp2hip.Jp2hipError, match="corrupt"):
        encoder.encode_tiff(bytes(data), jp2hip.LOSSLESS)


def test_corrupt_lzw_strip_fails_loudly(encoder):
    """An LZW strip whose first code (511) is past the table end fails."""
    img = im.synth_rgb8(64, 64, seed=1)
    data = bytearray(im.tiff_bytes_compressed(img, "tiff_lzw", rows_per_strip=32))
    lay, keep = jp2hip.tiff_layout(bytes(data))
    o, n = lay.strip_offsets[1], lay.strip_bytes[1]
    data[o:o + n] = b"\xff" * n
    with pytest.raises(jp2hip.Jp2hipError, match="corrupt"):
        encoder.encode_tiff(bytes(data), jp2hip.LOSSLESS)


@pytest.mark.parametrize("damage", ["header", "truncate", "bad_block"])
def test_corrupt_deflate_strip_fails_loudly(encoder, damage):
    """A bad zlib header, a strip whose byte count is cut to half its stream
    (the data runs out before the strip is full), or a reserved block type (3)
    all report a corrupt strip instead of encoding garbage."""
    from devmem import DeviceBytes
    img = im.synth_rgb8(64, 64, seed=1)
    data = bytearray(im.tiff_bytes_compressed(img, "tiff_adobe_deflate", rows_per_strip=32))
    lay, keep = jp2hip.tiff_layout(bytes(data))
    o, n = lay.strip_offsets[1], lay.strip_bytes[1]
    if damage == "truncate":
        keep[lay.nstrips + 1] = n // 2  # StripByteCounts[1] halved
        d = DeviceBytes(bytes(data))
        try:
            with pytest.raises(jp2hip.Jp2hipError, match="corrupt"):
                encoder.encode_device(d.ptr, d.nbytes, lay, jp2hip.LOSSLESS)
        finally:
            d.free()
        return
    if damage == "header":
        data[o] = 0x79  # CM 9: not Deflate
    else:
        data[o + 2] = 0x07  # BFINAL 1, BTYPE 3
    with pytest.raises(jp2hip.Jp2hipError, match="corrupt"):
        encoder.encode_tiff(bytes(data), jp2hip.LOSSLESS)


def test_corrupt_deflate_first_decode_of_fresh_context():
    """a corrupt Deflate strip as the FIRST Deflate decode of a new
    context (its link buffer fresh from hipMalloc, never holding valid links)
    fails as corrupt -- k_inflate fills the strip's unwritten links and
    k_inflate_links follows only backward links -- and the context then
    encodes a good Deflate TIFF normally."""
    img = im.synth_rgb8(64, 64, seed=1)
    good = im.tiff_bytes_compressed(img, "tiff_adobe_deflate", rows_per_strip=32)
    data = bytearray(good)
    lay, keep = jp2hip.tiff_layout(bytes(data))
    data[lay.strip_offsets[1] + 2] = 0x07  # BFINAL 1, BTYPE 3 (reserved)
    enc = jp2hip.Encoder(0)
    try:
        with pytest.raises(jp2hip.Jp2hipError, match="corrupt"):
            enc.encode_tiff(bytes(data), jp2hip.LOSSLESS)
        got, _ = enc.encode_tiff(good, jp2hip.LOSSLESS)
        assert got == ol.encode(img, ol.copy_recipe(jp2hip.recipe(jp2hip.LOSSLESS)))
    finally:
        enc.close()


def test_inflate_every_match_distance_and_length(encoder):
    """the lane-strided match copies (dist >= 64 rounds and the
    overlapping dist < 64 pattern) and the window flushes, on crafted
    streams -- two strips, each one fixed-Huffman block coding every match
    distance 1..70 at lengths 3..258 plus long distances up to 32768
    (imaging.crafted_match_tokens) -- against the same pixels uncompressed
    (the writer itself is pinned to zlib.decompress in test_abi)."""
    w = 311
    toks = [im.crafted_match_tokens(seed) for seed in (7, 8)]
    rows = max(-(-len(im.deflate_tokens(t)[1]) // w) for t in toks)
    strips, raws = [], []
    for t in toks:
        n = len(im.deflate_tokens(t)[1])
        st, raw = im.deflate_tokens(t + [(11 * k) & 0xFF for k in range(rows * w - n)])
        strips.append(st)
        raws.append(raw)
    img = np.frombuffer(b"".join(raws), np.uint8).reshape(2 * rows, w).copy()
    it = iter(strips)
    data = im.tiff_bytes(img, rows_per_strip=rows, strip_codec=lambda raw: next(it), compression=8)
    got, _ = encoder.encode_tiff(data, jp2hip.LOSSLESS)
    want, _ = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSLESS)
    assert got == want


@pytest.mark.parametrize("comp", ["tiff_lzw", "tiff_adobe_deflate", "packbits"])
def test_compressed_strip_longer_than_needed_is_cut(encoder, comp):
    """A last strip that decodes to more rows than ImageLength leaves is cut
    at the image's end, as libtiff does, not rejected."""
    img = im.synth_rgb8(107, 90, seed=3)
    data = im.tiff_set_tag(im.tiff_bytes_compressed(img, comp, rows_per_strip=16), 257, 101)
    got, _ = encoder.encode_tiff(data, jp2hip.LOSSLESS)
    want, _ = encoder.encode_tiff(im.tiff_bytes(img[:101].copy()), jp2hip.LOSSLESS)
    assert got == want


@pytest.mark.parametrize("clear_every", [700, 3000, 1])
def test_lzw_encoder_variants_same_output(encoder, clear_every):
    """LZW strips from an encoder that clears early (every 700 / 3000 codes:
    more, shorter segments) or after every code (more segments than the
    segment tables hold: the serial decoder takes the strip) decode to the
    same pixels as libtiff's strips (tests/imaging.py lzw_encode)."""
    img = im.synth_rgb8(300, 400, seed=11)
    data = im.tiff_bytes(img, rows_per_strip=64, compression=5,
                         strip_codec=lambda x: im.lzw_encode(x, clear_every=clear_every))
    got, _ = encoder.encode_tiff(data, jp2hip.LOSSY)
    want, _ = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSY)
    assert got == want


def test_old_style_lzw_rejected_by_name(encoder):
    img = im.synth_rgb8(32, 32, seed=1)
    data = bytearray(im.tiff_bytes_compressed(img, "tiff_lzw", rows_per_strip=32))
    lay, keep = jp2hip.tiff_layout(bytes(data))
    o = lay.strip_offsets[0]
    data[o:o + 2] = b"\x00\x01"  # LSB-first clear code: pre-TIFF 6.0 LZW
    with pytest.raises(jp2hip.Jp2hipError, match="old-style"):
        encoder.encode_tiff(bytes(data), jp2hip.LOSSLESS)


def test_device_layout_outside_source_fails_before_any_kernel(encoder):
    """jp2hip_encode_device checks a caller's strip table against src_len
    (ADVICE r1): an offset past the buffer is an error, not a GPU fault."""
    from devmem import DeviceBytes
    img = im.synth_rgb8(64, 64, seed=2)
    tif = im.tiff_bytes(img, rows_per_strip=16)
    lay, keep = jp2hip.tiff_layout(tif)
    d = DeviceBytes(tif)
    try:
        keep[3] = len(tif) - 10  # last strip runs past the end
        with pytest.raises(jp2hip.Jp2hipError, match="outside the source buffer"):
            encoder.encode_device(d.ptr, d.nbytes, lay, jp2hip.LOSSLESS)
        keep[3] = (1 << 64) - 64  # wraps when added to the strip size
        with pytest.raises(jp2hip.Jp2hipError, match="outside the source buffer"):
            encoder.encode_device(d.ptr, d.nbytes, lay, jp2hip.LOSSLESS)
    finally:
        d.free()


def test_encode_file_atomic(encoder, tmp_path):
    img = _img(120, 160, 3, 8, seed=6)
    src = tmp_path / "in.tif"
    src.write_bytes(im.tiff_bytes(img))
    out = tmp_path / "out.jpx"
    encoder.encode_file(str(src), str(out), jp2hip.LOSSLESS)
    assert np.array_equal(im.decode_pillow(out.read_bytes()), img)
    bad = tmp_path / "bad.tif"
    bad.write_bytes(b"II*\0garbage")
    out2 = tmp_path / "never.jpx"
    with pytest.raises(jp2hip.Jp2hipError):
        encoder.encode_file(str(bad), str(out2), jp2hip.LOSSLESS)
    assert not out2.exists()
    assert not any(p.name.startswith("never.jpx") for p in tmp_path.iterdir())


def test_gpu_converter_like_kakadu_converter_test(tmp_path, testjpx_pixels):
    """Mirror of KakaduConverterTest.testConvert (KakaduConverterTest.java:96-115)."""
    from jp2hip.converters import Conversion, ConverterFactory, GpuConverter
    tif = tmp_path / "test.tif"
    tif.write_bytes(im.tiff_bytes(testjpx_pixels))
    conv = ConverterFactory.get_converter(GpuConverter)
    for image_id in ("ark:/21198/zz0019pp86", "熵"):
        jpx = conv.convert(image_id, tif, Conversion.LOSSLESS)
        assert jpx.exists() and jpx.name.endswith(".jpx")
        assert jpx.stat().st_size > 30000
        assert np.array_equal(im.decode_pillow(jpx.read_bytes()), testjpx_pixels)
        jpx.unlink()
    with pytest.raises(IOError, match="Failed to convert TIFF to JP2"):
        conv.convert("missing", tmp_path / "nope.tif", Conversion.LOSSY)
    ConverterFactory.reset()


def test_unicode_tiff_path(tmp_path, testjpx_pixels):
    """ImageUploadKakaduIT converts /images/熵.tif (ImageUploadKakaduIT.java:69):
    a non-ASCII TIFF path through GpuConverter.convert and, below it, the C
    ABI's jp2hip_encode_file (UTF-8 path bytes, both directions)."""
    from jp2hip.converters import Conversion, ConverterFactory, GpuConverter
    d = tmp_path / "图像"
    d.mkdir()
    tif = d / "熵.tif"
    tif.write_bytes(im.tiff_bytes(testjpx_pixels))
    conv = ConverterFactory.get_converter(GpuConverter)
    jpx = conv.convert("熵", tif, Conversion.LOSSLESS)
    assert jpx.exists() and jpx.stat().st_size > 30000
    assert np.array_equal(im.decode_pillow(jpx.read_bytes()), testjpx_pixels)
    jpx.unlink()
    ConverterFactory.reset()
    enc = jp2hip.Encoder(0)
    try:
        out = d / "熵.jpx"
        enc.encode_file(str(tif), str(out), jp2hip.LOSSLESS)
        assert np.array_equal(im.decode_pillow(out.read_bytes()), testjpx_pixels)
        with pytest.raises(jp2hip.Jp2hipError, match="cannot open TIFF"):
            enc.encode_file(str(d / "熵-missing.tif"), str(d / "x.jpx"), jp2hip.LOSSLESS)
    finally:
        enc.close()


def test_concurrent_callers(tmp_path):
    from jp2hip.converters import Conversion, GpuConverter
    conv = GpuConverter(devices=[0, 0])
    imgs = [_img(200 + 37 * i, 300, 3, 8, seed=i) for i in range(4)]
    paths = []
    for i, a in enumerate(imgs):
        p = tmp_path / f"in{i}.tif"
        p.write_bytes(im.tiff_bytes(a))
        paths.append(p)
    results = {}

    def work(i):
        results[i] = conv.convert(f"id{i}", paths[i], Conversion.LOSSLESS).read_bytes()

    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i, a in enumerate(imgs):
        assert np.array_equal(im.decode_pillow(results[i]), a)
    conv.close()


def test_concurrent_contexts_stay_byte_identical():
    """Round 5's one unexplained mismatch was a batch-queue
    file whose code-stream length differed while three contexts encoded at
    once.  Guard against any state shared between contexts: four contexts
    encode eight different images (both conversions, ragged sizes, two flush
    stripes) in parallel threads, three rounds in shuffled orders, and every
    file must equal the oracle's."""
    import random
    cases = []
    for i in range(8):
        img = im.synth_rgb8(300 + 97 * i, 420 - 23 * i + (700 if i % 3 == 0 else 0), seed=500 + i)
        conv = jp2hip.LOSSLESS if i % 2 == 0 else jp2hip.LOSSY
        rc = jp2hip.recipe(conv)
        cases.append((im.tiff_bytes(img, rows_per_strip=16 + i), conv, rc, ol.encode(img, ol.copy_recipe(rc))))
    encs = [jp2hip.Encoder(0) for _ in range(4)]
    errors = []
    try:
        for rnd in range(3):
            order = list(range(len(cases)))
            random.Random(rnd).shuffle(order)

            def work(k):
                try:
                    for j in order[k::4]:
                        tif, conv, rc, want = cases[j]
                        got, _ = encs[k].encode_tiff(tif, conv, rc)
                        if got != want:
                            errors.append((rnd, j, len(got), len(want)))
                except Exception as e:  # noqa: BLE001 -- reported below
                    errors.append(repr(e))
            th = [threading.Thread(target=work, args=(k,)) for k in range(4)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        assert errors == []
    finally:
        for e in encs:
            e.close()
