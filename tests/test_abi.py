"""The C-ABI boundary (include/jp2hip.h) and the converter API mirror, on CPU.

No compute calls here: only that libjp2hip loads, exports every declared
symbol, parses TIFF headers, exposes the Kakadu recipe, and that the Python
mirror of converters/* behaves like the reference when no GPU / Kakadu exists.
"""
import os
import re

import numpy as np
import pytest

import imaging as im
import jp2hip
from jp2hip import _lib
from jp2hip.converters import (Conversion, ConverterFactory, GpuConverter, KakaduConverter,
                               KakaduNotFoundError, OpenJPEGConverter, _jpx_name)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "jp2hip.h")).read()
    return sorted(set(re.findall(r"\b(jp2hip_[a-z_]+)\s*\(", txt)))


def test_header_declares_what_the_binding_expects():
    assert _declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for sym in _declared_symbols():
        assert hasattr(L, sym), sym


def test_version_and_probe():
    assert "gfx950" in jp2hip.version()
    assert jp2hip.probe() in (True, False)


def test_recipe_is_the_kakadu_recipe():
    # KakaduConverter.java:38-44
    for conv, lossless in ((jp2hip.LOSSLESS, True), (jp2hip.LOSSY, False)):
        r = jp2hip.recipe(conv)
        assert (r.levels, r.layers, r.tile_w, r.tile_h) == (6, 6, 512, 512)
        assert (r.cblk_w_log2, r.cblk_h_log2) == (6, 6)
        assert r.nprecincts == 3 and list(r.prec_w_log2[:3]) == [8, 8, 7]
        assert (r.progression, r.sop, r.eph, r.plt, r.tparts_r) == (2, 1, 1, 1, 1)
        assert r.reversible == (1 if lossless else 0)
        assert r.rate_bpp == (0.0 if lossless else 3.0)
        assert r.format == jp2hip.FORMAT_JPX


def test_recipe_identical_to_oracle_recipe():
    import oracle_lib as ol
    for conv in (jp2hip.LOSSLESS, jp2hip.LOSSY):
        a = jp2hip.recipe(conv)
        b = ol.recipe(conv == jp2hip.LOSSLESS)
        for name, _ in _lib.Recipe._fields_:
            va, vb = getattr(a, name), getattr(b, name)
            if name.startswith("prec_"):
                assert list(va) == list(vb)
            else:
                assert va == vb, name


@pytest.mark.parametrize("kw", [{}, {"planar": True}, {"big_endian": True}, {"rows_per_strip": 3}])
def test_tiff_layout(kw):
    img = im.synth_rgb8(37, 53, seed=1)
    data = im.tiff_bytes(img, **kw)
    lay, offs = jp2hip.tiff_layout(data)
    assert (lay.width, lay.height, lay.components, lay.bits) == (53, 37, 3, 8)
    assert lay.planar == (2 if kw.get("planar") else 1)
    assert lay.big_endian == (1 if kw.get("big_endian") else 0)
    rps = kw.get("rows_per_strip", 64)
    assert lay.rows_per_strip == min(rps, 37)
    # strip 0 holds row 0
    o = offs[0]
    if not kw.get("planar"):
        assert data[o:o + 3] == img[0, 0].tobytes()


def test_tiff_layout_16bit():
    img = im.synth_u16(20, 30, comps=1)
    lay, offs = jp2hip.tiff_layout(im.tiff_bytes(img, big_endian=True))
    assert (lay.bits, lay.components, lay.big_endian) == (16, 1, 1)


@pytest.mark.parametrize("bad,msg", [(b"XX*\0" + b"\0" * 16, "byte-order"),
                                     (b"II+\0" + b"\0" * 16, "BigTIFF"),
                                     (b"II*\0", "short")])
def test_tiff_layout_rejects(bad, msg):
    with pytest.raises(jp2hip.Jp2hipError, match=msg):
        jp2hip.tiff_layout(bad)


def test_tiff_layout_rejects_unsupported_compression():
    data = bytearray(im.tiff_bytes(im.synth_rgb8(8, 8)))
    # Compression tag (259) value -> 7 (JPEG)
    i = data.find(bytes([0x03, 0x01, 0x03, 0x00, 0x01, 0x00, 0x00, 0x00, 0x01, 0x00]))
    assert i > 0
    data[i + 8] = 7
    with pytest.raises(jp2hip.Jp2hipError, match="compression 7"):
        jp2hip.tiff_layout(bytes(data))


def test_tiff_layout_rows_per_strip_zero_is_one_strip():
    """RowsPerStrip = 0 (invalid) reads as one strip, as libtiff does, instead
    of dividing by zero (one bad upload must not kill the JVM)."""
    img = im.synth_rgb8(40, 30, seed=1)
    data = im.tiff_set_tag(im.tiff_bytes(img, rows_per_strip=64), 278, 0)
    lay, offs = jp2hip.tiff_layout(data)
    assert lay.rows_per_strip == 40 and lay.nstrips == 1


def test_tiff_layout_rejects_wrapped_bigtiff_offset():
    """A LONG8 strip offset near 2^64 must not wrap the bounds check."""
    img = im.synth_rgb8(16, 16, seed=2)
    data = im.tiff_set_tag(im.bigtiff_bytes(img, rows_per_strip=16), 273, (1 << 64) - 8)
    with pytest.raises(jp2hip.Jp2hipError, match="out of range"):
        jp2hip.tiff_layout(data)


@pytest.mark.parametrize("photo,nc,msg", [(0, 1, "WhiteIsZero"), (3, 1, "Photometric"), (5, 4, "Photometric"),
                                          (6, 3, "Photometric"), (2, 1, "RGB needs"), (1, 3, "BlackIsZero")])
def test_tiff_layout_rejects_unsupported_photometric(photo, nc, msg):
    """Only BlackIsZero gray (+alpha) and RGB (+alpha) are encoded; palette,
    CMYK, YCbCr and WhiteIsZero fail with a message."""
    img = im.synth_rgb8(8, 8)
    img = img[..., 0].copy() if nc == 1 else (np.dstack([img, img[..., :1]]) if nc == 4 else img)
    data = im.tiff_set_tag(im.tiff_bytes(img), 262, photo)
    with pytest.raises(jp2hip.Jp2hipError, match=msg):
        jp2hip.tiff_layout(data)


@pytest.mark.parametrize("comp,code,pred", [("tiff_lzw", 5, False), ("tiff_lzw", 5, True), ("packbits", 32773, False),
                                            ("tiff_adobe_deflate", 8, False), ("tiff_adobe_deflate", 8, True),
                                            ("tiff_deflate", 32946, False)])
def test_tiff_layout_compressed_strips(comp, code, pred):
    """LZW / Deflate / PackBits strips: offsets, then byte counts, match the file's tags."""
    from PIL import Image
    import io
    img = im.synth_rgb8(70, 90, seed=2)
    data = im.tiff_bytes_compressed(img, comp, predictor=pred, rows_per_strip=16)
    lay, keep = jp2hip.tiff_layout(data)
    tags = Image.open(io.BytesIO(data)).tag_v2
    assert lay.compression == code and lay.predictor == (2 if pred else 1)
    assert lay.rows_per_strip == 16 and lay.nstrips == 5
    assert [lay.strip_offsets[i] for i in range(5)] == list(tags[273])
    assert [lay.strip_bytes[i] for i in range(5)] == list(tags[279])


@pytest.mark.parametrize("big_endian", [False, True])
def test_tiff_layout_bigtiff(big_endian):
    """BigTIFF (version 43, LONG8 offsets) parses to the same layout as the
    classic file of the same pixels, offsets aside."""
    img = im.synth_rgb8(100, 70, seed=4)
    lay, keep = jp2hip.tiff_layout(im.bigtiff_bytes(img, rows_per_strip=16, big_endian=big_endian))
    ref, _ = jp2hip.tiff_layout(im.tiff_bytes(img, rows_per_strip=16, big_endian=big_endian))
    for f in ("width", "height", "components", "bits", "planar", "big_endian", "rows_per_strip", "nstrips"):
        assert getattr(lay, f) == getattr(ref, f), f
    data = im.bigtiff_bytes(img, rows_per_strip=16, big_endian=big_endian)
    row = 70 * 3
    for s in range(lay.nstrips):
        o = lay.strip_offsets[s]
        rows = min(16, 100 - 16 * s)
        got = np.frombuffer(data[o:o + row * rows], np.uint8).reshape(rows, 70, 3)
        assert np.array_equal(got, img[16 * s:16 * s + rows])


@pytest.mark.parametrize("kw", [{}, {"packbits": True}, {"planar": True, "big_endian": True}])
def test_tiff_layout_tiled(kw):
    img = im.synth_rgb8(70, 90, seed=3)
    lay, keep = jp2hip.tiff_layout(im.tiled_tiff_bytes(img, tile=(32, 48), **kw))
    assert (lay.tile_width, lay.tile_height) == (32, 48)
    assert lay.nstrips == 3 * 2 * (3 if kw.get("planar") else 1)
    assert lay.compression == (32773 if kw.get("packbits") else 1)
    unit = 32 * 48 * (1 if kw.get("planar") else 3)
    sizes = [lay.strip_bytes[i] for i in range(lay.nstrips)]
    assert all(n == unit for n in sizes) if not kw.get("packbits") else all(n > unit for n in sizes)


def test_conversion_ordinals_match_reference():
    assert int(Conversion.LOSSY) == 0 and int(Conversion.LOSSLESS) == 1


def test_jpx_name_is_url_encoded():
    # KakaduConverter.java:57 URLEncoder.encode(id, UTF-8) + ".jpx"
    assert _jpx_name("ark:/21198/zz0019pp86") == "ark%3A%2F21198%2Fzz0019pp86.jpx"
    assert _jpx_name("a b") == "a+b.jpx"
    assert _jpx_name("熵") == "%E7%86%B5.jpx"


def test_kakadu_executable_honours_kakadu_home(monkeypatch):
    # KakaduConverterTest.testGetExecutable (KakaduConverterTest.java:77-87)
    monkeypatch.setenv("KAKADU_HOME", "/opt/kakadu")
    assert KakaduConverter.get_executable() == "/opt/kakadu/kdu_compress"
    monkeypatch.delenv("KAKADU_HOME")
    assert KakaduConverter.get_executable() == "kdu_compress"


@pytest.mark.skipif(jp2hip.probe(), reason="factory fallback is only observable without a GPU")
def test_factory_without_gpu_or_kakadu(monkeypatch):
    monkeypatch.delenv("KAKADU_HOME", raising=False)
    ConverterFactory.reset()
    assert isinstance(ConverterFactory.get_converter(), OpenJPEGConverter)
    assert ConverterFactory.get_converter(OpenJPEGConverter).convert("x", "y.tif", Conversion.LOSSLESS) is None
    with pytest.raises(KakaduNotFoundError):
        ConverterFactory.get_converter(KakaduConverter)
    # the GPU branch never raises (ImageWorkerVerticle.java:106 catches only
    # IOException/InterruptedException): without a GPU or Kakadu it hands out
    # a converter whose convert() raises IOError with the BUCKETEER-001 text
    conv = ConverterFactory.get_converter(GpuConverter)
    assert isinstance(conv, GpuConverter) and conv.unavailable
    with pytest.raises(IOError, match="Failed to convert TIFF to JP2: img1"):
        conv.convert("img1", "y.tif", Conversion.LOSSLESS)
    assert jp2hip.device_count() == 0
    assert jp2hip.device_ordinals() == []
    with pytest.raises(ValueError):
        ConverterFactory.get_converter(str)
    ConverterFactory.reset()


@pytest.mark.skipif(jp2hip.probe(), reason="needs a machine without a GPU")
def test_encoder_fails_loudly_without_gpu():
    with pytest.raises(jp2hip.Jp2hipError, match="no HIP device"):
        jp2hip.Encoder(0)


def test_output_view_keeps_the_pinned_buffer_alive(monkeypatch):
    """a view of an Output must outlive the Output (and its
    close()) without the buffer going back to jp2hip's pool under it."""
    import ctypes
    import gc
    freed = []

    class FakeLib:
        def jp2hip_free(self, p):
            freed.append(ctypes.addressof(p.contents))

    monkeypatch.setattr(_lib, "lib", lambda: FakeLib())
    store = (ctypes.c_uint8 * 8)(*b"JP2HIP!!")
    ptr = ctypes.cast(store, ctypes.POINTER(ctypes.c_uint8))
    v = _lib.Output(ptr, 8).view()  # the temporary Output is dropped at once
    gc.collect()
    assert freed == [] and bytes(v) == b"JP2HIP!!"
    del v
    gc.collect()
    assert freed == [ctypes.addressof(store)]
    freed.clear()
    o = _lib.Output(ptr, 8)
    v = o.view()
    o.close()
    gc.collect()
    assert freed == [] and bytes(v[:3]) == b"JP2"
    with pytest.raises(ValueError):
        o.view()
    v.release()
    del v
    gc.collect()
    assert len(freed) == 1
    o2 = _lib.Output(ptr, 8)
    o2.close()
    assert len(freed) == 2


def test_tiff_pixels_reads_only_the_header(tmp_path):
    """jp2hip_tiff_pixels: a converter's routing check (split context for
    oversized images) -- no GPU needed, errors through jp2hip_last_error."""
    img = im.synth_rgb8(37, 53, seed=1)
    p = tmp_path / "熵.tif"
    p.write_bytes(im.tiff_bytes(img))
    assert jp2hip._lib.tiff_pixels(p) == 37 * 53
    bad = tmp_path / "bad.tif"
    bad.write_bytes(b"II*\0garbage")
    with pytest.raises(jp2hip.Jp2hipError):
        jp2hip._lib.tiff_pixels(bad)
    with pytest.raises(jp2hip.Jp2hipError, match="cannot open"):
        jp2hip._lib.tiff_pixels(tmp_path / "missing.tif")


def test_env_check_without_contexts(monkeypatch):
    """jp2hip_env_check reads the process environment at the call and
    compares GPU_MAX_HW_QUEUES with the live contexts: none without a GPU,
    so nothing to advise whatever the variable says (the GPU side:
    test_gpu_api.py::test_env_check_names_too_few_queues)."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")
    assert jp2hip._lib.env_check() == ""


def test_crafted_deflate_writer_matches_zlib():
    """The fixed-Huffman token writer behind the GPU inflate test decodes,
    under zlib, to exactly the bytes it says (every distance 1..70, lengths
    3..258, distances up to 32768)."""
    import zlib
    toks = im.crafted_match_tokens(7)
    assert {t[1] for t in toks if isinstance(t, tuple)} >= set(range(1, 71)) | {32768}
    assert {t[0] for t in toks if isinstance(t, tuple)} >= {3, 4, 5, 257, 258}
    stream, raw = im.deflate_tokens(toks)
    assert zlib.decompress(stream) == raw and len(raw) > 100_000
