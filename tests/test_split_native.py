"""The tile-split behind Converter.convert (jp2hip_split_peers): no Python
group object, no callback -- jp2hip_encode_file / jp2hip_encode_tiff on a
context with peers split an oversized image across the context and its peers
(threads of the call, exchanges summed on the host) and write one file,
byte-identical to the single-GPU encode.  Reference entry point:
Converter.java:22, reached from ImageWorkerVerticle.java:58-64.  On the
one-GPU box every member sits on device 0."""
import numpy as np
import pytest

import imaging as im
import jp2hip

pytestmark = pytest.mark.gpu


def _file_pair(tmp_path, tif, conv, rc, peers, min_pixels=0, name="x"):
    src = tmp_path / f"{name}.tif"
    src.write_bytes(tif)
    single = jp2hip.Encoder(0)
    split = jp2hip.Encoder(0)
    try:
        split.split_peers(peers, min_pixels)
        a, b = tmp_path / f"{name}_single.jpx", tmp_path / f"{name}_split.jpx"
        single.encode_file(str(src), str(a), conv, rc)
        st = split.encode_file(str(src), str(b), conv, rc)
        return a.read_bytes(), b.read_bytes(), st
    finally:
        single.close()
        split.close()


@pytest.mark.parametrize("conv", [jp2hip.LOSSY, jp2hip.LOSSLESS], ids=["lossy", "lossless"])
def test_encode_file_world2_identical(tmp_path, conv):
    """>= 8 k rows (16 tile rows, the last ragged), world 2, default recipe."""
    img = im.synth_gray16_rows(0, 8300, 1900)
    a, b, st = _file_pair(tmp_path, im.tiff_bytes(img), conv, jp2hip.recipe(conv), [0])
    assert a == b
    assert st.out_bytes == len(b)
    if conv == jp2hip.LOSSLESS:
        assert np.array_equal(im.decode_opj(b).reshape(img.shape), img)


def test_encode_tiff_world3_compressed_master_identical(encoder):
    """encode_tiff (bytes in memory) with two peers on an LZW master whose
    48-row strips band boundaries cut; the min_pixels gate leaves a small
    image on the single-GPU path."""
    img = im.synth_rgb8(2600, 700, seed=31)
    tif = im.tiff_bytes(img, rows_per_strip=48, strip_codec=im.lzw_encode, compression=5)
    rc = jp2hip.recipe(jp2hip.LOSSY, tile_w=256, tile_h=256)
    want, _ = encoder.encode_tiff(im.tiff_bytes(img), jp2hip.LOSSY, rc)
    e = jp2hip.Encoder(0)
    try:
        e.split_peers([0, 0], min_pixels=1_000_000)
        got, st = e.encode_tiff(tif, jp2hip.LOSSY, rc)
        assert got == want
        small = im.synth_rgb8(300, 400, seed=2)
        got_small, st_small = e.encode_tiff(im.tiff_bytes(small), jp2hip.LOSSY, rc)
        assert got_small == encoder.encode_tiff(im.tiff_bytes(small), jp2hip.LOSSY, rc)[0]
        assert st_small.codeblocks < st.codeblocks
    finally:
        e.close()


def test_more_ranks_than_tile_rows(tmp_path):
    """World 4 on an image of two tile rows: ranks 2 and 3 hold nothing but
    still take part in every exchange."""
    img = im.synth_rgb8(900, 500, seed=7)
    a, b, _ = _file_pair(tmp_path, im.tiff_bytes(img, rows_per_strip=37), jp2hip.LOSSLESS,
                         jp2hip.recipe(jp2hip.LOSSLESS, flush_period=0), [0, 0, 0])
    assert a == b
    assert np.array_equal(im.decode_pillow(b), img)


def test_empty_ranks_with_a_compressed_master(tmp_path):
    """world 4 on an LZW master of two tile rows -- two ranks
    decode nothing and still join every exchange; the ragged last strip
    (900 = 18 x 48 + 36 rows) ends the last band."""
    img = im.synth_rgb8(900, 500, seed=17)
    tif = im.tiff_bytes(img, rows_per_strip=48, strip_codec=im.lzw_encode, compression=5)
    a, b, _ = _file_pair(tmp_path, tif, jp2hip.LOSSY, jp2hip.recipe(jp2hip.LOSSY, flush_period=0), [0, 0, 0])
    assert a == b


def test_one_rank_fails_every_rank_fails_no_file(tmp_path):
    """A corrupt strip in the last rank's band: the call fails with that
    rank's error, the others stop at their next exchange, no file is left."""
    img = im.synth_rgb8(1100, 500, seed=9)
    data = bytearray(im.tiff_bytes_compressed(img, "packbits", rows_per_strip=64))
    lay, keep = jp2hip.tiff_layout(bytes(data))
    o, n = lay.strip_offsets[lay.nstrips - 1], lay.strip_bytes[lay.nstrips - 1]
    data[o:o + n] = bytes([0x80]) * n  # PackBits no-ops: the strip decodes short
    src = tmp_path / "bad.tif"
    src.write_bytes(bytes(data))
    out = tmp_path / "bad.jpx"
    e = jp2hip.Encoder(0)
    try:
        e.split_peers([0], 0)
        with pytest.raises(jp2hip.Jp2hipError, match="corrupt"):
            e.encode_file(str(src), str(out), jp2hip.LOSSLESS, jp2hip.recipe(jp2hip.LOSSLESS, tile_w=256, tile_h=256))
        assert not any(p.name.startswith("bad.jpx") for p in tmp_path.iterdir())
        # the context and its peers stay usable
        ok = tmp_path / "ok.tif"
        ok.write_bytes(im.tiff_bytes(img))
        e.encode_file(str(ok), str(tmp_path / "ok.jpx"), jp2hip.LOSSLESS)
        assert np.array_equal(im.decode_pillow((tmp_path / "ok.jpx").read_bytes()), img)
    finally:
        e.close()


def test_gpu_converter_splits_oversized_images(tmp_path):
    """The Python mirror of the Java GpuConverter: a split context over the
    device list, used for images of at least split_min_pixels."""
    from jp2hip.converters import Conversion, GpuConverter
    img = im.synth_gray16_rows(0, 2100, 1300)
    tif = tmp_path / "big.tif"
    tif.write_bytes(im.tiff_bytes(img))
    plain = GpuConverter(devices=[0])
    conv = GpuConverter(devices=[0], split_devices=[0, 0], split_min_pixels=1_000_000)
    try:
        a = plain.convert("ark:/1/a", tif, Conversion.LOSSY).read_bytes()
        b = conv.convert("ark:/1/b", tif, Conversion.LOSSY).read_bytes()
        assert a == b
        assert conv.split_world == 2
    finally:
        plain.close()
        conv.close()
