"""GPU parity sweep: a seeded, randomized set of geometries and recipes
(tests/sweep_cases.py), each encoded by libjp2hip through the C ABI and
byte-compared with the CPU oracle.

Round 3's lesson: twenty hand-picked shapes passed while a 6-byte tier-2
header error showed up on the smoke image (a 300x530 RGB8 lossless encode
with the default recipe).  That image is a named case here, and the sweep
varies every field of the kdu recipe (KakaduConverter.java:38-44) --
levels 0-7, tiles 128-2048 (square and not), code-blocks 16-64 (square and
not), 1-12 layers, precincts, rates 0.5-4 bpp with slope prediction on and
off, flush periods, formats and COM markers -- over 1-4 components, 8/16
bits, ragged edges and content that leaves packets empty in some layers.
"""
import numpy as np
import pytest

import imaging as im
import jp2hip
import oracle_lib as ol
import sweep_cases as sc

pytestmark = pytest.mark.gpu

CASES = sc.cases()


@pytest.mark.parametrize("conv", [jp2hip.LOSSLESS, jp2hip.LOSSY], ids=["lossless", "lossy"])
def test_smoke_image_identical_to_oracle(encoder, conv):
    """__graft_entry__.smoke()'s image and recipe, as a named GPU case."""
    img = im.synth_rgb8(300, 530, seed=3)
    rc = jp2hip.recipe(conv)
    got, _ = encoder.encode_tiff(im.tiff_bytes(img), conv, rc)
    want = ol.encode(img, ol.copy_recipe(rc))
    assert len(got) == len(want)
    assert got == want
    if conv == jp2hip.LOSSLESS:
        assert np.array_equal(im.decode_pillow(got), img)


@pytest.mark.parametrize("case", CASES, ids=[sc.case_id(c) for c in CASES])
def test_sweep_identical_to_oracle(encoder, case):
    img = sc.image(case)
    conv = jp2hip.LOSSLESS if case["lossless"] else jp2hip.LOSSY
    rc = jp2hip.recipe(conv, **case["recipe"])
    got, st = encoder.encode_tiff(im.tiff_bytes(img), conv, rc)
    want = ol.encode(img, ol.copy_recipe(rc))
    if got != want:
        # name the first differing byte and the tile-part it falls in
        n = min(len(got), len(want))
        d = next((i for i in range(n) if got[i] != want[i]), n)
        raise AssertionError(f"{len(got)} vs {len(want)} bytes, first difference at byte {d}")
    if case["lossless"] and case["recipe"]["rate_bpp"] <= 0:
        ext = [".j2k", ".jp2", ".jpx"][case["recipe"]["format"]]
        assert np.array_equal(im.decode_opj(got, ext).reshape(img.shape), img)
