"""The oracle over the sweep of tests/sweep_cases.py (CPU only): every case
encodes, the reference decoder (opj_decompress, OpenJPEG 2.4.0) reads the
file back, lossless files decode to the source pixels exactly, and
rate-driven files stay within their byte target.  This is what lets the GPU
sweep (tests/test_gpu_sweep.py) treat the oracle's bytes as the answer."""
import numpy as np
import pytest

import imaging as im
import jp2hip
import oracle_lib as ol
import sweep_cases as sc

CASES = sc.cases()


@pytest.mark.parametrize("case", CASES, ids=[sc.case_id(c) for c in CASES])
def test_oracle_sweep_case_decodes(case):
    img = sc.image(case)
    conv = jp2hip.LOSSLESS if case["lossless"] else jp2hip.LOSSY
    r = case["recipe"]
    cs = ol.encode(img, ol.recipe(case["lossless"], **{k: v for k, v in r.items()}))
    ext = [".j2k", ".jp2", ".jpx"][r["format"]]
    dec = im.decode_opj(cs, ext).reshape(img.shape)
    if case["lossless"] and r["rate_bpp"] <= 0:
        assert np.array_equal(dec, img)
    else:
        target = r["rate_bpp"] * case["h"] * case["w"] / 8
        if target > 20000:  # below that the packet headers alone can exceed it
            assert len(im.codestream(cs)) <= target + 0.5
            assert im.psnr(img, dec, case["bits"]) > 8.0
    assert conv in (jp2hip.LOSSLESS, jp2hip.LOSSY)
