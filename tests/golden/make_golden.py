#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json (run in the build container).

Sources of truth, none of them part of the product:
  * tests/golden/test.jpx -- byte copy of the reference's only image fixture,
    src/test/resources/images/test.jpx (Kakadu 7.10.6 output of the lossless
    recipe, KakaduConverter.java:38-44).  We record its
    main-header segments, packet/tile-part structure and the SHA-256 of its
    decoded pixels (opj_decompress 2.4.0 and Pillow/OpenJPEG 2.5.4 agree).
  * opj_compress 2.4.0 (/opt/conda/bin) -- the CPU reference encoder that
    north_star names when Kakadu is unlicensed -- run with the Appendix A
    mapping of the recipe, to pin the lossy yardstick: PSNR at a given bpp.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import imaging as im  # noqa: E402

# usage: make_golden.py            -- everything (about 15 minutes)
#        make_golden.py NAME ...   -- only these lossy cases / "c5_full" / "c3_full"

PREC = "[256,256],[256,256],[128,128],[128,128],[128,128],[128,128],[128,128]"


def opj_encode(img: np.ndarray, ratios: str, lossy: bool, levels=6, tile=512) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.tif"), os.path.join(d, "out.j2k")
        with open(src, "wb") as f:
            f.write(im.tiff_bytes(img))
        prec = ",".join(["[256,256]", "[256,256]"] + ["[128,128]"] * (levels - 1))
        cmd = [im.opj("opj_compress"), "-i", src, "-o", dst, "-n", str(levels + 1), "-t", f"{tile},{tile}",
               "-b", "64,64", "-p", "RPCL", "-SOP", "-EPH", "-PLT", "-TP", "R", "-c", prec, "-r", ratios]
        if lossy:
            cmd.insert(1, "-I")
        subprocess.run(cmd, check=True, capture_output=True)
        return open(dst, "rb").read()


def opj_psnr_at(img, bits, target_bytes, levels=6):
    """opj lossy PSNR with the final layer sized to `target_bytes` (same bpp)."""
    raw_bits = img.size * bits
    r = raw_bits / (8.0 * target_bytes)
    ratios = ",".join(f"{r * 2 ** k:.4f}" for k in range(5, -1, -1))
    cs = opj_encode(img, ratios, True, levels)
    dec = im.decode_opj(cs, ".j2k")
    return len(cs), im.psnr(img, dec, bits)


def c5_full_sha(w=40000, h=30000):
    """SHA-256 of the oracle's file for the full C5 image (BASELINE.json
    configs[4]: 40000x30000 Gray16, 7 levels, lossy 3 bpp, JPX), so the GPU
    tile-split encode is compared with the oracle without running it there
    (about 8 minutes and 20 GB of RAM here)."""
    import hashlib
    import oracle_lib as ol
    img = im.synth_gray16_rows(0, h, w)
    cs = ol.encode(img, ol.recipe(False, levels=7))
    return {"name": "c5_gray16_40000x30000_jpx", "oracle_bytes": len(cs),
            "oracle_sha256": hashlib.sha256(cs).hexdigest()}


def c3_full_sha():
    """SHA-256 of the oracle's file for the full C3 image (BASELINE.json
    configs[2]: 10000x8000 RGB16, lossless 5/3, 1024^2 tiles, JPX; the bench
    image, seed 2), so bench.py's lossless_c3 leg checks its output against
    the oracle without running it on the GPU box."""
    import hashlib
    import oracle_lib as ol
    img = im.synth_u16(8000, 10000, comps=3, seed=2)
    cs = ol.encode(img, ol.recipe(True, tile_w=1024, tile_h=1024))
    assert np.array_equal(im.decode_opj(cs), img)
    return {"name": "c3_rgb16_10000x8000_lossless_jpx", "oracle_bytes": len(cs),
            "oracle_sha256": hashlib.sha256(cs).hexdigest()}


def c4_lossless():
    """Lossless at full C4 size (BASELINE.json configs[3]: one 5000x7000 RGB8
    batch image, seed 0, JPX as the batch writes it): the oracle file's
    SHA-256 pins the GPU batch output without running the oracle there."""
    import hashlib
    import oracle_lib as ol
    img = im.synth_rgb8(7000, 5000, seed=0)
    cs = ol.encode(img, ol.recipe(True))
    assert np.array_equal(im.decode_pillow(cs), img)
    return [{"name": "c4_synth_rgb8_5000x7000_seed0_jpx", "oracle_bytes": len(cs),
             "oracle_sha256": hashlib.sha256(cs).hexdigest()}]


def kdu_layer_info(cs):
    """(log2 slope, bytes) per quality layer from a Kdu-Layer-Info COM."""
    p = cs.find(b"Kdu-Layer-Info")
    n = int.from_bytes(cs[p - 4:p - 2], "big")
    lines = cs[p:p + n - 4].decode("latin-1").splitlines()[1:]
    return [[float(x.split(",")[0]), float(x.split(",")[1])] for x in lines]


def main(only=None):
    if only:
        # recompute the named lossy cases / the C5 file / the C4 lossless
        # file / test.jpx's layer info only, keep the rest
        g = json.load(open(os.path.join(HERE, "golden.json")))
        tj = open(os.path.join(HERE, "test.jpx"), "rb").read()
        pix = im.decode_opj(tj, ".j2k")
        if "c5_full" in only:
            g["c5_full"] = c5_full_sha()
            print(g["c5_full"])
        if "c3_full" in only:
            g["c3_full"] = c3_full_sha()
            print(g["c3_full"])
        if "lossless" in only:
            g["lossless"] = c4_lossless()
            print(g["lossless"])
        if "testjpx_layers" in only:
            g["testjpx"]["kdu_layer_info"] = kdu_layer_info(tj)
        g["lossy"] = [c for c in g["lossy"] if c["name"] not in only]
        g["lossy"] += lossy_cases(pix, only)
        with open(os.path.join(HERE, "golden.json"), "w") as f:
            json.dump(g, f, indent=1)
        return
    g = {}
    tj = open(os.path.join(HERE, "test.jpx"), "rb").read()
    pix = im.decode_opj(tj, ".j2k")
    pil = im.decode_pillow(tj)
    assert np.array_equal(pix, pil)
    seg = im.main_header_segments(tj)
    g["testjpx"] = {
        "size": len(tj),
        "shape": list(pix.shape),
        "sha256": im.sha256(pix),
        "siz": seg["ff51"].hex(), "cod": seg["ff52"].hex(), "qcd": seg["ff5c"].hex(),
        "sop": im.count_marker(tj, b"\xff\x91"),
        "tileparts": len(im.tile_parts(tj)),
        # every tile-part: (Isot, TPsot, TNsot), in code-stream order
        "tp_order": [[t[0], t[2], t[3]] for t in im.tile_parts(tj)],
        "min_size_assert": 30000,   # KakaduConverterTest.java:107
        # Kakadu's (log2 slope, code-stream bytes through the layer) per layer
        "kdu_layer_info": kdu_layer_info(tj),
    }
    g["lossy"] = lossy_cases(pix)
    g["lossless"] = c4_lossless()
    print(g["lossless"])
    g["c5_full"] = c5_full_sha()
    g["c3_full"] = c3_full_sha()
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
    print(json.dumps(g["testjpx"], indent=1))


LOSSY_SOURCES = {
    "synth_rgb8_1024x1536": (lambda pix: im.synth_rgb8(1024, 1536, seed=1234), 8, 6),
    "testjpx_rgb_crop_1024": (lambda pix: pix[:1024, :1024, :3].copy(), 8, 6),
    "synth_gray16_1024": (lambda pix: im.synth_u16(1024, 1024, comps=1, seed=5), 16, 7),
    # full-size C2 (BASELINE.json configs[1]) in both SURVEY.md 8(d)
    # content classes; the oracle file's SHA-256 pins the GPU output
    "c2_synth_rgb8_6000x4000": (lambda pix: im.synth_rgb8(4000, 6000, seed=1234), 8, 6),
    "c2_testjpx_tiled_6000x4000": (lambda pix: im.testjpx_tiled(pix), 8, 6),
    # C5's recipe (7 levels, lossy 3 bpp) and content generator on a 4096^2
    # window of the map scan: the Gray16 class's opj +-0.1 dB yardstick
    "c5_gray16_4096x4096": (lambda pix: im.synth_gray16_rows(0, 4096, 4096), 16, 7),
}


def lossy_cases(pix, only=None):
    """Lossy yardsticks: opj at exactly the oracle's output size."""
    import hashlib
    import oracle_lib as ol
    cases = []
    for name, (make, bits, lv) in LOSSY_SOURCES.items():
        if only and name not in only:
            continue
        img = make(pix)
        rc = ol.recipe(False, levels=lv, format=0)
        cs = ol.encode(img, rc)
        dec = im.decode_opj(cs, ".j2k")
        ps = im.psnr(img, dec, bits)
        n_opj, ps_opj = opj_psnr_at(img, bits, len(cs), lv)
        cases.append({"name": name, "bits": bits, "levels": lv, "oracle_bytes": len(cs),
                      "oracle_sha256": hashlib.sha256(cs).hexdigest(),
                      "oracle_psnr": round(ps, 4), "opj_bytes": n_opj, "opj_psnr": round(ps_opj, 4),
                      "bpp": round(8.0 * len(cs) / (img.shape[0] * img.shape[1]), 5)})
        if n_opj < 0.99 * len(cs):
            # every pass fits under the rate and opj's all-pass file is the
            # smaller one: the fair comparison is the oracle at opj's bytes
            # (the same recipe, rate target = opj's file size)
            rc2 = ol.recipe(False, levels=lv, format=0, rate_bpp=8.0 * n_opj / (img.shape[0] * img.shape[1]))
            cs2 = ol.encode(img, rc2)
            cases[-1]["oracle_at_opj_bytes"] = {"bytes": len(cs2),
                                                "psnr": round(im.psnr(img, im.decode_opj(cs2, ".j2k"), bits), 4)}
        print(cases[-1])
    return cases


if __name__ == "__main__":
    main(sys.argv[1:] or None)
