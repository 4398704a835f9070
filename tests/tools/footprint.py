#!/usr/bin/env python3
"""Device memory one context holds after encoding each configuration
(jp2hip_device_bytes; DESIGN.md 3 "Footprint"), on an MI355X:
  C2  6000x4000 RGB8, lossy 3 bpp
  C4  5000x7000 RGB8, lossless (one batch image)
  C3  10000x8000 RGB16, lossless, 1024^2 tiles
  C5  40000x30000 Gray16, 7 levels, lossy 3 bpp (one context, no split)
Each on a fresh context with the soft limit off, so the number is what the
image needs.  Writes one JSON object per line to argv[1] (or stdout)."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "jp2-bucketeer_amd"))
import numpy as np  # noqa: E402

import imaging as im  # noqa: E402
import jp2hip  # noqa: E402

out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
only = sys.argv[2].split(",") if len(sys.argv) > 2 else ["C2", "C4", "C3", "C5"]


def c5_image():
    h, w = 30000, 40000
    img = np.empty((h, w), np.uint16)
    for r in range(0, h, 2048):
        img[r:r + 2048] = im.synth_gray16_rows(r, min(h, r + 2048), w, seed=5, band=512)
    return img


cases = {
    "C2": (lambda: im.synth_rgb8(4000, 6000, seed=1234), jp2hip.LOSSY, {}),
    "C4": (lambda: im.synth_rgb8(7000, 5000, seed=0), jp2hip.LOSSLESS, {}),
    "C3": (lambda: im.synth_u16(8000, 10000, comps=3, seed=2), jp2hip.LOSSLESS, {"tile_w": 1024, "tile_h": 1024}),
    "C5": (c5_image, jp2hip.LOSSY, {"levels": 7}),
}
for name in only:
    make, conv, over = cases[name]
    img = make()
    tif = im.tiff_bytes(img)
    del img
    enc = jp2hip.Encoder(0)
    enc.set_memory_limits(soft=1 << 62)
    t0 = time.time()
    data, st = enc.encode_tiff(tif, conv, jp2hip.recipe(conv, **over))
    rec = {"config": name, "pixels": st.codeblocks and None, "device_bytes": enc.device_bytes(),
           "mp": None, "out_bytes": len(data), "encode_s": round(time.time() - t0, 3)}
    h, w = {"C2": (4000, 6000), "C4": (7000, 5000), "C3": (8000, 10000), "C5": (30000, 40000)}[name]
    rec["mp"] = h * w / 1e6
    rec["bytes_per_px"] = round(rec["device_bytes"] / (h * w), 2)
    rec.pop("pixels")
    print(json.dumps(rec), file=out, flush=True)
    enc.close()
    del tif, data
