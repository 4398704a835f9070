#!/usr/bin/env python3
"""One Deflate C2 TIFF encode (6000x4000 RGB8, 64-row strips) for a
rocprofv3 --pmc pass over k_inflate (measurement tool, not a test)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jp2-bucketeer_amd"))
import imaging as im  # noqa: E402
import jp2hip  # noqa: E402

img = im.synth_rgb8(4000, 6000, seed=1234)
tif = im.tiff_bytes_compressed(img, "tiff_adobe_deflate", rows_per_strip=64)
enc = jp2hip.Encoder(0)
for _ in range(2):
    out, st = enc.encode_tiff(tif, jp2hip.LOSSY)
print(len(out), st.total_ms)
