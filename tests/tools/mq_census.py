#!/usr/bin/env python3
"""Per-block MQ census on the GPU (debug): decisions vs shader cycles."""
import os, sys, tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
import imaging as im, jp2hip
img = im.synth_rgb8(4000, 6000, seed=1234)
tif = im.tiff_bytes(img)
enc = jp2hip.Encoder(0, profile=True)
enc.encode_tiff(tif, jp2hip.LOSSY)
d = tempfile.mkdtemp(); os.environ["JP2HIP_DUMP_DIR"] = d
out, st = enc.encode_tiff(tif, jp2hip.LOSSY)
a = np.fromfile(os.path.join(d, "mqdbg.bin"), dtype=np.int64).reshape(-1, 4)
dec, cyc, wall = a[:, 0], a[:, 1], a[:, 2]
m = dec > 0
print("t1_mq_ms", st.t1_mq_ms, "blocks", m.sum(), "dec total", dec.sum(), "max", dec.max())
print("cycles: max", cyc.max(), "wall ticks max", wall.max(), "=> clock GHz", cyc.max() / wall.max() / 10)
r = cyc[m] / dec[m]
print("cycles/decision: median", np.median(r), "p10", np.percentile(r, 10), "p90", np.percentile(r, 90))
o = np.argsort(-cyc)[:8]
for i in o: print(i, a[i])
