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



o = np.argsort(-cyc)[:8]
for i in o: print(i, a[i])
print("decisions per block: mean", dec[m].mean(), "p50", np.median(dec[m]), "p99", np.percentile(dec[m], 99))
wt = wall[m] / 100.0  # us
print("per-block wall us: mean", wt.mean(), "p50", np.median(wt), "p99", np.percentile(wt, 99), "max", wt.max())
print("sum decisions / t1_mq_ms => Gdec/s", dec.sum() / (st.t1_mq_ms * 1e-3) / 1e9)
print("stages", st.as_dict())
gi = a[:, 3]
lanes = int(os.environ.get("JP2HIP_MQ_LANES", "64"))
wv = gi[m] // lanes
import collections
print("ns per decision (per block wall/dec): p10 %.1f p50 %.1f p90 %.1f" % tuple(np.percentile(wall[m] * 10.0 / dec[m], [10, 50, 90])))
for q in (0, 1, 2, 10, 100, 300, 1000):
    sel = wv == q
    if sel.any():
        print("wave", q, "dec max", dec[m][sel].max(), "min", dec[m][sel].min(), "wall us max", wall[m][sel].max() / 100.0)
