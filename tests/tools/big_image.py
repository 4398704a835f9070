#!/usr/bin/env python3
"""Diagnostic: one C2-recipe image of F x F C2 images (the bench's image tiled)
through ONE context -- every kernel launch F^2 times larger, one stream, no
concurrency between contexts -- against the bench's 16 contexts of C2
images.  Prints device-resident encode MP/s per run.
  python tests/tools/big_image.py [F]"""
import os, sys, time
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "jp2-bucketeer_amd"))
import imaging as im
import jp2hip

F = int(sys.argv[1]) if len(sys.argv) > 1 else 4
img = np.tile(im.synth_rgb8(4000, 6000, seed=1234), (F, F, 1))
tif = im.tiff_bytes(img, rows_per_strip=64)
lay, _ = jp2hip.tiff_layout(tif)
d = torch.frombuffer(bytearray(tif), dtype=torch.uint8).to("cuda:0")
torch.cuda.synchronize()
e = jp2hip.Encoder(0, host_threads=16, profile=True)
rc = jp2hip.recipe(jp2hip.LOSSY)
mp = img.shape[0] * img.shape[1] / 1e6
for i in range(4):
    t = time.perf_counter()
    out, st = e.encode_device(d.data_ptr(), d.numel(), lay, jp2hip.LOSSY, rc, copy=False)
    dt = time.perf_counter() - t
    n = len(out.view())
    out.close()
    s = st.as_dict()
    print(f"F={F} {mp:.0f} MP run {i}: {dt*1e3:.1f} ms  {mp/dt:.0f} MP/s  bytes {n}  "
          + " ".join(f"{k}={v:.2f}" for k, v in s.items() if k.endswith("_ms")), flush=True)
e.close()
