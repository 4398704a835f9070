#!/usr/bin/env python3
"""Lossless C3 (10000x8000 RGB16) with N contexts in flight at the C call:
  python tests/tools/c3_inflight.py N [N ...]
(first line: one image's stats -- decisions, tier-1 bytes, stage times)."""
import os, sys, json
ns = [int(x) for x in sys.argv[1:]] or [4]
if not os.environ.get("JP2HIP_KEEP_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(ns) + 4))  # as bench.py (the box default is 4)
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import torch  # noqa: E402
torch.cuda.init()  # torch's runtime first (as bench.py), then the library's
import bench  # noqa: E402
import jp2hip  # noqa: E402
import imaging as im  # noqa: E402
enc = jp2hip.Encoder(0, host_threads=16, profile=True)
img = bench.make_image("c3", seed=2)
tif = im.tiff_bytes(img, rows_per_strip=64)
lay, _ = jp2hip.tiff_layout(tif)
d_src = torch.frombuffer(bytearray(tif), dtype=torch.uint8).cuda()
torch.cuda.synchronize()
rc = jp2hip.recipe(jp2hip.LOSSLESS, tile_w=1024, tile_h=1024)
for _ in range(2):
    out, st = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSLESS, rc, copy=False)
    out.close()
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.as_dict().items()}), flush=True)
del d_src
for n in ns:
    r = bench.lossless_c3(enc, inflight=n, n_each=int(os.environ.get("C3_EACH", "3")))
    print(json.dumps({"inflight": n, "mp_per_s_inflight_c_api": r["mp_per_s_inflight_c_api"],
                      "mp_per_s_c_api": r["mp_per_s_c_api"], "roofline_pcie": r["roofline_pcie"]["frac"]}), flush=True)
enc.close()
