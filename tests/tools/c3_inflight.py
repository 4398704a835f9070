#!/usr/bin/env python3
"""Lossless C3 (10000x8000 RGB16) with N contexts in flight at the C call:
  python tests/tools/c3_inflight.py N [N ...]"""
import os, sys, json
ns = [int(x) for x in sys.argv[1:]] or [4]
os.environ.setdefault("GPU_MAX_HW_QUEUES", str(min(32, max(ns) + 4)))
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import torch  # noqa: E402
torch.cuda.init()  # torch's runtime first (as bench.py), then the library's
import bench  # noqa: E402
import jp2hip  # noqa: E402
enc = jp2hip.Encoder(0, host_threads=16, profile=True)
for n in ns:
    r = bench.lossless_c3(enc, inflight=n, n_each=3)
    print(json.dumps({"inflight": n, "mp_per_s_inflight_c_api": r["mp_per_s_inflight_c_api"],
                      "mp_per_s_c_api": r["mp_per_s_c_api"], "roofline_pcie": r["roofline_pcie"]["frac"]}), flush=True)
enc.close()
