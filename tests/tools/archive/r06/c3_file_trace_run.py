#!/usr/bin/env python3
"""bench.c3_file_span (C3 TIFF files -> lossless JPX files through the batch
queue) once, for a rocprofv3 kernel / memory-copy trace:
  python tests/tools/c3_file_trace_run.py > out.json"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import bench  # noqa: E402

r = bench.c3_file_span(0)
print(json.dumps({k: v for k, v in r.items() if k in ("value", "seconds", "busy", "roofline_pcie")}), flush=True)
