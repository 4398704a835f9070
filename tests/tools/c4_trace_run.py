#!/usr/bin/env python3
"""One C4 batch leg (bench.c4_batch: 12 contexts, 6 readers, 8 uploaders) for
a rocprofv3 kernel / memory-copy trace; analyse with
  python tests/tools/c3_timeline.py <trace dir> <rows>
  python tests/tools/c4_trace_run.py [rows] > out.json"""
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

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 512
busy = {}
v, dt, res, read = bench.c4_batch(0, rows=rows, ndistinct=16, contexts=12, reader_threads=6, uploader_threads=8,
                                  busy=busy)
busy.pop("def", None)
print(json.dumps({"rows": rows, "mp_per_s": round(v, 1), "seconds": round(dt, 3), "busy": busy}), flush=True)
