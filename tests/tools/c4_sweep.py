#!/usr/bin/env python3
"""C4 batch leg (bench.c4_batch) over reader / uploader thread counts and
contexts, with each stage's busy fraction: which stage bounds the batch.
  python tests/tools/c4_sweep.py [rows] > out.jsonl"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "20")
import bench  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 512
for ctx, rd, up in [(12, 4, 4), (12, 4, 8), (12, 6, 8), (12, 4, 12), (16, 6, 12), (12, 8, 16)]:
    busy = {}
    v, dt, res, read = bench.c4_batch(0, rows=rows, ndistinct=16, contexts=ctx, reader_threads=rd,
                                      uploader_threads=up, busy=busy)
    busy.pop("def", None)
    print(json.dumps({"contexts": ctx, "readers": rd, "uploaders": up, "mp_per_s": round(v, 1),
                      "seconds": round(dt, 3), "tiff_gb_per_s": round(read / dt / 1e9, 2),
                      "jpx_gb_per_s": round(sum(r["out_bytes"] for r in res) / dt / 1e9, 2), "busy": busy}),
          flush=True)
