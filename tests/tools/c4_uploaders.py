import json, os, sys
HERE = os.path.join(os.getcwd(), "tests", "tools")
ROOT = os.getcwd()
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import bench
for up in [int(x) for x in sys.argv[1:]]:
    busy = {}
    v, dt, res, read = bench.c4_batch(0, rows=4096, ndistinct=16, contexts=12, reader_threads=6, uploader_threads=up, busy=busy)
    busy.pop("def", None)
    print(json.dumps({"uploaders": up, "mp_per_s": round(v, 1), "seconds": round(dt, 2), "busy": busy}), flush=True)
