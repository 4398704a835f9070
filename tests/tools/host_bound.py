#!/usr/bin/env python3
"""Is the C2 bench bound by host work?  Times K encodes over N contexts three
ways: the bench's call (output copied into a Python bytes object), the same
call with the output left in the library's pinned buffer (no Python copy),
and the copy alone (ctypes.string_at of a JPX-sized buffer).

  python tests/tools/host_bound.py [--steps 96] [--inflight 12]
"""
import argparse, ctypes, os, sys, threading, time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=96)
ap.add_argument("--inflight", type=int, default=12)
args = ap.parse_args()
os.environ.setdefault("GPU_MAX_HW_QUEUES", str(min(32, args.inflight + 4)))

import torch  # noqa: E402
import bench  # noqa: E402
import imaging as im  # noqa: E402
import jp2hip  # noqa: E402
from jp2hip import _lib as L  # noqa: E402

img = bench.make_image("c2", seed=1234)
tif = im.tiff_bytes(img, rows_per_strip=64)
lay, offs = jp2hip.tiff_layout(tif)
d_src = torch.frombuffer(bytearray(tif), dtype=torch.uint8).to("cuda:0")
torch.cuda.synchronize()
encs = [jp2hip.Encoder(0, host_threads=2) for _ in range(args.inflight)]
rc = jp2hip.recipe(jp2hip.LOSSY)
for e in encs:
    e.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)


def nocopy(e):
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    st = L.Stats()
    r = L.lib().jp2hip_encode_device(e._h, ctypes.c_void_p(d_src.data_ptr()), d_src.numel(), ctypes.byref(lay),
                                     jp2hip.LOSSY, ctypes.byref(rc), ctypes.byref(out), ctypes.byref(n),
                                     ctypes.byref(st))
    assert r == 0
    L.lib().jp2hip_free(out)


def timed(fn):
    nxt = [0]
    mu = threading.Lock()

    def worker(k):
        while True:
            with mu:
                s = nxt[0]
                nxt[0] += 1
            if s >= args.steps:
                return
            fn(encs[k])

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(k,)) for k in range(args.inflight)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return time.perf_counter() - t0


mp = img.shape[0] * img.shape[1] / 1e6
res = {}
for name, fn in [("bench_call", lambda e: e.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)),
                 ("no_python_copy", nocopy)] * 2:
    dt = timed(fn)
    res[name] = round(mp * args.steps / dt, 1)
buf = ctypes.create_string_buffer(9 << 20)
t = time.perf_counter()
for _ in range(20):
    ctypes.string_at(buf, 9 << 20)
res["string_at_9MiB_ms"] = round((time.perf_counter() - t) / 20 * 1e3, 3)
print(res)
