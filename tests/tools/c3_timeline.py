#!/usr/bin/env python3
"""C3 in-flight timeline from a rocprofv3 --kernel-trace --memory-copy-trace
run of tests/tools/c3_inflight.py N (C3_EACH=k): over the timed round (the
last N*k images, from the first DWT launch to the last image's code-stream
D2H), the fraction of time any kernel runs, the D2H busy fraction, and the
longest window with no kernel on the GPU.
  python tests/tools/c3_timeline.py <trace dir> <images in the timed round>"""
import csv
import sys

d, nimg = sys.argv[1], int(sys.argv[2])
K = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
M = sorted(csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
t0 = int([r for r in K if "k_dwt_l1s" in r["Kernel_Name"]][-nimg]["Start_Timestamp"])
rel = [int(r["End_Timestamp"]) for r in K if "k_release_dma" in r["Kernel_Name"] and int(r["End_Timestamp"]) > t0]
d2h = [(int(m["Start_Timestamp"]), int(m["End_Timestamp"])) for m in M if "DEVICE_TO_HOST" in m["Direction"]]
last_rel = sorted(rel)[nimg - 1] if len(rel) >= nimg else max(rel)
t1 = max(e for s, e in d2h if s <= last_rel + 1_000_000)  # the copy the last release let go


def union(iv):
    out = []
    for s, e in sorted(iv):
        s, e = max(s, t0), min(e, t1)
        if e <= s:
            continue
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


ku = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in K])
cu = union(d2h)
W = t1 - t0
gaps = [b[0] - a[1] for a, b in zip(ku, ku[1:])] + [ku[0][0] - t0] if ku else [W]
print({"window_ms": round(W / 1e6, 1), "kernels_busy": round(sum(e - s for s, e in ku) / W, 3),
       "d2h_busy": round(sum(e - s for s, e in cu) / W, 3), "longest_no_kernel_ms": round(max(gaps) / 1e6, 2),
       "images_per_s": round(nimg / (W / 1e9), 1)})
