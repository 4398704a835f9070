#!/usr/bin/env python3
"""GPU occupancy from a rocprofv3 kernel trace: busy fraction (union of kernel
intervals), kernel concurrency histogram and per-queue busy time over the
densest window (the bench's timed region)."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], r["Queue_Id"])
            for r in rows)
# timed region ~ last `frac` of the trace (the warm-up/latency part is first)
t0 = iv[int(len(iv) * float(sys.argv[2]) if len(sys.argv) > 2 else 0)][0]
t1 = max(e for _, e, _, _ in iv)
iv = [x for x in iv if x[0] >= t0]
ev = []
for s, e, n, q in iv:
    ev.append((s, 1)); ev.append((e, -1))
ev.sort()
conc = collections.Counter()
cur, last = 0, t0
for t, d in ev:
    conc[cur] += t - last
    cur += d; last = t
span = t1 - t0
busy = span - conc[0]
print(f"window {span/1e6:.2f} ms, kernels {len(iv)}, busy {busy/span*100:.1f}%")
for k in sorted(conc):
    print(f"  {k} concurrent: {conc[k]/span*100:.1f}%")
tot = collections.Counter(); qs = collections.Counter()
for s, e, n, q in iv:
    tot[n] += e - s; qs[q] += e - s
for n, v in tot.most_common(8):
    print(f"  {n:40s} {v/1e6:8.2f} ms")
print("queues:", {q: round(v / span, 2) for q, v in sorted(qs.items())})
