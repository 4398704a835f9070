#!/usr/bin/env python3
"""Per-stream timeline of a rocprofv3 kernel trace: for the busiest window
(the bench's timed loop), how much of each stream's time is spent inside its
kernels / copies, and how the gaps between them are distributed (host waits
show up as long gaps).  Usage: stream_gaps.py run_kernel_trace.csv [from_frac]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.35
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-28:],
             r["Stream_Id"]) for r in rows)
t0 = ev[int(len(ev) * frac)][0]
t1 = ev[-1][1]
ev = [e for e in ev if e[0] >= t0]
by = collections.defaultdict(list)
for s, e, n, st in ev:
    by[st].append((s, e, n))
span = t1 - t0
print(f"window {span / 1e6:.2f} ms, {len(ev)} dispatches, {len(by)} streams")
gapk = collections.Counter()
tot_busy = tot_gap = 0
gap_hist = collections.Counter()
for st, lst in sorted(by.items()):
    busy = sum(e - s for s, e, _ in lst)
    gaps = [(lst[i + 1][0] - lst[i][1], lst[i][2], lst[i + 1][2]) for i in range(len(lst) - 1)]
    g = sum(max(0, x[0]) for x in gaps)
    tot_busy += busy
    tot_gap += g
    for d, a, b in gaps:
        gapk[(a, b)] += max(0, d)
        gap_hist[min(6, len(str(max(1, d // 1000))))] += max(0, d)
print(f"in kernels {tot_busy / (tot_busy + tot_gap) * 100:.1f}% of stream time, gaps {tot_gap / (tot_busy + tot_gap) * 100:.1f}%")
print("gap time by size (us digits):", {k: round(v / tot_gap, 3) for k, v in sorted(gap_hist.items())})
print("largest gap totals (after -> before), ms per stream:")
for (a, b), v in gapk.most_common(12):
    print(f"  {a:28s} -> {b:28s} {v / 1e6 / len(by):8.3f}")
