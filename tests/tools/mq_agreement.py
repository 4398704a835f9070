#!/usr/bin/env python3
"""HIP-event vs rocprofv3 agreement for the roofline kernel.

bench.py's roofline.avg_launch_ms averages k_t1_mq's HIP-event time over every
C2 launch of the run (warm-up, alone, timed); with --no-extras those are all
the k_t1_mq launches a rocprofv3 kernel trace of the same command sees.  Also
lists blit-kernel launches (there should be none with SDMA on) and each
kernel's average under load.
usage: mq_agreement.py bench.json <rocprofv3 -d dir>"""
import csv
import glob
import json
import sys

line = [x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1]
b = json.loads(line)
stats = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(stats[0])))
mq = [r for r in rows if "k_t1_mq" in r["Name"]][0]
ev = b["roofline"]["avg_launch_ms"]
pr = float(mq["AverageNs"]) / 1e6
print(f"k_t1_mq launches: bench {b['roofline']['launches_averaged']}, rocprofv3 {mq['Calls']}")
print(f"k_t1_mq average: HIP events {ev:.4f} ms, rocprofv3 {pr:.4f} ms, ratio {ev / pr:.4f}")
print(f"hw_queues {b['config']['hw_queues']}, value {b['value']} MP/s")
blits = [r for r in rows if "copyBuffer" in r["Name"] or "fillBuffer" in r["Name"]]
print("blit kernels:", ", ".join(f"{r['Name'][:40]} x{r['Calls']}" for r in blits) or "none")
print("kernels by total time:")
tot = sum(int(r["TotalDurationNs"]) for r in rows)
for r in rows[:24]:
    print(f"  {r['Name'].split('(')[0].replace('void ', '')[:46]:46s} calls {int(r['Calls']):6d} "
          f"avg {float(r['AverageNs']) / 1e3:9.1f} us  share {int(r['TotalDurationNs']) / tot:6.3f}")
