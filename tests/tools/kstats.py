#!/usr/bin/env python3
"""Per-image kernel time table from a rocprofv3 --stats CSV (kernel_stats.csv):
calls and ms per image, images = k_t1_mq launches."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int([r for r in rows if "k_t1_mq" in r["Name"]][0]["Calls"])
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print(f"images {n}  kernel ms per image {tot / n / 1e6:.3f}")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    name = r["Name"].split("(")[0].replace("void ", "").replace("jp2hip::", "")[:44]
    print(f"  {name:44s} {int(r['Calls']) / n:5.1f}/img {float(r['AverageNs']) / 1e3:9.1f} us {int(r['TotalDurationNs']) / n / 1e6:7.3f} ms/img")
