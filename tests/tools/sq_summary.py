#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc pass of SQ counters into per-kernel occupancy /
VALU figures (north_star: tier-1 "with occupancy and VALU counters from
rocprof").

  python tests/tools/sq_summary.py DIR [DIR ...] --out profiles/rNN/t1_sq_counters.json

Counters are summed over the dispatch's SEs/XCDs as rocprofv3 reports them and
averaged over launches.  Derived (same units on both sides of each ratio):
  valu_busy      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES  (share of a wave's
                   lifetime spent issuing VALU)
  wait_share     = SQ_WAIT_ANY / SQ_WAVE_CYCLES           (waiting on s_waitcnt)
  waves_resident = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES        (mean waves in flight
                   per SQ-busy cycle, the occupancy the kernel reaches)
"""
import argparse, csv, glob, json, os, re
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name.split("(")[0][:60]


ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--out", required=True)
args = ap.parse_args()
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for d in args.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
out = {"meta": {"source": "rocprofv3 --pmc SQ_* passes", "derived": {
    "valu_busy": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES", "wait_share": "SQ_WAIT_ANY / SQ_WAVE_CYCLES",
    "waves_resident": "SQ_WAVE_CYCLES / SQ_BUSY_CYCLES"}}, "kernels": {}}
for k, cs in per.items():
    avg = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    e = {c: round(v) for c, v in avg.items()}
    e["launches"] = max(len(v) for v in cs.values())
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        if "SQ_ACTIVE_INST_VALU" in avg: e["valu_busy"] = round(avg["SQ_ACTIVE_INST_VALU"] / wc, 4)
        if "SQ_WAIT_ANY" in avg: e["wait_share"] = round(avg["SQ_WAIT_ANY"] / wc, 4)
        if avg.get("SQ_BUSY_CYCLES"): e["waves_resident"] = round(wc / avg["SQ_BUSY_CYCLES"], 3)
    out["kernels"][k] = e
os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
json.dump(out, open(args.out, "w"), indent=1)
print(json.dumps({k: {x: v[x] for x in ("valu_busy", "wait_share", "waves_resident", "launches") if x in v}
                  for k, v in out["kernels"].items()}, indent=1))
