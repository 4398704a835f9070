#!/usr/bin/env python3
"""Experiment: how many of the MQ decisions the slope prediction lets through
are discarded by PCRD-opt, by pass type (oracle, ORACLE_PASS_WASTE hook).
  python tests/tools/pass_waste.py [c2|c5small] [margin]"""
import json, os, sys, tempfile
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
if len(sys.argv) > 2:
    os.environ["ORACLE_SKIP_MARGIN"] = sys.argv[2]
out = tempfile.mktemp(suffix=".jsonl")
os.environ["ORACLE_PASS_WASTE"] = out
import subprocess  # noqa: E402
import bench  # noqa: E402
import oracle_lib as ol  # noqa: E402
# the hooks exist only in the experiments build of the oracle
subprocess.run(["make", "-s", "-C", os.path.join(HERE, "..", "..", "oracle"), "experiments"], check=True)
ol.LIB = os.path.join(os.path.dirname(ol.LIB), "liboracle_exp.so")
img = bench.make_image("c2", seed=1234)
rc = ol.recipe(False)
data = ol.encode(img, rc)
r = json.loads(open(out).read().splitlines()[-1])
r["file_bytes"] = len(data)
r["lost_frac"] = round(1 - r["kept"] / r["decisions"], 4)
print(json.dumps(r))
import imaging as im  # noqa: E402
dec = im.decode_pillow(data)
print(json.dumps({"margin": os.environ.get("ORACLE_SKIP_MARGIN", "12"), "psnr": round(im.psnr(img, dec), 4)}))
