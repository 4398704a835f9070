#!/usr/bin/env python3
"""Concatenate the parts split_worker.py wrote and compare them with the
single-GPU encode and with the oracle (fresh process, after the ranks exited).

  python tests/tools/split_compare.py OUT [lossy|lossless]
"""
import glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import imaging as im  # noqa: E402
import jp2hip  # noqa: E402
import oracle_lib as ol  # noqa: E402

out = sys.argv[1]
conv = jp2hip.LOSSLESS if (len(sys.argv) > 2 and sys.argv[2] == "lossless") else jp2hip.LOSSY
metas = sorted((json.load(open(f)) for f in glob.glob(os.path.join(out, "part*.json"))), key=lambda m: m["rank"])
parts = [open(os.path.join(out, f"part{m['rank']}.bin"), "rb").read() for m in metas]
data = b"".join(parts)
off = 0
for m, p in zip(metas, parts):
    assert m["offset"] == off and m["file_bytes"] == len(data), (m, off, len(data))
    off += len(p)
img = im.synth_rgb8(1300, 700, seed=2000)
rc = jp2hip.recipe(conv, tile_w=256, tile_h=256)
enc = jp2hip.Encoder(0)
single, _ = enc.encode_tiff(im.tiff_bytes(img), conv, rc)
oracle = ol.encode(img, ol.copy_recipe(rc))
res = {"world": len(parts), "backend": metas[0]["backend"], "rows": [m["rows"] for m in metas],
       "part_bytes": [len(p) for p in parts], "file_bytes": len(data),
       "equals_single_gpu": data == single, "equals_oracle": data == oracle}
print(json.dumps(res))
sys.exit(0 if res["equals_single_gpu"] and res["equals_oracle"] else 1)
