#!/usr/bin/env python3
"""Fits the lossless layer fractions (oracle/jp2_oracle.c kLosslessFrac6) to
the reference fixture test.jpx: encodes its decoded pixels with the lossless
recipe through the experiments build of the oracle (ORACLE_LAYER_FRACS
overrides the five lower layers' fractions, 1/65536 of each flush stripe's
tier-1 bytes) and compares the Kdu-Layer-Info byte column with Kakadu's.
  python tests/tools/fit_layers.py [f0,f1,f2,f3,f4]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, os.path.join(HERE, ".."))
subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "experiments"], check=True)
import imaging as im  # noqa: E402
import oracle_lib as ol  # noqa: E402
ol.LIB = os.path.join(os.path.dirname(ol.LIB), "liboracle_exp.so")


def layer_info(cs):
    p = cs.find(b"Kdu-Layer-Info")
    n = int.from_bytes(cs[p - 4:p - 2], "big")
    txt = cs[p:p + n - 4].decode("latin-1").splitlines()[1:]
    return [(float(x.split(",")[0]), float(x.split(",")[1])) for x in txt]


ref_bytes = open(os.path.join(ROOT, "tests", "golden", "test.jpx"), "rb").read()
ref = layer_info(ref_bytes)
pix = im.decode_pillow(ref_bytes)
if len(sys.argv) > 1:
    os.environ["ORACLE_LAYER_FRACS"] = sys.argv[1]
# exact layer ends: the oracle prints them (ORACLE_LAYER_END) in a child
# process, since the hook writes to the C stderr
code = ("import sys; sys.path.insert(0, %r); import imaging as im, oracle_lib as ol; ol.LIB = %r; "
        "ol.encode(im.decode_pillow(open(%r, 'rb').read()), ol.recipe(True, format=0))"
        % (os.path.join(HERE, ".."), ol.LIB, os.path.join(ROOT, "tests", "golden", "test.jpx")))
env = dict(os.environ, ORACLE_LAYER_END="1")
err = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stderr
exact = [int(x.split()[2]) for x in err.splitlines() if x.startswith("layer_end")]
cs = ol.encode(pix, ol.recipe(True, format=0))
got = layer_info(cs)
for (rs, rl), (gs, gl), ex in zip(ref, got, exact):
    print(f"kakadu {rs:7.1f} {rl:9.0f}   ours {gs:7.1f} {ex:9d}   L ratio {ex / rl:.3f}")
print("file bytes", len(cs), "kakadu", len(ref_bytes))
