#!/usr/bin/env python3
"""Fits the lossless layer fractions (oracle/jp2_oracle.c kLosslessFrac6,
plan.cpp lossless_layer_frac) to the reference fixture test.jpx: each of the
five lower layers' fraction (1/65536 of each -flush_period stripe's tier-1
bytes) is bisected until the oracle's file, decoded through that layer by
opj_decompress -l, has test.jpx's RGB PSNR at the same layer.

This is a FIT (five numbers to five numbers); tests/test_oracle.py's
per-layer PSNR check on test.jpx is a fit check, not independent parity.
What round 6 found while doing it: Kakadu's Kdu-Layer-Info
L column (5.1e4 .. 3.0e5) is its first flush stripe's bytes projected to the
image height, not the bytes a decoder of the first l layers reads (test.jpx's
packets, parsed by SOP: 80.1e3 / 99.2e3 / 117.8e3 / 137.6e3 / 197.0e3), which
is why round 5's fit to that column gave layers 0.5-4.3 dB below Kakadu's.

  python tests/tools/fit_layers.py            # fit, print the table
  python tests/tools/fit_layers.py f0,..,f4   # evaluate given fractions"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, os.path.join(HERE, ".."))
subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "experiments"], check=True)
import imaging as im  # noqa: E402
import oracle_lib as ol  # noqa: E402
ol.LIB = os.path.join(os.path.dirname(ol.LIB), "liboracle_exp.so")

ref = open(os.path.join(ROOT, "tests", "golden", "test.jpx"), "rb").read()
pix = im.decode_pillow(ref)


def layer_psnr(cs, l):
    return im.psnr(im.decode_opj(cs, ext=".j2k", layers=l)[..., :3], pix[..., :3])


target = [layer_psnr(ref, l) for l in range(1, 6)]


def encode(fr):
    os.environ["ORACLE_LAYER_FRACS"] = ",".join(str(int(x)) for x in fr)
    return ol.encode(pix, ol.recipe(True, format=0))


if len(sys.argv) > 1:
    fr = [int(x) for x in sys.argv[1].split(",")]
else:
    fr = [9340, 12200, 15100, 19240, 35220]
    for l in range(5):  # a layer's PSNR depends on its own fraction only
        lo, hi = 1000, 65000
        while hi - lo > 1:
            mid = (lo + hi) // 2
            trial = list(fr)
            trial[l] = mid
            if layer_psnr(encode(trial), l + 1) < target[l]:
                lo = mid
            else:
                hi = mid
        fr[l] = hi
cs = encode(fr)
got = [layer_psnr(cs, l) for l in range(1, 6)]
print("fractions (layers 1..5):", ",".join(map(str, fr)))
print("table (layers below the top):", [65536] + fr[::-1])
kp = np.cumsum(im.packet_bytes_by_layer(ref, 6))
op = np.cumsum(im.packet_bytes_by_layer(cs, 6))
for l in range(5):
    print(f"layer {l + 1}: PSNR kakadu {target[l]:6.2f} ours {got[l]:6.2f}   "
          f"packet bytes kakadu {kp[l]:7d} ours {op[l]:7d}")
print("file bytes", len(cs), "kakadu", len(ref))
