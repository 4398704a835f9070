#!/usr/bin/env python3
"""Tier-1 workload census with the oracle (CPU): MQ decisions per code-block.

Shows how the tier-1 work of an image is distributed over code-blocks (the
GPU kernel's critical path is its heaviest block).  Debug tool, not a test.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import imaging as im  # noqa: E402
import oracle_lib as ol  # noqa: E402


def blocks_of_tile(coef, L):
    th, tw = coef.shape
    W, H = [tw], [th]
    for d in range(1, L + 1):
        W.append((W[-1] + 1) // 2)
        H.append((H[-1] + 1) // 2)
    out = []
    for d in range(1, L + 1):
        for band in (1, 2, 3):
            hx, hy = band in (1, 3), band in (2, 3)
            x0, y0 = (W[d] if hx else 0), (H[d] if hy else 0)
            bw, bh = (W[d - 1] - W[d] if hx else W[d]), (H[d - 1] - H[d] if hy else H[d])
            for cy in range(0, bh, 64):
                for cx in range(0, bw, 64):
                    out.append((d, band, coef[y0 + cy:y0 + min(bh, cy + 64), x0 + cx:x0 + min(bw, cx + 64)]))
    out.append((L, 0, coef[:H[L], :W[L]]))
    return out


def main():
    lossless = "--lossless" in sys.argv
    h, w = 2048, 2048
    img = im.synth_rgb8(h, w, seed=1234).astype(np.int32) - 128
    R, G, B = img[..., 0].astype(np.float32), img[..., 1].astype(np.float32), img[..., 2].astype(np.float32)
    f32 = np.float32
    Y = f32(0.299) * R; Y = Y + f32(0.587) * G; Y = Y + f32(0.114) * B
    L = ol.lib()
    L.oracle_debug_decisions.restype = ctypes.c_int64
    rc = ol.recipe(lossless)
    # use band quantiser from the product's plan via the oracle QCD is awkward; use the
    # oracle's full encode only for the step sizes: approximate with Delta = 1 in lossless
    stats = []
    tile = Y[:512, :512].copy()
    coef = ol.fdwt(tile.astype(np.int32) if lossless else tile, 6, lossless)
    import jp2hip  # noqa: F401  (plan/quantiser are product-internal; recompute inv_delta here)
    for d, band, blk in blocks_of_tile(coef, 6):
        if lossless:
            v = np.abs(blk).astype(np.uint32)
        else:
            # Delta_b = Qstep*2^B/sqrt(G_b) -- same formula as band_quant (plan.cpp)
            v = np.floor(np.abs(blk) * np.float32(1.0 / DELTA[(d, band)])).astype(np.uint32)
        sm = (((blk < 0).astype(np.uint32) << 31) | v).view(np.int32)
        L.oracle_debug_decisions()
        b, r, dd, P = ol.t1_encode(sm, band, lossless)
        stats.append((L.oracle_debug_decisions(), d, band, blk.shape, P, len(r), len(b)))
    stats.sort(reverse=True)
    tot = sum(s[0] for s in stats)
    print(f"blocks {len(stats)} decisions total {tot} mean {tot / len(stats):.0f}")
    for s in stats[:12]:
        print(s)


def _deltas():
    from math import sqrt
    import subprocess  # noqa: F401
    out = {}
    # synthesis energies from the oracle's own definition are not exported; use opj-like
    # gains measured by a unit impulse through ol.fdwt's inverse is not available either.
    return out


DELTA = {}
if __name__ == "__main__":
    main()
