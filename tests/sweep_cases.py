"""Seeded, randomized recipe / geometry sweep shared by the GPU parity sweep
(tests/test_gpu_sweep.py) and the oracle's own round-trip check
(tests/test_oracle_sweep.py).

Every case varies what KakaduConverter.java:38-44 fixes -- levels, layers,
tiles, code-blocks, precincts, rate, the flush period, the file format and
the COM markers -- plus the image geometry (1-4 components, 8/16 bits, ragged
edges) and its content.  Content kinds are chosen to stress tier-2 as well as
tier-1: flat images with one textured patch and sparse spikes give precincts
whose packets are empty in some layers and not in others (the tag-tree
states the round-3 mid-round divergence came from), uniform noise gives deep
bit-planes and long MQ streams.
"""
from __future__ import annotations

import numpy as np

import imaging as im

SEED = 20261017
N_CASES = 96


def _content(kind, h, w, nc, bits, seed):
    rng = np.random.default_rng(seed)
    top = (1 << bits) - 1
    dt = np.uint8 if bits == 8 else np.uint16
    if kind == "synth":
        if bits == 16:
            a = im.synth_u16(h, w, comps=nc, seed=seed)
            return a
        a = im.synth_rgb8(h, w, seed=seed)
        if nc == 1:
            return a[..., 0].copy()
        if nc == 2:
            return np.ascontiguousarray(np.dstack([a[..., 0], a[..., 2]]))
        if nc == 4:
            return np.ascontiguousarray(np.dstack([a, (a[..., 1] // 3 + 40).astype(np.uint8)]))
        return a
    shape = (h, w) if nc == 1 else (h, w, nc)
    if kind == "noise":
        return rng.integers(0, top + 1, size=shape, dtype=np.int64).astype(dt)
    if kind == "flat":
        a = np.full(shape, top // 3, dtype=dt)
        ph, pw = max(1, h // 4), max(1, w // 5)
        y0, x0 = int(rng.integers(0, h - ph + 1)), int(rng.integers(0, w - pw + 1))
        patch = rng.normal(top / 2, top / 8, size=(ph, pw) + shape[2:])
        a[y0:y0 + ph, x0:x0 + pw] = np.clip(patch, 0, top).astype(dt)
        return a
    if kind == "sparse":
        a = np.zeros(shape, dtype=dt)
        n = max(1, (h * w) // 2000)
        ys, xs = rng.integers(0, h, n), rng.integers(0, w, n)
        a[ys, xs] = top
        return a
    raise ValueError(kind)


def cases():
    """N_CASES dicts: geometry, content and recipe overrides (jp2hip.recipe
    keywords).  Deterministic: the same list on every box."""
    rng = np.random.default_rng(SEED)
    out = []
    tiles = (128, 256, 384, 512, 640, 768, 1024, 2048)
    for i in range(N_CASES):
        nc = int(rng.integers(1, 5))
        bits = 16 if rng.random() < 0.35 else 8
        lossless = bool(rng.random() < 0.5)
        levels = int(rng.integers(0, 8))
        tw = int(rng.choice(tiles))
        th = tw if rng.random() < 0.7 else int(rng.choice(tiles))
        # ragged images, about 1.2 MP per component at most, edge strips included
        r = rng.random()
        if r < 0.08:
            h, w = 1 + int(rng.integers(0, 3)), int(rng.integers(1, 1500))
        elif r < 0.16:
            h, w = int(rng.integers(1, 1500)), 1 + int(rng.integers(0, 3))
        else:
            h, w = int(rng.integers(8, 1300)), int(rng.integers(8, 1300))
        cb = [(6, 6), (6, 6), (5, 5), (4, 4), (6, 4), (4, 6), (5, 6), (6, 5)][int(rng.integers(0, 8))]
        layers = int(rng.choice([1, 2, 3, 6, 6, 8, 12]))
        pr = rng.random()
        if pr < 0.6:
            prec = dict(nprecincts=3, prec_w_log2=[8, 8, 7], prec_h_log2=[8, 8, 7])
        elif pr < 0.8:
            p = int(rng.integers(6, 9))
            prec = dict(nprecincts=1, prec_w_log2=[p], prec_h_log2=[p])
        elif pr < 0.9:
            prec = dict(nprecincts=2, prec_w_log2=[8, 6], prec_h_log2=[7, 6])
        else:
            prec = dict(nprecincts=0)
        if lossless:
            rate = 0.0 if rng.random() < 0.8 else round(float(rng.uniform(1.0, 6.0)), 2)
        else:
            rate = round(float(rng.uniform(0.5, 4.0)), 2)
        ov = dict(levels=levels, layers=layers, tile_w=tw, tile_h=th, cblk_w_log2=cb[0],
                  cblk_h_log2=cb[1], rate_bpp=rate, slope_skip=int(rng.random() < 0.6),
                  flush_period=int(rng.choice([1024, 1024, 0, 512, 2048])),
                  format=int(rng.integers(0, 3)), comment=int(rng.random() < 0.7), **prec)
        kind = str(rng.choice(["synth", "synth", "flat", "noise", "sparse"]))
        out.append(dict(idx=i, h=h, w=w, nc=nc, bits=bits, lossless=lossless, kind=kind,
                        seed=SEED + i, recipe=ov))
    # tag-tree stress: the most layers the recipe allows, so most blocks are
    # first included in a late layer after empty packets; 16x16 blocks give
    # precincts of 64 blocks (the wave-per-precinct tier-2 kernel, deepest
    # trees) and of 256 (the serial fallback)
    base = dict(levels=5, tile_w=512, tile_h=512, cblk_w_log2=4, cblk_h_log2=4, slope_skip=1,
                flush_period=1024, format=0, comment=1, nprecincts=3, prec_w_log2=[8, 8, 7],
                prec_h_log2=[8, 8, 7])
    for j, (kind, lossless, layers, rate) in enumerate([("sparse", True, 32, 0.0), ("flat", True, 32, 0.0),
                                                       ("synth", False, 32, 0.7), ("flat", False, 20, 2.0),
                                                       ("sparse", False, 32, 3.0), ("synth", True, 17, 0.0)]):
        i = N_CASES + j
        out.append(dict(idx=i, h=700 + 37 * j, w=900 - 29 * j, nc=1 + j % 3, bits=8 if j % 2 else 16,
                        lossless=lossless, kind=kind, seed=SEED + i,
                        recipe=dict(base, layers=layers, rate_bpp=rate)))
    return out


def case_id(c):
    r = c["recipe"]
    return (f"{c['idx']:02d}_{c['h']}x{c['w']}x{c['nc']}_{c['bits']}b_{'ll' if c['lossless'] else 'ly'}"
            f"_{c['kind']}_L{r['levels']}_T{r['tile_w']}x{r['tile_h']}_cb{r['cblk_w_log2']}{r['cblk_h_log2']}"
            f"_ly{r['layers']}_r{r['rate_bpp']}")


def image(c):
    return _content(c["kind"], c["h"], c["w"], c["nc"], c["bits"], c["seed"])
