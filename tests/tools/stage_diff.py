#!/usr/bin/env python3
"""Stage-by-stage comparison of libjp2hip against the CPU oracle (debug tool).

Runs one encode with JP2HIP_DUMP_DIR set, then checks, in pipeline order,
DWT + quantiser indices -> tier-1 (bytes, truncation lengths, distortion)
-> final code-stream, and prints the first divergence.  Needs a GPU.

  python tests/tools/stage_diff.py --w 700 --h 600 --nc 3 --bits 8 [--lossy]
  python tests/tools/stage_diff.py --image testjpx
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))

import imaging as im  # noqa: E402
import oracle_lib as ol  # noqa: E402

BLOCK_DT = np.dtype([("tc", "<i4"), ("x0", "<i2"), ("y0", "<i2"), ("w", "<i2"), ("h", "<i2"),
                     ("band", "i1"), ("Mb", "i1"), ("p0", "i1"), ("p1", "i1"),
                     ("inv_delta", "<f4"), ("p2", "<u4"), ("bp_off", "<u8"), ("sm_off", "<u8"),
                     ("out_off", "<u8"), ("out_cap", "<u4"), ("p3", "<u4")])
MAXP = 96


def make_image(args):
    if args.image == "testjpx":
        return im.decode_pillow(open(os.path.join(ROOT, "tests/golden/test.jpx"), "rb").read())
    if args.bits == 8:
        a = im.synth_rgb8(args.h, args.w, seed=args.seed)
        if args.nc == 1:
            return a[..., 0].copy()
        if args.nc == 4:
            return np.dstack([a, (np.arange(args.w)[None, :] + np.zeros((args.h, 1), int)) % 256]).astype(np.uint8)
        return a[..., :args.nc].copy()
    return im.synth_u16(args.h, args.w, comps=args.nc, seed=args.seed)


def expected_ingest(img, rc):
    a = img if img.ndim == 3 else img[..., None]
    B = a.dtype.itemsize * 8
    s = a.astype(np.int32) - (1 << (B - 1))
    nc = a.shape[2]
    if rc.reversible:
        out = s.copy()
        if rc.mct and nc >= 3:
            R, G, Bl = s[..., 0], s[..., 1], s[..., 2]
            out[..., 0] = (R + 2 * G + Bl) >> 2
            out[..., 1] = Bl - G
            out[..., 2] = R - G
        return out
    f = s.astype(np.float32)
    if rc.mct and nc >= 3:
        R, G, Bl = f[..., 0], f[..., 1], f[..., 2]
        f32 = np.float32
        y0 = f32(0.299) * R; y0 = y0 + f32(0.587) * G; y0 = y0 + f32(0.114) * Bl
        cb = f32(-0.16875) * R; cb = cb - f32(0.33126) * G; cb = cb + f32(0.5) * Bl
        cr = f32(0.5) * R; cr = cr - f32(0.41869) * G; cr = cr - f32(0.08131) * Bl
        f = f.copy()
        f[..., 0], f[..., 1], f[..., 2] = y0, cb, cr
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", default="synth")
    ap.add_argument("--w", type=int, default=700)
    ap.add_argument("--h", type=int, default=600)
    ap.add_argument("--nc", type=int, default=3)
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--lossy", action="store_true")
    ap.add_argument("--levels", type=int, default=6)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--max-report", type=int, default=5)
    args = ap.parse_args()

    import jp2hip
    img = make_image(args)
    conv = jp2hip.LOSSY if args.lossy else jp2hip.LOSSLESS
    rc = jp2hip.recipe(conv, levels=args.levels, tile_w=args.tile, tile_h=args.tile)
    orc = ol.copy_recipe(rc)
    tif = im.tiff_bytes(img)
    d = tempfile.mkdtemp(prefix="jp2hip_dump_")
    os.environ["JP2HIP_DUMP_DIR"] = d
    enc = jp2hip.Encoder(0)
    got, st = enc.encode_tiff(tif, conv, rc)
    del os.environ["JP2HIP_DUMP_DIR"]
    want = ol.encode(img, orc)
    print(f"image {img.shape} {img.dtype} {'lossy' if args.lossy else 'lossless'}: product {len(got)} B, oracle {len(want)} B")
    if got == want:
        print("CODESTREAM IDENTICAL")
        return 0
    # ---------------- stage checks ----------------
    # dwt.bin holds the quantisation indices the DWT writes (sign-magnitude,
    # 16-bit words for 8-bit sources, else 32-bit): checked per code-block
    # against the oracle's transform of the expected ingest, quantised
    H, W = img.shape[:2]
    nc = 1 if img.ndim == 2 else img.shape[2]
    T = args.tile
    ntx, nty = -(-W // T), -(-H // T)
    ntc = ntx * nty * nc
    raw = np.fromfile(os.path.join(d, "dwt.bin"), dtype=np.uint8)
    q16 = raw.size == ntc * T * T * 2
    dwt = raw.view(np.uint16 if q16 else np.uint32).reshape(ntc, T, T).astype(np.uint32)
    sbit = 15 if q16 else 31
    exp = expected_ingest(img, rc)
    ref = {}
    for ty in range(nty):
        for tx in range(ntx):
            for c in range(nc):
                tc = (ty * ntx + tx) * nc + c
                x0, y0 = tx * T, ty * T
                tw, th = min(W, x0 + T) - x0, min(H, y0 + T) - y0
                ref[tc] = ol.fdwt(np.ascontiguousarray(exp[y0:y0 + th, x0:x0 + tw, c]), args.levels, bool(rc.reversible))
    blocks = np.fromfile(os.path.join(d, "blocks.bin"), dtype=BLOCK_DT)
    sm = np.fromfile(os.path.join(d, "sm.bin"), dtype=np.int32)
    P = np.fromfile(os.path.join(d, "P.bin"), dtype=np.uint8)
    t1 = np.fromfile(os.path.join(d, "t1out.bin"), dtype=np.uint8)
    lens = np.fromfile(os.path.join(d, "lengths.bin"), dtype=np.int32)
    npas = np.fromfile(os.path.join(d, "npasses.bin"), dtype=np.uint8)
    rates = np.fromfile(os.path.join(d, "rates.bin"), dtype=np.int32).reshape(-1, MAXP)
    dists = np.fromfile(os.path.join(d, "dists.bin"), dtype=np.int64).reshape(-1, MAXP)
    nbad = 0
    for i, b in enumerate(blocks):
        w, h = int(b["w"]), int(b["h"])
        coef = ref[int(b["tc"])][b["y0"]:b["y0"] + h, b["x0"]:b["x0"] + w]
        if rc.reversible:
            v = np.abs(coef).astype(np.uint32)
            s = (coef < 0).astype(np.uint32)
        else:
            f = coef.astype(np.float32)
            v = np.floor(np.abs(f) * np.float32(b["inv_delta"])).astype(np.uint32)
            s = (f < 0).astype(np.uint32)
        v = np.minimum(v, (1 << int(b["Mb"])) - 1)
        esm = ((s << 31) | v).astype(np.uint32).view(np.int32)
        gq = dwt[b["tc"], b["y0"]:b["y0"] + h, b["x0"]:b["x0"] + w]
        gv, gs = gq & ((1 << sbit) - 1), gq >> sbit
        if not (np.array_equal(gv, v) and np.array_equal(gs[v != 0], s[v != 0])):
            print(f"DWT/QUANT index mismatch block {i} tc={b['tc']} band={b['band']} {w}x{h} "
                  f"n={int(np.count_nonzero(gv != v))}")
            nbad += 1
            if nbad > args.max_report:
                return 1
            continue
        gsm = sm[b["sm_off"]:b["sm_off"] + 64 * h].reshape(h, 64)[:, :w]
        if not np.array_equal(esm.view(np.uint32) & 0x7FFFFFFF, gsm.view(np.uint32) & 0x7FFFFFFF):
            print(f"QUANT mismatch block {i} band={b['band']} {w}x{h}")
            nbad += 1
            if nbad > args.max_report:
                return 1
            continue
        obytes, orates, odists, oP = ol.t1_encode(esm, int(b["band"]), bool(rc.reversible))
        gb = bytes(t1[b["out_off"]:b["out_off"] + lens[i]])
        n = int(npas[i])
        if oP != P[i] or obytes != gb or n != len(orates) or not np.array_equal(orates, rates[i, :n]) \
                or not np.array_equal(odists, dists[i, :n]):
            print(f"T1 mismatch block {i} band={b['band']} {w}x{h} P={P[i]}/{oP} len={lens[i]}/{len(obytes)} "
                  f"npasses={n}/{len(orates)}")
            if len(obytes) and len(gb):
                k = next((j for j in range(min(len(obytes), len(gb))) if obytes[j] != gb[j]), None)
                print(f"   first differing byte {k}")
            if n == len(orates):
                rb = np.nonzero(orates != rates[i, :n])[0]
                db = np.nonzero(odists != dists[i, :n])[0]
                print(f"   rate diffs at passes {rb[:8].tolist()}  dist diffs at {db[:8].tolist()}")
                if len(db):
                    j = db[0]
                    print(f"   pass {j}: dist product {dists[i, j]} oracle {odists[j]}")
            nbad += 1
            if nbad > args.max_report:
                return 1
    if nbad:
        return 1
    print("quantiser + tier-1 identical for all blocks; divergence is in PCRD/tier-2")
    k = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), None)
    print(f"first differing byte of file: {k} (sizes {len(got)} vs {len(want)})")
    return 1


if __name__ == "__main__":
    sys.exit(main())
