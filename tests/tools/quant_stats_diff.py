#!/usr/bin/env python3
"""Quantiser statistics of libjp2hip (per-plane predicted sizes `est` and
distortion decreases dref + dsig) against their oracle definition
(oracle/jp2_oracle.c plane_stats), block by block (debug tool, needs a GPU).

  python tests/tools/quant_stats_diff.py --w 260 --h 300 --nc 4 [--lossy]
"""
import argparse, os, sys, tempfile
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "tools"))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
import imaging as im  # noqa: E402
from stage_diff import BLOCK_DT  # noqa: E402


def dist_at(v, p, lossless):
    t2 = 2 * v + (0 if lossless else 1)
    r2 = np.where((v >> p) != 0, 2 * ((v >> p) << p) + (0 if (lossless and p == 0) else (1 << p)), 0)
    e = t2 - r2
    return e * e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=260)
    ap.add_argument("--h", type=int, default=300)
    ap.add_argument("--nc", type=int, default=4)
    ap.add_argument("--lossy", action="store_true")
    args = ap.parse_args()
    import jp2hip
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import _img
    img = _img(args.h, args.w, args.nc, 8, seed=args.h * 7 + args.w)
    conv = jp2hip.LOSSY if args.lossy else jp2hip.LOSSLESS
    rc = jp2hip.recipe(conv)
    d = tempfile.mkdtemp(prefix="jp2hip_q_")
    os.environ["JP2HIP_DUMP_DIR"] = d
    enc = jp2hip.Encoder(0)
    enc.encode_tiff(im.tiff_bytes(img), conv, rc)
    blocks = np.fromfile(os.path.join(d, "blocks.bin"), dtype=BLOCK_DT)
    sm = np.fromfile(os.path.join(d, "sm.bin"), dtype=np.int32).view(np.uint32)
    P = np.fromfile(os.path.join(d, "P.bin"), dtype=np.uint8)
    est = np.fromfile(os.path.join(d, "est.bin"), dtype=np.uint32).reshape(-1, 32)
    dref = np.fromfile(os.path.join(d, "dref.bin"), dtype=np.int64).reshape(-1, 32)
    dsig = np.fromfile(os.path.join(d, "dsig.bin"), dtype=np.int64).reshape(-1, 32)
    lossless = not args.lossy
    nbad = 0
    for i, b in enumerate(blocks):
        w, h = int(b["w"]), int(b["h"])
        v = (sm[b["sm_off"]:b["sm_off"] + 64 * h].reshape(h, 64)[:, :w] & 0x7FFFFFFF).astype(np.int64)
        for p in range(int(P[i])):
            sig = (v >> p) != 0
            nref = int(((v >> (p + 1)) != 0).sum())
            nnew = int(sig.sum()) - nref
            pad = np.pad(sig, 1)
            nbm = np.zeros_like(sig)
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    if dy or dx:
                        nbm |= pad[1 + dy:1 + dy + h, 1 + dx:1 + dx + w]
            nnb = int((nbm & ~sig).sum())
            e = 16 * nref + 56 * nnew + 5 * nnb
            pd = int(((dist_at(v, p + 1, lossless) - dist_at(v, p, lossless)) * sig).sum())
            g = int(dref[i, p] + dsig[i, p])
            if e != est[i, p] or pd != g:
                print(f"block {i} band {b['band']} {w}x{h} Mb {b['Mb']} P {P[i]} plane {p}: est {est[i, p]} "
                      f"want {e} (ref {nref} new {nnew} nb {nnb}); pd {g} want {pd}")
                nbad += 1
                if nbad > 10:
                    return 1
    print("blocks", len(blocks), "mismatches", nbad)
    return 1 if nbad else 0


if __name__ == "__main__":
    sys.exit(main())
