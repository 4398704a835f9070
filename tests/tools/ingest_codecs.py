"""Cost of compressed TIFF ingest on the GPU (measurement tool, not a test).

Encodes the C2 image (6000x4000 RGB8, lossy 3 bpp) from an uncompressed strip
TIFF and from LZW / Deflate / PackBits TIFFs of the same pixels (Pillow's
libtiff writes them), checks every file equals the uncompressed encode, and
prints the median wall and per-stage times.  The strip decoders run one lane
per strip, so the rows per strip set how many lanes decode at once.

    python tests/tools/ingest_codecs.py [--rps 64 8] [--reps 3]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jp2-bucketeer_amd"))

import imaging as im  # noqa: E402
import jp2hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rps", type=int, nargs="+", default=[64, 8])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    img = im.synth_rgb8(4000, 6000, seed=1234)
    enc = jp2hip.Encoder(0, profile=True)
    conv = jp2hip.LOSSY
    ref, _ = enc.encode_tiff(im.tiff_bytes(img, rows_per_strip=64), conv)
    cases = [("none", None, False)]
    cases += [(c, c, p) for c in ("tiff_lzw", "tiff_adobe_deflate", "packbits") for p in (False, True)
              if not (c == "packbits" and p)]
    for rps in args.rps:
        for name, comp, pred in cases:
            data = im.tiff_bytes(img, rows_per_strip=rps) if comp is None else \
                im.tiff_bytes_compressed(img, comp, predictor=pred, rows_per_strip=rps)
            walls, stats = [], []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                out, st = enc.encode_tiff(data, conv)
                walls.append((time.perf_counter() - t0) * 1e3)
                stats.append(st.as_dict())
            assert out == ref, (name, pred, rps)
            mid = sorted(range(len(walls)), key=lambda i: walls[i])[len(walls) // 2]
            s = stats[mid]
            print(json.dumps({"compression": name, "predictor": 2 if pred else 1, "rows_per_strip": rps,
                              "strips": (4000 + rps - 1) // rps, "tiff_mb": round(len(data) / 1e6, 2),
                              "wall_ms": round(statistics.median(walls), 2), "total_ms": round(s["total_ms"], 2),
                              "h2d_ms": round(s["h2d_ms"], 2), "ingest_ms": round(s["ingest_ms"], 2),
                              "dwt_ms": round(s["dwt_ms"], 2), "t1_ms": round(s["t1_ms"], 2),
                              "identical": True}), flush=True)


if __name__ == "__main__":
    main()
