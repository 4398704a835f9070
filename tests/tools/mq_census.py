#!/usr/bin/env python3
"""Per-block MQ census on the GPU (debug library): decisions, and the shader
cycles of the modeller and coder waves (k_t1_mq), with the part of each spent
at the chunk barrier -- which of the two chains sets the pace.

  make -C jp2-bucketeer_amd/csrc debug
  JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/libjp2hip_debug.so python tests/tools/mq_census.py
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
import imaging as im  # noqa: E402
import jp2hip  # noqa: E402

img = im.synth_rgb8(4000, 6000, seed=1234)
tif = im.tiff_bytes(img)
enc = jp2hip.Encoder(0, profile=True)
try:
    enc.encode_tiff(tif, jp2hip.LOSSY)
except jp2hip.Jp2hipError:
    pass
d = tempfile.mkdtemp()
os.environ["JP2HIP_DUMP_DIR"] = d
try:
    out, st = enc.encode_tiff(tif, jp2hip.LOSSY)
except jp2hip.Jp2hipError as ex:  # census experiment builds (JP2HIP_MQ_EXP) do not produce valid files
    print("encode:", ex)

    class _St:
        t1_mq_ms = float("nan")
    st = _St()
a = np.fromfile(os.path.join(d, "mqdbg.bin"), dtype=np.int64).reshape(-1, 6)
dec, mcyc, mwait, ccyc, cwait, pos = (a[:, i] for i in range(6))
m = dec > 0
print("t1_mq_ms %.3f  blocks %d  decisions %d  max/block %d" % (st.t1_mq_ms, m.sum(), dec.sum(), dec.max()))
wave = pos[m] // 64
for w in (0, 1, 2, 5, 20, 100):
    sel = wave == w
    if not sel.any():
        continue
    dm = dec[m][sel].max()
    mc, mw = mcyc[m][sel].max(), mwait[m][sel].max()
    cc, cw = ccyc[m][sel].max(), cwait[m][sel].max()
    print(f"wave {w:4d}: decisions max {dm:6d}  modeller {mc / dm:6.1f} cyc/dec ({mw / mc * 100:4.1f}% at barrier)"
          f"  coder {cc / dm:6.1f} cyc/dec ({(cw / cc * 100) if cc else 0:4.1f}% at barrier)")
if hasattr(st, "as_dict"):
    print("stages", {k: round(v, 3) for k, v in st.as_dict().items() if k.endswith("_ms")})
sel = os.path.join(d, "seldbg.bin")
if os.path.exists(sel):
    s = np.fromfile(sel, dtype=np.int64)
    n = int(s[0])
    print("k_select (last call): lists", n, "sizes", s[1:1 + n].tolist(), "rounds", s[33:39].tolist(),
          "survivors", s[65:71].tolist())
