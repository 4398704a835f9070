#!/usr/bin/env python3
"""One rank of a multi-process tile-split encode (torch.distributed, one
process per rank; on a one-GPU box every rank uses cuda:0 with gloo).  Writes
this rank's part and its (offset, file length) to OUT/part<rank>.bin/.json.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29613 tests/tools/split_worker.py OUT [lossy|lossless]
"""
import json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import imaging as im  # noqa: E402
import jp2hip  # noqa: E402
from jp2hip import split as js  # noqa: E402

out = sys.argv[1]
conv = jp2hip.LOSSLESS if (len(sys.argv) > 2 and sys.argv[2] == "lossless") else jp2hip.LOSSY
dist.init_process_group(os.environ.get("JP2HIP_BENCH_BACKEND", "gloo"))
rank, world = dist.get_rank(), dist.get_world_size()
dev = int(os.environ.get("JP2HIP_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
img = im.synth_rgb8(1300, 700, seed=2000)
rc = jp2hip.recipe(conv, tile_w=256, tile_h=256)
tif = im.tiff_bytes(img)
lay, offs = jp2hip.tiff_layout(tif)
r0, r1 = js.split_rows(lay.height, rc.tile_h, rank, world, rc.flush_period)
buf, blay, keep = js.band_strips(tif, lay, offs, r0, r1)  # this rank uploads only its band's strips
d = torch.frombuffer(bytearray(buf or b"\0"), dtype=torch.uint8).to(f"cuda:{dev}")
enc = jp2hip.Encoder(dev)
part, off, flen, st = enc.encode_device_split(d.data_ptr(), d.numel(), blay, conv, js.TorchGroup().split(), rc)
os.makedirs(out, exist_ok=True)
open(os.path.join(out, f"part{rank}.bin"), "wb").write(part)
json.dump({"rank": rank, "world": world, "rows": [r0, r1], "offset": off, "file_bytes": flen,
           "backend": dist.get_backend()}, open(os.path.join(out, f"part{rank}.json"), "w"))
enc.close()
dist.barrier()
dist.destroy_process_group()
