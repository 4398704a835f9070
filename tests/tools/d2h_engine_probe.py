#!/usr/bin/env python3
"""Which engine moves a device -> pinned-host copy (the code-stream D2H):
run under rocprofv3 --kernel-trace; a __amd_rocclr_copyBuffer dispatch per
copy means a blit kernel on the CUs, none means a DMA engine.  Prints the
copy rate.  Env settings are given by the caller."""
import os
import time

import torch

n = 256 << 20
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d.fill_(7)
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
s = torch.cuda.Stream()
torch.cuda.synchronize()
with torch.cuda.stream(s):
    h.copy_(d, non_blocking=True)
s.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(s):
    for _ in range(8):
        h.copy_(d, non_blocking=True)
s.synchronize()
dt = time.perf_counter() - t0
env = {k: v for k, v in os.environ.items() if k.startswith(("HSA_", "GPU_", "ROC_", "DEBUG_CLR"))}
print({"env": env, "GBps": round(8 * n / dt / 1e9, 2)}, flush=True)
