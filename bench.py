#!/usr/bin/env python3
"""Benchmark: encoded megapixels/s of the MI355X JPEG 2000 path (libjp2hip).

Workload (BASELINE.json configs[1], "C2"): a 6000x4000 8-bit RGB TIFF,
lossy 9/7 at 3 bpp with the Bucketeer/Kakadu recipe (6 levels, 6 layers, 512^2
tiles, 64^2 blocks, RPCL, SOP/EPH/PLT, tile-parts per resolution), JPX out.
One step = one batch of full encodes per GPU (--batch images, default one per
in-flight context, 16): TIFF strips already resident in HBM -> JPX bytes in
host memory (ingest, DWT, quantiser, tier-1, PCRD, tier-2) for every image of
the batch; value = megapixels of every image encoded / timed seconds.  Images are independent, so N GPUs run N replicas (weak scaling,
no collective on the data path); the barrier/max are only for timing.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

# (HSA_ENABLE_SDMA is not set: the runtime copies device -> pinned host with
# its blit kernel whatever it says -- profiles/r04/sdma_probe.txt)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jp2-bucketeer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "encoded megapixels/sec (node), lossless 5/3 + lossy 9/7, at 1/2/4/8 MI355X"
HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md chip table (spec)


def dwt_bytes_per_px(C, s, L, e=4):
    """DWT bytes per pixel: level 1 reads the s-byte TIFF samples, level k > 1
    reads the previous LL (4-byte words); each level writes its three high
    bands as e-byte final coefficients and its LL as 4-byte words (the last
    level's LL final, e bytes).  e = 4 is SURVEY.md 8(d)'s B_dwt = C*[s + 4 +
    (8/3)(1 - 4^-(L-1))] (up to the last LL); the DWT writes 16-bit
    quantisation indices (e = 2) wherever every band fits 15 magnitude
    bit-planes (csrc/plan.cpp quant_tab: 8-bit sources, and lossy 16-bit)."""
    b = 0.0
    for k in range(1, L + 1):
        f = 4.0 ** (-(k - 1))  # samples of level k's input, per pixel and component
        b += (s if k == 1 else 4 * f) + f * (0.75 * e + 0.25 * (4 if k < L else e))
    return C * b


def coef_bytes(bits, lossy):
    """Bytes per final coefficient the DWT writes and k_quant reads."""
    return 2 if (bits == 8 or lossy) else 4


def make_image(kind: str, seed: int):
    import imaging as im
    if kind == "c2":
        return im.synth_rgb8(4000, 6000, seed=seed)
    if kind == "c3":
        return im.synth_u16(8000, 10000, comps=3, seed=seed)
    raise ValueError(kind)


def dist_setup(n_gpus):
    """(world, rank, local device) of this process; for N > 1 ranks the
    process group is up and its size checked against --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # single-box rehearsal of the N-rank path: every rank on one GPU
    # (JP2HIP_BENCH_DEVICE=0, with JP2HIP_BENCH_BACKEND=gloo)
    if os.environ.get("JP2HIP_BENCH_DEVICE"):
        local = int(os.environ["JP2HIP_BENCH_DEVICE"])
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("JP2HIP_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend=backend)
        if dist.get_world_size() != n_gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {n_gpus}")
    return world, rank, local


def local_device():
    if os.environ.get("JP2HIP_BENCH_DEVICE"):
        return int(os.environ["JP2HIP_BENCH_DEVICE"])
    return int(os.environ.get("LOCAL_RANK", "0"))


def ranks_seen(world):
    if world <= 1:
        return 1
    import torch.distributed as dist
    return dist.get_world_size()


def barrier_max(world, value, device):
    """Barrier + max over ranks (RCCL all-reduce of one float)."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(world, value, device):
    if world == 1:
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.int64, device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def host_cpu():
    """(cores this process may use, CPU model) of the host the bench runs on:
    the affinity mask, capped by the cgroup CPU quota (a GPU box's share of a
    large host) and OMP_NUM_THREADS when the pool sets it."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            cores = min(cores, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, max(1, int(os.environ["OMP_NUM_THREADS"])))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, model


def cpu_oracle_not_a_reference(img, budget_s=8.0):
    """This repo's own C restatement (oracle/jp2_oracle.c, 1 thread) on a
    1024x2048 crop -- NOT a reference converter, reported for scale only."""
    import oracle_lib as ol
    crop = np.ascontiguousarray(img[:1024, :2048])
    rc = ol.recipe(False)
    t0 = time.perf_counter()
    n = 0
    while True:
        ol.encode(crop, rc)
        n += 1
        if time.perf_counter() - t0 > budget_s or n >= 32:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * crop.shape[0] * crop.shape[1] / 1e6 / dt, 4), "unit": "MP/s", "cores": 1,
            "kind": "not a reference (this repo's C restatement, oracle/jp2_oracle.c)", "seconds": round(dt, 2),
            "sample": f"{n}x encode of a 1024x2048 crop of the C2 image, lossy 9/7 3 bpp, 1 thread"}


def cpu_reference_opj(img):
    """north_star's CPU reference converter: kdu_compress is proprietary and
    absent, so opj_compress (OpenJPEG 2.4.0) with the
    Appendix A mapping of the recipe.  BASELINE.md steps 1-3: the full C2
    image (6000x4000 RGB8, lossy 3 bpp) encoded by `nproc` concurrent
    single-image processes (OpenJPEG's encoder does not scale with -threads),
    on the host cores of this same run; value = images x 24 MP / wall time."""
    import imaging as im
    tool = im.opj("opj_compress")
    if tool is None:
        return None
    cores, model = host_cpu()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "c2.tif")
        with open(src, "wb") as f:
            f.write(im.tiff_bytes(img))
        # -r: rate ratios of the 6 layers, the last = 24 bpp raw / 3 bpp
        cmd = [tool, "-i", src, "-I", "-n", "7", "-t", "512,512", "-b", "64,64", "-p", "RPCL", "-SOP",
               "-EPH", "-PLT", "-TP", "R", "-c",
               "[256,256],[256,256],[128,128],[128,128],[128,128],[128,128],[128,128]",
               "-r", "256,128,64,32,16,8"]
        t0 = time.perf_counter()
        ps = [subprocess.Popen(cmd + ["-o", os.path.join(d, f"o{i}.j2k")], stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL) for i in range(cores)]
        ok = all(p.wait() == 0 for p in ps)
        dt = time.perf_counter() - t0
        nbytes = os.path.getsize(os.path.join(d, "o0.j2k")) if ok else 0
        # one process with every core gives the
        # single-image latency (beside the GPU's config.single_image_latency_ms)
        lat = None
        if ok:
            t0 = time.perf_counter()
            if subprocess.run(cmd + ["-threads", str(cores), "-o", os.path.join(d, "lat.j2k")],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL).returncode == 0:
                lat = time.perf_counter() - t0
    if not ok:
        return None
    mp = cores * img.shape[0] * img.shape[1] / 1e6
    return {"value": round(mp / dt, 3), "unit": "MP/s", "cores": cores, "kind": "reference",
            "tool": "opj_compress 2.4.0 (north_star's stand-in for the proprietary kdu_compress)",
            "cpu_model": model, "seconds": round(dt, 2), "bytes_per_image": nbytes,
            "sample": f"{cores} concurrent processes, each one full 6000x4000 RGB8 C2 image, lossy 3 bpp, "
                      "Appendix A recipe",
            "single_image_latency_ms": round(lat * 1e3, 1) if lat else None,
            "latency_sample": f"one process, -threads {cores}, the same image and recipe"}


def cpu_reference_opj_lossless(crop_h=4096, crop_w=2048):
    """The lossless CPU baseline (the conversion the reference's service runs,
    ImageWorkerVerticle.java:64): opj_compress lossless 5/3 with C3's recipe
    (1024^2 tiles, Appendix A mapping) on a BOUNDED sample -- a 4096x2048 crop
    of the C3 image per process, `nproc` concurrent processes on this run's
    host cores (a full 80 MP C3 image takes opj ~140 s per core, far past the
    bench's budget).  value = processes x crop MP / wall time."""
    import imaging as im
    tool = im.opj("opj_compress")
    if tool is None:
        return None
    cores, model = host_cpu()
    crop = np.ascontiguousarray(make_image("c3", seed=2)[:crop_h, :crop_w])
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "c3crop.tif")
        with open(src, "wb") as f:
            f.write(im.tiff_bytes(crop))
        cmd = [tool, "-i", src, "-n", "7", "-t", "1024,1024", "-b", "64,64", "-p", "RPCL", "-SOP", "-EPH", "-PLT",
               "-TP", "R", "-c", "[256,256],[256,256],[128,128],[128,128],[128,128],[128,128],[128,128]",
               "-r", "64,32,16,8,4,1"]
        t0 = time.perf_counter()
        ps = [subprocess.Popen(cmd + ["-o", os.path.join(d, f"o{i}.j2k")], stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL) for i in range(cores)]
        ok = all(p.wait() == 0 for p in ps)
        dt = time.perf_counter() - t0
    if not ok:
        return None
    mp = cores * crop_h * crop_w / 1e6
    return {"value": round(mp / dt, 3), "unit": "MP/s", "cores": cores, "kind": "reference",
            "tool": "opj_compress 2.4.0 (north_star's stand-in for the proprietary kdu_compress)",
            "cpu_model": model, "seconds": round(dt, 2),
            "sample": f"{cores} concurrent processes, each a {crop_w}x{crop_h} crop of the C3 image "
                      "(RGB16), lossless 5/3, C3 recipe (1024^2 tiles)"}


def cpu_reference_opj_c4():
    """SURVEY.md 8(d) item 3, the C4 CPU baseline: `nproc` concurrent
    opj_compress processes, each one full 5000x7000 RGB8 C4 image (the seed-0
    file, as SURVEY.md 8(d) item 2 runs `nproc` copies),
    lossless 5/3 with the Bucketeer recipe (512^2 tiles, Appendix A) -- one
    image per core of the 10k-row list (the list itself would take hours).
    value = processes x 35 MP / wall time."""
    import imaging as im
    tool = im.opj("opj_compress")
    if tool is None:
        return None
    cores, model = host_cpu()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "c4.tif")
        with open(src, "wb") as f:
            f.write(im.tiff_bytes(im.synth_rgb8(7000, 5000, seed=0)))
        srcs = [src] * cores
        cmd = [tool, "-n", "7", "-t", "512,512", "-b", "64,64", "-p", "RPCL", "-SOP", "-EPH", "-PLT", "-TP", "R",
               "-c", "[256,256],[256,256],[128,128],[128,128],[128,128],[128,128],[128,128]",
               "-r", "64,32,16,8,4,1"]
        t0 = time.perf_counter()
        ps = [subprocess.Popen(cmd + ["-i", srcs[i], "-o", os.path.join(d, f"o{i}.j2k")], stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL) for i in range(cores)]
        ok = all(p.wait() == 0 for p in ps)
        dt = time.perf_counter() - t0
    if not ok:
        return None
    return {"value": round(cores * 35.0 / dt, 3), "unit": "MP/s", "cores": cores, "kind": "reference",
            "tool": "opj_compress 2.4.0 (north_star's stand-in for the proprietary kdu_compress)",
            "cpu_model": model, "seconds": round(dt, 2),
            "sample": f"{cores} concurrent processes, each one full 5000x7000 RGB8 C4 image (the seed-0 file), "
                      "lossless 5/3, Bucketeer recipe"}


def d2h_peak(nbytes=256 << 20, reps=5):
    """Device -> pinned host copy rate (GB/s) on this box: the bound of a
    lossless encode, whose code-stream (~34 bpp for C3) must cross PCIe."""
    import torch
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        h.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
    return best


def h2d_peak(nbytes=256 << 20, reps=5):
    """Pinned host -> device copy rate (GB/s) on this box: the bound of the
    file-to-file span, whose TIFF bytes (72 MB per C2 image) cross PCIe."""
    import torch
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
    return best


def evict_from_page_cache(paths):
    """Drop the files' pages from the page cache (written pages are flushed
    first), so the timed region reads them from the device, not from RAM."""
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN/pmc_traffic.json, made by tests/tools/pmc_summary.py from two
    rocprofv3 --pmc passes of this bench); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    if not files:
        return None, None
    try:
        k = json.load(open(files[-1]))["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None, None
    if not k:
        return None, None
    return k["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def sq_counters(kernel):
    """Occupancy / VALU figures of `kernel` from the newest committed SQ PMC
    summary (profiles/rNN/t1_sq_counters.json, tests/tools/sq_summary.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "t1_sq_counters.json")))
    if not files:
        return None
    try:
        k = json.load(open(files[-1]))["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    if not k:
        return None
    keep = {x: k[x] for x in ("valu_busy", "wait_share", "waves_resident", "SQ_WAVES", "SQ_INSTS_VALU",
                              "SQ_INSTS_SALU", "SQ_INSTS_LDS") if x in k}
    keep["source"] = os.path.relpath(files[-1], ROOT)
    return keep


def run(args):
    import threading

    import torch  # device memory + distributed plumbing only

    import jp2hip
    import imaging as im

    world, rank, local = dist_setup(args.gpus)
    device = f"cuda:{local}"
    torch.cuda.set_device(local)
    img = make_image("c2", seed=1234 + rank)
    tif = im.tiff_bytes(img, rows_per_strip=64)
    lay, offs = jp2hip.tiff_layout(tif)
    d_src = torch.frombuffer(bytearray(tif), dtype=torch.uint8).to(device)
    # the same TIFF in pinned host memory, for the PCIe-inclusive variant
    h_src = torch.frombuffer(bytearray(tif), dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    # `inflight` independent images per GPU, each on its own libjp2hip
    # context (own HIP stream and buffers): the batch path's per-GPU queue.
    # Steps are spread evenly over the contexts (no context does an extra
    # image after the others have drained).
    # a step is one batch of `batch` images (default: one per in-flight
    # context), spread over the contexts from a shared counter
    nf = max(1, args.inflight)
    batch = max(1, args.batch or nf)
    total = args.steps * batch
    host_threads = max(2, 16 // nf)
    prof = os.environ.get("JP2HIP_BENCH_PROFILE", "1") != "0"  # stage times from HIP events (roofline below)
    encs = [jp2hip.Encoder(local, host_threads=host_threads, profile=prof) for _ in range(nf)]
    rc = jp2hip.recipe(jp2hip.LOSSY)
    # every C2 launch's stage times, so the kernel averages cover the same
    # launches a rocprofv3 --kernel-trace of this command sees
    all_stats = []
    for e in encs:
        for _ in range(args.warmup):
            _, st = e.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)
            all_stats.append(st.as_dict())
    # single-image latency (one context, nothing else in flight)
    lat, alone = [], []
    for _ in range(3):
        t = time.perf_counter()
        _, st = encs[0].encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)
        lat.append(time.perf_counter() - t)
        all_stats.append(st.as_dict())
        alone.append(st.as_dict())

    host_delay = float(os.environ.get("JP2HIP_BENCH_HOST_DELAY_MS", "0")) / 1e3

    def timed(encode):
        """K steps over the contexts from a shared counter; (seconds, stats)."""
        stages, errors = [], []
        nxt = [0]
        mu = threading.Lock()

        def worker(k):
            try:
                while True:
                    with mu:
                        step = nxt[0]
                        nxt[0] += 1
                    if step >= total:
                        return
                    out, st = encode(encs[k])
                    if host_delay:  # experiment only: a longer host turnaround per encode
                        time.sleep(host_delay)
                    # the file stays in the library's pinned buffer (no copy
                    # into a Python bytes object); check it ends in EOC.  The
                    # stats stay ctypes structs until the timed region ends:
                    # the Python work between two encodes holds the GIL the
                    # other 15 workers need
                    ok = out.tail(2) == b"\xff\xd9"
                    out.close()
                    if not ok:
                        raise RuntimeError("encode output does not end in EOC")
                    stages.append(st)  # (list.append is atomic under the GIL)
            except Exception as ex:  # surfaced after the timed region
                errors.append(ex)

        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=worker, args=(k,)) for k in range(nf)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        barrier(world)
        dt = time.perf_counter() - t0
        if errors:
            raise errors[0]
        return dt, [s.as_dict() for s in stages]

    # the contract's value: TIFF resident in HBM -> JPX bytes in host memory
    dt, stages = timed(lambda e: e.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc, copy=False))
    dt_max = barrier_max(world, dt, device)
    mp = img.shape[0] * img.shape[1] / 1e6
    value = world * mp * total / dt_max
    # PCIe-inclusive: TIFF bytes in pinned host memory -> jp2hip_encode_tiff
    # (header parse, H2D of the 72 MB file, encode) -> JPX bytes in host memory
    dt_h_max = None
    if not args.no_pcie:
        dt_h, _ = timed(lambda e: e.encode_tiff_ptr(h_src.data_ptr(), h_src.numel(), jp2hip.LOSSY, rc, copy=False))
        dt_h_max = barrier_max(world, dt_h, device)
    res = None
    if rank == 0:
        flat = stages
        avg = {k: float(np.mean([s[k] for s in flat])) for k in flat[0]}
        every = flat + all_stats
        avg_all = {k: float(np.mean([s[k] for s in every])) for k in every[0]}
        # the dominant kernel by rocprofv3 kernel time (~60 % of all kernel
        # time, profiles/r02/final/kernel_stats_*.csv): k_t1_mq, timed with
        # HIP events on its context's stream around the launch (what
        # rocprofv3's dispatch duration measures; under load that includes
        # waiting for CUs other images hold), averaged over every launch of
        # this run
        dom = "k_t1_mq"
        C, L = 3, 6
        npx = img.shape[0] * img.shape[1]
        # algorithmic bytes per k_t1_mq launch: it reads one decision-stream
        # byte per MQ decision and writes the MQ code bytes (the per-pass
        # counts / distortions it also reads are < 1 %)
        mq_alg = avg_all["mq_decisions"] + avg_all["t1_bytes"]
        ach = mq_alg / (avg_all["t1_mq_ms"] * 1e-3) / 1e9 if avg_all["t1_mq_ms"] > 0 else 0.0
        ce = coef_bytes(8, True)
        dwt_alg = dwt_bytes_per_px(C, 1, L, ce) * npx
        dwt_alone = float(np.mean([x["dwt_ms"] for x in alone]))
        traffic, traffic_src = pmc_traffic(dom)
        # SURVEY.md 8(d) full path: B_path = B_dwt + (coefficient read) C +
        # 3*bpp/8 per pixel (4C there: 4-byte coefficients)
        bpp = 8 * avg["out_bytes"] / npx
        b_path = dwt_bytes_per_px(C, 1, L, ce) + ce * C + 3 * bpp / 8
        px_per_s_gpu = value / world * 1e6
        res = {
            "metric": METRIC, "value": round(value, 3), "unit": "MP/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt_max * 1e3 / args.steps, 3),
            "images_per_step": batch,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32+i32",
            "data": "synthetic (sinusoids + checker + N(0,6) noise, seed 1234+rank), in-memory baseline TIFF",
            "config": {"workload": "C2: 6000x4000 RGB8 TIFF -> JPX, lossy 9/7 3 bpp, Kakadu recipe "
                                   "(6 levels, 6 layers, 512^2 tiles, 64^2 blocks, RPCL, SOP/EPH/PLT, TP=R)",
                       "image": "6000x4000x3 u8", "step": f"one batch of {batch} C2 images per GPU",
                       "images_per_step": batch, "images_in_flight_per_gpu": nf, "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "timed_span": "TIFF resident in HBM -> JPX bytes in host memory (jp2hip_encode_device; "
                                     "the file is left in the library's pinned buffer, not copied into Python)",
                       "parallelism": f"replicas x{world}", "ranks_in_process_group": ranks_seen(world),
                       "out_bytes": int(avg["out_bytes"]),
                       "bpp": round(8 * avg["out_bytes"] / npx, 4),
                       "single_image_latency_ms": round(1e3 * min(lat), 3),
                       "host_waits_per_encode": int(max(a["host_waits"] for a in alone)),
                       "rate_iterations": int(max(a["rate_iterations"] for a in alone))},
            # the same steps with the TIFF in pinned host memory and the H2D
            # inside the timed span (PCIe-inclusive rate)
            "value_pcie_inclusive": ({"value": round(world * mp * total / dt_h_max, 3), "unit": "MP/s",
                                      "ms_per_step": round(dt_h_max * 1e3 / args.steps, 3),
                                      "timed_span": "TIFF bytes in pinned host memory -> jp2hip_encode_tiff (parse, "
                                                    "H2D, encode) -> JPX bytes in host memory"}
                                     if dt_h_max else None),
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2),
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": round(ach * 1e9 / HBM_PEAK, 5),
                         "traffic": round(traffic) if traffic is not None else None,
                         "traffic_source": traffic_src,
                         "alg_bytes_per_launch": int(mq_alg),
                         "alg_bytes_def": "decision-stream bytes read (1 per MQ decision) + MQ code bytes written",
                         "avg_launch_ms": round(avg_all["t1_mq_ms"], 4), "launches_averaged": len(every),
                         "mq_decisions_per_launch": int(avg_all["mq_decisions"]),
                         "note": "tier-1 MQ is a serial dependency chain per code-block: latency-bound; "
                                 "its byte roofline is tiny by nature (SURVEY.md 8(d))"},
            "roofline_path": {"bound": "hbm", "bytes_per_px": round(b_path, 3),
                              "achieved": round(b_path * px_per_s_gpu / 1e9, 2), "peak": HBM_PEAK / 1e9,
                              "unit": "GB/s", "frac": round(b_path * px_per_s_gpu / HBM_PEAK, 5)},
            # DWT stage time from HIP events on the context's stream: under
            # load (the event span includes waiting for CUs other images
            # hold) and alone (one image on the GPU)
            "roofline_dwt": ({"bound": "hbm", "achieved": round(dwt_alg / (avg["dwt_ms"] * 1e-3) / 1e9, 2),
                             "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                             "frac": round(dwt_alg / (avg["dwt_ms"] * 1e-3) / HBM_PEAK, 5),
                             "alg_bytes_per_px": round(dwt_bytes_per_px(C, 1, L, ce), 3),
                             "coef_bytes": ce,
                             "stage_ms": round(avg["dwt_ms"], 4),
                             "alone": {"stage_ms": round(dwt_alone, 4),
                                       "achieved": round(dwt_alg / (dwt_alone * 1e-3) / 1e9, 2),
                                       "frac": round(dwt_alg / (dwt_alone * 1e-3) / HBM_PEAK, 5)}}
                             if avg["dwt_ms"] > 0 and dwt_alone > 0 else None),
            # SQ counters are per launch (one launch per image: sq_summary.py
            # averages the rocprofv3 --pmc rows over the launches)
            "t1_counters": {"units": "per kernel launch (one per image)",
                            "k_t1_mq": sq_counters("k_t1_mq"), "k_t1_cm3": sq_counters("k_t1_cm3"),
                            "k_quant": sq_counters("k_quant")},
            "stages_ms": {k: round(avg[k], 4) for k in ("ingest_ms", "dwt_ms", "quant_ms", "t1_cm_ms",
                                                        "t1_mq_ms", "pcrd_ms", "d2h_ms", "t2_ms",
                                                        "total_ms")},
            "t1": {"codeblocks": int(avg["codeblocks"]), "coded_passes": int(avg["coded_passes"]),
                   "mq_bytes": int(avg["t1_bytes"]), "mq_decisions": int(avg["mq_decisions"])},
        }
    if rank == 0:
        res["validation"] = validate_c2(encs[0], d_src, lay, rc, img, rank)
    for e in encs[1:]:  # their HBM and streams back before the lossless legs
        e.close()
    return res, img, world, rank, encs[0]


def validate_c2(enc, d_src, lay, rc, img, rank):
    """validation (decode and compare) is mandatory but not
    timed.  One more encode of the bench image after the timed region: its
    code-stream against the oracle's SHA-256 committed for this image
    (tests/golden/golden.json c2_synth_rgb8_6000x4000, seed 1234 -- rank 0's
    image), and its opj_decompress decode against the pixels (PSNR)."""
    import hashlib

    import jp2hip
    import imaging as im
    got, _ = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)
    cs = im.codestream(got)
    sha = hashlib.sha256(cs).hexdigest()
    out = {"codestream_bytes": len(cs), "codestream_sha256": sha, "equals_oracle_sha256": None, "psnr_db": None,
           "oracle_psnr_db": None, "golden": "tests/golden/golden.json c2_synth_rgb8_6000x4000"}
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            g = [x for x in json.load(f)["lossy"] if x["name"] == "c2_synth_rgb8_6000x4000"][0]
        if rank == 0:
            out["equals_oracle_sha256"] = sha == g["oracle_sha256"]
        out["oracle_psnr_db"] = g.get("oracle_psnr")
    except (OSError, KeyError, IndexError, ValueError):
        pass
    try:
        out["psnr_db"] = round(im.psnr(im.decode_opj(got), img, 8), 4)
    except Exception as ex:  # the decoder is a check, not the product: record why it is absent
        out["psnr_db"] = f"not decoded: {ex}"
    return out


C5 = {"w": 40000, "h": 30000, "levels": 7, "tile": 512, "rps": 64, "seed": 5}


def c5_band(rank, world, threads=16):
    """This rank's band of the C5 image as TIFF strips (generated strip by
    strip, never whole in RAM): (bytes, Layout, offsets keep-alive, rows)."""
    from concurrent.futures import ThreadPoolExecutor
    from ctypes import POINTER, c_uint64, cast

    import imaging as im
    import jp2hip
    from jp2hip import split as js
    from jp2hip._lib import Layout
    w, h, rps = C5["w"], C5["h"], C5["rps"]
    # the band the encoder reads: its own recipe's tile height and flush period
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=C5["levels"])
    r0, r1 = js.split_rows(h, rc.tile_h, rank, world, rc.flush_period)
    buf = np.empty((r1 - r0, w), "<u2")
    groups = list(range(r0, r1, C5["tile"]))

    def fill(g):
        e = min(r1, g + C5["tile"])
        buf[g - r0:e - r0] = im.synth_gray16_rows(g, e, w, seed=C5["seed"], band=C5["tile"])

    with ThreadPoolExecutor(max(1, threads)) as ex:
        list(ex.map(fill, groups))
    nstrips = (h + rps - 1) // rps
    offs = (c_uint64 * nstrips)()
    for s in range(r0 // rps, (r1 + rps - 1) // rps):
        offs[s] = (s * rps - r0) * w * 2
    lay = Layout(w, h, 1, 16, 1, 0, rps, nstrips, cast(offs, POINTER(c_uint64)))
    return buf.tobytes(), lay, offs, (r0, r1)


def run_c4(args):
    """C4 (configs[3]) at reduced size: a Bucketeer batch CSV of synthetic
    5000x7000 RGB8 TIFFs (cycling over a few distinct files, as SURVEY.md 8(d)
    prescribes for the 10k-row batch), lossless (ImageWorker hard-codes it),
    through one GPU's native batch queue per rank: TIFF read -> encode -> JPX
    write -> stub upload (reads every byte) -> delete.  The timed span runs from
    the first submit to the last upload, file I/O included; rows are pulled
    by the ranks from one shared claim counter (work stealing through the
    process group's store; no collective on the data path)."""
    import csv as _csv
    import shutil

    import imaging as im
    from jp2hip import batch as jb

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # single-box rehearsal of the N-rank path: every rank on one GPU
    # (JP2HIP_BENCH_DEVICE=0, with JP2HIP_BENCH_BACKEND=gloo)
    if os.environ.get("JP2HIP_BENCH_DEVICE"):
        local = int(os.environ["JP2HIP_BENCH_DEVICE"])
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    work = tempfile.mkdtemp(prefix=f"jp2hip_c4_{rank}_")
    try:
        ndistinct, rows = 4, args.steps
        paths = []
        for i in range(ndistinct):
            pth = os.path.join(work, f"synth{i:02d}.tif")
            with open(pth, "wb") as f:
                f.write(im.tiff_bytes(im.synth_rgb8(7000, 5000, seed=i), rows_per_strip=64))
            paths.append(pth)
        csv_path = os.path.join(work, "batch.csv")
        with open(csv_path, "w", newline="", encoding="utf-8") as f:
            wr = _csv.writer(f)
            wr.writerow(["Item ARK", "File Name"])
            for i in range(rows * world):
                wr.writerow([f"ark:/99999/synth{i:05d}", os.path.basename(paths[i % ndistinct])])
        items = jb.read_batch_csv(csv_path, path_prefix=work)
        # rows go to the ranks by work stealing: each rank's queue pulls the
        # next unclaimed row from the process group's store (an atomic add;
        # no data-path collective), so a faster GPU takes more rows
        claims = None
        if world > 1:
            from torch.distributed import distributed_c10d as c10d
            claims = jb.StoreClaims(c10d._get_default_store(), len(items), key="jp2hip/c4/next")
        out_dir = os.path.join(work, "out")
        os.makedirs(out_dir, exist_ok=True)
        with jb.BatchQueue(device=local, reader_threads=6, uploader_threads=8) as q:
            # warm-up: one image per context, so device buffers exist
            for k, it in enumerate(items[:12]):
                q.submit(-1 - k, it.image_id, it.tiff, os.path.join(out_dir, "warm%d.jpx" % k))
            q.drain()
            evict_from_page_cache(paths)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            res = jb.run_batch_dynamic(items, out_dir, [q], claims=claims, depth=32)
            dt = time.perf_counter() - t0
        ok = sum(1 for r in res if r["status"] == 0)
        mp = 5000 * 7000 / 1e6 * ok
        rows_by_rank = [ok]
        if world > 1:
            import torch
            t = torch.tensor([dt, mp], dtype=torch.float64)
            dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
            dt, mp = float(t[0]), float(t[1])
            per = torch.zeros(world, dtype=torch.int64)
            per[rank] = ok
            dist.all_reduce(per, op=dist.ReduceOp.SUM)  # (bookkeeping after the timed region)
            rows_by_rank = [int(x) for x in per]
            dist.destroy_process_group()
        if rank != 0:
            return None
        return {"metric": METRIC, "value": round(mp / dt, 3), "unit": "MP/s", "n_gpus": world,
                "steps": rows, "warmup": 1, "ms_per_step": round(dt * 1e3 / rows, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "i32",
                "data": f"synthetic 5000x7000 RGB8 TIFFs ({ndistinct} distinct, seeds 0..{ndistinct - 1}) on local "
                        "disk, evicted from the page cache before the timed region",
                "config": {"workload": "C4: Bucketeer batch CSV -> per-GPU native queue (read, lossless 5/3 encode, "
                                       "JPX write, stub upload, delete-after-upload), Kakadu recipe",
                           "rows_per_gpu": rows, "images_ok": sum(rows_by_rank), "rows_by_rank": rows_by_rank,
                           "parallelism": f"work stealing x{world}",
                           "ranks_in_process_group": world}}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def run_c5(args):
    """C5 (configs[4]): one 40000x30000 Gray16 image, lossy 9/7 3 bpp, 7
    levels, tile-split across the ranks (jp2hip.split).  One step = the whole
    image encoded once by all ranks together (strong scaling: total work is
    fixed).  The exchange is RCCL all-reduces of <= 64 int64 (PCRD threshold
    bisection, sizes); no pixel crosses GPUs."""
    import torch

    import jp2hip
    from jp2hip import split as js

    world, rank, local = dist_setup(args.gpus)
    device = f"cuda:{local}"
    torch.cuda.set_device(local)
    band, lay, offs, rows = c5_band(rank, world)
    d_src = torch.frombuffer(bytearray(band) if band else bytearray(1), dtype=torch.uint8).to(device)
    torch.cuda.synchronize()
    enc = jp2hip.Encoder(local, host_threads=16, profile=True)
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=C5["levels"])
    group = js.TorchGroup() if world > 1 else js.SingleGroup()

    def step():
        return enc.encode_device_split(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, group.split(), rc)

    for _ in range(args.warmup):
        part, off, flen, st = step()
    identical = None
    if world == 1:  # the split path at world 1 must be the single-image encode
        single, _ = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)
        identical = single == part
        if not identical:
            raise SystemExit("C5: split encode differs from the single-image encode")
    barrier(world)
    torch.cuda.synchronize()
    stats = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        part, off, flen, st = step()
        stats.append(st.as_dict())
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    dt_max = barrier_max(world, dt, device)
    npx = C5["w"] * C5["h"]
    value = npx / 1e6 * args.steps / dt_max
    # the parts tile the file: their sizes add up to its length on every rank
    parts_total = allreduce_sum(world, len(part), device)
    if parts_total != flen:
        raise SystemExit(f"C5: parts add up to {parts_total} bytes, file length {flen}")
    if rank != 0:
        return None
    avg = {k: float(np.mean([s[k] for s in stats])) for k in stats[0]}
    dwt_alg = dwt_bytes_per_px(1, 2, C5["levels"], coef_bytes(16, True)) * (rows[1] - rows[0]) * C5["w"]
    return {
        "metric": METRIC, "value": round(value, 3), "unit": "MP/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt_max * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32+i32",
        "data": "synthetic Gray16 (sinusoids + N(0,400), seed 5 per 512-row band), generated per rank band",
        "config": {"workload": "C5: 40000x30000 Gray16 -> JPX, lossy 9/7 3 bpp, 7 levels, 6 layers, 512^2 tiles, "
                               "tile-split across ranks (bands of tile rows, RCCL all-reduce of PCRD sums)",
                   "image": "40000x30000x1 u16", "parallelism": f"tile-split x{world}",
                   "file_bytes": int(flen), "bpp": round(8 * flen / npx, 4),
                   "rank0_rows": list(rows), "rank0_part_bytes": len(part), "parts_total_bytes": parts_total,
                   "backend": os.environ.get("JP2HIP_BENCH_BACKEND", "nccl") if world > 1 else None,
                   "ranks_in_process_group": ranks_seen(world)},
        "roofline_dwt": {"bound": "hbm", "achieved": round(dwt_alg / (avg["dwt_ms"] * 1e-3) / 1e9, 2),
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": round(dwt_alg / (avg["dwt_ms"] * 1e-3) / HBM_PEAK, 5),
                         "alg_bytes_per_px": round(dwt_bytes_per_px(1, 2, C5["levels"], coef_bytes(16, True)), 3)},
        "stages_ms_rank0": {k: round(avg[k], 4) for k in ("ingest_ms", "dwt_ms", "quant_ms", "t1_cm_ms",
                                                          "t1_mq_ms", "pcrd_ms", "d2h_ms", "t2_ms", "total_ms")},
        "rate_iterations": int(avg["rate_iterations"]),
        "split_equals_single_encode": identical,
    }


def spawn_ranks(n):
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the environment):
    start N rank processes through torch.distributed.run, before anything here
    touches a GPU, and exit with their status (a child process, not an exec)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--inflight", type=int, default=int(os.environ.get("JP2HIP_INFLIGHT", "16")),
                    help="independent images in flight per GPU (separate contexts/streams)")
    ap.add_argument("--batch", type=int, default=0,
                    help="images per step (default: --inflight); value = MP of every image / time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lossless", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive C2 leg")
    ap.add_argument("--no-extras", action="store_true",
                    help="C2 timed leg only: no PCIe-inclusive leg, lossless C3/C4, file-span, C5 or CPU "
                         "baselines (the profiled configuration)")
    ap.add_argument("--workload", choices=("c2", "c4", "c5"), default="c2",
                    help="c2: the headline (replicas); c4: CSV batch through the native per-GPU queue; "
                         "c5: one oversized image tile-split across ranks")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.no_extras:
        args.no_pcie = args.no_lossless = args.no_cpu_baseline = True
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}")
    # one hardware queue per in-flight context plus a few for the runtime's
    # own streams: with HIP's default of 4 (exported as such on the GPU
    # boxes) the 12 contexts share 4 queues, and the kernels of a shared
    # queue run one at a time -- the tier-1 MQ kernel (few waves, long) then
    # runs alone for a fifth of the time.  The deployment sets the same for
    # the Bucketeer JVM.  Must be set before anything
    # initialises HIP.  Sweep: profiles/r02/hwq_sweep.txt
    if not os.environ.get("JP2HIP_KEEP_HW_QUEUES"):
        os.environ["GPU_MAX_HW_QUEUES"] = str(max(4, min(32, args.inflight + 4)))
    if args.workload == "c4":
        res = run_c4(args)
        if res is not None:
            print(json.dumps(res), flush=True)
        return
    if args.workload == "c5":
        res = run_c5(args)
        if res is not None:
            print(json.dumps(res), flush=True)
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    res, img, world, rank, enc = run(args)
    if rank == 0 and world == 1:
        if not args.no_lossless:
            res["lossless_c3"] = lossless_c3(enc)
            if not args.no_extras:
                res["lossless_c3"]["value_file_span"] = c3_file_span(local_device())
            res["lossless_c4"] = lossless_c4(local_device())
        if not args.no_extras:
            res["value_file_span"] = c2_file_span(local_device())
            res["c5"] = c5_single_gpu(enc)
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_reference_opj(img)
            res["cpu_baseline_lossless"] = cpu_reference_opj_lossless()
            res["cpu_baseline_c4"] = cpu_reference_opj_c4()
            if res.get("lossless_c4") and res["cpu_baseline_c4"]:
                res["lossless_c4"]["vs_cpu_baseline_c4"] = round(
                    res["lossless_c4"]["mp_per_s"] / res["cpu_baseline_c4"]["value"], 2)
            if res.get("lossless_c3") and res["cpu_baseline_lossless"]:
                res["lossless_c3"]["vs_cpu_baseline_lossless"] = round(
                    res["lossless_c3"]["mp_per_s_inflight_c_api"] / res["cpu_baseline_lossless"]["value"], 2)
            res["cpu_not_a_reference"] = cpu_oracle_not_a_reference(img)
    if rank == 0:
        import jp2hip
        res["dma_engines"] = jp2hip._lib.dma_engines()  # engine choice differs per box: record it
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def lossless_c3(enc, steps=2, inflight=12, n_each=8):
    """C3 (configs[2]): 10000x8000 RGB16 lossless 5/3, 1024^2 tiles, the
    conversion the reference's service runs (ImageWorkerVerticle.java:64).
    One image alone (latency at the C call) and `inflight` images at once on
    separate contexts (throughput): TIFF resident in HBM -> JPX bytes in host
    memory, timed around the C calls, the file left in the library's pinned
    buffer (no Python copy); each context's code-stream D2H overlaps the
    other contexts' kernels."""
    import threading

    import torch

    import jp2hip
    import imaging as im
    img = make_image("c3", seed=2)
    tif = im.tiff_bytes(img, rows_per_strip=64)
    lay, offs = jp2hip.tiff_layout(tif)
    d_src = torch.frombuffer(bytearray(tif), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    rc = jp2hip.recipe(jp2hip.LOSSLESS, tile_w=1024, tile_h=1024)
    out, st = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSLESS, rc, copy=False)
    out.close()
    lat = []
    for _ in range(steps):
        t0 = time.perf_counter()
        out, st = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSLESS, rc, copy=False)
        lat.append(time.perf_counter() - t0)
        nbytes = len(out)
        out.close()
    npx = img.shape[0] * img.shape[1]
    bpp = 8 * nbytes / npx
    res = {"workload": "C3: 10000x8000 RGB16 lossless 5/3, 1024^2 tiles", "bpp": round(bpp, 4),
           "ms_c_api": round(1e3 * min(lat), 2), "mp_per_s_c_api": round(npx / 1e6 / min(lat), 3),
           "stages_ms": {k: round(v, 3) for k, v in st.as_dict().items() if k.endswith("_ms")}}
    encs = [enc] + [jp2hip.Encoder(torch.cuda.current_device(), host_threads=4, profile=True)
                    for _ in range(inflight - 1)]
    errors = []

    def work(e, n):
        try:
            for _ in range(n):
                o, _ = e.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSLESS, rc, copy=False)
                o.close()
        except Exception as ex:
            errors.append(ex)

    def round_(n):
        th = [threading.Thread(target=work, args=(e, n)) for e in encs]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errors:
            raise errors[0]

    # warm-up: every context at once, so the library's pinned output pool
    # holds `inflight` buffers of this size before the timed region (a cold
    # pool pins ~390 MB per first encode inside it: hipHostMalloc stalls the
    # caller for tens of ms -- gpurun_out/c3prof, 50-290 ms before k_t2_tp_emit)
    # (two rounds: the first call of a process measured 3-8 % below a repeat
    # after one, gpurun_out/r06_c3each; the timed window is 8 images per
    # context, 96 in all, so its ramp and tail are a small part of it)
    round_(1)
    round_(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    round_(n_each)
    dt = time.perf_counter() - t0
    value = npx / 1e6 * n_each * inflight / dt
    # SURVEY.md 8(d) full path at the measured bpp: B_dwt + 4C + 3 bpp / 8
    b_path = dwt_bytes_per_px(3, 2, 6, coef_bytes(16, False)) + coef_bytes(16, False) * 3 + 3 * bpp / 8
    # the bound that matters for lossless: every code-stream byte (~34 bpp
    # for C3) crosses PCIe to the host; device->pinned-host peak measured here
    d2h = d2h_peak()
    out_gbs = value * 1e6 * bpp / 8 / 1e9
    res.update({"inflight": inflight, "images": n_each * inflight, "mp_per_s_inflight_c_api": round(value, 3),
                "roofline_pcie": {"bound": "pcie_d2h", "achieved": round(out_gbs, 2), "peak": round(d2h, 2),
                                  "unit": "GB/s", "frac": round(out_gbs / d2h, 4),
                                  "def": "code-stream bytes/s leaving the GPU (MP/s x bpp / 8) / measured "
                                         "device->pinned-host copy rate"},
                "roofline_path": {"bound": "hbm", "bytes_per_px": round(b_path, 3),
                                  "achieved": round(b_path * value * 1e6 / 1e9, 2), "peak": HBM_PEAK / 1e9,
                                  "unit": "GB/s", "frac": round(b_path * value * 1e6 / HBM_PEAK, 5),
                                  "note": "not the bound of a lossless encode: see roofline_pcie"}})
    for e in encs[1:]:
        e.close()
    # SURVEY.md 8(d) validation, untimed: one more encode against the SHA-256
    # of the oracle's file for this image (tests/golden/make_golden.py c3_full)
    import hashlib
    got, _ = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSLESS, rc)
    val = {"bytes": len(got), "sha256": hashlib.sha256(got).hexdigest(), "equals_oracle_sha256": None,
           "golden": "tests/golden/golden.json c3_full"}
    del got
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            val["equals_oracle_sha256"] = val["sha256"] == json.load(f)["c3_full"]["oracle_sha256"]
    except (OSError, KeyError, ValueError):
        pass
    res["validation"] = val
    return res


def golden_sha(which):
    """The oracle's SHA-256 for a bench image from tests/golden/golden.json
    (committed fixtures; None when absent): "c2" (its code-stream), "c3" and
    "c4" (the whole file)."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            g = json.load(f)
        if which == "c2":
            return [x for x in g["lossy"] if x["name"] == "c2_synth_rgb8_6000x4000"][0]["oracle_sha256"]
        if which == "c3":
            return g["c3_full"]["oracle_sha256"]
        if which == "c4":
            return [x for x in g["lossless"] if x["name"] == "c4_synth_rgb8_5000x7000_seed0_jpx"][0]["oracle_sha256"]
    except (OSError, KeyError, IndexError, ValueError):
        return None
    return None


def c4_batch(device, rows=16, ndistinct=2, contexts=8, conversion=None, make=None, reader_threads=4,
             uploader_threads=4, shape=(7000, 5000), gen_threads=8, rcp=None, busy=None, validate=None):
    """C4 (configs[3]) on one GPU: a Bucketeer batch CSV of `rows` synthetic
    5000x7000 RGB8 TIFFs (cycling over `ndistinct` files, as SURVEY.md 8(d)
    prescribes for the 10k-row batch) through the native batch queue: TIFF
    read from disk -> lossless encode -> JPX write -> stub upload (reads every
    byte) -> delete.  The files are evicted from the page cache before the
    timed region (POSIX_FADV_DONTNEED), which runs from the first submit to
    the last upload, file I/O included; rows beyond the first `ndistinct`
    re-read files the first pass left in the page cache.  `rcp`: the recipe
    of every row (None: the Bucketeer recipe of the conversion).  `busy`
    (a dict) receives the stages' busy fractions over the timed span: each
    stage's summed per-image time / (its threads x span).  `validate` (a
    dict with "golden": a golden_sha() name) receives, untimed, the SHA-256
    of the first distinct file's JPX from one more pass through a queue that
    keeps its output, and whether it equals the oracle's.  Returns (MP/s,
    seconds, results, bytes of TIFF read)."""
    import csv as _csv
    import shutil
    from concurrent.futures import ThreadPoolExecutor

    import imaging as im
    import jp2hip
    from jp2hip import batch as jb
    conv = jp2hip.LOSSLESS if conversion is None else conversion
    make = make or (lambda i: im.synth_rgb8(7000, 5000, seed=i))
    work = tempfile.mkdtemp(prefix="jp2hip_c4_")
    try:
        def gen(i):
            pth = os.path.join(work, f"synth{i:02d}.tif")
            with open(pth, "wb") as f:
                f.write(im.tiff_bytes(make(i), rows_per_strip=64))
            return pth

        with ThreadPoolExecutor(min(ndistinct, gen_threads)) as ex:
            paths = list(ex.map(gen, range(ndistinct)))
        sizes = {p: os.path.getsize(p) for p in paths}
        csv_path = os.path.join(work, "batch.csv")
        with open(csv_path, "w", newline="", encoding="utf-8") as f:
            wr = _csv.writer(f)
            wr.writerow(["Item ARK", "File Name"])
            for i in range(rows):
                wr.writerow([f"ark:/99999/synth{i:05d}", os.path.basename(paths[i % ndistinct])])
        items = jb.read_batch_csv(csv_path, path_prefix=work)
        out_dir = os.path.join(work, "out")
        os.makedirs(out_dir, exist_ok=True)
        with jb.BatchQueue(device=device, contexts=contexts, reader_threads=reader_threads,
                           uploader_threads=uploader_threads) as q:
            # warm-up: every context's device buffers, and the pinned host
            # buffers of a full pipeline -- files read ahead, in the contexts,
            # queued for and in the uploaders (pinning a 480 MB C3 buffer took
            # 16-500 ms; without this the first rows of the timed region
            # pinned them)
            nwarm = 2 * contexts + reader_threads + uploader_threads
            for k in range(nwarm):
                it = items[k % len(items)]
                q.submit(-1 - k, it.image_id, it.tiff, os.path.join(out_dir, "warm%d.jpx" % k), conv, rcp)
            q.drain()
            evict_from_page_cache(paths)
            t0 = time.perf_counter()
            for it in items:
                q.submit(it.job, it.image_id, it.tiff, os.path.join(out_dir, jb.jpx_name(it.image_id)), conv, rcp)
            res = q.drain()
            dt = time.perf_counter() - t0
        if validate is not None:  # decode-and-compare, untimed
            import hashlib
            vout = os.path.join(out_dir, "validate.jpx")
            with jb.BatchQueue(device=device, contexts=1, reader_threads=1, uploader_threads=1,
                               delete_after_upload=False) as vq:
                vq.submit(-1, "validate", paths[0], vout, conv, rcp)
                vres = vq.drain()
            sha = None
            if vres and vres[0]["status"] == 0 and os.path.exists(vout):
                with open(vout, "rb") as f:
                    data = f.read()
                sha = hashlib.sha256(im.codestream(data) if validate.get("golden") == "c2" else data).hexdigest()
            want = golden_sha(validate.get("golden"))
            validate.update({"file": "the first distinct file (row 0) through a one-context queue that keeps its "
                                     "output", "sha256": sha,
                             "equals_oracle_sha256": (sha == want) if (sha and want) else None})
        ok = sum(1 for r in res if r["status"] == 0)
        if busy is not None:
            busy.update({
                "readers": round(sum(r["read_ms"] for r in res) / 1e3 / (reader_threads * dt), 3),
                "contexts": round(sum(r["encode_ms"] for r in res) / 1e3 / (contexts * dt), 3),
                "uploaders": round(sum(r["upload_ms"] for r in res) / 1e3 / (uploader_threads * dt), 3),
                "def": "summed per-image stage time / (stage threads x timed span); a stage near 1.0 is the "
                       "bound (contexts: host time from a context taking the image to its JPX bytes in host "
                       "memory, GPU work and waits included)"})
        read = sum(sizes[paths[i % ndistinct]] for i in range(rows))
        return shape[0] * shape[1] / 1e6 * ok / dt, dt, res, read
    finally:
        shutil.rmtree(work, ignore_errors=True)


def lossless_c4(device, rows=10000, ndistinct=16, sweep=(8, 12, 16), sweep_rows=512):
    """a 10 000-row CSV (16 distinct files of seeds 0-15;
    the survey's 64 would be 6.7 GB of fixtures per bench run), 12 contexts
    (the queue's default), plus a shorter sweep over the context count with
    each stage's busy fraction, which names the bound."""
    busy = {}
    # 6 readers / 8 uploaders: with 4 uploaders (the queue's default) the
    # upload stage -- JPX write, stub read-back, delete -- is the bound
    # (busy 0.95-1.0; profiles/r06/c4_sweep.jsonl), with 8 the contexts are
    val = {"golden": "c4"}
    value, dt, res, read = c4_batch(device, rows=rows, ndistinct=ndistinct, contexts=12, busy=busy,
                                    reader_threads=6, uploader_threads=8, validate=val)
    ok = [r for r in res if r["status"] == 0]
    peak_h2d = h2d_peak()
    sweep_res = []
    for c in sweep:
        b = {}
        v, d, rr, rd = c4_batch(device, rows=sweep_rows, ndistinct=ndistinct, contexts=c, busy=b,
                                reader_threads=6, uploader_threads=8)
        sweep_res.append({"contexts": c, "mp_per_s": round(v, 3), "seconds": round(d, 3),
                          "tiff_read_gb_per_s": round(rd / d / 1e9, 2),
                          "jpx_gb_per_s": round(sum(r["out_bytes"] for r in rr) / d / 1e9, 2), "busy": b})
    bpp = 8 * float(np.mean([r["out_bytes"] for r in ok])) / (5000 * 7000) if ok else 0.0
    b_path = dwt_bytes_per_px(3, 1, 6, coef_bytes(8, False)) + coef_bytes(8, False) * 3 + 3 * bpp / 8
    return {"workload": f"C4: Bucketeer batch CSV of 5000x7000 RGB8 TIFFs ({ndistinct} distinct, seeds 0-"
                        f"{ndistinct - 1}) -> native per-GPU queue (disk read, lossless 5/3 encode, JPX write, "
                        "stub upload, delete)",
            "rows": rows, "distinct_files": ndistinct, "contexts": 12, "reader_threads": 6, "uploader_threads": 8,
            "page_cache": f"the {ndistinct} files are evicted before the timed region; rows after the first "
                          f"{ndistinct} re-read them from the page cache",
            "images_ok": len(ok), "mp_per_s": round(value, 3), "seconds": round(dt, 3),
            "bpp": round(bpp, 4), "timed_span": "first submit -> last upload, file I/O included",
            "busy": busy, "validation": val,
            "roofline_pcie": {"bound": "pcie_h2d", "achieved": round(read / dt / 1e9, 2), "peak": round(peak_h2d, 2),
                              "unit": "GB/s", "frac": round(read / dt / 1e9 / peak_h2d, 4),
                              "def": "TIFF bytes read per second (every byte is uploaded) / measured pinned "
                                     "host->device copy rate"},
            "contexts_sweep": sweep_res,
            "roofline_path": {"bound": "hbm", "bytes_per_px": round(b_path, 3),
                              "achieved": round(b_path * value * 1e6 / 1e9, 2), "peak": HBM_PEAK / 1e9,
                              "unit": "GB/s", "frac": round(b_path * value * 1e6 / HBM_PEAK, 5)}}


def c2_file_span(device, images=1024, contexts=16, ndistinct=16):
    """SURVEY.md 8(d)'s span for the headline workload: C2 (lossy 3 bpp) from
    TIFF files on disk to JPX files written, through the native per-GPU queue
    (reader threads: file -> pinned buffer + header parse; `contexts` encodes
    in flight; uploader threads: atomic JPX write, stub upload reading every
    byte, delete-after-upload), `images` images cycling over `ndistinct`
    distinct files evicted from the page cache first, timed from the first
    submit to the last upload.  Every TIFF byte crosses PCIe host -> device:
    roofline_pcie is that rate against the measured pinned H2D rate."""
    import imaging as im
    import jp2hip
    val = {"golden": "c2"}
    value, dt, res, read = c4_batch(device, rows=images, ndistinct=ndistinct, contexts=contexts,
                                    conversion=jp2hip.LOSSY,
                                    make=lambda i: im.synth_rgb8(4000, 6000, seed=1234 + i), reader_threads=8,
                                    uploader_threads=8, shape=(4000, 6000), validate=val)
    ok = [r for r in res if r["status"] == 0]
    peak = h2d_peak()
    h2d = read / dt / 1e9
    return {"value": round(value, 3), "unit": "MP/s", "images": images, "images_ok": len(ok), "validation": val,
            "distinct_files": ndistinct,
            "page_cache": f"the {ndistinct} files are evicted before the timed region; images after the first "
                          f"{ndistinct} re-read them from the page cache",
            "seconds": round(dt, 3), "contexts": contexts,
            "out_bytes": int(np.mean([r["out_bytes"] for r in ok])) if ok else 0,
            "roofline_pcie": {"bound": "pcie_h2d", "achieved": round(h2d, 2), "peak": round(peak, 2), "unit": "GB/s",
                              "frac": round(h2d / peak, 4),
                              "def": "TIFF bytes read per second (every byte is uploaded) / measured pinned "
                                     "host->device copy rate"},
            "timed_span": "first TIFF open -> last JPX written, uploaded (stub) and deleted; "
                          "file read, H2D, encode, D2H, file write included"}


def c3_file_span(device, images=64, contexts=8, ndistinct=4):
    """SURVEY.md 8(d)'s span for the production conversion at C3 size:
    10000x8000 RGB16 TIFF files (480 MB each) on disk -> lossless JPX files
    written, through the native per-GPU queue (reader threads, `contexts`
    encodes in flight, uploader threads: atomic JPX write, stub upload reading
    every byte, delete), `images` rows cycling over `ndistinct` distinct files
    evicted from the page cache first.  Both PCIe directions carry the image:
    every TIFF byte goes host -> device, every code-stream byte device ->
    host; roofline_pcie gives each against its measured pinned copy rate."""
    import imaging as im
    import jp2hip
    busy = {}
    rc = jp2hip.recipe(jp2hip.LOSSLESS, tile_w=1024, tile_h=1024)
    val = {"golden": "c3"}
    value, dt, res, read = c4_batch(device, rows=images, ndistinct=ndistinct, contexts=contexts,
                                    conversion=jp2hip.LOSSLESS, rcp=rc,
                                    make=lambda i: im.synth_u16(8000, 10000, comps=3, seed=2 + i), reader_threads=6,
                                    uploader_threads=8, shape=(8000, 10000), gen_threads=4, busy=busy,
                                    validate=val)
    ok = [r for r in res if r["status"] == 0]
    out = sum(r["out_bytes"] for r in ok)
    ph, pd = h2d_peak(), d2h_peak()
    return {"value": round(value, 3), "unit": "MP/s", "images": images, "images_ok": len(ok), "validation": val,
            "distinct_files": ndistinct, "contexts": contexts,
            "page_cache": f"the {ndistinct} files are evicted before the timed region; images after the first "
                          f"{ndistinct} re-read them from the page cache",
            "seconds": round(dt, 3), "bpp": round(8 * out / max(1, len(ok)) / 80e6, 4), "busy": busy,
            "roofline_pcie": {
                "h2d": {"achieved": round(read / dt / 1e9, 2), "peak": round(ph, 2), "unit": "GB/s",
                        "frac": round(read / dt / 1e9 / ph, 4), "def": "TIFF bytes read per second / pinned H2D rate"},
                "d2h": {"achieved": round(out / dt / 1e9, 2), "peak": round(pd, 2), "unit": "GB/s",
                        "frac": round(out / dt / 1e9 / pd, 4),
                        "def": "code-stream bytes per second / pinned D2H rate"}},
            "timed_span": "first TIFF open -> last JPX written, uploaded (stub) and deleted; "
                          "file read, H2D, encode, D2H, file write included"}


def c5_single_gpu(enc, steps=2):
    """C5 (configs[4]) at N=1: the full 40000x30000 Gray16 image, lossy 3 bpp,
    7 levels, through the tile-split entry (jp2hip_encode_device_split) at
    world 1, checked byte-equal to the single-image encode and, when the
    committed fixture holds it, to the oracle's file (SHA-256 from
    tests/golden/make_golden.py c5_full).  TIFF resident in HBM -> JPX bytes
    in host memory, as the headline."""
    import hashlib

    import torch

    import jp2hip
    from jp2hip import split as js
    band, lay, offs, rows = c5_band(0, 1)
    d_src = torch.frombuffer(bytearray(band), dtype=torch.uint8).cuda()
    del band
    torch.cuda.synchronize()
    rc = jp2hip.recipe(jp2hip.LOSSY, levels=C5["levels"])
    sp = js.SingleGroup()
    part, off, flen, st = enc.encode_device_split(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, sp.split(), rc)
    single, _ = enc.encode_device(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY, rc)
    identical = single == part
    sha = hashlib.sha256(single).hexdigest()
    del single
    oracle = None
    try:
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
        if "c5_full" in g:
            oracle = sha == g["c5_full"]["oracle_sha256"]
    except (OSError, ValueError):
        pass
    times = []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        part, off, flen, st = enc.encode_device_split(d_src.data_ptr(), d_src.numel(), lay, jp2hip.LOSSY,
                                                      sp.split(), rc)
        times.append(time.perf_counter() - t0)
    npx = C5["w"] * C5["h"]
    dt = min(times)
    del d_src
    torch.cuda.empty_cache()
    return {"workload": "C5: 40000x30000 Gray16 -> JPX, lossy 9/7 3 bpp, 7 levels, 6 layers, 512^2 tiles, "
                        "tile-split entry at world 1", "n_gpus": 1, "value": round(npx / 1e6 / dt, 3),
            "unit": "MP/s", "seconds": round(dt, 4), "file_bytes": int(flen), "bpp": round(8 * flen / npx, 4),
            "split_equals_single_encode": identical, "equals_oracle_sha256": oracle,
            "codeblocks": int(st.codeblocks), "rate_iterations": int(st.rate_iterations),
            "timed_span": "TIFF resident in HBM -> JPX bytes in host memory"}


if __name__ == "__main__":
    main()
