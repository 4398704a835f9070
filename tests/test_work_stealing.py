"""Work stealing across GPU queues in the batch path (static
round-robin plus work stealing).

CPU only: the queues are fakes with the native queue's contract (submit /
pending / wait, pending counting images not yet collected) whose "contexts"
are threads that sleep in proportion to the image's size, so mixed archival
sizes are modelled. Covers N queues in one process (LocalClaims) and one
queue per process over a world-2 gloo group sharing the store's atomic
counter (StoreClaims)."""
import os
import threading
import time
from collections import deque

import numpy as np
import pytest

from jp2hip import batch as jb

UNIT_S = 0.004  # seconds of "encode" per size unit


class FakeQueue:
    def __init__(self, contexts=2, speed=1.0):
        self.speed = speed
        self._todo, self._done = deque(), deque()
        self._cv = threading.Condition()
        self._pending = 0
        self._closed = False
        self.encoded = []
        self._workers = [threading.Thread(target=self._work, daemon=True) for _ in range(contexts)]
        for w in self._workers:
            w.start()

    def _work(self):
        while True:
            with self._cv:
                while not self._todo and not self._closed:
                    self._cv.wait()
                if self._closed and not self._todo:
                    return
                job, tiff = self._todo.popleft()
            time.sleep(float(os.path.basename(str(tiff)).split("_")[1]) * UNIT_S / self.speed)
            with self._cv:
                self._done.append({"job": job, "status": 0})
                self.encoded.append(job)
                self._cv.notify_all()

    def submit(self, job, image_id, tiff, jpx, conversion=1, rcp=None):
        with self._cv:
            self._todo.append((job, tiff))
            self._pending += 1
            self._cv.notify_all()

    def pending(self):
        with self._cv:
            return self._pending

    def wait(self, max_results=64, timeout_ms=-1):
        with self._cv:
            ready = lambda: self._done or self._pending == 0  # noqa: E731 (the native queue's rule)
            if timeout_ms < 0:
                self._cv.wait_for(ready)
            else:
                self._cv.wait_for(ready, timeout_ms / 1000)
            out = []
            while self._done and len(out) < max_results:
                out.append(self._done.popleft())
                self._pending -= 1
            return out

    def close(self):
        with self._cv:
            self._closed = True
            self._cv.notify_all()


def mixed_items(n, seed):
    """Archival batches mix sizes: most images small, some 8x larger."""
    rng = np.random.default_rng(seed)
    sizes = np.where(rng.random(n) < 0.25, 8, 1)
    return [jb.BatchItem(i, f"ark:/99999/m{i:04d}", f"/in/img_{s}_{i}.tif") for i, s in enumerate(sizes)], sizes


def idle_gaps(trace, nq, n_items, min_gap):
    """Intervals (queue, start, end) longer than min_gap in which a queue
    held nothing while rows were still unclaimed."""
    out = []
    held = [0] * nq
    submitted = 0
    empty_since = [None] * nq  # the initial fill is not a gap: a queue counts once it has drained
    for t, q, ev, _ in sorted(trace, key=lambda e: (e[0], e[2] != "done")):
        if ev == "submit":
            if held[q] == 0 and empty_since[q] is not None and t - empty_since[q] > min_gap:
                out.append((q, empty_since[q], t))
            held[q] += 1
            submitted += 1
        else:
            held[q] -= 1
            if held[q] == 0:
                empty_since[q] = t
    return out


def test_dynamic_keeps_every_queue_busy_with_mixed_sizes(tmp_path):
    items, sizes = mixed_items(120, seed=3)
    queues = [FakeQueue(contexts=2), FakeQueue(contexts=2), FakeQueue(contexts=2)]
    trace = []
    try:
        res = jb.run_batch_dynamic(items, tmp_path, queues, depth=3, trace=trace)
    finally:
        for q in queues:
            q.close()
    assert sorted(r["job"] for r in res) == list(range(120))  # every row exactly once
    assert sorted(j for q in queues for j in q.encoded) == list(range(120))
    # no queue sits empty while rows remain unclaimed (beyond a few ms of
    # hand-off latency)
    assert idle_gaps(trace, 3, 120, min_gap=0.010) == []
    # and every queue holds at most `depth` images: nothing piles up behind a
    # slow GPU while another runs dry
    held, top = [0, 0, 0], [0, 0, 0]
    for _, q, ev, _ in sorted(trace, key=lambda e: (e[0], e[2] != "done")):
        held[q] += 1 if ev == "submit" else -1
        top[q] = max(top[q], held[q])
    assert max(top) <= 3
    # finish times differ by at most about one large image
    last = [max(t for t, q, ev, _ in trace if q == k and ev == "done") for k in range(3)]
    assert max(last) - min(last) <= 8 * UNIT_S * 2 + 0.05


def test_dynamic_beats_static_shards_when_sizes_cluster(tmp_path):
    """The static round-robin split (shard) hands one GPU all the large
    images when sizes cluster by position; stealing evens the load."""
    n = 48
    items = [jb.BatchItem(i, f"id{i}", f"/in/img_{8 if i % 2 == 0 else 1}_{i}.tif") for i in range(n)]
    t0 = time.perf_counter()
    qs = [FakeQueue(contexts=1), FakeQueue(contexts=1)]
    try:
        threads = []
        for r, q in enumerate(qs):
            part = jb.shard(items, r, 2)
            threads.append(threading.Thread(target=jb.run_batch_dynamic,
                                            args=(part, tmp_path / f"s{r}", [q]), kwargs={"depth": 2}))
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        static_s = time.perf_counter() - t0
        assert sorted(qs[0].encoded) == list(range(0, n, 2))  # rank 0: every large image
    finally:
        for q in qs:
            q.close()
    t0 = time.perf_counter()
    qs = [FakeQueue(contexts=1), FakeQueue(contexts=1)]
    try:
        jb.run_batch_dynamic(items, tmp_path / "d", qs, depth=2)
        dynamic_s = time.perf_counter() - t0
    finally:
        for q in qs:
            q.close()
    # static: 24 x 8 units on one queue; dynamic: about (24 x 8 + 24) / 2
    assert dynamic_s < 0.75 * static_s, (dynamic_s, static_s)


def test_local_claims_each_row_once_under_contention():
    c = jb.LocalClaims(10000)
    got = []
    mu = threading.Lock()

    def take():
        mine = []
        while (i := c.next()) is not None:
            mine.append(i)
        with mu:
            got.extend(mine)
    ts = [threading.Thread(target=take) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert sorted(got) == list(range(10000))


def _rank_main(rank, world, store_path, out_path, n):
    import json

    import torch.distributed as dist
    store = dist.FileStore(store_path, world)
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
    items = [jb.BatchItem(i, f"id{i}", f"/in/img_{1 + (i % 3)}_{i}.tif") for i in range(n)]
    q = FakeQueue(contexts=2, speed=3.0 if rank == 1 else 1.0)  # rank 1's GPU is 3x faster
    try:
        dist.barrier()
        # the process group's own store, as bench.py --workload c4 takes it
        from torch.distributed import distributed_c10d as c10d
        claims = jb.StoreClaims(c10d._get_default_store(), n)
        out_dir = os.path.join(os.path.dirname(out_path), f"jpx{rank}")
        res = jb.run_batch_dynamic(items, out_dir, [q], claims=claims, depth=2)
    finally:
        q.close()
    dist.barrier()
    with open(out_path, "w") as f:
        json.dump(sorted(r["job"] for r in res), f)
    dist.destroy_process_group()


def test_store_claims_share_rows_across_two_ranks(tmp_path):
    """World 2 over gloo: both ranks pull rows from the store's atomic
    counter (no data-path collective); every row is encoded exactly once and
    the faster rank takes more of them."""
    import json

    import torch.multiprocessing as mp
    n = 90
    store_path = str(tmp_path / "store")
    outs = [str(tmp_path / f"r{r}.json") for r in range(2)]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank_main, args=(r, 2, store_path, outs[r], n)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    got = [json.load(open(o)) for o in outs]
    assert sorted(got[0] + got[1]) == list(range(n))
    assert len(got[1]) > 1.5 * len(got[0]), (len(got[0]), len(got[1]))


@pytest.mark.parametrize("world", [1, 3])
def test_store_claims_end_at_n(world):
    import torch.distributed as dist
    store = dist.HashStore()
    cl = [jb.StoreClaims(store, 7) for _ in range(world)]
    seen = []
    k = 0
    while True:
        i = cl[k % world].next()
        k += 1
        if i is None:
            break
        seen.append(i)
    assert seen == list(range(7))
    assert all(c.next() is None for c in cl)
