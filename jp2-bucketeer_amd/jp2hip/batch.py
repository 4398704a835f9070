"""Batch path: a CSV batch through one GPU's native work queue.

Mirrors the route a CSV row takes in the reference (paths under
src/main/java/edu/ucla/library/bucketeer/):

  JobFactory.java:86-330       CSV -> items; the columns used here are
                               "Item ARK" (Metadata.java:12) and "File Name"
                               (Metadata.java:17), each at most once (BUCKETEER-516)
  LoadCsvHandler.java:250-289  queue every item that has a file
  LargeImageVerticle.java:65-108 -> ImageWorkerVerticle.java:54-110
                               convert LOSSLESS, then hand the JPX to
  S3BucketVerticle.java:88-211 upload under the JPX file name, delete it
                               after a successful upload (:286-303)

The queue itself is native (libjp2hip ``jp2hip_batch_*``, csrc/batch.cpp):
reader threads, one encoder thread per GPU context, uploader threads.  Images
are independent, so no collective touches the data.  Rows reach the GPUs by
work stealing: every GPU's queue pulls the next unclaimed
row whenever it holds fewer than ``depth`` images, from one shared claim
counter -- ``LocalClaims`` for N queues in one process, ``StoreClaims``
(the torch.distributed store's atomic ``add``) for one queue per process --
so a GPU that drew small images takes more of them and none sits idle while
rows remain (``run_batch_dynamic``).  ``shard`` (static round-robin) stays
for callers that want a fixed partition.
"""
from __future__ import annotations

import csv
import ctypes
import os
import threading
import time
import urllib.parse
from ctypes import CFUNCTYPE, POINTER, Structure, byref, c_char, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p
from dataclasses import dataclass
from pathlib import Path

from . import _lib

ITEM_ID = "Item ARK"      # Metadata.java:12
FILE_NAME = "File Name"   # Metadata.java:17

OK, CONVERT_FAILED, UPLOAD_FAILED = 0, -1, -2


class BatchConfig(Structure):
    _fields_ = [("device", c_int32), ("contexts", c_int32), ("reader_threads", c_int32),
                ("uploader_threads", c_int32), ("host_threads", c_int32),
                ("delete_after_upload", c_int32), ("write_output", c_int32), ("reserved", c_int32)]


class BatchResult(Structure):
    _fields_ = [("job", c_int64), ("status", c_int32), ("reserved", c_int32), ("in_bytes", c_int64),
                ("out_bytes", c_int64), ("pixels", c_int64), ("read_ms", c_double),
                ("encode_ms", c_double), ("upload_ms", c_double), ("message", c_char * 240)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("reserved", "message")}
        d["message"] = self.message.decode("utf-8", "replace")
        return d


UPLOAD_FN = CFUNCTYPE(c_int, c_void_p, c_char_p, c_char_p)

BATCH_EXPORTS = ("jp2hip_batch_create", "jp2hip_batch_submit", "jp2hip_batch_wait",
                 "jp2hip_batch_pending", "jp2hip_batch_destroy")


def _bind():
    L = _lib.lib()
    if getattr(L, "_batch_bound", False):
        return L
    L.jp2hip_batch_create.argtypes = [POINTER(c_void_p), POINTER(BatchConfig), c_void_p, c_void_p]
    L.jp2hip_batch_submit.argtypes = [c_void_p, c_int64, c_char_p, c_char_p, c_char_p, c_int,
                                      POINTER(_lib.Recipe)]
    L.jp2hip_batch_wait.argtypes = [c_void_p, POINTER(BatchResult), c_int, c_int]
    L.jp2hip_batch_pending.argtypes = [c_void_p]
    L.jp2hip_batch_pending.restype = c_int64
    L.jp2hip_batch_destroy.argtypes = [c_void_p]
    L._batch_bound = True
    return L


@dataclass
class BatchItem:
    job: int
    image_id: str
    tiff: str


class CsvError(ValueError):
    """A batch CSV the reference would reject (JobFactory.hasHeaderErrors)."""


def read_batch_csv(path: os.PathLike | str, path_prefix: str = "") -> list[BatchItem]:
    """Items of a Bucketeer batch CSV: (Item ARK, File Name) per row.

    Header rules follow JobFactory.hasHeaderErrors (JobFactory.java:280-330):
    each of the two columns must appear exactly once.  Rows without a file
    name are not converted (the reference marks them and moves on)."""
    with open(path, newline="", encoding="utf-8") as f:
        rows = list(csv.reader(f))
    if not rows:
        raise CsvError(f"{path}: empty CSV")
    head = rows[0]
    for col in (ITEM_ID, FILE_NAME):
        n = head.count(col)
        if n != 1:
            raise CsvError(f"{path}: column '{col}' appears {n} times")
    iid, ifn = head.index(ITEM_ID), head.index(FILE_NAME)
    items = []
    for i, r in enumerate(rows[1:]):
        if len(r) <= max(iid, ifn) or not r[ifn].strip():
            continue
        items.append(BatchItem(i, r[iid].strip(), os.path.join(path_prefix, r[ifn].strip())))
    return items


def shard(items: list, rank: int, world: int) -> list:
    """Static round-robin share of one GPU process (images are independent)."""
    return items[rank::world]


class LocalClaims:
    """Claims on rows 0..n-1 shared by the queues of one process."""

    def __init__(self, n: int):
        self._n, self._next, self._mu = n, 0, threading.Lock()

    def next(self) -> int | None:
        with self._mu:
            if self._next >= self._n:
                return None
            i = self._next
            self._next += 1
            return i


class StoreClaims:
    """Claims on rows 0..n-1 shared by every rank of a job, through a
    torch.distributed store (TCPStore / FileStore / HashStore): ``add`` is
    atomic on the store's server, so each row goes to exactly one rank. Only
    the row index crosses processes -- control plane, not data path."""

    def __init__(self, store, n: int, key: str = "jp2hip/batch/next"):
        self._store, self._n, self._key = store, n, key

    def next(self) -> int | None:
        i = int(self._store.add(self._key, 1)) - 1
        return i if i < self._n else None


def run_batch_dynamic(items: list[BatchItem], out_dir: os.PathLike | str, queues: list, claims=None,
                      depth: int = 16, conversion: int = _lib.LOSSLESS, poll_ms: int = 20,
                      trace: list | None = None) -> list[dict]:
    """Work stealing over ``queues`` (BatchQueue-like: submit / pending /
    wait): one feeder thread per queue tops its queue up to ``depth``
    images with the next unclaimed row and collects its results, so rows go
    to whichever GPU has room. ``claims`` defaults to LocalClaims over
    ``items``; pass StoreClaims to share rows with other processes.
    ``trace`` (a list) receives (t, queue, "submit" | "done", job) events.
    Returns every result, in completion order."""
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    claims = claims or LocalClaims(len(items))
    results, mu, errors = [], threading.Lock(), []
    t0 = time.perf_counter()

    def feed(qi, q):
        try:
            exhausted = False
            while True:
                while not exhausted and q.pending() < depth:
                    i = claims.next()
                    if i is None:
                        exhausted = True
                        break
                    it = items[i]
                    q.submit(it.job, it.image_id, it.tiff, out_dir / jpx_name(it.image_id), conversion)
                    if trace is not None:
                        with mu:
                            trace.append((time.perf_counter() - t0, qi, "submit", it.job))
                if exhausted and q.pending() == 0:
                    return
                got = q.wait(timeout_ms=poll_ms)
                with mu:
                    results.extend(got)
                    if trace is not None:
                        trace.extend((time.perf_counter() - t0, qi, "done", r["job"]) for r in got)
        except Exception as e:  # surfaced below, after every feeder stopped
            errors.append(e)

    threads = [threading.Thread(target=feed, args=(k, q), name=f"jp2hip-feed-{k}") for k, q in enumerate(queues)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return results


def jpx_name(image_id: str) -> str:
    """URLEncoder.encode(id) + ".jpx" (KakaduConverter.java:57)."""
    return urllib.parse.quote_plus(image_id, safe="*-._") + ".jpx"


class BatchQueue:
    """One GPU's native batch queue (jp2hip_batch_*).

    ``upload(image_id, jpx_path) -> bool`` is the S3 stand-in; None selects
    the built-in stub that reads every byte of the file."""

    def __init__(self, device: int = 0, contexts: int = 12, reader_threads: int = 4,
                 uploader_threads: int = 4, host_threads: int = 0, delete_after_upload: bool = True,
                 write_output: bool = True, upload=None):
        # one HW queue per context (+4 for the runtime); only takes effect if
        # nothing in this process has initialised HIP yet
        os.environ.setdefault("GPU_MAX_HW_QUEUES", str(max(4, min(32, (contexts or 12) + 4))))
        L = _bind()
        cfg = BatchConfig(device, contexts, reader_threads, uploader_threads, host_threads,
                          1 if delete_after_upload else 0, 1 if write_output else 0, 0)
        self._cb = None
        if upload is not None:
            def _cb(_user, iid, path):
                try:
                    return 0 if upload(iid.decode("utf-8"), path.decode("utf-8")) else 1
                except Exception:  # an upload failure, never a crash of the queue
                    return 1
            self._cb = UPLOAD_FN(_cb)
        h = c_void_p()
        if L.jp2hip_batch_create(byref(h), byref(cfg), ctypes.cast(self._cb, c_void_p) if self._cb else None,
                                 None) != 0:
            raise _lib.Jp2hipError(_lib.last_error())
        self._h = h

    def submit(self, job: int, image_id: str, tiff: os.PathLike | str, jpx: os.PathLike | str,
               conversion: int = _lib.LOSSLESS, rcp: _lib.Recipe | None = None):
        rc = _bind().jp2hip_batch_submit(self._h, job, image_id.encode("utf-8"), os.fsencode(str(tiff)),
                                         os.fsencode(str(jpx)), conversion,
                                         byref(rcp) if rcp is not None else None)
        if rc != 0:
            raise _lib.Jp2hipError("batch queue is closed")

    def pending(self) -> int:
        return int(_bind().jp2hip_batch_pending(self._h))

    def wait(self, max_results: int = 64, timeout_ms: int = -1) -> list[dict]:
        arr = (BatchResult * max_results)()
        n = _bind().jp2hip_batch_wait(self._h, arr, max_results, timeout_ms)
        return [arr[i].as_dict() for i in range(n)]

    def drain(self) -> list[dict]:
        out = []
        while self.pending() > 0:
            out.extend(self.wait())
        return out

    def close(self):
        if self._h:
            _bind().jp2hip_batch_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_batch(items: list[BatchItem], out_dir: os.PathLike | str, conversion: int = _lib.LOSSLESS,
              **queue_kw) -> list[dict]:
    """Convert + upload every item through one GPU's queue; one result per item
    (ImageWorker's reply / callback status), in completion order."""
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    with BatchQueue(**queue_kw) as q:
        for it in items:
            q.submit(it.job, it.image_id, it.tiff, out_dir / jpx_name(it.image_id), conversion)
        return q.drain()
