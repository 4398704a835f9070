"""Tile-split path: one oversized image encoded by several GPUs.

The reference has no such path -- ``kdu_compress`` encodes one image in one
process (KakaduConverter.java:61-71) -- so this is the north_star's "RCCL only
if a single oversized image is split across GPUs".  JPEG 2000 tiles are
independent through DWT, tier-1 and the per-block rate/distortion hulls, so
rank ``r`` of ``world`` encodes the contiguous band of tile rows
``split_rows()`` names and nothing else.  The one exchange step is the PCRD
layer-threshold search (csrc/split.cpp): a bisection over the slope-key space
with one all-reduce(sum) of ``layers`` int64 per step, plus a few more
all-reduces for the lossless total, the rate loop's code-stream size and the
part sizes.  No pixel or coefficient crosses GPUs; the concatenation of every
rank's part in rank order is byte-identical to the single-GPU file.

``group`` objects supply the all-reduce:

* ``TorchGroup`` -- ``torch.distributed`` (backend "nccl" = RCCL over xGMI on
  the node; "gloo" for CPU rehearsals), one process per GPU;
* ``ThreadGroup`` -- ranks as threads of one process (several contexts on one
  GPU: tests and single-box rehearsals).
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, byref, c_int32, c_int64, c_uint64

import numpy as np

from . import _lib
from ._lib import ALLREDUCE_FN, Jp2hipError, Layout, Split


def split_rows(height: int, tile_h: int, rank: int, world: int, flush_period: int) -> tuple[int, int]:
    """Image rows [row0, row1) whose tiles rank ``rank`` of ``world`` encodes
    (whole -flush_period stripes of tile rows).  Pass the encode's own
    recipe.tile_h and recipe.flush_period (no default: a band computed with
    another period is not the band the encoder reads)."""
    r0, r1 = c_int32(), c_int32()
    _lib.lib().jp2hip_split_rows(height, tile_h, flush_period, rank, world, byref(r0), byref(r1))
    return r0.value, r1.value


class _Group:
    """Holds the ctypes callback alive for as long as the Split struct is used."""

    rank = 0
    world = 1

    def _sum(self, values: np.ndarray) -> None:  # in place
        raise NotImplementedError

    def split(self) -> Split:
        def cb(_user, ptr, n):
            try:
                arr = np.ctypeslib.as_array(ptr, shape=(n,))
                self._sum(arr)
                return 0
            except Exception:  # reported to the C side as a failed exchange
                return -1

        self._cb = ALLREDUCE_FN(cb)
        return Split(self.rank, self.world, self._cb, None)


class ThreadGroup:
    """``world`` ranks as threads of one process; ``member(rank)`` per thread."""

    def __init__(self, world: int):
        self.world = world
        self._bar = threading.Barrier(world)
        self._slots: list[np.ndarray | None] = [None] * world
        self._out: np.ndarray | None = None

    def member(self, rank: int) -> "_ThreadMember":
        return _ThreadMember(self, rank)

    def _allreduce(self, rank: int, values: np.ndarray) -> None:
        self._slots[rank] = values.copy()
        if self._bar.wait() == 0:
            self._out = np.sum(np.stack(self._slots), axis=0)
        self._bar.wait()
        values[:] = self._out
        self._bar.wait()  # nobody overwrites _out before everyone copied it

    def abort(self) -> None:
        self._bar.abort()


class _ThreadMember(_Group):
    def __init__(self, group: ThreadGroup, rank: int):
        self.group, self.rank, self.world = group, rank, group.world

    def _sum(self, values):
        self.group._allreduce(self.rank, values)


class TorchGroup(_Group):
    """All-reduce over the default ``torch.distributed`` process group.

    With backend "nccl" (RCCL) the int64 vector goes through device memory on
    ``device``; with "gloo" it stays on the host.
    """

    def __init__(self, device=None):
        import torch
        import torch.distributed as dist
        self._torch, self._dist = torch, dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        nccl = dist.get_backend() == "nccl"
        self._device = (device if device is not None else torch.device("cuda", torch.cuda.current_device())) \
            if nccl else torch.device("cpu")

    def _sum(self, values):
        t = self._torch.from_numpy(values.astype(np.int64, copy=True)).to(self._device)
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM)
        values[:] = t.cpu().numpy()


class SingleGroup(_Group):
    """world == 1: the split path with no exchange."""

    def _sum(self, values):
        pass


def thresholds(keys, cum, budgets, group: _Group | None = None) -> np.ndarray:
    """Global layer thresholds K[l] = min{k : sum over ranks of bytes with key >= k <= budgets[l]}.

    ``keys`` are this rank's hull-segment slope keys in descending order and
    ``cum`` their inclusive running byte sums (csrc/split.cpp)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    cum = np.ascontiguousarray(cum, dtype=np.int64)
    budgets = np.ascontiguousarray(budgets, dtype=np.int64)
    if keys.shape != cum.shape:
        raise ValueError("keys and cum differ in length")
    K = np.zeros(len(budgets), dtype=np.uint64)
    sp = (group or SingleGroup()).split()
    rc = _lib.lib().jp2hip_split_thresholds(
        keys.ctypes.data_as(POINTER(c_uint64)), cum.ctypes.data_as(POINTER(c_int64)), len(keys),
        budgets.ctypes.data_as(POINTER(c_int64)), len(budgets), byref(sp),
        K.ctypes.data_as(POINTER(c_uint64)))
    if rc != 0:
        raise Jp2hipError(f"split thresholds failed ({rc})")
    return K


def band_strips(tif: bytes, layout: Layout, offsets, row0: int, row1: int):
    """The strips a rank reads for image rows [row0, row1), packed back to back.

    Returns (buffer, Layout, offsets) with offsets rebased to the buffer, so a
    rank uploads only its band of a multi-GB TIFF.  Offsets of strips outside
    the band are 0 and never read (kernels.hip k_ingest / dwt.hip band_load
    touch only the rows of their band).  Compressed strips and tiles are
    packed whole, with their byte counts (the ``offsets`` array then holds
    the offsets followed by the counts, as jp2hip.tiff_layout returns them);
    the encoder decodes only the band's units (api.cpp unpack_band)."""
    if layout.compression > 1 or layout.tile_width > 0:
        return _band_units(tif, layout, offsets, row0, row1)
    rps, h, w = layout.rows_per_strip, layout.height, layout.width
    per_plane = (h + rps - 1) // rps
    planes = layout.components if layout.planar == 2 else 1
    row_bytes = w * (1 if layout.planar == 2 else layout.components) * (layout.bits // 8)
    s0, s1 = row0 // rps, (row1 + rps - 1) // rps if row1 > row0 else row0 // rps
    new = (c_uint64 * (per_plane * planes))()
    chunks, pos = [], 0
    for p in range(planes):
        for s in range(s0, s1):
            idx = p * per_plane + s
            nbytes = (min(h, (s + 1) * rps) - s * rps) * row_bytes
            o = int(offsets[idx])
            chunks.append(tif[o:o + nbytes])
            new[idx] = pos
            pos += nbytes
    lay = Layout(layout.width, layout.height, layout.components, layout.bits, layout.planar,
                 layout.big_endian, layout.rows_per_strip, layout.nstrips,
                 ctypes.cast(new, POINTER(c_uint64)))
    return b"".join(chunks), lay, new


def _band_units(tif: bytes, layout: Layout, offsets, row0: int, row1: int):
    """band_strips for compressed strips or tiles: every unit (strip, or tile
    of a tile row) that rows [row0, row1) touch, with its byte count."""
    tiled = layout.tile_width > 0
    uh = layout.tile_height if tiled else layout.rows_per_strip
    across = -(-layout.width // layout.tile_width) if tiled else 1
    urows = -(-layout.height // uh)
    per_plane = across * urows
    planes = layout.components if layout.planar == 2 else 1
    n = layout.nstrips
    u0, u1 = row0 // uh, min(urows, -(-row1 // uh)) if row1 > row0 else row0 // uh
    new = (c_uint64 * (2 * n))()
    chunks, pos = [], 0
    for p in range(planes):
        for u in range(u0, u1):
            for x in range(across):
                idx = p * per_plane + u * across + x
                o, nb = int(offsets[idx]), int(offsets[n + idx])
                chunks.append(tif[o:o + nb])
                new[idx], new[n + idx] = pos, nb
                pos += nb
    lay = Layout(layout.width, layout.height, layout.components, layout.bits, layout.planar,
                 layout.big_endian, layout.rows_per_strip, n, ctypes.cast(new, POINTER(c_uint64)),
                 layout.compression, layout.predictor, ctypes.cast(ctypes.byref(new, 8 * n), POINTER(c_uint64)),
                 layout.tile_width, layout.tile_height)
    return b"".join(chunks), lay, new


def encode_split(encoder, d_ptr: int, nbytes: int, layout: Layout, conversion: int,
                 group: _Group | None = None, rcp=None):
    """This rank's part: (bytes, file_offset, file_len, Stats).  Collective."""
    sp = (group or SingleGroup()).split()
    return encoder.encode_device_split(d_ptr, nbytes, layout, conversion, sp, rcp)


def write_part(path: str, part: bytes, offset: int, file_len: int) -> None:
    """Every rank writes its part at its offset of one shared file (pwrite).

    The caller barriers after every rank wrote, then one rank renames the
    temp file into place, so a reader never sees a partial file."""
    fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
    try:
        if os.fstat(fd).st_size < file_len:
            os.ftruncate(fd, file_len)
        view = memoryview(part)
        done = 0
        while done < len(view):
            done += os.pwrite(fd, view[done:], offset + done)
        os.fsync(fd)
    finally:
        os.close(fd)
