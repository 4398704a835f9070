"""ctypes binding of libjp2hip (include/jp2hip.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C jp2-bucketeer_amd/csrc``) next to this file.  There is no fallback:
if the library or a gfx950 device is missing, calls raise ``Jp2hipError``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (CFUNCTYPE, POINTER, Structure, byref, c_char_p, c_double, c_int, c_int32,
                    c_int64, c_size_t, c_uint8, c_uint64, c_void_p)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JP2HIP_LIBRARY") or os.path.join(HERE, "libjp2hip.so")  # override: experiments only

LOSSY = 0      # Conversion.LOSSY    (Conversion.java:9)
LOSSLESS = 1   # Conversion.LOSSLESS (Conversion.java:9)
FORMAT_J2K, FORMAT_JP2, FORMAT_JPX = 0, 1, 2


class Jp2hipError(OSError):
    """Raised for every libjp2hip failure (maps to IOException on the Java side)."""


class Config(Structure):
    _fields_ = [("device", c_int32), ("host_threads", c_int32), ("profile", c_int32),
                ("reserved", c_int32)]


class Recipe(Structure):
    _fields_ = [("levels", c_int32), ("layers", c_int32), ("tile_w", c_int32), ("tile_h", c_int32),
                ("cblk_w_log2", c_int32), ("cblk_h_log2", c_int32), ("nprecincts", c_int32),
                ("prec_w_log2", c_int32 * 16), ("prec_h_log2", c_int32 * 16),
                ("progression", c_int32), ("sop", c_int32), ("eph", c_int32), ("plt", c_int32),
                ("tparts_r", c_int32), ("guard_bits", c_int32), ("reversible", c_int32),
                ("mct", c_int32), ("qstep", c_double), ("rate_bpp", c_double),
                ("format", c_int32), ("comment", c_int32), ("slope_skip", c_int32),
                ("flush_period", c_int32)]


class Layout(Structure):
    _fields_ = [("width", c_int32), ("height", c_int32), ("components", c_int32),
                ("bits", c_int32), ("planar", c_int32), ("big_endian", c_int32),
                ("rows_per_strip", c_int32), ("nstrips", c_int32),
                ("strip_offsets", POINTER(c_uint64)),
                ("compression", c_int32), ("predictor", c_int32),
                ("strip_bytes", POINTER(c_uint64)),
                ("tile_width", c_int32), ("tile_height", c_int32)]


class Stats(Structure):
    _fields_ = [("total_ms", c_double), ("h2d_ms", c_double), ("ingest_ms", c_double),
                ("dwt_ms", c_double), ("quant_ms", c_double), ("t1_ms", c_double),
                ("pcrd_ms", c_double), ("d2h_ms", c_double), ("t2_ms", c_double),
                ("codeblocks", c_int64), ("coded_passes", c_int64), ("t1_bytes", c_int64),
                ("out_bytes", c_int64), ("rate_iterations", c_int32), ("host_waits", c_int32),
                ("t1_cm_ms", c_double), ("t1_mq_ms", c_double), ("mq_decisions", c_int64),
                ("stream_pool_bytes", c_int64), ("stream_need_bytes", c_int64), ("pool_grows", c_int32),
                ("reserved", c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every symbol include/jp2hip.h declares
EXPORTS = ("jp2hip_version", "jp2hip_last_error", "jp2hip_probe", "jp2hip_device_count", "jp2hip_device_ordinals",
           "jp2hip_recipe_init",
           "jp2hip_create", "jp2hip_destroy", "jp2hip_encode_file", "jp2hip_encode_tiff",
           "jp2hip_tiff_layout", "jp2hip_encode_device", "jp2hip_free",
           # batch path (csrc/batch.cpp; bound in jp2hip.batch)
           "jp2hip_batch_create", "jp2hip_batch_submit", "jp2hip_batch_wait", "jp2hip_batch_pending",
           "jp2hip_batch_destroy",
           # tile-split path (csrc/split.cpp + api.cpp; bound in jp2hip.split)
           "jp2hip_split_rows", "jp2hip_encode_device_split", "jp2hip_split_thresholds",
           "jp2hip_split_peers", "jp2hip_tiff_pixels", "jp2hip_env_check",
           # device-memory policy (api.cpp)
           "jp2hip_device_bytes", "jp2hip_set_memory_limits", "jp2hip_device_memory", "jp2hip_dma_engines")


# int (*)(void *user, int64_t *values, int32_t n): in-place sum over ranks, 0 ok
ALLREDUCE_FN = CFUNCTYPE(c_int, c_void_p, POINTER(c_int64), c_int32)


class Split(Structure):
    _fields_ = [("rank", c_int32), ("world", c_int32), ("allreduce_sum", ALLREDUCE_FN),
                ("user", c_void_p)]

_lib = None


def lib():
    """Load libjp2hip.so once; raise if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Jp2hipError(f"libjp2hip is not built ({LIB_PATH} missing); run __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    L.jp2hip_version.restype = c_char_p
    L.jp2hip_last_error.restype = c_char_p
    L.jp2hip_probe.restype = c_int
    L.jp2hip_device_count.restype = c_int
    L.jp2hip_device_ordinals.argtypes = [POINTER(c_int32), c_int32]
    L.jp2hip_device_ordinals.restype = c_int
    L.jp2hip_recipe_init.argtypes = [POINTER(Recipe), c_int]
    L.jp2hip_create.argtypes = [POINTER(c_void_p), POINTER(Config)]
    L.jp2hip_destroy.argtypes = [c_void_p]
    L.jp2hip_encode_file.argtypes = [c_void_p, c_char_p, c_char_p, c_int, POINTER(Recipe),
                                     POINTER(Stats)]
    L.jp2hip_encode_tiff.argtypes = [c_void_p, c_void_p, c_size_t, c_int, POINTER(Recipe),
                                     POINTER(POINTER(c_uint8)), POINTER(c_size_t), POINTER(Stats)]
    L.jp2hip_tiff_layout.argtypes = [c_void_p, c_size_t, POINTER(Layout), POINTER(c_uint64),
                                     c_int32]
    L.jp2hip_encode_device.argtypes = [c_void_p, c_void_p, c_size_t, POINTER(Layout), c_int,
                                       POINTER(Recipe), POINTER(POINTER(c_uint8)),
                                       POINTER(c_size_t), POINTER(Stats)]
    L.jp2hip_free.argtypes = [c_void_p]
    L.jp2hip_split_rows.argtypes = [c_int32, c_int32, c_int32, c_int32, c_int32, POINTER(c_int32),
                                    POINTER(c_int32)]
    L.jp2hip_split_rows.restype = None
    L.jp2hip_encode_device_split.argtypes = [c_void_p, c_void_p, c_size_t, POINTER(Layout), c_int,
                                             POINTER(Recipe), POINTER(Split),
                                             POINTER(POINTER(c_uint8)), POINTER(c_size_t),
                                             POINTER(c_uint64), POINTER(c_uint64), POINTER(Stats)]
    L.jp2hip_split_peers.argtypes = [c_void_p, POINTER(c_int32), c_int32, c_int64]
    L.jp2hip_env_check.restype = c_char_p
    L.jp2hip_tiff_pixels.argtypes = [c_char_p]
    L.jp2hip_tiff_pixels.restype = c_int64
    L.jp2hip_split_thresholds.argtypes = [POINTER(c_uint64), POINTER(c_int64), c_int64,
                                          POINTER(c_int64), c_int32, POINTER(Split),
                                          POINTER(c_uint64)]
    L.jp2hip_device_bytes.argtypes = [c_void_p]
    L.jp2hip_device_bytes.restype = c_int64
    L.jp2hip_set_memory_limits.argtypes = [c_void_p, c_int64, c_int64]
    L.jp2hip_device_memory.argtypes = [c_int, POINTER(c_int64), POINTER(c_int64)]
    L.jp2hip_dma_engines.restype = c_char_p
    _lib = L
    return L


def last_error() -> str:
    return lib().jp2hip_last_error().decode("utf-8", "replace")


def version() -> str:
    return lib().jp2hip_version().decode()


def probe() -> bool:
    return bool(lib().jp2hip_probe())


def device_count() -> int:
    """gfx950 devices visible to libjp2hip (0 without a GPU)."""
    return int(lib().jp2hip_device_count())


def device_ordinals() -> list[int]:
    """HIP ordinals of the visible gfx950 devices (Encoder(device=...) takes these)."""
    n = int(lib().jp2hip_device_ordinals(None, 0))
    if n <= 0:
        return []
    buf = (c_int32 * n)()
    n = min(n, int(lib().jp2hip_device_ordinals(buf, n)))
    return [int(buf[i]) for i in range(n)]


def env_check() -> str:
    """"" or what the process environment should change for the contexts
    alive in it (jp2hip_env_check: GPU_MAX_HW_QUEUES)."""
    return lib().jp2hip_env_check().decode()


def dma_engines() -> str:
    """The SDMA engines the code-stream copies use and their probed rates."""
    return lib().jp2hip_dma_engines().decode()


def device_memory(device: int) -> tuple[int, int]:
    """(free, total) bytes of HIP device `device` (jp2hip_device_memory)."""
    fr, tot = c_int64(), c_int64()
    if lib().jp2hip_device_memory(device, byref(fr), byref(tot)) != 0:
        raise Jp2hipError(last_error())
    return int(fr.value), int(tot.value)


# what one context holds for the images a converter usually sees (C4-class
# 5000 x 7000 RGB8 lossless, DESIGN.md 3 "Footprint"); a pool is sized from it
CONTEXT_BUDGET_BYTES = 8 << 30


def contexts_for_memory(free_bytes: int, budget: int = CONTEXT_BUDGET_BYTES, cap: int = 16) -> int:
    """Contexts per GPU that fit 75 % of the device's free memory at `budget`
    bytes each (at least 1, at most `cap`)."""
    return max(1, min(cap, int(free_bytes * 0.75) // max(1, budget)))


def tiff_pixels(path) -> int:
    """Width x height of a TIFF file, from its header (jp2hip_tiff_pixels)."""
    n = int(lib().jp2hip_tiff_pixels(os.fsencode(path)))
    if n < 0:
        raise Jp2hipError(last_error())
    return n


def recipe(conversion: int, **overrides) -> Recipe:
    r = Recipe()
    lib().jp2hip_recipe_init(byref(r), conversion)
    for k, v in overrides.items():
        if k in ("prec_w_log2", "prec_h_log2"):
            arr = getattr(r, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(r, k, v)
    return r


def tiff_layout(data: bytes):
    """Parse a baseline TIFF header; returns (Layout, offsets array)."""
    lay = Layout()
    cap = 1 << 20
    offs = (c_uint64 * cap)()
    buf = ctypes.create_string_buffer(data, len(data))
    if lib().jp2hip_tiff_layout(buf, len(data), byref(lay), offs, cap) != 0:
        raise Jp2hipError(last_error())
    n = lay.nstrips
    packed = lay.compression > 1 or lay.tile_width > 0
    m = 2 * n if packed else n  # compressed / tiled: offsets, then byte counts
    keep = (c_uint64 * m)(*offs[:m])
    lay.strip_offsets = ctypes.cast(keep, POINTER(c_uint64))
    if packed:
        lay.strip_bytes = ctypes.cast(ctypes.byref(keep, 8 * n), POINTER(c_uint64))
    return lay, keep


class _PinnedBuffer:
    """Owns one *out buffer of the encode calls; returns it to jp2hip's pool
    (jp2hip_free) when the last holder -- the Output or a view of it -- goes."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        try:
            lib().jp2hip_free(self.ptr)
        except Exception:
            pass


class Output:
    """An encode's file bytes, left where the library wrote them (pinned host
    memory from jp2hip's pool) instead of copied into a Python bytes object.
    close() (or collection) releases the Output's hold; the buffer goes back
    to the pool once no view() of it is alive either, so a view never sees
    another encode's bytes."""

    def __init__(self, ptr, n: int):
        self._buf = _PinnedBuffer(ptr)
        self._n = n

    def __len__(self):
        return self._n

    def view(self) -> memoryview:
        if self._buf is None:
            raise ValueError("released output")
        arr = (c_uint8 * self._n).from_address(ctypes.addressof(self._buf.ptr.contents))
        arr._jp2hip_owner = self._buf  # the view keeps the pinned buffer alive
        return memoryview(arr)

    def tobytes(self) -> bytes:
        return bytes(self.view())

    def tail(self, k: int) -> bytes:
        """The last k bytes, read in place (no array type, no view)."""
        if self._buf is None:
            raise ValueError("released output")
        k = min(k, self._n)
        return ctypes.string_at(ctypes.addressof(self._buf.ptr.contents) + self._n - k, k)

    def close(self):
        self._buf = None


class Encoder:
    """One libjp2hip context bound to one GPU (thread-safe, calls serialise).
    The encode_* methods return the file as bytes, or with copy=False as an
    Output over the library's buffer (no host copy of the result)."""

    def __init__(self, device: int = 0, host_threads: int = 0, profile: bool = False):
        cfg = Config(device, host_threads, 1 if profile else 0, 0)
        h = c_void_p()
        if lib().jp2hip_create(byref(h), byref(cfg)) != 0:
            raise Jp2hipError(last_error())
        self._h = h

    def close(self):
        if self._h:
            lib().jp2hip_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_bytes(self) -> int:
        """Device memory held by this context (jp2hip_device_bytes)."""
        return int(lib().jp2hip_device_bytes(self._h))

    def set_memory_limits(self, soft: int = 0, hard: int = 0):
        """jp2hip_set_memory_limits: <= 0 keeps the default of each."""
        if lib().jp2hip_set_memory_limits(self._h, int(soft), int(hard)) != 0:
            raise Jp2hipError(last_error())

    def _take(self, out, n, copy=True):
        if not copy:
            return Output(out, n.value)
        try:
            return ctypes.string_at(out, n.value)
        finally:
            lib().jp2hip_free(out)

    def encode_tiff(self, data: bytes, conversion: int, rcp: Recipe | None = None):
        out = POINTER(c_uint8)()
        n = c_size_t()
        st = Stats()
        buf = ctypes.create_string_buffer(data, len(data))
        rc = lib().jp2hip_encode_tiff(self._h, buf, len(data), conversion,
                                      byref(rcp) if rcp is not None else None,
                                      byref(out), byref(n), byref(st))
        if rc != 0:
            raise Jp2hipError(last_error())
        return self._take(out, n), st

    def encode_tiff_ptr(self, h_ptr: int, nbytes: int, conversion: int, rcp: Recipe | None = None,
                        copy: bool = True):
        """encode_tiff on TIFF bytes already in host memory at h_ptr (pinned
        memory makes the H2D a plain DMA)."""
        out = POINTER(c_uint8)()
        n = c_size_t()
        st = Stats()
        rc = lib().jp2hip_encode_tiff(self._h, c_void_p(h_ptr), nbytes, conversion,
                                      byref(rcp) if rcp is not None else None,
                                      byref(out), byref(n), byref(st))
        if rc != 0:
            raise Jp2hipError(last_error())
        return self._take(out, n, copy), st

    def encode_device(self, d_ptr: int, nbytes: int, layout: Layout, conversion: int,
                      rcp: Recipe | None = None, copy: bool = True):
        out = POINTER(c_uint8)()
        n = c_size_t()
        st = Stats()
        rc = lib().jp2hip_encode_device(self._h, c_void_p(d_ptr), nbytes, byref(layout), conversion,
                                        byref(rcp) if rcp is not None else None,
                                        byref(out), byref(n), byref(st))
        if rc != 0:
            raise Jp2hipError(last_error())
        return self._take(out, n, copy), st

    def encode_device_split(self, d_ptr: int, nbytes: int, layout: Layout, conversion: int,
                            split: Split, rcp: Recipe | None = None):
        """This rank's part of a tile-split encode: (bytes, file_offset, file_len, Stats)."""
        out = POINTER(c_uint8)()
        n = c_size_t()
        off = c_uint64()
        flen = c_uint64()
        st = Stats()
        rc = lib().jp2hip_encode_device_split(self._h, c_void_p(d_ptr), nbytes, byref(layout),
                                              conversion, byref(rcp) if rcp is not None else None,
                                              byref(split), byref(out), byref(n), byref(off),
                                              byref(flen), byref(st))
        if rc != 0:
            raise Jp2hipError(last_error())
        return self._take(out, n), off.value, flen.value, st

    def split_peers(self, ordinals: list[int], min_pixels: int = 0):
        """Tile-split this encoder's images of >= min_pixels pixels across
        itself and one peer context per entry of ``ordinals``
        (jp2hip_split_peers); ``[]`` removes the peers."""
        arr = (c_int32 * max(1, len(ordinals)))(*ordinals)
        if lib().jp2hip_split_peers(self._h, arr, len(ordinals), min_pixels) != 0:
            raise Jp2hipError(last_error())

    def encode_file(self, tiff_path: str, out_path: str, conversion: int,
                    rcp: Recipe | None = None):
        st = Stats()
        rc = lib().jp2hip_encode_file(self._h, os.fsencode(tiff_path), os.fsencode(out_path),
                                      conversion, byref(rcp) if rcp is not None else None,
                                      byref(st))
        if rc != 0:
            raise Jp2hipError(last_error())
        return st
