"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker, never the thing measured
or shipped.  Built by ``make -C oracle`` (``__graft_entry__.build()`` does it).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, byref, c_double, c_int, c_int32, c_int64, c_size_t, c_uint8

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


class OracleRecipe(Structure):
    _fields_ = [("levels", c_int32), ("layers", c_int32), ("tile_w", c_int32), ("tile_h", c_int32),
                ("cblk_w_log2", c_int32), ("cblk_h_log2", c_int32), ("nprecincts", c_int32),
                ("prec_w_log2", c_int32 * 16), ("prec_h_log2", c_int32 * 16),
                ("progression", c_int32), ("sop", c_int32), ("eph", c_int32), ("plt", c_int32),
                ("tparts_r", c_int32), ("guard_bits", c_int32), ("reversible", c_int32),
                ("mct", c_int32), ("qstep", c_double), ("rate_bpp", c_double),
                ("format", c_int32), ("comment", c_int32), ("slope_skip", c_int32),
                ("flush_period", c_int32)]


_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           capture_output=True)
        L = ctypes.CDLL(LIB)
        L.oracle_recipe_init.argtypes = [POINTER(OracleRecipe), c_int]
        L.oracle_encode.argtypes = [ctypes.c_void_p, c_int, c_int, c_int, c_int,
                                    POINTER(OracleRecipe), POINTER(POINTER(c_uint8)),
                                    POINTER(c_size_t)]
        L.oracle_encode_tiff.argtypes = [ctypes.c_void_p, c_size_t, POINTER(OracleRecipe),
                                         POINTER(POINTER(c_uint8)), POINTER(c_size_t)]
        L.oracle_fdwt.argtypes = [ctypes.c_void_p, c_int, c_int, c_int, c_int]
        L.oracle_t1_encode.argtypes = [ctypes.c_void_p, c_int, c_int, c_int, c_int,
                                       ctypes.c_void_p, c_int, POINTER(c_int), ctypes.c_void_p,
                                       ctypes.c_void_p, POINTER(c_int)]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_last_error.restype = ctypes.c_char_p
        _L = L
    return _L


def recipe(lossless: bool, **overrides) -> OracleRecipe:
    r = OracleRecipe()
    lib().oracle_recipe_init(byref(r), 1 if lossless else 0)
    for k, v in overrides.items():
        if k in ("prec_w_log2", "prec_h_log2"):
            arr = getattr(r, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(r, k, v)
    return r


def copy_recipe(src) -> OracleRecipe:
    """Oracle recipe with the same field values as a jp2hip Recipe."""
    r = OracleRecipe()
    for name, _ in OracleRecipe._fields_:
        v = getattr(src, name)
        if name in ("prec_w_log2", "prec_h_log2"):
            arr = getattr(r, name)
            for i in range(16):
                arr[i] = v[i]
        else:
            setattr(r, name, v)
    return r


def _take(out, n) -> bytes:
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib().oracle_free(out)


def encode(img: np.ndarray, rcp: OracleRecipe) -> bytes:
    a = np.ascontiguousarray(img)
    if a.ndim == 2:
        h, w, nc = a.shape[0], a.shape[1], 1
    else:
        h, w, nc = a.shape
    bits = a.dtype.itemsize * 8
    out = POINTER(c_uint8)()
    n = c_size_t()
    if lib().oracle_encode(a.ctypes.data, w, h, nc, bits, byref(rcp), byref(out), byref(n)):
        raise RuntimeError(lib().oracle_last_error().decode())
    return _take(out, n)


def encode_tiff(data: bytes, rcp: OracleRecipe) -> bytes:
    buf = ctypes.create_string_buffer(data, len(data))
    out = POINTER(c_uint8)()
    n = c_size_t()
    if lib().oracle_encode_tiff(buf, len(data), byref(rcp), byref(out), byref(n)):
        raise RuntimeError(lib().oracle_last_error().decode())
    return _take(out, n)


def fdwt(plane: np.ndarray, levels: int, reversible: bool) -> np.ndarray:
    a = np.ascontiguousarray(plane.astype(np.int32 if reversible else np.float32))
    lib().oracle_fdwt(a.ctypes.data, a.shape[1], a.shape[0], levels, 1 if reversible else 0)
    return a


def t1_encode(sm: np.ndarray, band: int, lossless: bool):
    """Tier-1 of one block of sign-magnitude int32 samples -> (bytes, rates, dists, P)."""
    a = np.ascontiguousarray(sm.astype(np.int32))
    h, w = a.shape
    cap = w * h * 8 + 256
    buf = (c_uint8 * cap)()
    rates = np.zeros(100, np.int32)
    dists = np.zeros(100, np.int64)
    n = c_int()
    P = c_int()
    np_ = lib().oracle_t1_encode(a.ctypes.data, w, h, band, 1 if lossless else 0, buf, cap,
                                 byref(n), rates.ctypes.data, dists.ctypes.data, byref(P))
    if np_ < 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return bytes(buf[:n.value]), rates[:np_].copy(), dists[:np_].copy(), P.value
