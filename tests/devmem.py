"""Device buffers for GPU tests through the HIP runtime libjp2hip links
(/opt/rocm/lib/libamdhip64.so), not torch's bundled copy: a second HIP
runtime initialised after libjp2hip's finds no devices in this process."""
import ctypes
import os

_hip = None


def _rt():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamdhip64.so"))
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
        _hip.hipSetDevice.argtypes = [ctypes.c_int]
    return _hip


class DeviceBytes:
    """`data` copied into device memory of `device`; .ptr / .nbytes; free()."""

    def __init__(self, data, device: int = 0):
        """`data`: bytes, or a C-contiguous numpy array (copied without an
        intermediate bytes object)."""
        rt = _rt()
        if rt.hipSetDevice(device) != 0:
            raise RuntimeError("hipSetDevice failed")
        if hasattr(data, "ctypes"):
            n, src = int(data.nbytes), ctypes.c_void_p(data.ctypes.data)
        else:
            n, src = len(data), data
        self.nbytes = max(1, n)
        p = ctypes.c_void_p()
        if rt.hipMalloc(ctypes.byref(p), self.nbytes) != 0:
            raise RuntimeError("hipMalloc failed")
        self.ptr = p.value
        if n and rt.hipMemcpy(self.ptr, src, n, 1) != 0:  # hipMemcpyHostToDevice
            self.free()
            raise RuntimeError("hipMemcpy failed")

    def free(self):
        if self.ptr:
            _rt().hipFree(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()
