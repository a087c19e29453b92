"""Loader for the in-tree native library (fails loudly when it is absent)."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FHE_AMD_LIB: an alternative in-tree build of the same library (A/B experiments only)
lib_path = os.environ.get("FHE_AMD_LIB") or os.path.join(_HERE, "libfhe_amd.so")

vp = ctypes.c_void_p
u64 = ctypes.c_uint64
sz = ctypes.c_size_t


class FheHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fhe_hip error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """The loaded libfhe_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(lib_path):
            raise FheHipError(-11, f"native library not built: {lib_path} (run fhe_amd.build.build())")
        L = ctypes.CDLL(lib_path)
        L.fhe_hip_last_error.restype = ctypes.c_char_p
        L.fhe_hip_ntt_plan_create.argtypes = [u64, u64, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(vp),
                                              ctypes.POINTER(u64)]
        L.fhe_hip_ntt_plan_destroy.argtypes = [vp]
        L.fhe_hip_ntt_plan_destroy.restype = None
        L.fhe_hip_ntt_batch.argtypes = [vp, vp, sz, ctypes.c_int]
        L.fhe_hip_ntt_batch_device.argtypes = [vp, vp, vp, sz, ctypes.c_int, vp]
        L.fhe_hip_ntt_plan_stream.argtypes = [vp]
        L.fhe_hip_ntt_plan_stream.restype = vp
        L.fhe_hip_alloc.argtypes = [ctypes.c_int, sz, ctypes.POINTER(vp)]
        L.fhe_hip_free.argtypes = [vp]
        L.fhe_hip_copy_to_device.argtypes = [vp, vp, sz]
        L.fhe_hip_copy_to_host.argtypes = [vp, vp, sz]
        L.fhe_hip_synchronize.argtypes = [ctypes.c_int]
        L.fhe_hip_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise FheHipError(rc, lib().fhe_hip_last_error().decode())
    return rc


def ptr(a):
    """ctypes pointer to a C-contiguous numpy array."""
    if not a.flags.c_contiguous:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data_as(vp)
