"""Binding of the bench-only library libshf_hb_bench.so
(include/shf_hash_batch_ceiling.h): the on-box HBM and VALU ceilings bench.py
reports every hashing kernel against. Not part of the product: the product
library libshf_hash_batch.so neither contains nor exports these kernels, and
nothing in sharedhashfile_amd/__init__.py loads this one.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
BENCH_LIB_PATH = os.path.join(_PKG, "libshf_hb_bench.so")

CEIL_COPY = 0
CEIL_READ16 = 1
CEIL_GATHER128 = 2
CEIL_STREAM16U = 3
CEIL_VALU_ADD = 4
CEIL_VALU_MUL = 5
CEIL_COPY4 = 6
CEIL_COPY_PLAIN = 7
CEIL_COPY_NT = 8
CEIL_COPY_SLEEP = 9
CEIL_COPY2 = 10
CEIL_READ16_NT = 11
CEIL_READ16_W1 = 12
CEIL_PROBE_ROWS = 13

_lib = None


def load():
    """Load libshf_hb_bench.so (raises when it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(BENCH_LIB_PATH):
        raise RuntimeError("libshf_hb_bench.so not built (%s); run python -m sharedhashfile_amd.build"
                           % BENCH_LIB_PATH)
    import sharedhashfile_amd as hb

    hb.load()  # the same HIP runtime (torch's) serves both libraries
    lib = ctypes.CDLL(BENCH_LIB_PATH)
    v = ctypes.c_void_p
    lib.shf_hb_ceiling_async.argtypes = [ctypes.c_int, v, ctypes.c_uint64, v, v, ctypes.c_uint64, v]
    lib.shf_hb_ceiling_async.restype = ctypes.c_int
    lib.shf_hb_host_device_ptr.argtypes = [v, ctypes.POINTER(v)]
    lib.shf_hb_host_device_ptr.restype = ctypes.c_int
    _lib = lib
    return lib


def host_device_ptr(host_ptr):
    """Device address (int) of page-locked host memory at host_ptr."""
    d = ctypes.c_void_p()
    rc = load().shf_hb_host_device_ptr(ctypes.c_void_p(host_ptr), ctypes.byref(d))
    if rc:
        raise RuntimeError("shf_hb_host_device_ptr: %d" % rc)
    return d.value
