"""MI355X batch key hashing for SharedHashFile (Python side of the C ABI).

The product is the C-ABI library ``libshf_hash_batch.so`` (include/shf_hash_batch.h).
This module only binds it with ctypes so the tests and bench.py can drive it with
torch device buffers or numpy host buffers. It mirrors the reference seam:

    shf_make_hash(key, key_len)            /root/reference/src/shf.c:450-462
      -> SHF_HASH {u64[0]=h1, u64[1]=h2}   /root/reference/src/shf.private.h:180-185

for a whole batch: results are (n, 2) uint64 arrays, row i = SHF_HASH of key i.

There is no CPU fallback. If the library is missing or cannot run on the device,
every call raises ShfHashBatchError / RuntimeError.
"""
import ctypes
import os

import numpy as np

SEED = 12345  # src/shf.c:456

OK = 0
ERR_ARG = -1
ERR_NODEV = -2
ERR_HIP = -3
ERR_NOMEM = -4
ERR_ARCH = -5
ERR_FORKED = -6  # a fork() child of a process that had used the library (include/shf_hash_batch.h "fork")

MEM_DEVICE = 0
MEM_HOST = 1

KERNEL_AUTO = 0
KERNEL_FIXED16 = 1
KERNEL_TILED = 2
KERNEL_GENERIC = 3
KERNEL_SPAN = 4
KERNEL_ROUND = 5
KERNEL_SPAN_PP = 6

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libshf_hash_batch.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "shf_hash_batch.h")

_lib = None


class ShfHashBatchError(RuntimeError):
    def __init__(self, status, where, hip_error=0):
        self.status = status
        self.hip_error = hip_error
        msg = "%s failed: %s (status %d" % (where, _strerror(status), status)
        if hip_error:
            msg += ", hipError %d" % hip_error
        super().__init__(msg + ")")


def _strerror(status):
    try:
        return load().shf_hash_batch_strerror(status).decode()
    except Exception:  # pragma: no cover - only when the library itself is broken
        return "status %d" % status


_VP = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_INT = ctypes.c_int

_SIGS = {
    "shf_hash_batch_fixed": [_VP, _U32, _U64, _U32, _VP, _INT],
    "shf_hash_batch_fixed_async": [_VP, _U32, _U64, _U32, _VP, _VP],
    "shf_hash_batch_var": [_VP, _VP, _U64, _U32, _VP, _INT],
    "shf_hash_batch_var_async": [_VP, _VP, _U64, _U32, _VP, _VP],
    "shf_uid_parts_batch_fixed": [_VP, _U32, _U64, _U32, _VP, _INT],
    "shf_uid_parts_batch_var": [_VP, _VP, _U64, _U32, _VP, _INT],
    "shf_uid_parts_batch_fixed_multi": [_VP, _U32, _U64, _U32, _VP, _INT],
    "shf_uid_parts_batch_var_multi": [_VP, _VP, _U64, _U32, _VP, _INT],
    "shf_uid_parts_batch_fixed_async": [_VP, _U32, _U64, _U32, _VP, _VP],
    "shf_uid_parts_batch_var_async": [_VP, _VP, _U64, _U32, _VP, _VP],
    "shf_hash_batch_fixed_multi": [_VP, _U32, _U64, _U32, _VP, _INT],
    "shf_hash_batch_var_multi": [_VP, _VP, _U64, _U32, _VP, _INT],
    "shf_hash_batch_fixed_kernel_async": [_VP, _U32, _U64, _U32, _VP, _INT, _VP],
    "shf_hash_batch_var_kernel_async": [_VP, _VP, _U64, _U32, _VP, _INT, _VP],
    "shf_hash_batch_var_sized_async": [_VP, _VP, _U64, _U64, _U32, _VP, _VP],
    "shf_hash_batch_var_sized_kernel_async": [_VP, _VP, _U64, _U64, _U32, _VP, _INT, _VP],
    "shf_row_index_create": [_U64, ctypes.POINTER(_VP)],
    "shf_row_index_destroy": [_VP],
    "shf_row_index_set_tabs": [_VP, _VP],
    "shf_row_index_set_rows": [_VP, _U64, _U64, _VP],
    "shf_row_index_device_ptrs": [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.POINTER(_U64)],
    "shf_probe_batch_fixed_async": [_VP, _VP, _U32, _U64, _U32, _VP, _VP, _VP],
    "shf_probe_batch_var_async": [_VP, _VP, _VP, _U64, _U32, _VP, _VP, _VP],
    "shf_probe_batch_hashes_async": [_VP, _VP, _U64, _VP, _VP],
    "shf_probe_batch_fixed": [_VP, _VP, _U32, _U64, _U32, _VP, _VP, _INT],
    "shf_probe_batch_var": [_VP, _VP, _VP, _U64, _U32, _VP, _VP, _INT],
    "shf_probe_batch_fixed_kernel_async": [_VP, _VP, _U32, _U64, _U32, _VP, _VP, _INT, _VP],
    "shf_hash_batch_status": [_VP],
    "shf_tab_copy_batch_async": [_VP, _U64, _VP, _U64, _VP, _U32, _VP, _U32, _VP, _VP],
    "shf_tab_copy_batch": [_VP, _U64, _VP, _U64, _VP, _U32, _VP, _U32, _VP, _INT],
    "shf_tab_part_redirect": [_VP, _U32, _U32],
    "shf_win_order_workspace_bytes": [_U64],
    "shf_win_order_async": [_VP, _U64, _VP, _VP, _VP, ctypes.c_size_t, _VP],
    "shf_win_order": [_VP, _U64, _VP, _VP, _INT],
    "shf_hash_batch_fixed_win": [_VP, _U32, _U64, _U32, _VP, _VP, _VP, _INT],
    "shf_uid_parts_batch_fixed_win": [_VP, _U32, _U64, _U32, _VP, _VP, _VP, _INT],
    "shf_uid_parts_batch_var_win": [_VP, _VP, _U64, _U32, _VP, _VP, _VP, _INT],
    "shf_hash_batch_var_win": [_VP, _VP, _U64, _U32, _VP, _VP, _VP, _INT],
    "shf_hash_batch_fixed_win_async": [_VP, _U32, _U64, _U32, _VP, _VP, _VP, _VP, ctypes.c_size_t, _VP],
    "shf_hash_batch_var_win_async": [_VP, _VP, _U64, _U32, _VP, _VP, _VP, _VP, ctypes.c_size_t, _VP],
    "shf_hash_batch_fixed_win_kernel_async": [_VP, _U32, _U64, _U32, _VP, _VP, _VP, _VP, ctypes.c_size_t, _INT,
                                              _VP],
    "shf_hash_batch_var_win_kernel_async": [_VP, _VP, _U64, _U32, _VP, _VP, _VP, _VP, ctypes.c_size_t, _INT, _VP],
    "shf_hash_batch_device_count": [],
    "shf_hash_batch_check_device": [],
    "shf_hash_batch_last_hip_error": [],
    "shf_hash_batch_release": [],
    "shf_hash_batch_strerror": [_INT],
    "shf_hash_batch_version": [],
}


_RESTYPES = {"shf_hash_batch_strerror": ctypes.c_char_p, "shf_hash_batch_version": ctypes.c_char_p,
             "shf_win_order_workspace_bytes": ctypes.c_size_t}


def load(path=None):
    """Load the C-ABI library (raises loudly when it is not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError("libshf_hash_batch.so not built (%s); run python -m sharedhashfile_amd.build" % p)
    try:  # torch first: its bundled libamdhip64 (SONAME libamdhip64.so.7) then serves this library too,
        import torch  # noqa: F401  so one HIP runtime owns every stream, event and buffer of the process
    except ImportError:
        pass
    lib = ctypes.CDLL(p)
    for name, args in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if path is None:  # the in-tree build must export everything
                raise RuntimeError("%s does not export %s: rebuild it" % (p, name))
            continue  # an older variant loaded side by side for an A/B (tools/ab.py)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if path is None:
        _lib = lib
    return lib


def header_functions(header=HEADER_PATH):
    """Names of every function include/shf_hash_batch.h declares."""
    import re

    txt = open(header).read()
    return sorted(set(re.findall(r"SHF_HB_API\s+(?:const\s+char\s*\*|int|size_t)\s*(shf_\w+)\s*\(", txt)))


def _check(rc, where):
    if rc != OK:
        raise ShfHashBatchError(rc, where, load().shf_hash_batch_last_hip_error())


# ---------------------------------------------------------------------------
# torch device-resident helpers (pointers are HBM addresses)
# ---------------------------------------------------------------------------
def _record(tensors, stream):
    """Tensors allocated here on the current stream and used by kernels on `stream`:
    the kernels may still run after the call returns, so keep the caching allocator
    from handing their bytes out before `stream` gets there."""
    if stream is not None:
        for t in tensors:
            t.record_stream(stream)


def _stream_handle(stream):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _require_cuda(t, name, dtypes):
    import torch

    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise TypeError("%s must be a CUDA (HIP) tensor" % name)
    if t.dtype not in dtypes:
        raise TypeError("%s must be %s, not %s" % (name, " or ".join(str(d) for d in dtypes), t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)


def _require_cuda_u8(t, name):
    import torch

    _require_cuda(t, name, (torch.uint8,))


def _offset_dtypes():
    import torch

    return tuple(d for d in (torch.int64, getattr(torch, "uint64", None)) if d is not None)


def _require_offsets(offsets, data):
    """offsets: contiguous 1-D int64/uint64 CUDA tensor of n + 1 >= 1 entries on data's device."""
    _require_cuda(offsets, "offsets", _offset_dtypes())
    if offsets.dim() != 1 or offsets.numel() < 1:
        raise ValueError("offsets must be 1-D with n + 1 >= 1 entries")
    if offsets.device != data.device:
        raise ValueError("offsets (%s) and data (%s) must be on the same GPU" % (offsets.device, data.device))
    return offsets.numel() - 1


def _require_out(out, shape, dtypes, device):
    _require_cuda(out, "out", dtypes)
    if tuple(out.shape) != tuple(shape):
        raise ValueError("out must have shape %s, not %s" % (tuple(shape), tuple(out.shape)))
    if out.device != device:
        raise ValueError("out (%s) must be on %s" % (out.device, device))


def _on(t):
    """The device context of tensor t: the library runs on the calling thread's
    current device and stream, so every call is made on t's device."""
    import torch

    return torch.cuda.device(t.device)


def status(stream=None):
    """shf_hash_batch_status(): raises ShfHashBatchError(ERR_ARG) if an async
    variable-length call of this thread met an invalid key since the last query."""
    _check(load().shf_hash_batch_status(_stream_handle(stream)), "shf_hash_batch_status")


def hash_fixed(keys, key_len=None, seed=SEED, out=None, stream=None, kernel=KERNEL_AUTO):
    """Hash n fixed-length keys resident on the GPU.

    keys: uint8 CUDA tensor (n, key_len) or flat with key_len given.
    Returns an int64 CUDA tensor (n, 2) holding the uint64 bit patterns of
    (h1, h2) = SHF_HASH.u64[0..1] per key. Asynchronous on `stream`.
    """
    import torch

    _require_cuda_u8(keys, "keys")
    if key_len is None:
        if keys.dim() != 2:
            raise ValueError("pass key_len for a flat key buffer")
        n, key_len = keys.shape
    else:
        n = keys.numel() // key_len if key_len else 0
    mine = []
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=keys.device)
        mine.append(out)
    _require_out(out, (n, 2), (torch.int64,), keys.device)
    with _on(keys):
        rc = load().shf_hash_batch_fixed_kernel_async(
            ctypes.c_void_p(keys.data_ptr()), key_len, n, seed, ctypes.c_void_p(out.data_ptr()), kernel,
            _stream_handle(stream))
    _check(rc, "shf_hash_batch_fixed_kernel_async")
    _record(mine, stream)
    return out


def hash_var(data, offsets, seed=SEED, out=None, stream=None, kernel=KERNEL_AUTO, key_bytes=None):
    """Hash n variable-length keys on the GPU: key i = data[offsets[i]:offsets[i+1]].

    data: uint8 CUDA tensor; offsets: int64 CUDA tensor of n + 1 entries.
    key_bytes: offsets[n] - offsets[0] if known (sizes the span kernel's LDS
    window: shf_hash_batch_var_sized_kernel_async); None = unknown.
    """
    import torch

    _require_cuda_u8(data, "data")
    n = _require_offsets(offsets, data)
    mine = []
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=data.device)
        mine.append(out)
    _require_out(out, (n, 2), (torch.int64,), data.device)
    with _on(data):
        if key_bytes is None:
            rc = load().shf_hash_batch_var_kernel_async(
                ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offsets.data_ptr()), n, seed,
                ctypes.c_void_p(out.data_ptr()), kernel, _stream_handle(stream))
            name = "shf_hash_batch_var_kernel_async"
        else:
            rc = load().shf_hash_batch_var_sized_kernel_async(
                ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offsets.data_ptr()), n, int(key_bytes), seed,
                ctypes.c_void_p(out.data_ptr()), kernel, _stream_handle(stream))
            name = "shf_hash_batch_var_sized_kernel_async"
    _check(rc, name)
    _record(mine, stream)
    return out


def uid_parts_fixed(keys, key_len=None, seed=SEED, out=None, stream=None):
    """Packed win/tab/row/rnd (include/shf_hash_batch.h SHF_UID_PARTS_*) per key."""
    import torch

    _require_cuda_u8(keys, "keys")
    if key_len is None:
        n, key_len = keys.shape
    else:
        n = keys.numel() // key_len if key_len else 0
    mine = []
    if out is None:
        out = torch.empty((n,), dtype=torch.int64, device=keys.device)
        mine.append(out)
    _require_out(out, (n,), (torch.int64,), keys.device)
    with _on(keys):
        rc = load().shf_uid_parts_batch_fixed_async(
            ctypes.c_void_p(keys.data_ptr()), key_len, n, seed, ctypes.c_void_p(out.data_ptr()),
            _stream_handle(stream))
    _check(rc, "shf_uid_parts_batch_fixed_async")
    _record(mine, stream)
    return out


def uid_parts_var(data, offsets, seed=SEED, out=None, stream=None):
    import torch

    _require_cuda_u8(data, "data")
    n = _require_offsets(offsets, data)
    mine = []
    if out is None:
        out = torch.empty((n,), dtype=torch.int64, device=data.device)
        mine.append(out)
    _require_out(out, (n,), (torch.int64,), data.device)
    with _on(data):
        rc = load().shf_uid_parts_batch_var_async(
            ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offsets.data_ptr()), n, seed,
            ctypes.c_void_p(out.data_ptr()), _stream_handle(stream))
    _check(rc, "shf_uid_parts_batch_var_async")
    _record(mine, stream)
    return out


# ---------------------------------------------------------------------------
# Row pre-probe (include/shf_hash_batch.h "row pre-probe")
# ---------------------------------------------------------------------------
PROBE_NONE = 0xFFFFFFFF
ROW_INDEX_TABS = 256 * 2048
ROW_INDEX_SLOT_BYTES = 65536


def _buffer(a, np_dtype):
    """(pointer, nbytes) of a contiguous numpy array or CUDA tensor, plus the object to keep alive."""
    try:
        import torch

        if isinstance(a, torch.Tensor):
            if not a.is_cuda or not a.is_contiguous():
                raise ValueError("tensors must be contiguous CUDA tensors")
            return (ctypes.c_void_p(a.data_ptr()), a.numel() * a.element_size()), a
    except ImportError:  # pragma: no cover
        pass
    arr = np.ascontiguousarray(a)
    if arr.dtype != np_dtype:
        arr = arr.view(np_dtype) if arr.dtype.itemsize == np.dtype(np_dtype).itemsize or np_dtype == np.uint8 \
            else arr.astype(np_dtype)
    return (ctypes.c_void_p(arr.ctypes.data), arr.nbytes), arr


class RowIndex:
    """Device copy of a store's rows (shf_row_index): tab_slot map + n_slots x 64 KiB.

    tab_slot: (256*2048,) uint32 host array, entry (slot << 11) | tab or PROBE_NONE.
    rows: (n_slots * 65536,) uint8 host array of SHF_TAB_MMAP.row[] blocks.
    Either may be omitted and filled later (set_tabs / set_rows / device_ptrs).
    """

    def __init__(self, n_slots, tab_slot=None, rows=None):
        lib = load()
        h = ctypes.c_void_p()
        _check(lib.shf_row_index_create(int(n_slots), ctypes.byref(h)), "shf_row_index_create")
        self._h = h
        self.n_slots = int(n_slots)
        if tab_slot is not None:
            self.set_tabs(tab_slot)
        if rows is not None:
            self.set_rows(0, rows)

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("row index destroyed")
        return self._h

    def set_tabs(self, tab_slot):
        """tab_slot: numpy uint32 array or CUDA tensor (int32/uint32 bits) of 256*2048 entries."""
        t, keep = _buffer(tab_slot, np.uint32)
        if t[1] != ROW_INDEX_TABS * 4:
            raise ValueError("tab_slot needs %d entries" % ROW_INDEX_TABS)
        _check(load().shf_row_index_set_tabs(self.handle, t[0]), "shf_row_index_set_tabs")
        del keep

    def set_rows(self, first, rows):
        """rows: whole 64 KiB slots, numpy array or CUDA tensor."""
        r, keep = _buffer(rows, np.uint8)
        if r[1] % ROW_INDEX_SLOT_BYTES:
            raise ValueError("rows must be whole 64 KiB slots")
        _check(load().shf_row_index_set_rows(self.handle, int(first), r[1] // ROW_INDEX_SLOT_BYTES, r[0]),
               "shf_row_index_set_rows")
        del keep

    def device_ptrs(self):
        ts, rows, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        _check(load().shf_row_index_device_ptrs(self.handle, ctypes.byref(ts), ctypes.byref(rows), ctypes.byref(n)),
               "shf_row_index_device_ptrs")
        return ts.value, rows.value, n.value

    def close(self):
        if self._h is not None:
            load().shf_row_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def probe_fixed(index, keys, key_len=None, seed=SEED, out=None, hashes=False, stream=None, kernel=KERNEL_AUTO):
    """Hash + row pre-probe of fixed-length keys on the GPU.

    Returns an int32 CUDA tensor (n, 4): {uid, pos, mask | tab << 16, slot} per key
    (struct shf_probe), and with hashes=True also the (n, 2) int64 hash tensor.
    """
    import torch

    _require_cuda_u8(keys, "keys")
    if key_len is None:
        n, key_len = keys.shape
    else:
        n = keys.numel() // key_len if key_len else 0
    mine = []
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=keys.device)
        mine.append(out)
    _require_out(out, (n, 4), (torch.int32,), keys.device)
    hout = torch.empty((n, 2), dtype=torch.int64, device=keys.device) if hashes else None
    if hout is not None:
        mine.append(hout)
    with _on(keys):
        rc = load().shf_probe_batch_fixed_kernel_async(
            index.handle, ctypes.c_void_p(keys.data_ptr()), key_len, n, seed,
            ctypes.c_void_p(hout.data_ptr() if hout is not None else 0), ctypes.c_void_p(out.data_ptr()), kernel,
            _stream_handle(stream))
    _check(rc, "shf_probe_batch_fixed_kernel_async")
    _record(mine, stream)
    return (out, hout) if hashes else out


def probe_var(index, data, offsets, seed=SEED, out=None, hashes=False, stream=None):
    import torch

    _require_cuda_u8(data, "data")
    n = _require_offsets(offsets, data)
    mine = []
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=data.device)
        mine.append(out)
    _require_out(out, (n, 4), (torch.int32,), data.device)
    hout = torch.empty((n, 2), dtype=torch.int64, device=data.device) if hashes else None
    if hout is not None:
        mine.append(hout)
    with _on(data):
        rc = load().shf_probe_batch_var_async(
            index.handle, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offsets.data_ptr()), n, seed,
            ctypes.c_void_p(hout.data_ptr() if hout is not None else 0), ctypes.c_void_p(out.data_ptr()),
            _stream_handle(stream))
    _check(rc, "shf_probe_batch_var_async")
    _record(mine, stream)
    return (out, hout) if hashes else out


def probe_hashes(index, hashes, out=None, stream=None):
    """Row pre-probe of precomputed (n, 2) int64 CUDA hashes."""
    import torch

    _require_cuda(hashes, "hashes", _offset_dtypes())
    if hashes.dim() != 2 or hashes.shape[1] != 2:
        raise ValueError("hashes must have shape (n, 2)")
    n = hashes.shape[0]
    mine = []
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=hashes.device)
        mine.append(out)
    _require_out(out, (n, 4), (torch.int32,), hashes.device)
    with _on(hashes):
        rc = load().shf_probe_batch_hashes_async(index.handle, ctypes.c_void_p(hashes.data_ptr()), n,
                                                 ctypes.c_void_p(out.data_ptr()), _stream_handle(stream))
    _check(rc, "shf_probe_batch_hashes_async")
    _record(mine, stream)
    return out


def win_order(hashes, perm=None, win_start=None, workspace=None, stream=None):
    """Window order of (n, 2) int64/uint64 CUDA hashes (shf_win_order_async):
    returns (perm, win_start), int32 CUDA tensors of n and 257 entries (the
    indices are unsigned 32-bit: view them as such past 2^31 keys)."""
    import torch

    _require_cuda(hashes, "hashes", _offset_dtypes())
    if hashes.dim() != 2 or hashes.shape[1] != 2:
        raise ValueError("hashes must have shape (n, 2)")
    n = hashes.shape[0]
    dev = hashes.device
    mine = []  # tensors allocated here (on the current stream)
    if perm is None:
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        mine.append(perm)
    _require_out(perm, (n,), (torch.int32,), dev)
    if win_start is None:
        win_start = torch.empty(257, dtype=torch.int32, device=dev)
        mine.append(win_start)
    _require_out(win_start, (257,), (torch.int32,), dev)
    lib = load()
    need = lib.shf_win_order_workspace_bytes(n)
    if workspace is None:
        workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        mine.append(workspace)
    _require_cuda_u8(workspace, "workspace")
    with _on(hashes):
        rc = lib.shf_win_order_async(ctypes.c_void_p(hashes.data_ptr()), n, ctypes.c_void_p(perm.data_ptr()),
                                     ctypes.c_void_p(win_start.data_ptr()), ctypes.c_void_p(workspace.data_ptr()),
                                     workspace.numel(), _stream_handle(stream))
    _check(rc, "shf_win_order_async")
    _record(mine, stream)
    return perm, win_start


def _win_outputs(n, dev, out, perm, win_start, workspace):
    import torch

    mine = []  # tensors allocated here (on the current stream)
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        mine.append(out)
    _require_out(out, (n, 2), _offset_dtypes(), dev)
    if perm is None:
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        mine.append(perm)
    _require_out(perm, (n,), (torch.int32,), dev)
    if win_start is None:
        win_start = torch.empty(257, dtype=torch.int32, device=dev)
        mine.append(win_start)
    _require_out(win_start, (257,), (torch.int32,), dev)
    if workspace is None:
        workspace = torch.empty(max(load().shf_win_order_workspace_bytes(n), 1), dtype=torch.uint8, device=dev)
        mine.append(workspace)
    _require_cuda_u8(workspace, "workspace")
    return out, perm, win_start, workspace, mine


def hash_fixed_win(keys, key_len, seed=SEED, out=None, perm=None, win_start=None, workspace=None, stream=None,
                   kernel=KERNEL_AUTO):
    """Hash + window order in one call (shf_hash_batch_fixed_win_async):
    returns (hashes (n, 2) int64, perm int32[n], win_start int32[257]), the
    order exactly what win_order(hashes) gives, computed without reading the
    records back (16-B keys: the hashing kernel ranks each chunk itself; other
    lengths: it writes each key's window byte beside its record)."""
    _require_cuda_u8(keys, "keys")
    if key_len <= 0 or keys.numel() % key_len:
        raise ValueError("keys.numel() must be a multiple of key_len")
    n = keys.numel() // key_len
    out, perm, win_start, workspace, mine = _win_outputs(n, keys.device, out, perm, win_start, workspace)
    with _on(keys):
        rc = load().shf_hash_batch_fixed_win_kernel_async(
            ctypes.c_void_p(keys.data_ptr()), key_len, n, seed, ctypes.c_void_p(out.data_ptr()),
            ctypes.c_void_p(perm.data_ptr()), ctypes.c_void_p(win_start.data_ptr()),
            ctypes.c_void_p(workspace.data_ptr()), workspace.numel(), kernel, _stream_handle(stream))
    _check(rc, "shf_hash_batch_fixed_win_kernel_async")
    _record(mine, stream)
    return out, perm, win_start


def hash_var_win(data, offsets, seed=SEED, out=None, perm=None, win_start=None, workspace=None, stream=None,
                 kernel=KERNEL_AUTO):
    """Variable-length keys: hash + window order in one call (shf_hash_batch_var_win_async)."""
    _require_cuda_u8(data, "data")
    _require_cuda(offsets, "offsets", _offset_dtypes())
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets needs n + 1 entries")
    out, perm, win_start, workspace, mine = _win_outputs(n, data.device, out, perm, win_start, workspace)
    with _on(data):
        rc = load().shf_hash_batch_var_win_kernel_async(
            ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offsets.data_ptr()), n, seed,
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(perm.data_ptr()), ctypes.c_void_p(win_start.data_ptr()),
            ctypes.c_void_p(workspace.data_ptr()), workspace.numel(), kernel, _stream_handle(stream))
    _check(rc, "shf_hash_batch_var_win_kernel_async")
    _record(mine, stream)
    return out, perm, win_start


def hash_fixed_win_host(keys, key_len=None, seed=SEED):
    """Host keys in; host (hashes (n, 2) uint64, perm uint32[n], win_start uint32[257]) out
    (shf_hash_batch_fixed_win, SHF_HASH_MEM_HOST: the window bytes stay on the device)."""
    keys = _np_u8(keys)
    if key_len is None:
        key_len = keys.shape[-1] if keys.ndim == 2 else 16
    flat = keys.reshape(-1)
    n = flat.size // key_len if key_len else 0
    out = np.empty((n, 2), dtype=np.uint64)
    perm = np.empty(n, dtype=np.uint32)
    ws = np.empty(257, dtype=np.uint32)
    rc = load().shf_hash_batch_fixed_win(flat.ctypes.data, key_len, n, seed, out.ctypes.data, perm.ctypes.data,
                                         ws.ctypes.data, MEM_HOST)
    _check(rc, "shf_hash_batch_fixed_win")
    return out, perm, ws


def hash_var_win_host(data, offsets, seed=SEED):
    """Variable-length host keys: (hashes, perm, win_start) (shf_hash_batch_var_win, SHF_HASH_MEM_HOST)."""
    data = _np_u8(data).reshape(-1)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = off.size - 1
    out = np.empty((n, 2), dtype=np.uint64)
    perm = np.empty(n, dtype=np.uint32)
    ws = np.empty(257, dtype=np.uint32)
    rc = load().shf_hash_batch_var_win(data.ctypes.data, off.ctypes.data, n, seed, out.ctypes.data,
                                       perm.ctypes.data, ws.ctypes.data, MEM_HOST)
    _check(rc, "shf_hash_batch_var_win")
    return out, perm, ws


def uid_parts_fixed_win_host(keys, key_len=None, seed=SEED):
    """Host keys in; host (parts uint64[n], perm uint32[n], win_start uint32[257]) out
    (shf_uid_parts_batch_fixed_win, SHF_HASH_MEM_HOST)."""
    keys = _np_u8(keys)
    if key_len is None:
        key_len = keys.shape[-1] if keys.ndim == 2 else 16
    flat = keys.reshape(-1)
    n = flat.size // key_len if key_len else 0
    parts = np.empty(n, dtype=np.uint64)
    perm = np.empty(n, dtype=np.uint32)
    ws = np.empty(257, dtype=np.uint32)
    _check(load().shf_uid_parts_batch_fixed_win(flat.ctypes.data, key_len, n, seed, parts.ctypes.data,
                                                perm.ctypes.data, ws.ctypes.data, MEM_HOST),
           "shf_uid_parts_batch_fixed_win")
    return parts, perm, ws


def uid_parts_var_win_host(data, offsets, seed=SEED):
    """Variable-length host keys: (parts, perm, win_start) (shf_uid_parts_batch_var_win, SHF_HASH_MEM_HOST)."""
    data = _np_u8(data).reshape(-1)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = off.size - 1
    parts = np.empty(n, dtype=np.uint64)
    perm = np.empty(n, dtype=np.uint32)
    ws = np.empty(257, dtype=np.uint32)
    _check(load().shf_uid_parts_batch_var_win(data.ctypes.data, off.ctypes.data, n, seed, parts.ctypes.data,
                                              perm.ctypes.data, ws.ctypes.data, MEM_HOST),
           "shf_uid_parts_batch_var_win")
    return parts, perm, ws


def win_order_host(hashes):
    """Host (n, 2) uint64 hashes in, host (perm uint32[n], win_start uint32[257]) out (shf_win_order)."""
    h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
    n = h.shape[0]
    perm = np.empty(n, dtype=np.uint32)
    ws = np.empty(257, dtype=np.uint32)
    rc = load().shf_win_order(h.ctypes.data, n, perm.ctypes.data, ws.ctypes.data, MEM_HOST)
    _check(rc, "shf_win_order")
    return perm, ws


def probe_fixed_host(index, keys, key_len=None, seed=SEED, hashes=False):
    """Host buffers in and out: (n, 4) uint32 probe records (+ (n, 2) uint64 hashes)."""
    keys = _np_u8(keys)
    if key_len is None:
        n, key_len = keys.shape
    else:
        n = keys.size // key_len if key_len else 0
    rec = np.empty((n, 4), dtype=np.uint32)
    h = np.empty((n, 2), dtype=np.uint64) if hashes else None
    rc = load().shf_probe_batch_fixed(index.handle, keys.ctypes.data, key_len, n, seed,
                                      h.ctypes.data if h is not None else None, rec.ctypes.data, MEM_HOST)
    _check(rc, "shf_probe_batch_fixed")
    return (rec, h) if hashes else rec


def probe_var_host(index, data, offsets, seed=SEED, hashes=False):
    data = _np_u8(data)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = max(offsets.size - 1, 0)
    rec = np.empty((n, 4), dtype=np.uint32)
    h = np.empty((n, 2), dtype=np.uint64) if hashes else None
    rc = load().shf_probe_batch_var(index.handle, data.ctypes.data, offsets.ctypes.data, n, seed,
                                    h.ctypes.data if h is not None else None, rec.ctypes.data, MEM_HOST)
    _check(rc, "shf_probe_batch_var")
    return (rec, h) if hashes else rec


# ---------------------------------------------------------------------------
# numpy host-memory helpers (library stages through pinned buffers)
# ---------------------------------------------------------------------------
def _np_u8(a):
    a = np.ascontiguousarray(a)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a


def hash_fixed_host(keys, key_len=None, seed=SEED, n_devices=None):
    """Host buffers in, host (n, 2) uint64 out. n_devices: None = current device only."""
    keys = _np_u8(keys)
    if key_len is None:
        n, key_len = keys.shape
    else:
        n = keys.size // key_len if key_len else 0
    out = np.empty((n, 2), dtype=np.uint64)
    lib = load()
    if n_devices is None:
        rc = lib.shf_hash_batch_fixed(keys.ctypes.data, key_len, n, seed, out.ctypes.data, MEM_HOST)
        _check(rc, "shf_hash_batch_fixed")
    else:
        rc = lib.shf_hash_batch_fixed_multi(keys.ctypes.data, key_len, n, seed, out.ctypes.data, n_devices)
        _check(rc, "shf_hash_batch_fixed_multi")
    return out


def uid_parts_fixed_host(keys, key_len=None, seed=SEED, n_devices=None):
    """Host keys in, host uint64[n] UID parts out (shf_uid_parts_batch_fixed,
    SHF_HASH_MEM_HOST: 8 B per key back instead of 16). n_devices: None = the
    current device only, else shf_uid_parts_batch_fixed_multi."""
    keys = _np_u8(keys)
    if key_len is None:
        n, key_len = keys.shape
    else:
        n = keys.size // key_len if key_len else 0
    out = np.empty(n, dtype=np.uint64)
    if n_devices is None:
        _check(load().shf_uid_parts_batch_fixed(keys.ctypes.data, key_len, n, seed, out.ctypes.data, MEM_HOST),
               "shf_uid_parts_batch_fixed")
    else:
        _check(load().shf_uid_parts_batch_fixed_multi(keys.ctypes.data, key_len, n, seed, out.ctypes.data,
                                                      n_devices), "shf_uid_parts_batch_fixed_multi")
    return out


def uid_parts_var_host(data, offsets, seed=SEED, n_devices=None):
    """Variable-length host keys in, host uint64[n] UID parts out (shf_uid_parts_batch_var, SHF_HASH_MEM_HOST;
    n_devices as uid_parts_fixed_host)."""
    data = _np_u8(data)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = max(offsets.size - 1, 0)
    out = np.empty(n, dtype=np.uint64)
    if n_devices is None:
        _check(load().shf_uid_parts_batch_var(data.ctypes.data, offsets.ctypes.data, n, seed, out.ctypes.data,
                                              MEM_HOST), "shf_uid_parts_batch_var")
    else:
        _check(load().shf_uid_parts_batch_var_multi(data.ctypes.data, offsets.ctypes.data, n, seed, out.ctypes.data,
                                                    n_devices), "shf_uid_parts_batch_var_multi")
    return out


def hash_var_host(data, offsets, seed=SEED, n_devices=None):
    data = _np_u8(data)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty((max(n, 0), 2), dtype=np.uint64)
    lib = load()
    if n_devices is None:
        rc = lib.shf_hash_batch_var(data.ctypes.data, offsets.ctypes.data, max(n, 0), seed, out.ctypes.data, MEM_HOST)
        _check(rc, "shf_hash_batch_var")
    else:
        rc = lib.shf_hash_batch_var_multi(data.ctypes.data, offsets.ctypes.data, max(n, 0), seed, out.ctypes.data,
                                          n_devices)
        _check(rc, "shf_hash_batch_var_multi")
    return out


# ---------------------------------------------------------------------------
# Tab part / shrink copy (include/shf_hash_batch.h)
# ---------------------------------------------------------------------------
TAB_NONE = 0xFFFF
TAB_DATA = 24 + 512 * 16 * 8  # offsetof(SHF_TAB_MMAP, data)


class TabJob(ctypes.Structure):
    _fields_ = [("src", _U64), ("src_len", _U64), ("keep", _U64), ("move", _U64), ("cap", _U64), ("map", _U32),
                ("tab_new", ctypes.c_uint16), ("keep_type", ctypes.c_uint8), ("move_type", ctypes.c_uint8),
                ("status", ctypes.c_int32), ("reserved", _U32)]


class TabParams(ctypes.Structure):
    _fields_ = [("fixed", _U32), ("fixed_key_len", _U32), ("fixed_val_len", _U32), ("data_needed_factor", _U32)]


def tab_part_redirect(tab_map, tab_old, tab_new):
    """shf_tab_part()'s map redirect (a new uint16 array)."""
    m = np.array(tab_map, dtype=np.uint16)
    _check(load().shf_tab_part_redirect(m.ctypes.data, tab_old, tab_new), "shf_tab_part_redirect")
    return m


def tab_copy(images, maps=None, tab_new=None, fixed=0, key_len=0, val_len=0, factor=1, keep_type=0x3E,
             move_type=0x3E, cap=None, device=None):
    """Part / shrink copy of a batch of tab images on the GPU.

    images: list of uint8 numpy tab images; maps: list of 2048-entry uint16
    maps (after the redirect) per image (None for shrink-only);
    tab_new: list of new-tab numbers (TAB_NONE: shrink). Returns a list of
    (keep, move) uint8 numpy images of `cap` bytes each (zero past tab_used;
    move None for a shrink). keep_type / move_type: int or per-job lists.
    Device-resident: the images are packed into one HBM buffer and copied back.
    """
    import torch

    n = len(images)
    tab_new = [TAB_NONE] * n if tab_new is None else list(tab_new)
    kt = keep_type if isinstance(keep_type, (list, tuple)) else [keep_type] * n
    mt = move_type if isinstance(move_type, (list, tuple)) else [move_type] * n
    dev = device or torch.device("cuda", torch.cuda.current_device())
    al = lambda x: (x + 4095) // 4096 * 4096
    caps = [al(int(cap or img.size)) for img in images]
    src_off, off = [], 0
    for img in images:
        src_off.append(off)
        off += al(img.size)
    src = torch.zeros(max(off, 8), dtype=torch.uint8, device=dev)
    for o, img in zip(src_off, images):
        src[o:o + img.size] = torch.from_numpy(np.ascontiguousarray(img, dtype=np.uint8)).to(dev)
    jobs = (TabJob * n)()
    doff = 0
    for i in range(n):
        j = jobs[i]
        j.src, j.src_len, j.cap, j.map = src_off[i], images[i].size, caps[i], i if maps is not None else 0
        j.keep = doff
        doff += caps[i]
        j.tab_new = tab_new[i]
        if tab_new[i] != TAB_NONE:
            j.move = doff
            doff += caps[i]
        j.keep_type, j.move_type, j.status = kt[i], mt[i], 1
    dst = torch.zeros(max(doff, 8), dtype=torch.uint8, device=dev)
    d_jobs = torch.from_numpy(np.frombuffer(bytes(jobs), dtype=np.uint8).copy()).to(dev)
    d_maps = None
    if maps is not None:
        d_maps = torch.from_numpy(np.ascontiguousarray(np.stack([np.asarray(m, np.uint16) for m in maps]))
                                  .view(np.int16)).to(dev)
    prm = TabParams(int(bool(fixed)), key_len, val_len, factor)
    with _on(src):
        rc = load().shf_tab_copy_batch_async(
            ctypes.c_void_p(src.data_ptr()), src.numel(), ctypes.c_void_p(dst.data_ptr()), dst.numel(),
            ctypes.c_void_p(d_jobs.data_ptr()), n, ctypes.c_void_p(d_maps.data_ptr() if d_maps is not None else 0),
            n if d_maps is not None else 0, ctypes.byref(prm), _stream_handle(None))
    _check(rc, "shf_tab_copy_batch_async")
    torch.cuda.synchronize(dev)
    done = (TabJob * n).from_buffer_copy(d_jobs.cpu().numpy().tobytes())
    bad = [i for i in range(n) if done[i].status != OK]
    if bad:
        raise ShfHashBatchError(ERR_ARG, "shf_tab_copy_batch_async (jobs %s)" % bad[:8])
    out_h = dst.cpu().numpy()
    res = []
    for i in range(n):
        j = jobs[i]
        keep = out_h[j.keep:j.keep + caps[i]].copy()
        move = out_h[j.move:j.move + caps[i]].copy() if tab_new[i] != TAB_NONE else None
        res.append((keep, move))
    return res


def device_count():
    return load().shf_hash_batch_device_count()


def check_device():
    _check(load().shf_hash_batch_check_device(), "shf_hash_batch_check_device")


def release():
    """shf_hash_batch_release(): free the calling thread's per-device state, the
    state exited threads left for reuse, and the staging pools' idle slots."""
    _check(load().shf_hash_batch_release(), "shf_hash_batch_release")
