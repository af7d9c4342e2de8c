"""fork() after use (include/shf_hash_batch.h "fork").

SharedHashFile's load test forks up to 36 workers
(/root/reference/src/test.f.shf.c:248, :274-336). The HIP runtime and this
library's staging pools and copy threads do not survive a fork, so a child of a
process that has used the library must get an error, not a hang and not a call
into the parent's runtime state: every entry point that can reach HIP returns
SHF_HB_ERR_FORKED first.

CPU only (this container has no GPU): here every HIP call fails with
SHF_HB_ERR_NODEV, so a child that answers SHF_HB_ERR_FORKED instead proves the
guard ran before any HIP call. Skipped where a GPU is visible -- a process that
has initialised the GPU must not be forked on the GPU box. The copy workers'
own fork handling is tests/c/test_host_plan.cpp test_fork (ASan and TSan).
"""
import os
import subprocess
import sys

import pytest

import sharedhashfile_amd as hb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


EXEMPT = {"shf_win_order_workspace_bytes", "shf_tab_part_redirect", "shf_hash_batch_last_hip_error",
          "shf_hash_batch_strerror", "shf_hash_batch_version"}

CHILD = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import sharedhashfile_amd as hb
lib = ctypes.CDLL(hb.LIB_PATH)  # not hb.load(): no torch, nothing touches HIP before the calls below
for name, args in hb._SIGS.items():
    getattr(lib, name).argtypes = args
    getattr(lib, name).restype = hb._RESTYPES.get(name, ctypes.c_int)
exempt = set(sys.argv[2].split(","))
names = [f for f in hb.header_functions() if f not in exempt]

def fork_and(fn):
    pid = os.fork()
    if pid == 0:
        try:
            os._exit(fn())
        except BaseException:
            import traceback
            traceback.print_exc()
            sys.stderr.flush()
            os._exit(99)
    _, st = os.waitpid(pid, 0)
    return os.WEXITSTATUS(st) if os.WIFEXITED(st) else 100 + os.WTERMSIG(st)

# 1. forked before the parent's first call: a fresh process for the library (NODEV here, not FORKED)
assert fork_and(lambda: 0 if lib.shf_hash_batch_check_device() == hb.ERR_NODEV else 1) == 0, "fresh child"
# 2. the parent uses the library (a host batch: the call reaches HIP and fails with NODEV on this CPU box)
keys = np.zeros(16 * 1000, dtype=np.uint8)
out = np.zeros((1000, 2), dtype=np.uint64)
rc = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, 1000, 12345, out.ctypes.data, hb.MEM_HOST)
assert rc == hb.ERR_NODEV, rc

# 3. a child forked now: every entry point that can reach HIP answers FORKED, with any arguments
def every_entry():
    bad = []
    for f in names:
        fn = getattr(lib, f)
        zero = [None if a in (ctypes.c_void_p, ctypes.c_char_p) or issubclass(a, ctypes._Pointer) else 0
                for a in fn.argtypes]
        r = fn(*zero)
        if r != hb.ERR_FORKED:
            bad.append((f, r))
    # real arguments too: still refused before anything else
    r = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, 1000, 12345, out.ctypes.data, hb.MEM_HOST)
    parts = np.zeros(1000, dtype=np.uint64)
    r2 = lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 16, 1000, 12345, parts.ctypes.data, hb.MEM_HOST)
    if r != hb.ERR_FORKED or r2 != hb.ERR_FORKED:
        bad.append(("real args", r, r2))
    # the exempt ones still work
    m = (ctypes.c_uint16 * 2048)(*([3] * 2048))
    if lib.shf_tab_part_redirect(m, 3, 9) != 0 or list(m[:4]) != [3, 9, 3, 9]:
        bad.append("shf_tab_part_redirect")
    if b"fork" not in lib.shf_hash_batch_strerror(hb.ERR_FORKED):
        bad.append("strerror")
    if bad:
        print(bad, file=sys.stderr, flush=True)
    return 0 if not bad else 1

assert fork_and(every_entry) == 0, "forked child"
# 4. a grandchild too; the parent itself is unchanged (NODEV, not FORKED)
assert fork_and(lambda: fork_and(lambda: 0 if lib.shf_hash_batch_check_device() == hb.ERR_FORKED else 1)) == 0
assert lib.shf_hash_batch_check_device() == hb.ERR_NODEV
print("fork ok: %d entry points refuse in a child" % len(names))
"""


@pytest.mark.skipif(_has_gpu(), reason="forks a process that used the library: CPU box only")
def test_forked_child_gets_an_error_before_any_hip_call():
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT, ",".join(sorted(EXEMPT))], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "fork ok" in p.stdout


def test_every_header_function_is_guarded_or_exempt():
    """The guard's source contract: every extern "C" function of the library
    that is not exempt starts with HB_ENTER()."""
    import re

    src = open(os.path.join(ROOT, "sharedhashfile_amd", "csrc", "shf_hash_batch.hip")).read()
    for name in hb.header_functions():
        m = re.search(r"^(?:int|size_t|const char\*) %s\([^)]*\)\s*\{\s*([^\n]*)" % name, src, re.M)
        assert m, name
        first = m.group(1).strip()
        if name in EXEMPT:
            assert not first.startswith("HB_ENTER();"), name
        else:
            assert first.startswith("HB_ENTER();"), name


def test_forked_error_code_is_named():
    assert hb.ERR_FORKED == -6
    assert "fork" in hb.load().shf_hash_batch_strerror(hb.ERR_FORKED).decode()
