"""The C-ABI library: loads, exports every declared symbol, validates arguments
and fails loudly (never silently on the CPU) when no GPU is present.

No hashing is executed here; parity lives in tests/test_gpu_parity.py (-m gpu).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import sharedhashfile_amd as hbmod

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_library_exports_every_header_symbol(hb):
    declared = hbmod.header_functions()
    assert len(declared) >= 14
    # the product library exports exactly include/shf_hash_batch.h (the .h/.hpp seam headers are static inline)
    out = subprocess.check_output(["nm", "-D", "--defined-only", hbmod.LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    # nothing else leaks out of the shared object (hidden visibility), measurement kernels included
    extra = sorted(s for s in exported if s not in declared)
    assert not extra, extra
    assert not any(s.startswith("shf_hb_ceiling") for s in exported)
    assert "k_ceil" not in subprocess.check_output(["nm", "-C", hbmod.LIB_PATH]).decode()


def test_bench_library_is_separate():
    """The ceiling kernels (include/shf_hash_batch_ceiling.h) live in the
    bench-only libshf_hb_bench.so, which exports only them."""
    from sharedhashfile_amd import bench_ceiling

    ceiling = hbmod.header_functions(os.path.join(ROOT, "include", "shf_hash_batch_ceiling.h"))
    assert ceiling == ["shf_hb_ceiling_async", "shf_hb_host_device_ptr"]
    hbmod.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", bench_ceiling.BENCH_LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert exported == set(ceiling), exported
    assert bench_ceiling.load().shf_hb_ceiling_async(0, None, 0, None, None, 0, None) == hbmod.OK  # n == 0
    assert bench_ceiling.load().shf_hb_ceiling_async(99, 16, 16, None, 16, 1, None) == hbmod.ERR_ARG
    assert bench_ceiling.load().shf_hb_host_device_ptr(None, None) == hbmod.ERR_ARG


def test_header_compiles_as_c():
    src = '#include "shf_hash_batch.h"\nint main(void){ shf_hash128 h; (void)h; return SHF_HB_OK; }\n'
    p = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-x", "c", "-",
                        "-o", "/dev/null"], input=src.encode(), capture_output=True)
    assert p.returncode == 0, p.stderr.decode()


def test_record_layout_matches_shf_hash():
    # SHF_HASH: 16-byte packed union, u64[0]=h1, u64[1]=h2 (shf.private.h:180-185).
    src = ('#include <stddef.h>\n#include "shf_hash_batch.h"\n'
           '_Static_assert(sizeof(shf_hash128) == 16, "size");\n'
           '_Static_assert(offsetof(shf_hash128, h2) == 8, "h2");\n'
           # shf_probe: {uid, pos, mask, tab, slot} = 4 u32 words as the kernels write them
           '_Static_assert(sizeof(shf_probe) == 16, "probe");\n'
           '_Static_assert(offsetof(shf_probe, pos) == 4 && offsetof(shf_probe, mask) == 8, "p1");\n'
           '_Static_assert(offsetof(shf_probe, tab) == 10 && offsetof(shf_probe, slot) == 12, "p2");\n'
           'int main(void){return 0;}\n')
    p = subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-x", "c", "-", "-o", "/dev/null"],
                       input=src.encode(), capture_output=True)
    assert p.returncode == 0, p.stderr.decode()


def test_strerror_and_version(hb):
    lib = hb.load()
    names = {s: lib.shf_hash_batch_strerror(s).decode() for s in (0, -1, -2, -3, -4, -5, -99)}
    assert names[0] == "ok" and names[-99] == "unknown status"
    assert len(set(names.values())) == 7
    assert b"gfx950" in lib.shf_hash_batch_version()


def test_argument_validation_needs_no_device(hb):
    lib = hb.load()
    keys = np.zeros(64, dtype=np.uint8)
    out = np.zeros((4, 2), dtype=np.uint64)
    # n == 0 is a no-op success, whatever the pointers
    assert lib.shf_hash_batch_fixed(None, 16, 0, 12345, None, hbmod.MEM_HOST) == hbmod.OK
    assert lib.shf_hash_batch_var(None, None, 0, 12345, None, hbmod.MEM_DEVICE) == hbmod.OK
    # NULL output / NULL keys with key_len > 0
    assert lib.shf_hash_batch_fixed(keys.ctypes.data, 16, 4, 12345, None, hbmod.MEM_HOST) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_fixed(None, 16, 4, 12345, out.ctypes.data, hbmod.MEM_HOST) == hbmod.ERR_ARG
    # key_len >= 2^31 (reference takes `const int len`, murmurhash3.c:75)
    assert lib.shf_hash_batch_fixed(keys.ctypes.data, 0x80000000, 4, 12345, out.ctypes.data,
                                    hbmod.MEM_HOST) == hbmod.ERR_ARG
    # unknown memory kind
    assert lib.shf_hash_batch_fixed(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, 7) == hbmod.ERR_ARG
    # var: decreasing offsets / too-long key are rejected on the host path
    off = np.array([0, 8, 4], dtype=np.uint64)
    assert lib.shf_hash_batch_var(keys.ctypes.data, off.ctypes.data, 2, 12345, out.ctypes.data,
                                  hbmod.MEM_HOST) == hbmod.ERR_ARG
    off = np.array([0, 1 << 31], dtype=np.uint64)
    assert lib.shf_hash_batch_var(keys.ctypes.data, off.ctypes.data, 1, 12345, out.ctypes.data,
                                  hbmod.MEM_HOST) == hbmod.ERR_ARG
    # forced kernels with shapes they cannot take
    assert lib.shf_hash_batch_fixed_kernel_async(keys.ctypes.data, 17, 3, 12345, out.ctypes.data,
                                                 hbmod.KERNEL_FIXED16, None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_fixed_kernel_async(keys.ctypes.data, 24, 2, 12345, out.ctypes.data,
                                                 hbmod.KERNEL_TILED, None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_fixed_kernel_async(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, 9,
                                                 None) == hbmod.ERR_ARG
    # sized variable-length entry points
    assert lib.shf_hash_batch_var_sized_async(None, None, 0, 0, 12345, None, None) == hbmod.OK
    assert lib.shf_hash_batch_var_sized_async(keys.ctypes.data, None, 2, 16, 12345, out.ctypes.data,
                                              None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_var_sized_kernel_async(keys.ctypes.data, keys.ctypes.data, 2, 16, 12345, None,
                                                     hbmod.KERNEL_SPAN, None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_var_sized_kernel_async(keys.ctypes.data, keys.ctypes.data, 2, 16, 12345,
                                                     out.ctypes.data, hbmod.KERNEL_TILED, None) == hbmod.ERR_ARG
    # row pre-probe: no index / no output / bad handles
    assert lib.shf_probe_batch_fixed_async(None, keys.ctypes.data, 16, 4, 12345, None, out.ctypes.data,
                                           None) == hbmod.ERR_ARG
    assert lib.shf_probe_batch_var_async(None, keys.ctypes.data, keys.ctypes.data, 2, 12345, None,
                                         out.ctypes.data, None) == hbmod.ERR_ARG
    assert lib.shf_probe_batch_hashes_async(None, out.ctypes.data, 4, out.ctypes.data, None) == hbmod.ERR_ARG
    assert lib.shf_probe_batch_hashes_async(None, None, 0, None, None) == hbmod.OK
    assert lib.shf_probe_batch_fixed(None, keys.ctypes.data, 16, 4, 12345, None, out.ctypes.data,
                                     hbmod.MEM_HOST) == hbmod.ERR_ARG
    assert lib.shf_probe_batch_var(None, keys.ctypes.data, keys.ctypes.data, 2, 12345, None, None,
                                   hbmod.MEM_HOST) == hbmod.ERR_ARG
    assert lib.shf_row_index_create(0, None) == hbmod.ERR_ARG
    assert lib.shf_row_index_create(1 << 22, ctypes.byref(ctypes.c_void_p())) == hbmod.ERR_ARG
    assert lib.shf_row_index_destroy(None) == hbmod.OK
    assert lib.shf_row_index_set_tabs(None, keys.ctypes.data) == hbmod.ERR_ARG
    assert lib.shf_row_index_set_rows(None, 0, 1, keys.ctypes.data) == hbmod.ERR_ARG
    assert lib.shf_row_index_device_ptrs(None, None, None, None) == hbmod.ERR_ARG
    # hash + window order: argument checks come before any device work
    perm = np.zeros(4, dtype=np.uint32)
    ws = np.zeros(1 << 20, dtype=np.uint8)
    assert lib.shf_hash_batch_fixed_win_async(None, 16, 0, 12345, None, None, None, None, 0, None) == hbmod.OK
    assert lib.shf_hash_batch_fixed_win_async(keys.ctypes.data, 16, 4, 12345, None, perm.ctypes.data, None,
                                              ws.ctypes.data, ws.size, None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_fixed_win_async(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, perm.ctypes.data,
                                              None, ws.ctypes.data, 16, None) == hbmod.ERR_ARG  # workspace too small
    assert lib.shf_hash_batch_fixed_win_kernel_async(keys.ctypes.data, 17, 3, 12345, out.ctypes.data,
                                                     perm.ctypes.data, None, ws.ctypes.data, ws.size,
                                                     hbmod.KERNEL_FIXED16, None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_var_win_async(keys.ctypes.data, None, 2, 12345, out.ctypes.data, perm.ctypes.data,
                                            None, ws.ctypes.data, ws.size, None) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_fixed_win(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, perm.ctypes.data, None,
                                        7) == hbmod.ERR_ARG
    assert lib.shf_hash_batch_var_win(keys.ctypes.data, None, 2, 12345, out.ctypes.data, perm.ctypes.data, None,
                                      hbmod.MEM_HOST) == hbmod.ERR_ARG


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device behaviour")
def test_no_device_fails_loudly_not_on_cpu(hb):
    lib = hb.load()
    keys = np.zeros(64, dtype=np.uint8)
    out = np.zeros((4, 2), dtype=np.uint64)
    rc = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, hbmod.MEM_HOST)
    assert rc in (hbmod.ERR_NODEV, hbmod.ERR_HIP)
    assert not out.any()  # nothing computed on the CPU behind our back
    assert lib.shf_hash_batch_check_device() in (hbmod.ERR_NODEV, hbmod.ERR_HIP)
    with pytest.raises(hbmod.ShfHashBatchError):
        hbmod.hash_fixed_host(keys.reshape(4, 16))
    assert lib.shf_hash_batch_fixed_multi(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, 0) in (
        hbmod.ERR_NODEV, hbmod.ERR_HIP)
    off = np.array([0, 16, 32], dtype=np.uint64)
    assert lib.shf_hash_batch_var_sized_async(keys.ctypes.data, off.ctypes.data, 2, 32, 12345, out.ctypes.data,
                                              None) in (hbmod.ERR_NODEV, hbmod.ERR_HIP)
    assert not out.any()
    h = ctypes.c_void_p()
    assert lib.shf_row_index_create(4, ctypes.byref(h)) in (hbmod.ERR_NODEV, hbmod.ERR_HIP)
    assert h.value is None
    with pytest.raises(hbmod.ShfHashBatchError):
        hbmod.RowIndex(4)
    prm = hbmod.TabParams(0, 0, 0, 1)
    jobs = (hbmod.TabJob * 1)()
    img = np.zeros(70000, dtype=np.uint8)
    assert lib.shf_tab_copy_batch(img.ctypes.data, img.size, img.ctypes.data, img.size, ctypes.addressof(jobs), 1,
                                  None, 0, ctypes.byref(prm), hbmod.MEM_HOST) in (hbmod.ERR_NODEV, hbmod.ERR_HIP)


def test_missing_library_raises(tmp_path):
    with pytest.raises(RuntimeError):
        hbmod.load(str(tmp_path / "nope.so"))


@pytest.mark.parametrize("source,min_kernels", [("kernels.hip", 30), ("tab_copy.hip", 1),
                                                ("../csrc_bench/hbm_ceiling.hip", 4), ("win_order.hip", 3)])
def test_kernels_compile_without_scratch(source, min_kernels):
    """Every kernel instantiation fits in registers (no scratch spills), as
    reported by hipcc's resource-usage remarks for gfx950."""
    import re
    import shutil
    import tempfile

    from sharedhashfile_amd import build as b

    if not shutil.which(b.hipcc()) and not os.path.exists(b.hipcc()):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        p = subprocess.run([b.hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                            "-I", os.path.join(ROOT, "include"), os.path.join(b.CSRC, source), "-o",
                            os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", p.stderr)]
    assert len(scratch) >= min_kernels and max(scratch) == 0, scratch


def test_no_untested_compile_time_alternates():
    """The library has one build: no preprocessor knob selects an alternative
    kernel body that no test compiles (alternatives live in git history)."""
    import re

    from sharedhashfile_amd import build as b

    for f in sorted(os.listdir(b.CSRC)):
        txt = open(os.path.join(b.CSRC, f)).read()
        conds = re.findall(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b(.*)$", txt, re.M)
        assert not conds, (f, conds)


def test_tab_part_redirect_on_the_host(hb, oracle):
    """shf_tab_part_redirect is host code (no device needed): the oracle's
    restatement of shf.c:683-692 on maps with 1-3 tabs."""
    lib = hb.load()
    rng = np.random.default_rng(9)
    for tabs in (1, 2, 3):
        m = (np.arange(2048) % tabs).astype(np.uint16)
        rng.shuffle(m)
        for old in range(tabs):
            got = hbmod.tab_part_redirect(m, old, tabs)
            assert np.array_equal(got, oracle.tab_part_redirect(m, old, tabs))
            assert (got == tabs).sum() == (m == old).sum() // 2
    m = np.zeros(2048, dtype=np.uint16)
    assert lib.shf_tab_part_redirect(None, 0, 1) == hbmod.ERR_ARG
    assert lib.shf_tab_part_redirect(m.ctypes.data, 3, 3) == hbmod.ERR_ARG
    assert lib.shf_tab_part_redirect(m.ctypes.data, 0, 2048) == hbmod.ERR_ARG


def test_tab_copy_argument_validation_needs_no_device(hb):
    lib = hb.load()
    prm = hbmod.TabParams(0, 0, 0, 1)
    buf = np.zeros(16, dtype=np.uint8)
    assert lib.shf_tab_copy_batch(None, 0, None, 0, None, 0, None, 0, None, hbmod.MEM_HOST) == hbmod.OK  # no jobs
    assert lib.shf_tab_copy_batch(None, 16, buf.ctypes.data, 16, buf.ctypes.data, 1, None, 0, ctypes.byref(prm),
                                  hbmod.MEM_HOST) == hbmod.ERR_ARG
    assert lib.shf_tab_copy_batch(buf.ctypes.data, 16, buf.ctypes.data, 16, buf.ctypes.data, 1, None, 0, None,
                                  hbmod.MEM_HOST) == hbmod.ERR_ARG
    assert lib.shf_tab_copy_batch(buf.ctypes.data, 16, buf.ctypes.data, 16, buf.ctypes.data, 1, None, 0,
                                  ctypes.byref(prm), 7) == hbmod.ERR_ARG
    assert lib.shf_tab_copy_batch_async(None, 0, buf.ctypes.data, 16, buf.ctypes.data, 1, None, 0,
                                        ctypes.byref(prm), None) == hbmod.ERR_ARG
