"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU
(SURVEY.md §5 plans ASan/UBSan for host code):

* tests/c/test_host_plan.cpp: the host pipelines' chunk arithmetic and the
  process staging pool (sharedhashfile_amd/csrc/host_plan.h, compiled into the
  product library) -- edge ranges: slots shorter than one key, key lengths and
  batches at the 2^31-byte limit of the reference's `const int len`
  (/root/reference/src/murmurhash3.c:75), 16 threads borrowing slots while the
  slot size changes and allocations fail;
* the same program under ThreadSanitizer (the pool's locking);
* tests/c/test_oracle_asan.c: the C oracle against every golden the reference
  produced (tests/golden/murmur3_golden.json), each key in a buffer of exactly
  its length so a tail over-read is a sanitizer report;
* the seam program (include/shf_hash_batch_shf.h, tests/c/test_seam.c) built the
  same way: on a machine without a GPU it must fail loudly and cleanly; on the
  GPU box tests/test_c_seam.py runs it end to end.

Built by `make -C tests/c sanitize` (gcc/g++, host code only).
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "c", "build")
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def built():
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c"), "sanitize"], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    return BUILD


def _no_reports(p):
    text = p.stdout + p.stderr
    assert "ERROR: AddressSanitizer" not in text and "runtime error:" not in text, text
    assert "ERROR: LeakSanitizer" not in text, text


def test_host_plan_under_sanitizers(built):
    p = subprocess.run([os.path.join(built, "test_host_plan_asan")], capture_output=True, text=True, timeout=300,
                       env=SAN_ENV)
    _no_reports(p)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all checks passed" in p.stdout


def test_host_plan_pool_under_thread_sanitizer(built):
    p = subprocess.run([os.path.join(built, "test_host_plan_tsan")], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert "WARNING: ThreadSanitizer" not in p.stdout + p.stderr, p.stderr
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all checks passed" in p.stdout


def test_oracle_under_sanitizers(built):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "murmur3_golden.json")))
    lines = ["%d %s %s %s" % (c["seed"], c["key_hex"] or "-", c["h1"], c["h2"]) for c in g["cases"]]
    p = subprocess.run([os.path.join(built, "test_oracle_asan")], input="\n".join(lines) + "\n", capture_output=True,
                       text=True, timeout=300, env=SAN_ENV)
    _no_reports(p)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "%d cases" % len(lines) in p.stdout and " 0 mismatches" in p.stdout, p.stdout


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device behaviour")
def test_seam_program_under_sanitizers_without_gpu(built):
    exe = os.path.join(built, "test_seam_asan")
    if not os.path.exists(exe):
        pytest.skip("tests/c/build/test_seam_asan not built (needs /root/reference headers at build time)")
    env = dict(SAN_ENV, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")  # the HIP runtime's own allocations
    p = subprocess.run([exe, "1000"], capture_output=True, text=True, timeout=120, env=env)
    _no_reports(p)
    assert p.returncode == 2 and "no usable GPU" in p.stderr, (p.returncode, p.stdout, p.stderr)
