"""Build the in-tree HIP library (gfx950) and the CPU oracle.

    python -m sharedhashfile_amd.build            # library + oracle (+ reference if present)

The library is a plain hipcc shared object, built in-tree so it travels to the
GPU box with the repository snapshot:
    sharedhashfile_amd/libshf_hash_batch.so   the product (include/shf_hash_batch.h)
    sharedhashfile_amd/libshf_hb_bench.so     bench-only ceiling kernels
                                              (include/shf_hash_batch_ceiling.h), never
                                              linked into the product
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libshf_hash_batch.so")
SOURCES = ["kernels.hip", "shf_hash_batch.hip", "tab_copy.hip", "win_order.hip"]
BENCH_CSRC = os.path.join(PKG, "csrc_bench")
BENCH_LIB = os.path.join(PKG, "libshf_hb_bench.so")
BENCH_SOURCES = ["hbm_ceiling.hip"]
HEADERS = ["kernels.h", "murmur3_mix.h", "win_rank.h", "host_plan.h"]
ARCH = "gfx950"


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _hipcc_shared(sources, headers, out, force, verbose):
    if not force and not _stale(out, sources + headers):
        return out
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fvisibility=hidden", "-Wall", "-I" + os.path.join(ROOT, "include")]
    cmd += sources + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_library(force=False, verbose=True):
    """The product library, then the bench-only ceiling library beside it."""
    inc = os.path.join(ROOT, "include")
    _hipcc_shared([os.path.join(CSRC, s) for s in SOURCES],
                  [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(inc, "shf_hash_batch.h")], LIB, force,
                  verbose)
    _hipcc_shared([os.path.join(BENCH_CSRC, s) for s in BENCH_SOURCES],
                  [os.path.join(inc, h) for h in ("shf_hash_batch.h", "shf_hash_batch_ceiling.h")], BENCH_LIB, force,
                  verbose)
    return LIB


def build_oracle(verbose=True):
    """oracle/_build/liboracle.so always; oracle/_ref/ only where /root/reference exists."""
    cmd = ["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"]
    if os.path.isdir("/root/reference/src"):
        cmd.append("ref")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build_c_tests(verbose=True):
    """tests/c/build/test_seam (the seam proven from C), where the reference's
    headers exist to compile it; elsewhere the prebuilt binary is used."""
    cmd = ["make", "-s", "-C", os.path.join(ROOT, "tests", "c")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    build_library(force="--force" in argv)
    build_oracle()
    build_c_tests()


if __name__ == "__main__":
    main()
