"""Build the in-tree HIP library (gfx950) and the CPU oracle.

    python -m sharedhashfile_amd.build            # library + oracle (+ reference if present)

The library is a plain hipcc shared object, built in-tree so it travels to the
GPU box with the repository snapshot:
    sharedhashfile_amd/libshf_hash_batch.so
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libshf_hash_batch.so")
SOURCES = ["kernels.hip", "shf_hash_batch.hip", "tab_copy.hip", "hbm_ceiling.hip", "win_order.hip"]
HEADERS = ["kernels.h", "murmur3_mix.h"]
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


def build_library(force=False, verbose=True):
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps += [os.path.join(ROOT, "include", h) for h in ("shf_hash_batch.h", "shf_hash_batch_ceiling.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fvisibility=hidden", "-Wall", "-I" + os.path.join(ROOT, "include")]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    cmd += ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
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
